// ngs_abi.cpp — the C ABI (include/ngram_search.h): handle registry, device residency of the
// index, per-call search contexts (stream + scratch) and result marshalling.
//
// Mirrors nGramSearch/dllmain.cpp (paths under /root/reference): the global shared_mutex
// (:22), smallest-free-handle allocation (:41-46), shared locks for searches (:63,84,100,122,
// 135,147) and exclusive locks for indexN/dispose (:39,112).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/ngram_search.h"
#include "ngs_build.h"
#include "ngs_index.h"
#include "ngs_kernels.h"

namespace ngs {
namespace {

constexpr char kDefaultValid[] = ".%$ @0123456789abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ";
constexpr uint32_t kInt32Max = (uint32_t)std::numeric_limits<int32_t>::max();
constexpr size_t kOutBudget = size_t(1) << 30;       // bytes of (key, score) output per chunk
constexpr size_t kGeneralBudget = size_t(2) << 30;   // bytes of dense general-path state
constexpr uint32_t kSmallBatch = 16;                 // host batches up to this many queries take the latency path
constexpr size_t kSmallBlock = size_t(1) << 20;      // ... if their output block is at most this many bytes
constexpr size_t kPartBudget = size_t(1) << 30;      // bytes of sliced tier-1b partial results per call
constexpr uint32_t kSmallSlices = 32;                // ... or term-id slices per query (sliced k_wave)
constexpr size_t kSmallQ = size_t(64) << 10;         // ... and if their offsets + bytes fit this many bytes
// the latency path's one block, device and pinned host: statistics | results | queries
constexpr size_t kSioStats = sizeof(DevStats) * (kStatSlots + 1);
constexpr size_t kSioBytes = kSioStats + kSmallBlock + kSmallQ;
constexpr int kRetryQcap = -6;                       // finish_search: rerun with the batch's byte count
constexpr uint32_t kCalmCalls = 16;                  // grown survivor slots unused this many calls: halved

// the last HIP failure on this thread (ngsLastError): the reference's entry points answer 0 on
// failure, indistinguishable from "no results", so callers that care ask afterwards
thread_local int t_last_error = 0;
// failures that are not HIP errors (include/ngram_search.h: NGS_ERR_*)
constexpr int kErrInternal = 0x10001;     // a kernel reported an internal error (finish_search -5)
constexpr int kErrQueryBuffer = 0x10002;  // the batch outgrew the normalised-query buffer twice

bool hip_ok(hipError_t e, const char* what) {
    if (e == hipSuccess) return true;
    std::fprintf(stderr, "ngram_search: %s failed: %s\n", what, hipGetErrorString(e));
    t_last_error = (int)e;
    return false;
}
#define HIP_CHECK(expr) hip_ok((expr), #expr)

// Phases of the host batch path (scoreBatch / searchBatch): nanoseconds summed over the calls since
// the last reset, read by ngsHostPhases (bench.py's detail.dropin). NGS_HOST_TIMING=1 also prints
// each phase (microseconds since the previous mark) to stderr.
enum HostPhase : int {
    kHpPack = 0,      // query lengths, offsets and bytes packed into pinned staging
    kHpQueue,         // H2D copies and the kernels queued
    kHpWait,          // the kernels, waited for
    kHpPackBack,      // the device pack of the results and the offsets back
    kHpRecords,       // the records back, marshalled into the new[]'d arrays as they land
    kHpCall,          // the whole call (scoreBatch / searchBatch)
    kHpCalls,         // (count) calls
    kHpReplays,       // (count) one-stream calls replayed from a graph (queue_search)
    kHpN
};
std::atomic<uint64_t> g_host_phase[kHpN];
struct HostTimer {
    bool on;
    std::chrono::steady_clock::time_point t;
    HostTimer() : on(std::getenv("NGS_HOST_TIMING") != nullptr), t(std::chrono::steady_clock::now()) {}
    void mark(int id, const char* what) {
        const auto n = std::chrono::steady_clock::now();
        g_host_phase[id].fetch_add((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(n - t).count(),
                                   std::memory_order_relaxed);
        if (on)
            std::fprintf(stderr, "[ngs host] %-28s %9.1f us\n", what,
                         std::chrono::duration<double, std::micro>(n - t).count());
        t = n;
    }
};

// Largest host batch (queries x limit entries) whose result arrays are allocated at capacity and
// filled as chunks finish (batch_query); larger ones collect the records first
constexpr uint64_t kDirectMax = uint64_t(1) << 25;


// body(lo, hi) over [0, n) on up to 8 host threads (one below `serial_below` items)
// A fixed pool of host worker threads for the batch path's packing and marshalling: spawning
// eight threads per use cost ~50 us each time (the pool's workers wait on a condition variable).
class HostPool {
  public:
    static HostPool& get() {
        static HostPool p;
        return p;
    }
    size_t size() const { return workers_.size() + 1; }
    // runs task(i) for i in [0, n) on the workers and the caller; returns when all are done
    void run(size_t n, const std::function<void(size_t)>& task) {
        std::unique_lock<std::mutex> lk(mu_);
        busy_.wait(lk, [&] { return !task_; });  // one parallel section at a time
        task_ = &task;
        n_ = n;
        next_ = 0;
        left_ = n;
        ++gen_;
        work_.notify_all();
        while (next_ < n_) {  // the caller takes items too
            const size_t i = next_++;
            lk.unlock();
            task(i);
            lk.lock();
            --left_;
        }
        done_.wait(lk, [&] { return left_ == 0; });
        task_ = nullptr;
        busy_.notify_all();
    }

  private:
    HostPool() {
        const size_t nt = std::min<size_t>(8, std::max(1u, std::thread::hardware_concurrency()));
        for (size_t t = 1; t < nt; ++t) workers_.emplace_back([this] { loop(); });
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            quit_ = true;
        }
        work_.notify_all();
        for (auto& w : workers_) w.join();
    }
    void loop() {
        std::unique_lock<std::mutex> lk(mu_);
        uint64_t seen = 0;
        for (;;) {
            work_.wait(lk, [&] { return quit_ || (task_ && gen_ != seen && next_ < n_); });
            if (quit_) return;
            seen = gen_;
            while (task_ && next_ < n_) {
                const size_t i = next_++;
                const std::function<void(size_t)>* t = task_;
                lk.unlock();
                (*t)(i);
                lk.lock();
                if (--left_ == 0) done_.notify_all();
            }
        }
    }
    std::vector<std::thread> workers_;
    std::mutex mu_;
    std::condition_variable work_, done_, busy_;
    const std::function<void(size_t)>* task_ = nullptr;
    size_t n_ = 0, next_ = 0, left_ = 0;
    uint64_t gen_ = 0;
    bool quit_ = false;
};

// body(lo, hi) over [0, n) on the host pool (serially below `serial_below` items)
template <class F>
void parallel_ranges(size_t n, size_t serial_below, F&& body) {
    HostPool& pool = HostPool::get();
    const size_t nt = n < serial_below ? 1 : pool.size();
    if (nt <= 1) {
        body(size_t(0), n);
        return;
    }
    const std::function<void(size_t)> task = [&](size_t t) { body(n * t / nt, n * (t + 1) / nt); };
    pool.run(nt, task);
}

// Persistent host threads for the parts of a batch split over replicas (dllmain.cpp:82-90 callers
// on an index placed on several devices): part 0 runs on the calling thread, part i on worker i - 1,
// each on its replica's device and contexts. One split at a time; a call that finds the workers
// busy (another thread's split) spawns threads of its own for that call.
class PartWorkers {
  public:
    explicit PartWorkers(size_t n) : n_(n), todo_(n, false) {
        for (size_t i = 0; i < n; ++i) th_.emplace_back([this, i] { loop(i); });
    }
    ~PartWorkers() {
        {
            std::lock_guard<std::mutex> g(mu_);
            quit_ = true;
        }
        work_.notify_all();
        for (auto& t : th_) t.join();
    }
    size_t size() const { return n_; }
    // f(i) for i in [0, parts): i = 0 here, the rest on the workers; false if busy (nothing ran)
    bool try_run(size_t parts, const std::function<void(size_t)>& f) {
        std::unique_lock<std::mutex> call(call_mu_, std::try_to_lock);
        if (!call.owns_lock() || parts > n_ + 1) return false;
        {
            std::lock_guard<std::mutex> g(mu_);
            f_ = &f;
            left_ = parts - 1;
            for (size_t i = 0; i + 1 < parts; ++i) todo_[i] = true;
        }
        work_.notify_all();
        f(0);
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [&] { return left_ == 0; });
        f_ = nullptr;
        return true;
    }

  private:
    void loop(size_t i) {
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            work_.wait(lk, [&] { return quit_ || todo_[i]; });
            if (quit_) return;
            todo_[i] = false;
            const std::function<void(size_t)>* f = f_;
            lk.unlock();
            (*f)(i + 1);
            lk.lock();
            if (--left_ == 0) done_.notify_all();
        }
    }
    size_t n_;
    std::vector<char> todo_;
    std::vector<std::thread> th_;
    std::mutex mu_, call_mu_;
    std::condition_variable work_, done_;
    const std::function<void(size_t)>* f_ = nullptr;
    size_t left_ = 0;
    bool quit_ = false;
};

// f(i) for the parts of a split: on the library's persistent workers, or threads of this call's own
template <class Workers>
void run_parts(Workers& w, size_t parts, const std::function<void(size_t)>& f) {
    if (w && w->try_run(parts, f)) return;
    std::vector<std::thread> th;
    for (size_t i = 1; i < parts; ++i) th.emplace_back(f, i);
    f(0);
    for (auto& t : th) t.join();
}

template <class T>
bool dev_alloc(T** p, size_t n) {
    *p = nullptr;
    return HIP_CHECK(hipMalloc((void**)p, std::max<size_t>(n, 1) * sizeof(T)));
}

template <class T>
bool dev_upload(T** p, const std::vector<T>& v, std::vector<void*>& owned, size_t pad = 0) {
    if (!dev_alloc(p, v.size() + pad)) return false;
    owned.push_back(*p);
    if (pad && !HIP_CHECK(hipMemset(*p + v.size(), 0, pad * sizeof(T)))) return false;
    return v.empty() || HIP_CHECK(hipMemcpy(*p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
}

// A page-locked host buffer, grown geometrically: the host entry points stage queries and
// results through these (asynchronous DMA at full PCIe rate instead of pageable bounce copies).
struct Pinned {
    void* p = nullptr;
    size_t cap = 0;
    bool grow(size_t bytes) {
        if (bytes <= cap) return true;
        const size_t nb = std::max<size_t>(bytes, cap * 2);
        if (p) hipHostFree(p);
        p = nullptr;
        cap = 0;
        if (!HIP_CHECK(hipHostMalloc(&p, std::max<size_t>(nb, 64), hipHostMallocDefault))) return false;
        cap = nb;
        return true;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
    ~Pinned() {
        if (p) hipHostFree(p);
    }
};

struct Context {
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t side = nullptr;      // the heavy list (cmin 2) beside tier 1a
    hipStream_t side2 = nullptr;     // tier 1b on the full list (cmin 1, short search) beside both
    hipEvent_t join = nullptr, join2 = nullptr;
    hipEvent_t prep_ev = nullptr, lists_ev = nullptr;  // k_prep done (s), heavy / full lists merged (side)
    hipEvent_t in_ev = nullptr;   // ngsSearchDeviceAsync: the caller's stream up to the call
    // d_stats needs no reset before the next call's k_prep (kPrepZero): k_prep zeroes the statistics
    // and the path counts, k_lists the list counters after reading them; false until a call has
    // queued both, and after a call that flagged *oflow
    bool stats_clean = false;
    hipEvent_t ev[6] = {};
    hipEvent_t piece_ev[kBackPieces] = {};  // finish_host_chunk: the read-back's pieces landed
    size_t qcap = 0, bcap = 0, ncap = 0, ocap = 0;
    uint32_t ecap = kEmitCap;  // survivor slots per query in d_est / d_esc (ensure_queries, emit_cap)
    uint32_t ecap_grow = 0;    // slots later calls ask for: raised when tier 1a ran out of them
    size_t ebcap = 0;          // ... for this many queries
    uint32_t calm = 0;         // calls in a row with grown slots that no query filled
    bool shrink = false;       // ... enough of them: the next call gives half the slots back
    uint8_t* d_raw = nullptr;
    uint64_t* d_off = nullptr;
    uint8_t* d_norm = nullptr;
    uint32_t* d_qm = nullptr;
    uint32_t* d_glist = nullptr;
    uint32_t* d_list2 = nullptr;
    uint32_t* d_gcount = nullptr;  // [0] general-path count, [1] tier-2 count, [2] tier-1b hand-overs, [3] heavy,
                                   // [4] hand-overs of the heavy list's lean launch, [5] full list,
                                   // [6] k_prep: a query past the normalised-query buffer (qcap)
    uint32_t* d_fb = nullptr;      // queries tier 1a handed to tier 1b
    uint32_t* d_fb2 = nullptr;     // ... from the heavy list (side stream)
    uint32_t* d_heavy = nullptr;   // queries the prep kernel listed as heavy (cmin 2)
    uint32_t* d_full = nullptr;    // ... for tier 1b (cmin 1, short search)
    uint32_t* d_lslots = nullptr;  // k_prep's slot lists of both (2 * kListSlots * ceil(B / kListSlots))
    uint32_t* d_esn = nullptr;     // tier 1a survivor lists for k_emit: count per query,
    uint32_t* d_est = nullptr;     // kEmitCap terms and
    uint8_t* d_esc = nullptr;      // kEmitCap hit counts per query
    // the survivor arena (SearchParams.at): ablocks blocks of kArenaBlock entries, a chain link per
    // block and a first block per query (ebcap rows); grown (arena_grow) after a call ran out of it
    uint32_t* d_eovf = nullptr;
    uint32_t* d_anext = nullptr;
    uint32_t* d_at = nullptr;
    uint8_t* d_ac = nullptr;
    uint32_t ablocks = 0, arena_grow = 0;
    // arena_calm: calls in a row that used under a quarter of a grown arena (kCalmCalls: halved);
    // arena_off: calls left to run without an arena after its allocation failed
    uint32_t arena_calm = 0, arena_off = 0, arena_shrink_to = 0;
    uint32_t heavy_items = 0;      // (query, slice) items of the last call's heavy launch (SearchParams.hgrid)
    size_t eorows = 0;
    uint64_t* d_prec = nullptr;    // sliced tier 1b: top-L records per (query, slice)
    uint32_t* d_pcnt = nullptr;    // ... and their counts
    size_t pcap = 0, pncap = 0;    // records d_prec holds, counts d_pcnt holds
    uint32_t* d_group = nullptr;
    // kStatSlots slots, then one holding d_gcount (one memset, one read-back), then the
    // 2 * kListSlots counter lines of k_prep's slot lists (d_lctr; same memset, not read back)
    DevStats* d_stats = nullptr;
    uint32_t* d_lctr = nullptr;
    DevStats* h_stats = nullptr;   // pinned host copy of the same
    // host-path outputs, one block holding [n (B + 1) | k (B * stride) | s (B * stride)] for the
    // call's B and stride, so that a small batch reads all of it back in one copy; packed copies
    // (launch_pack) for large batches
    uint32_t* d_out = nullptr;
    uint32_t* d_n = nullptr;
    uint32_t* d_k = nullptr;
    float* d_s = nullptr;
    uint32_t* d_pos = nullptr;  // [ncap + 1] packed offsets
    uint32_t* d_pk = nullptr;   // [2 * ocap] packed keys, or (pointer mode) u64 result pointers
    float* d_ps = nullptr;      // [ocap] packed scores
    void* d_ptemp = nullptr;    // scan scratch
    size_t ptemp_bytes = 0;
    GeneralBuffers gen;
    Pinned h_off, h_raw, h_res;  // queries in; results out
    uint8_t* d_sio = nullptr;     // the latency path's block (kSioBytes): one copy in, one copy out
    uint8_t* h_sio = nullptr;     // ... its pinned host image
    // one-stream calls (queue_search): calls built as graphs, replayed when a call's launch
    // arguments (the signature) repeat one of them; gseen: recent signatures, a call is built on
    // its second occurrence. Up to kGraphs of each (a pipelined caller rotates its output buffers
    // over the contexts in flight: C2's bench loop, 4 buffers over 3 contexts)
    static constexpr size_t kGraphs = 8;
    std::vector<std::pair<std::vector<uint8_t>, hipGraphExec_t>> graphs;
    std::vector<std::vector<uint8_t>> gseen;
    bool gfail = false;  // a graph failed to build: this context queues its calls one by one

    ~Context() {
        hipSetDevice(device);
        for (void* p : {(void*)d_raw, (void*)d_off, (void*)d_norm, (void*)d_qm, (void*)d_glist, (void*)d_list2, (void*)d_fb, (void*)d_fb2, (void*)d_heavy, (void*)d_full, (void*)d_lslots,
                        (void*)d_esn, (void*)d_est, (void*)d_esc, (void*)d_prec, (void*)d_pcnt,
                        (void*)d_eovf, (void*)d_anext, (void*)d_at, (void*)d_ac,
                        (void*)d_group, (void*)d_stats, (void*)d_sio, (void*)d_out, (void*)d_pos, (void*)d_pk, (void*)d_ps, d_ptemp, (void*)gen.cnt,
                        (void*)gen.kenc, (void*)gen.list, (void*)gen.sorted, (void*)gen.lcount, gen.temp})
            if (p) hipFree(p);
        for (auto& g : graphs) hipGraphExecDestroy(g.second);
        if (h_stats) hipHostFree(h_stats);
        if (h_sio) hipHostFree(h_sio);
        for (hipEvent_t e : ev)
            if (e) hipEventDestroy(e);
        for (hipEvent_t e : {join, join2, prep_ev, lists_ev, in_ev})
            if (e) hipEventDestroy(e);
        for (hipEvent_t e : piece_ev)
            if (e) hipEventDestroy(e);
        if (stream) hipStreamDestroy(stream);
        if (side && side != stream && !side_shared) hipStreamDestroy(side);
        if (side2 && side2 != side && side2 != stream) hipStreamDestroy(side2);
    }
    bool side_shared = false;  // side is the replica's (shared by its contexts)
};

// The side stream runs the heavy list's chain and then the full list's tier 1b (cmin 1, short
// search) beside tier 1a, at normal priority (at the highest one the main launches' streams starved:
// rejected in round 1 and again in round 5). A third stream per context for the full list made one
// context's main stream share a hardware queue (HIP's default is four, one of them the null
// stream's) with the other's side work (a pipelined scoreBatch measured 2x slower that way); the
// side stream is also shared by the replica's contexts (queue_search).
hipError_t make_side_stream(hipStream_t* s) { return hipStreamCreateWithFlags(s, hipStreamNonBlocking); }

// One copy of the index in one device's HBM, with its pool of per-call contexts. An index built
// after ngsSetDevices has one replica per listed device; batches are split across them.
struct Replica {
    int device = 0;
    DevIndex dev{};
    const float* wild_w = nullptr;  // the keys' wildcard weights (ngsSaveIndex reads them back)
    std::vector<void*> owned;
    std::mutex pool_mu;
    std::vector<std::unique_ptr<Context>> pool;
    // DevIndex.kt_flag per validChar set in use (indexes with kt_off only): made once per set, kept
    // until dispose (a launch in flight may still read an older set's)
    std::mutex kflag_mu;
    std::vector<std::pair<std::array<uint32_t, 8>, uint8_t*>> kflags;
    // the last main tier-1a launch of any call on this replica (launch_fast orders the next after it)
    std::mutex main_mu;
    hipEvent_t main_ev = nullptr;
    bool main_rec = false;
    hipStream_t shared_side = nullptr;  // one side stream for every context (made under main_mu)

    // the index as the kernels of a search under `valid` see it (kt_flag for that set); false on a
    // HIP failure
    bool index_for(const uint32_t valid[8], DevIndex& X) {
        X = dev;
        X.kt_flag = nullptr;
        if (!dev.kt_off) return true;
        std::array<uint32_t, 8> v;
        std::copy(valid, valid + 8, v.begin());
        std::lock_guard<std::mutex> g(kflag_mu);
        for (auto& e : kflags)
            if (e.first == v) {
                X.kt_flag = e.second;
                return true;
            }
        uint8_t* f = nullptr;
        if (!HIP_CHECK(hipSetDevice(device)) || !HIP_CHECK(hipMalloc(&f, std::max<size_t>(dev.n_keys, 1)))) return false;
        owned.push_back(f);
        // synchronously: a search on another stream may use the set as soon as it is listed
        if (!HIP_CHECK(build_key_flags(dev, valid, f, nullptr)) || !HIP_CHECK(hipStreamSynchronize(nullptr))) return false;
        kflags.emplace_back(v, f);
        X.kt_flag = f;
        return true;
    }

    ~Replica() {
        pool.clear();
        hipSetDevice(device);
        if (main_ev) hipEventDestroy(main_ev);
        if (shared_side) hipStreamDestroy(shared_side);
        for (void* p : owned) hipFree(p);
    }

    std::unique_ptr<Context> acquire() {
        {
            std::lock_guard<std::mutex> g(pool_mu);
            if (!pool.empty()) {
                auto c = std::move(pool.back());
                pool.pop_back();
                return c;
            }
        }
        auto c = std::make_unique<Context>();
        c->device = device;
        // (the side streams are made by the first call whose batch needs them, queue_search)
        if (!HIP_CHECK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) ||
            !HIP_CHECK(hipEventCreateWithFlags(&c->join, hipEventDisableTiming)) ||
            !HIP_CHECK(hipEventCreateWithFlags(&c->join2, hipEventDisableTiming)) ||
            !HIP_CHECK(hipEventCreateWithFlags(&c->prep_ev, hipEventDisableTiming)) ||
            !HIP_CHECK(hipEventCreateWithFlags(&c->lists_ev, hipEventDisableTiming)) ||
            !HIP_CHECK(hipEventCreateWithFlags(&c->in_ev, hipEventDisableTiming)))
            return nullptr;
        for (hipEvent_t& e : c->ev)
            if (!HIP_CHECK(hipEventCreate(&e))) return nullptr;
        for (hipEvent_t& e : c->piece_ev)
            if (!HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming))) return nullptr;
        if (!dev_alloc(&c->d_group, kGeneralMaxGroup) || !dev_alloc(&c->d_stats, kStatSlots + 1 + 2 * kListSlots) ||
            !dev_alloc(&c->d_sio, kSioBytes) ||
            !HIP_CHECK(hipMemsetAsync(c->d_sio, 0, kSioStats, c->stream)) ||
            !HIP_CHECK(hipStreamSynchronize(c->stream)) ||
            !HIP_CHECK(hipHostMalloc((void**)&c->h_sio, kSioBytes, hipHostMallocDefault)) ||
            !HIP_CHECK(hipHostMalloc((void**)&c->h_stats, sizeof(DevStats) * (kStatSlots + 1), hipHostMallocDefault)))
            return nullptr;
        c->d_gcount = reinterpret_cast<uint32_t*>(c->d_stats + kStatSlots);
        c->d_lctr = reinterpret_cast<uint32_t*>(c->d_stats + kStatSlots + 1);
        static_assert(sizeof(DevStats) == 16 * sizeof(uint32_t), "k_prep's counters are 16 words apart");
        static_assert(sizeof(DevStats) >= 7 * sizeof(uint32_t), "the path counts fit one stats slot");
        return c;
    }
    void give_back(std::unique_ptr<Context> c) {
        std::lock_guard<std::mutex> g(pool_mu);
        pool.push_back(std::move(c));
    }
};

// ngsServe: the low-latency score() path. A persistent kernel (k_serve) on a stream of its own,
// one wave per request slot, polls request blocks in coherent pinned host memory; score() takes a
// free slot, writes the normalised query there, publishes a request number and spins until the
// kernel publishes it back with the results: no launch, no copy, no stream wait per call, and up
// to kServeSlots callers served side by side. The kernel exits on stop, after kServeIdleMs without
// a request or after kServeLifeMs, and is relaunched on demand.
constexpr uint32_t kServeIdleMs = 200;
constexpr uint32_t kServeLifeMs = 10000;
// score()/search() start the server by themselves (no ngsServe call) from this many single-query
// calls on a library the server can answer (fewer than 16 skip buckets, narrow strings)
constexpr uint32_t kAutoServeAfter = 4;

struct Server {
    int device = 0;
    hipStream_t stream = nullptr;
    ServeBlock* h = nullptr;  // kServeSlots request blocks, coherent pinned host memory
    ServeBlock* d = nullptr;  // their device view
    DevStats* scratch = nullptr;
    uint32_t* list2 = nullptr;
    unsigned long long* t_any = nullptr;  // the latest request time of any slot (device memory)
    uint64_t seq[kServeSlots] = {};
    std::mutex slot_mu[kServeSlots];  // one request per slot at a time
    std::mutex launch_mu;             // one (re)launch at a time
    std::atomic<bool> launched{false};
    uint32_t launch_valid[8] = {};  // the validChar set of its DevIndex.kt_flag

    bool init(int dev) {
        device = dev;
        const size_t nst = (size_t)kServeSlots * (kStatSlots + 1);
        if (!HIP_CHECK(hipSetDevice(dev)) || !HIP_CHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking)) ||
            !HIP_CHECK(hipHostMalloc((void**)&h, sizeof(ServeBlock) * kServeSlots,
                                     hipHostMallocCoherent | hipHostMallocMapped)) ||
            !HIP_CHECK(hipHostGetDevicePointer((void**)&d, h, 0)) ||
            !HIP_CHECK(hipMalloc((void**)&scratch, sizeof(DevStats) * nst)) ||
            !HIP_CHECK(hipMalloc((void**)&list2, sizeof(uint32_t) * 4 * kServeSlots)) ||
            !HIP_CHECK(hipMalloc((void**)&t_any, sizeof(unsigned long long))))
            return false;
        std::memset((void*)h, 0, sizeof(ServeBlock) * kServeSlots);
        return HIP_CHECK(hipMemset(scratch, 0, sizeof(DevStats) * nst)) &&
               HIP_CHECK(hipMemset(t_any, 0, sizeof(unsigned long long)));
    }
    // the kernel has left (idle, lifetime, stop) or was never launched
    bool stopped() { return !launched || hipStreamQuery(stream) == hipSuccess; }
    void stop() {
        if (!h) return;
        __atomic_store_n(&h->stop, 1u, __ATOMIC_RELEASE);
        if (stream) hipStreamSynchronize(stream);  // it exits within one poll
        launched = false;
        __atomic_store_n(&h->stop, 0u, __ATOMIC_RELEASE);
    }
    ~Server() {
        if (h) stop();
        hipSetDevice(device);
        if (stream) hipStreamDestroy(stream);
        if (h) hipHostFree(h);
        if (scratch) hipFree(scratch);
        if (list2) hipFree(list2);
        if (t_any) hipFree(t_any);
    }
};

struct Library {
    std::unique_ptr<Server> server;  // ngsServe (null: off)
    std::atomic<bool> serving{false};  // server != null, for the unlocked test in one_query
    std::shared_mutex server_mu;     // creating / dropping / stopping it (exclusive); requests (shared)
    std::atomic<int> serve_pref{0};  // 0: automatic (kAutoServeAfter), 1: ngsServe(h, 1), -1: ngsServe(h, 0)
    std::atomic<uint32_t> single_calls{0};  // score()/search() calls so far (automatic start)
    // batch calls in flight: the server kernel is stopped while any runs and not relaunched until
    // they are done, so no batch kernel queues behind it on a shared hardware queue
    std::atomic<int> batches{0};
    HostIndex host;
    int device = 0;                              // first replica's device (or the build device)
    std::vector<std::unique_ptr<Replica>> reps;  // empty until the index is on a GPU
    std::mutex valid_mu;
    uint32_t valid[8] = {};
    std::atomic<bool> timing{false};
    std::mutex stats_mu;
    ngs_stats last{};
    bool tk_identity = false;  // DevIndex.tk_identity / tk_monotone / w_max, computed once for every replica
    bool tk_monotone = false;
    float w_max = 0.0f;
    bool rank_lists = false;   // DevIndex.rank_post: one weight (w_uniform), one pair per term, one term per key
    uint32_t w_uniform = 0;
    // DevIndex.kt_off / kt_term (keys with several pairs), built once in upload() for every replica
    std::vector<uint32_t> kt_off, kt_term;
    // the replicas a batch is split over (upload), and host threads for its parts past the first
    std::vector<uint32_t> split;
    std::unique_ptr<PartWorkers> workers;

    // ngsSearchDeviceAsync calls in flight: their context stays out of the pool until
    // ngsSearchDeviceWait (the general path and the statistics need the host afterwards)
    struct Pending {
        Replica* R = nullptr;
        std::unique_ptr<Context> c;
        SearchParams P{};
        const uint8_t* dq = nullptr;
        const uint64_t* doff = nullptr;
        uint32_t B = 0, Lm = 0, stride = 0;
        float thr = 0;
        uint32_t *dn = nullptr, *dk = nullptr;
        float* ds = nullptr;
        int rc = 0;  // queueing already failed
    };
    std::mutex pend_mu;
    std::unordered_map<uint64_t, Pending> pending;
    uint64_t next_ticket = 1;

    ~Library() {
        workers.reset();  // (idle: dispose holds the exclusive lock, so no split is running)
        server.reset();  // stops the kernel before the index it reads is freed
        for (auto& kv : pending)  // dispose: nothing may still run on the buffers freed below
            if (kv.second.c) hipStreamSynchronize(kv.second.c->stream);
        pending.clear();
        reps.clear();
    }
    // the replica on `dev`, or null
    Replica* replica_at(int dev) {
        for (auto& r : reps)
            if (r->device == dev) return r.get();
        return nullptr;
    }
};

std::shared_mutex g_lock;                                        // dllmain.cpp:22
std::unordered_map<uint32_t, std::unique_ptr<Library>> g_libs;   // dllmain.cpp:24
thread_local std::vector<int> t_devices;                          // ngsSetDevice(s): this thread's next builds

Library* find_lib(uint32_t h) {
    auto it = g_libs.find(h);
    return it == g_libs.end() ? nullptr : it->second.get();
}

// Places one copy of the host-built index on device R.device. The host arrays stay until every
// replica is uploaded (free_uploaded).
// `first`: the first replica settles the host index's gram fields (or builds the gram CSR on the
// host when the device build fails); later replicas are placed concurrently and only read them.
bool upload_replica(Library& L, Replica& R, bool keys_unique, bool first) {
    if (!HIP_CHECK(hipSetDevice(R.device))) return false;
    HostIndex& H = L.host;
    DevIndex& X = R.dev;
    X.n_terms = H.n_terms;
    X.n_short = H.n_short;
    X.n_keys = H.n_keys;
    X.keys_unique = keys_unique ? 1u : 0u;
    X.tk_identity = L.tk_identity ? 1u : 0u;
    X.tk_monotone = L.tk_monotone ? 1u : 0u;
    X.w_max = L.w_max;
    const std::vector<char>& kb = H.key_bytes;
    uint64_t *gram_off, *term_off, *key_off;
    uint32_t *post, *tk_off, *wild_key, *gram_row, *skip;
    uint8_t* term_bytes;
    char* key_bytes;
    uint2* tk;
    float *wild_w, *wild_score;
    // from here on the replica's destructor frees what was allocated
    PhaseTimer pt;
    bool ok = dev_upload(&term_off, H.term_off, R.owned) && dev_upload(&term_bytes, H.term_bytes, R.owned, 8) /* whole dwords, and a short term's second dword (myers_short) */ &&
              dev_upload(&tk_off, H.tk_off, R.owned) && dev_upload(&tk, H.tk, R.owned) &&
              dev_upload(&key_off, H.key_off, R.owned) && dev_upload(&key_bytes, kb, R.owned) &&
              dev_upload(&wild_w, H.wild_w, R.owned);
    if (!ok) return false;
    pt.mark("replica: arrays to HBM");
    bool dev_built = false;
    uint64_t n_post = H.post.size();
    if (!H.grams_built) {
        // the gram CSR and skip table from the terms now in HBM (ngs_build.hip); dictionary
        // indexes first find their distinct gram keys there and the host lays out the lookup table
        // from them (the first replica; the others reuse it). On failure the host builds them.
        DeviceGrams dg;
        const auto t0 = std::chrono::steady_clock::now();
        hipError_t e = hipSuccess;
        uint64_t* dict = nullptr;
        if (H.gram_mode == 1) {
            if (first) {
                std::vector<uint64_t> keys;
                e = gram_keys_device(term_off, term_bytes, H.n_short, H.n_terms, H.csize, H.gsz, keys);
                if (e == hipSuccess) set_gram_dict(H, std::move(keys));
            }
            if (e == hipSuccess) e = hipMalloc(&dict, sizeof(uint64_t) * std::max<size_t>(H.gram_keys.size(), 1));
            if (e == hipSuccess && !H.gram_keys.empty())
                e = hipMemcpy(dict, H.gram_keys.data(), sizeof(uint64_t) * H.gram_keys.size(), hipMemcpyHostToDevice);
        }
        if (e == hipSuccess)
            e = build_grams_device(term_off, term_bytes, H.n_short, H.n_terms, dg, dict, (uint32_t)H.gram_keys.size(),
                                   H.csize, H.gsz);
        if (dict) (void)hipFree(dict);
        if (std::getenv("NGS_BUILD_TIMING"))
            std::fprintf(stderr, "[ngs build] %-22s %8.3f s\n", "gram CSR + skip (GPU)",
                         std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
        if (e == hipSuccess) {
            for (void* p : {(void*)dg.gram_off, (void*)dg.post, (void*)dg.gram_row, (void*)dg.skip}) R.owned.push_back(p);
            gram_off = dg.gram_off;
            post = dg.post;
            gram_row = dg.gram_row;
            skip = dg.skip;
            n_post = dg.n_post;
            if (first) {
                H.n_grams = dg.n_grams;
                H.n_buckets = dg.n_buckets;
                H.bucket_span = dg.bucket_span;
            } else if (H.n_grams != dg.n_grams || H.n_buckets != dg.n_buckets || H.bucket_span != dg.bucket_span) {
                return false;  // cannot happen: every device builds the same CSR
            }
            dev_built = true;
        } else {
            (void)hipGetLastError();
            if (!first) return false;  // the host index is shared by the replicas placed concurrently
            build_grams_host(H);
            if (!H.grams_built) return false;
        }
    }
    if (!dev_built)  // host-built gram CSR (NGS_HOST_GRAMS, device-build failure)
        ok = dev_upload(&gram_off, H.gram_off, R.owned) && dev_upload(&post, H.post, R.owned, 4) /* k_wave stages whole 16-byte chunks */ &&
             dev_upload(&gram_row, H.gram_row, R.owned) && dev_upload(&skip, H.skip, R.owned);
    if (!ok) return false;
    uint64_t* ghash_key = nullptr;
    uint32_t* ghash_val = nullptr;
    if (H.gram_mode == 1 && !(dev_upload(&ghash_key, H.ghash_key, R.owned) && dev_upload(&ghash_val, H.ghash_val, R.owned)))
        return false;
    X.gsz = H.gsz;
    X.csize = H.csize;
    X.gram_mode = H.gram_mode;
    X.short_query_len = H.short_query_len;
    X.full_scan_len = H.full_scan_len;
    X.ghash_bits = H.ghash_bits;
    X.ghash_key = ghash_key;
    X.ghash_val = ghash_val;
    R.wild_w = wild_w;
    if (!dev_alloc(&wild_key, H.n_keys)) return false;
    R.owned.push_back(wild_key);
    if (!dev_alloc(&wild_score, H.n_keys)) return false;
    R.owned.push_back(wild_score);
    pt.mark("replica: gram CSR");
    if (!HIP_CHECK(build_wildcard(wild_w, H.n_keys, wild_key, wild_score, nullptr))) return false;
    X.kt_off = nullptr;
    X.kt_term = nullptr;
    if (!L.kt_off.empty()) {
        uint32_t *kt_off, *kt_term;
        if (!(dev_upload(&kt_off, L.kt_off, R.owned) && dev_upload(&kt_term, L.kt_term, R.owned))) return false;
        X.kt_off = kt_off;
        X.kt_term = kt_term;
    }
    X.rank_post = nullptr;
    X.w_uniform = L.w_uniform;
    if (L.rank_lists && n_post <= kRankMaxPostings) {
        // the threshold-0 shortcut's rank lists (4 bytes per posting); an index that cannot have them
        // (over 2^31 postings, or no memory for them) searches without them
        const uint32_t n_seg = H.gram_mode == 1 ? (uint32_t)H.gram_keys.size() : (uint32_t)kGramSpace;
        uint32_t* rp = nullptr;
        if (hipMalloc(&rp, sizeof(uint32_t) * (n_post + 4)) == hipSuccess) {
            const hipError_t e = build_rank_post(gram_off, n_seg, post, n_post, tk, H.n_short, H.n_keys, rp, nullptr);
            if (e == hipSuccess) {
                R.owned.push_back(rp);
                X.rank_post = rp;
            } else {
                (void)hipFree(rp);
                if (e != hipErrorNotSupported && !HIP_CHECK(e)) return false;
            }
        }
        (void)hipGetLastError();
        pt.mark("replica: rank lists");
    }
    X.gram_off = gram_off;
    X.post = post;
    X.gram_row = gram_row;
    X.skip = skip;
    X.n_buckets = H.n_buckets;
    X.bucket_span = H.bucket_span;
    X.post_per_row = (uint32_t)std::min<uint64_t>(UINT32_MAX, n_post / std::max<uint64_t>(H.n_grams, 1));
    X.term_off = term_off;
    X.term_bytes = term_bytes;
    X.tk_off = tk_off;
    X.tk = tk;
    X.key_off = key_off;
    X.key_bytes = reinterpret_cast<const uint8_t*>(key_bytes);
    X.wild_key = wild_key;
    X.wild_score = wild_score;
    // the build's null-stream work completes before any search stream (non-blocking) reads it
    const bool synced = HIP_CHECK(hipDeviceSynchronize());
    pt.mark("replica: wildcard answer");
    return synced;
}

// The device copies are authoritative for the search; keep only what marshalling needs.
void free_uploaded(HostIndex& H) {
    std::vector<uint64_t>().swap(H.gram_off);
    std::vector<uint32_t>().swap(H.post);
    std::vector<uint32_t>().swap(H.gram_row);
    std::vector<uint32_t>().swap(H.skip);
    std::vector<uint64_t>().swap(H.term_off);
    std::vector<uint8_t>().swap(H.term_bytes);
    std::vector<uint32_t>().swap(H.tk_off);
    std::vector<uint2>().swap(H.tk);
    std::vector<float>().swap(H.wild_w);
    std::vector<uint64_t>().swap(H.ghash_key);
    std::vector<uint32_t>().swap(H.ghash_val);
    std::vector<uint64_t>().swap(H.gram_keys);
}

// One replica per device in `devs` (repeats allowed: several replicas on one device split a batch
// like several devices do, which the one-GPU tests use).
bool upload(Library& L, const std::vector<int>& devs) {
    const HostIndex& H = L.host;
    PhaseTimer pt;
    bool keys_unique = true;
    {
        std::vector<uint8_t> seen(H.n_keys, 0);
        for (const uint2& kw : H.tk) {
            if (seen[kw.x]) { keys_unique = false; break; }
            seen[kw.x] = 1;
        }
    }
    // term -> pairs shape and the largest weight (term_pairs in ngs_kernels.hip)
    L.tk_identity = H.tk_off.size() == (size_t)H.n_terms + 1;
    for (size_t t = 0; L.tk_identity && t < H.tk_off.size(); ++t) L.tk_identity = H.tk_off[t] == t;
    // term ids in key-rank order: every key rank of term t is below every key rank of t + 1
    // (DevIndex.tk_monotone; the build orders terms by their best key rank, so this fails only
    // where a key has several terms or a short term's key ranks above a long one's)
    L.tk_monotone = true;
    {
        int64_t prev = -1;
        for (size_t t = 0; L.tk_monotone && t + 1 < H.tk_off.size(); ++t) {
            uint32_t lo = UINT32_MAX, hi = 0;
            for (uint32_t p = H.tk_off[t]; p < H.tk_off[t + 1]; ++p) {
                lo = std::min(lo, H.tk[p].x);
                hi = std::max(hi, H.tk[p].x);
            }
            if (lo == UINT32_MAX) continue;  // no pair
            L.tk_monotone = (int64_t)lo > prev;
            prev = hi;
        }
    }
    L.w_max = 0.0f;
    for (const uint2& kw : H.tk) {
        float w;
        std::memcpy(&w, &kw.y, sizeof w);
        if (w > L.w_max) L.w_max = w;  // NaN weights score +0 (pair_enc) and never raise the bound
    }
    // the threshold-0 shortcut (DevIndex.rank_post) needs one record shape per hit count: one weight.
    // Its one-hit prefix entries stand in for multi-hit records only while a one-hit score is at most
    // the record's own: w * fl(1/n) <= 100 (a promoted record) needs w <= 200 (n >= 2)
    L.rank_lists = keys_unique && L.tk_identity && !H.tk.empty() && !std::getenv("NGS_NO_RANK_LISTS");
    L.w_uniform = H.tk.empty() ? 0u : H.tk.front().y;
    for (size_t i = 0; L.rank_lists && i < H.tk.size(); ++i) L.rank_lists = H.tk[i].y == L.w_uniform;
    {
        float wu;
        std::memcpy(&wu, &L.w_uniform, sizeof wu);
        if (!(wu <= 200.0f)) L.rank_lists = false;
    }
    // key -> terms for keys with several pairs (DevIndex.kt_off, key_promoted_long)
    L.kt_off.clear();
    L.kt_term.clear();
    if (!keys_unique) {
        L.kt_off.assign((size_t)H.n_keys + 1, 0);
        for (const uint2& kw : H.tk) L.kt_off[kw.x + 1]++;
        for (uint32_t k = 0; k < H.n_keys; ++k) L.kt_off[k + 1] += L.kt_off[k];
        L.kt_term.resize(H.tk.size() + 1);
        std::vector<uint32_t> fill(L.kt_off.begin(), L.kt_off.end() - 1);
        for (uint32_t t = 0; (size_t)t + 1 < H.tk_off.size(); ++t)
            for (uint32_t p = H.tk_off[t]; p < H.tk_off[t + 1]; ++p) L.kt_term[fill[H.tk[p].x]++] = t;
    }
    pt.mark("upload: index shape checks");
    for (int d : devs) {
        L.reps.push_back(std::make_unique<Replica>());
        L.reps.back()->device = d;
    }
    // the first replica alone (it settles the host index's gram fields), then the others at once,
    // one host thread each: every device has its own PCIe link, so placing n replicas takes about
    // the time of one instead of n (C5 x 8: ~6.5 GB each)
    if (!upload_replica(L, *L.reps.front(), keys_unique, true)) return false;
    if (L.reps.size() > 1) {
        std::vector<char> rok(L.reps.size(), 0);
        std::vector<int> rerr(L.reps.size(), 0);
        std::vector<std::thread> th;
        for (size_t i = 1; i < L.reps.size(); ++i)
            th.emplace_back([&, i] {
                t_last_error = 0;
                rok[i] = upload_replica(L, *L.reps[i], keys_unique, false);
                rerr[i] = t_last_error;
            });
        for (auto& t : th) t.join();
        // a later replica whose device build failed is placed again on this thread, serially, with
        // the host-built gram CSR (what the first replica falls back to) instead of failing indexN
        for (size_t i = 1; i < L.reps.size(); ++i) {
            if (rok[i]) continue;
            if (rerr[i]) t_last_error = rerr[i];
            const int dev = L.reps[i]->device;
            L.reps[i] = std::make_unique<Replica>();
            L.reps[i]->device = dev;
            (void)hipSetDevice(dev);
            (void)hipGetLastError();
            if (!L.host.grams_built) build_grams_host(L.host);
            if (!L.host.grams_built || !upload_replica(L, *L.reps[i], keys_unique, false)) return false;
        }
    }
    L.device = devs.front();
    // the replicas a batch is split over: the first one on each device (NGS_SPLIT_SAME_DEVICE=1, a
    // test hook for one-GPU boxes: every replica). Two replicas on one device add no compute, and
    // their halves' streams share the device's hardware queues: at C3 a forced split ran 1.34x one
    // replica's time (profiles/r06_s2_dropin_replicas.txt)
    static const bool same_dev = [] {
        const char* e = std::getenv("NGS_SPLIT_SAME_DEVICE");
        return e && std::atoi(e) != 0;
    }();
    L.split.clear();
    for (size_t i = 0; i < L.reps.size(); ++i) {
        bool first = true;
        for (size_t j = 0; j < i && !same_dev; ++j) first &= L.reps[j]->device != L.reps[i]->device;
        if (first) L.split.push_back((uint32_t)i);
    }
    if (L.split.size() > 1) L.workers = std::make_unique<PartWorkers>(L.split.size() - 1);
    free_uploaded(L.host);
    std::vector<uint32_t>().swap(L.kt_off);
    std::vector<uint32_t>().swap(L.kt_term);
    pt.mark("upload: replicas placed");
    return true;
}

// Survivor slots per query of tier 1a (d_est / d_esc, 5 bytes each): the wide cap for batches
// up to kEmitWideBatch, at every threshold, halved until the slots fit kEmitWideBytes per context
// (4,096 up to 52,428 queries, 2,048 at 65,536, 1,024 at C5's 131,072). The main launch's queries
// with more survivors go on in the batch's survivor arena (ensure_arena), which holds only what
// they use: C4 (3,960 survivors per query on average, a long tail) takes 1.8 GiB per context this
// way against 2.2 GiB with 4,096 slots and 10 GiB with round 4's slots grown to 32,768
// (profiles/r05_s5_c4_arena.txt). Queries of the heavy list's launch have no arena: past their
// slots they go to tier 1b, and the slots grow when that is frequent (finish_search). Sizing the
// cap by threshold (wide only at thr <= 1/8) handed 26,594 C4 and 7,871 C5 queries per batch to
// tier 1b before the arena (profiles/r03_s4_ab_ecap.txt).
uint32_t emit_cap(size_t B) {
    static const uint32_t init = [] {  // NGS_ECAP_INIT: the slots a context starts with (tests)
        const char* e = std::getenv("NGS_ECAP_INIT");
        return e ? std::max<uint32_t>(kRankInfo + 64, (uint32_t)std::strtoul(e, nullptr, 0)) : 0u;
    }();
    if (init) return init;
    if (B > kEmitWideBatch) return kEmitCap;
    uint32_t cap = std::max(kEmitCap, kEmitCapWide);
    while (cap > kEmitCap && (uint64_t)B * cap * 5ull > kEmitWideBytes) cap /= 2;
    return cap;
}

// The most survivor slots per query a batch of B may grow to: powers of two up to kEmitCapMax,
// within kEmitBudget bytes per context (5 bytes a slot).
uint32_t emit_cap_max(size_t B) {
    uint32_t cap = kEmitCap;
    while (cap < kEmitCapMax && (uint64_t)std::max<size_t>(B, 1) * (cap * 2ull) * 5ull <= kEmitBudget) cap *= 2;
    return cap;
}

bool ensure_queries(Context& c, size_t B, size_t bytes) {
    if (B > c.bcap) {
        for (void** p : {(void**)&c.d_off, (void**)&c.d_qm, (void**)&c.d_glist, (void**)&c.d_list2, (void**)&c.d_fb,
                         (void**)&c.d_fb2, (void**)&c.d_heavy, (void**)&c.d_full, (void**)&c.d_lslots, (void**)&c.d_esn})
            if (*p) { hipFree(*p); *p = nullptr; }
        size_t nb = std::max<size_t>(B, 1024);
        if (!dev_alloc(&c.d_off, nb + 1) || !dev_alloc(&c.d_qm, nb) || !dev_alloc(&c.d_glist, nb) ||
            !dev_alloc(&c.d_list2, nb) || !dev_alloc(&c.d_fb, nb) || !dev_alloc(&c.d_fb2, nb) || !dev_alloc(&c.d_heavy, nb) || !dev_alloc(&c.d_full, nb) ||
            !dev_alloc(&c.d_lslots, 2 * (nb + kListSlots)) || !dev_alloc(&c.d_esn, nb))
            return false;
        c.bcap = nb;
    }
    // the survivor slots: (re)allocated when the batch or the cap this call needs outgrows them,
    // or when a grown cap is given back (finish_search). The rows are this call's batch (or the
    // rows held, if more and the cap is unchanged), and the cap is bounded by kEmitBudget at the
    // rows actually allocated: a context that once ran a large batch must not grow a small
    // batch's cap into rows x cap bytes past the budget.
    uint32_t want = emit_cap(B);
    if (c.ecap_grow > want) want = std::min(c.ecap_grow, std::max(want, emit_cap_max(B)));
    const bool give_back = c.shrink && c.d_est && want < c.ecap;
    c.shrink = false;
    if (!c.d_est || B > c.ebcap || want > c.ecap || give_back) {
        const size_t nb = (want == c.ecap && c.d_est) ? std::max<size_t>({B, 1024, c.ebcap}) : std::max<size_t>(B, 1024);
        want = std::max(emit_cap(B), std::min(want, emit_cap_max(nb)));
        for (void** p : {(void**)&c.d_est, (void**)&c.d_esc})
            if (*p) { hipFree(*p); *p = nullptr; }
        c.ebcap = 0;
        c.ecap = 0;
        if (!dev_alloc(&c.d_est, nb * want) || !dev_alloc(&c.d_esc, nb * want)) return false;
        c.ecap = want;
        c.ebcap = nb;
    }
    if (bytes > c.qcap) {
        for (void** p : {(void**)&c.d_raw, (void**)&c.d_norm})
            if (*p) { hipFree(*p); *p = nullptr; }
        size_t nb = std::max<size_t>(bytes, 1 << 16);
        if (!dev_alloc(&c.d_raw, nb) || !dev_alloc(&c.d_norm, nb)) return false;
        c.qcap = nb;
    }
    return true;
}

// The survivor arena of a context (SearchParams.at): kArenaInit blocks of kArenaBlock entries to
// start with (a C3 query has ~35 survivors, so only outliers ever use it), after a call that ran out
// 5/4 of the blocks it would have needed (each query it ran out for estimates its own need from the
// share of its postings counted), at least 3/2 as many, within
// kArenaBudget bytes. A query's first-block word per row of the batch.
constexpr uint32_t kArenaInit = 1024;                // 1M survivors, 5 MB
constexpr uint64_t kArenaBudget = 4ull << 30;
bool ensure_arena(Context& c, size_t B) {
    static const uint32_t init = [] {  // NGS_ARENA_INIT (tests): a smaller first arena
        const char* e = std::getenv("NGS_ARENA_INIT");
        return e ? std::max<uint32_t>(1, (uint32_t)std::strtoul(e, nullptr, 0)) : kArenaInit;
    }();
    if (!c.d_eovf || B > c.eorows) {  // the first-block words (also the heavy slices' words): required
        if (c.d_eovf) { hipFree(c.d_eovf); c.d_eovf = nullptr; }
        const size_t nb = std::max<size_t>(B, 1024);
        if (!dev_alloc(&c.d_eovf, nb)) return false;
        c.eorows = nb;
    }
    auto free_arena = [&c] {
        for (void** p : {(void**)&c.d_anext, (void**)&c.d_at, (void**)&c.d_ac})
            if (*p) { hipFree(*p); *p = nullptr; }
        c.ablocks = 0;
    };
    if (c.arena_shrink_to && c.arena_shrink_to < c.ablocks) {  // a grown arena left unused (finish_search)
        free_arena();
        c.arena_grow = c.arena_shrink_to;
    }
    c.arena_shrink_to = 0;
    // The arena is optional: the kernels run without one (SearchParams.at null; a query past its slots
    // goes to tier 1b). An allocation that fails leaves the call without it, drops the grown size and
    // waits kCalmCalls calls before trying again, so one out-of-memory event does not fail every later
    // call of the context.
    if (c.arena_off) {
        --c.arena_off;
        return true;
    }
    const uint32_t want = std::max<uint32_t>({init, c.ablocks, c.arena_grow});
    if (!c.d_at || want > c.ablocks) {
        free_arena();
        // plain hipMalloc, not dev_alloc: a refused arena is not an error of the call
        if (hipMalloc((void**)&c.d_anext, (size_t)want * sizeof(uint32_t)) != hipSuccess ||
            hipMalloc((void**)&c.d_at, (size_t)want * kArenaBlock * sizeof(uint32_t)) != hipSuccess ||
            hipMalloc((void**)&c.d_ac, (size_t)want * kArenaBlock) != hipSuccess) {
            (void)hipGetLastError();
            free_arena();
            c.arena_grow = 0;
            c.arena_off = kCalmCalls;
            return true;
        }
        c.ablocks = want;
    }
    return true;
}

// Sliced tier 1b's partial results: B * slices * limit records. Within kPartBudget bytes, else the
// call runs tier 1b unsliced (returns the slice count to use).
uint32_t ensure_parts(Context& c, size_t B, uint32_t limit, uint32_t slices) {
    if (slices <= 1 || limit > kWaveMaxLimit) return 1;
    const size_t need = B * slices * limit;
    if (need * sizeof(uint64_t) > kPartBudget) return 1;
    if (need > c.pcap) {
        if (c.d_prec) hipFree(c.d_prec);
        c.d_prec = nullptr;
        c.pcap = 0;
        const size_t nb = std::max<size_t>(need, 1 << 16);
        if (!dev_alloc(&c.d_prec, nb)) return 1;
        c.pcap = nb;
    }
    if (B * slices > c.pncap) {
        if (c.d_pcnt) hipFree(c.d_pcnt);
        c.d_pcnt = nullptr;
        c.pncap = 0;
        const size_t nb = std::max<size_t>(B * slices, 4096);
        if (!dev_alloc(&c.d_pcnt, nb)) return 1;
        c.pncap = nb;
    }
    return slices;
}

bool ensure_outputs(Context& c, size_t B, size_t stride) {
    const size_t need = B * stride;
    if (!c.d_out || B > c.ncap || need > c.ocap) {
        for (void** p : {(void**)&c.d_out, (void**)&c.d_pos, (void**)&c.d_pk, (void**)&c.d_ps, &c.d_ptemp})
            if (*p) { hipFree(*p); *p = nullptr; }
        c.d_n = c.d_k = nullptr;
        c.d_s = nullptr;
        const size_t nb = std::max(B, c.ncap), ob = std::max(need, c.ocap);
        if (!dev_alloc(&c.d_out, nb + 1 + 2 * ob) || !dev_alloc(&c.d_pos, nb + 1) || !dev_alloc(&c.d_pk, 2 * ob) ||
            !dev_alloc(&c.d_ps, ob))
            return false;
        c.ptemp_bytes = pack_temp_bytes((uint32_t)nb);
        if (!HIP_CHECK(hipMalloc(&c.d_ptemp, std::max<size_t>(c.ptemp_bytes, 1)))) return false;
        c.ncap = nb;
        c.ocap = ob;
    }
    // this call's views: [n (B + 1) | k (B * stride) | s (B * stride)] from the block's start
    c.d_n = c.d_out;
    c.d_k = c.d_out + B + 1;
    c.d_s = reinterpret_cast<float*>(c.d_k + need);
    return true;
}

bool ensure_general(const Replica& R, Context& c, hipStream_t s) {
    if (c.gen.G) return true;
    const DevIndex& X = R.dev;
    const uint64_t n_long = X.n_terms - X.n_short;
    const uint64_t kst = gen_kstride(X.n_keys);
    const uint64_t per = n_long * 4 + kst * 4 + (uint64_t)X.n_keys * 8 + 64;
    uint32_t G = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(kGeneralMaxGroup, kGeneralBudget / per));
    if ((uint64_t)G * std::max<uint64_t>(kst, 1) > (uint64_t)kInt32Max) G = 1;
    GeneralBuffers& W = c.gen;
    if (!dev_alloc(&W.cnt, (size_t)G * n_long) || !dev_alloc(&W.kenc, (size_t)G * kst) ||
        !dev_alloc(&W.list, (size_t)G * X.n_keys) || !dev_alloc(&W.sorted, X.n_keys) || !dev_alloc(&W.lcount, G))
        return false;
    W.temp_bytes = general_sort_temp_bytes(X.n_keys);
    if (!HIP_CHECK(hipMalloc(&W.temp, std::max<size_t>(W.temp_bytes, 1)))) return false;
    // on the call's stream: a plain hipMemset runs on the null stream, which the context's
    // non-blocking streams do not wait for (the first group's counts raced with it)
    if (!HIP_CHECK(hipMemsetAsync(W.cnt, 0, sizeof(uint32_t) * std::max<size_t>((size_t)G * n_long, 1), s)) ||
        !HIP_CHECK(hipMemsetAsync(W.kenc, 0, sizeof(uint32_t) * std::max<size_t>((size_t)G * kst, 1), s)))
        return false;
    W.G = G;
    return true;
}

// The search pipeline over B queries already in device memory, in two halves: queue_search
// queues the normalisation, the tier kernels and the read-back of the statistics and path
// counts; finish_search waits for them, runs the general path for the queries listed for it
// and records the statistics. small: one kernel per tier on the call's stream (no routing
// lists, no side streams; the latency path of score() and small batches).
int queue_search(Library& L, Replica& R, Context& c, const uint8_t* d_raw, const uint64_t* d_off, uint32_t B,
                 uint64_t qbytes, float thr, uint32_t limit, uint32_t stride, uint32_t* d_n, uint32_t* d_k,
                 float* d_s, hipStream_t s, SearchParams& P, bool small) {
    // small: the statistics go to the latency block (zeroed by k_prep, read back by the caller
    // together with the results)
    DevStats* sd = small ? reinterpret_cast<DevStats*>(c.d_sio) : c.d_stats;
    uint32_t* gc = reinterpret_cast<uint32_t*>(sd + kStatSlots);
    std::memset(&P, 0, sizeof(P));  // (padding too: the bytes are a replay signature, Context::gsig)
    P.thr = thr;
    P.limit = limit;
    P.out_stride = stride;
    P.n_queries = B;
    static const uint32_t dbg = [] {
        const char* e = std::getenv("NGS_DEBUG");
        return e ? (uint32_t)std::strtoul(e, nullptr, 0) : 0u;
    }();
    P.dbg = dbg;
    static const uint32_t hslices = [] {  // NGS_HEAVY_SLICES: term-id slices per heavy query (0: auto)
        const char* e = std::getenv("NGS_HEAVY_SLICES");
        return e ? std::min<uint32_t>((uint32_t)std::strtoul(e, nullptr, 0), kHeavyMaxSlices) : 0u;
    }();
    P.hslices = hslices;
    P.hbase = 0;
    P.hgrid = c.heavy_items ? c.heavy_items + c.heavy_items / 8 + 64 : 0u;  // (a margin: batches change)
    // tier 1: the lean kernel with tier 1b on its hand-overs (batches), or tier 1b alone (the latency path)
    P.waves = small ? 1u : 0u;
    {
        std::lock_guard<std::mutex> g(L.valid_mu);
        std::memcpy(P.valid, L.valid, sizeof(P.valid));
    }
    if (!ensure_queries(c, B, qbytes)) return -4;
    P.esn = c.d_esn;
    P.est = c.d_est;
    P.esc = c.d_esc;
    P.ecap = c.ecap;
    if (!small) {  // (the latency path runs tier 1b alone: no tier-1a survivors)
        if (!ensure_arena(c, B)) return -4;
        P.eovf = c.d_eovf;
        P.anext = c.ablocks ? c.d_anext : nullptr;
        P.at = c.ablocks ? c.d_at : nullptr;  // null: no arena this call (ensure_arena)
        P.ac = c.ablocks ? c.d_ac : nullptr;
        P.ablocks = c.ablocks;
        P.actr = gc + kArenaCtrWord;
    }
    constexpr uint32_t list_slices = kSlices;        // term-id slices of the hand-over / full lists' tier 1b
    constexpr uint32_t small_slices = kSmallSlices;  // ... and of every query of the latency path
    if (small) {
        // one query's postings over several CUs: a wave per (query, slice of at least 8 skip
        // buckets), then k_merge; a small library stays on one wave per query
        const uint32_t sl = std::min<uint32_t>(small_slices, R.dev.n_buckets / 8);
        P.nslices = sl > 1 ? ensure_parts(c, B, P.limit, sl) : 1u;
        if (P.nslices > 1) P.waves = 1;
    } else {
        P.nslices = ensure_parts(c, B, P.limit, list_slices);
    }
    P.qcap = c.qcap;
    P.oflow = gc + 6;
    if (small) {
        P.zero_stats = reinterpret_cast<uint32_t*>(sd);
        // the slots this batch's queries add to (q & (kStatSlots - 1), errors in slot 0); the
        // others stay zero from the block's allocation
        P.zero_words = (uint32_t)(std::min<size_t>(B, kStatSlots) * sizeof(DevStats) / sizeof(uint32_t));
    }
    P.prec = c.d_prec;
    P.pcnt = c.d_pcnt;
    const bool timing = L.timing.load();
    // A small batch whose queries are all on the heavy list (C2: 4,096 queries at threshold 0) is a
    // few waves per CU of long per-query chains, so throughput comes from batches in flight, not from
    // the main and side streams
    // of one call overlapping: its side work goes on the call's own stream, in order, and a context
    // that only ever runs such batches never makes its side streams. Three pipelined calls then hold
    // three hardware queues (HIP maps streams to its four queues round-robin as they are made) instead
    // of six streams sharing four (C2 28.6 -> 34.8 Mq/s at three in flight)
    constexpr uint32_t one_stream_batch = kOneStreamBatch;
    // (only where every lean query is on the heavy list, cmin <= kHeavyCmin for any gram count up to
    // kWaveMaxGrams, as at threshold 0: with a mix, the heavy chain on its own stream overlaps the
    // main launch, and in order after it a call of 8,192 C3-like queries took 0.23 ms longer)
    const bool all_heavy = !((float)kHeavyCmin / (float)kWaveMaxGrams < thr);
    hipStream_t side = s, side2 = s;
    // one side stream for all of the replica's contexts: two calls in flight then hold three streams
    // beside the null stream, one per hardware queue at HIP's default of four; with a side stream per
    // context, one context's main and side streams shared a queue and its tail waited behind its own
    // heavy chain (C3 +1.0 %, six passes on two boxes; profiles/r05_s27_ab_hw_queues.txt)
    if (B > one_stream_batch || !all_heavy) {
        if (!c.side) {
            std::lock_guard<std::mutex> g(R.main_mu);
            if (!R.shared_side && !HIP_CHECK(make_side_stream(&R.shared_side))) return -4;
            c.side = c.side2 = R.shared_side;
            c.side_shared = true;
        }
        side = c.side;
        side2 = c.side2;
    }
    // statistics, path counts and list counters: reset by k_prep and k_lists when the context's last
    // call left them so (the memset's fill kernel waited ~200 us for a workgroup slot behind the
    // previous call's tail in the pipelined trace)
    const bool zero_in_prep = !small && c.stats_clean && P.waves == 0;
    c.stats_clean = false;
    if (zero_in_prep) {
        P.zero_stats = reinterpret_cast<uint32_t*>(c.d_stats);
        P.zero_words = (uint32_t)(kStatSlots * sizeof(DevStats) / sizeof(uint32_t));
    }
    DevIndex X;
    if (!R.index_for(P.valid, X)) return -4;
    // A one-stream call (side == s: batches up to kOneStreamBatch queries that are all heavy, C2) is
    // ~0.1 ms of GPU work for ~12 queued operations, 50 us of host time per call. When a call's
    // launch arguments repeat an earlier call of the context (a server's or a bench's batches into
    // the same buffers), the sequence is built as a graph on the second occurrence and replayed
    // from then on (one submission: ~4 us of host time for 10 launches against ~30,
    // tools/ubench/graph_launch.hip). Such calls leave the replica's main-launch order alone
    // (main_ev): their main launch only routes, every lean query being on the heavy list.
    static const bool no_graphs = std::getenv("NGS_SYNC_DEBUG") != nullptr;
    bool capture = false;
    std::vector<uint8_t> sig;
    // (not on the null stream)
    if (!small && side == s && s && !timing && !no_graphs && !c.gfail) {
        auto put = [&](const void* p, size_t n) {
            sig.insert(sig.end(), static_cast<const uint8_t*>(p), static_cast<const uint8_t*>(p) + n);
        };
        const void* ptrs[] = {d_raw, d_off, d_n, d_k, d_s, s, c.d_norm, c.d_qm, c.d_list2, c.d_fb, c.d_fb2,
                              c.d_heavy, c.d_full, c.d_glist, c.d_lslots, c.d_lctr, c.d_stats, c.h_stats};
        put(ptrs, sizeof(ptrs));
        put(&X, sizeof(X));
        put(&P, sizeof(P));
        const uint32_t flags[] = {B, all_heavy ? 1u : 0u, zero_in_prep ? 1u : 0u};
        put(flags, sizeof(flags));
        for (auto& g : c.graphs) {
            if (g.first != sig) continue;
            if (!HIP_CHECK(hipGraphLaunch(g.second, s))) return -4;
            c.stats_clean = true;
            g_host_phase[kHpReplays].fetch_add(1, std::memory_order_relaxed);
            return 0;
        }
        capture = std::find(c.gseen.begin(), c.gseen.end(), sig) != c.gseen.end();
        if (!capture) {
            if (c.gseen.size() >= Context::kGraphs) c.gseen.erase(c.gseen.begin());
            c.gseen.push_back(sig);
        }
    }
    // the call's operations, queued on s, or with gb appended to a graph being built (one-stream calls)
    auto queue_ops = [&](GraphBuild* gb) -> bool {
        const size_t stat_bytes = sizeof(DevStats) * (kStatSlots + 1 + 2 * kListSlots);
        if (!zero_in_prep && !small) {
            if (gb) {
                hipMemsetParams mp{};
                mp.dst = c.d_stats;
                mp.value = 0;
                mp.elementSize = 4;
                mp.width = stat_bytes / 4;
                mp.height = 1;
                if (!HIP_CHECK(hipGraphAddMemsetNode(&gb->last, gb->graph, nullptr, 0, &mp))) return false;
            } else if (!HIP_CHECK(hipMemsetAsync(c.d_stats, 0, stat_bytes, s))) {
                return false;
            }
        }
        if (timing) HIP_CHECK(hipEventRecord(c.ev[0], s));
        if (!HIP_CHECK(launch_prep(d_raw, d_off, B, P, c.d_norm, c.d_qm, X.csize, X, c.d_heavy, gc + 3, c.d_full,
                                   gc + 5, c.d_lslots, c.d_lctr, s, side, c.prep_ev, c.lists_ev, gb)))
            return false;
        if (timing) HIP_CHECK(hipEventRecord(c.ev[1], s));  // the end of k_prep is the start of the tier-1 phase
        // the main tier-1a launches of this replica's calls one after another: with two calls in flight
        // the second call's main launch otherwise starts in the first one's and the two share the GPU
        // (C3, one box, three passes each: 31.3-31.6 against 30.1-30.6 Mq/s,
        // profiles/r05_s15_ab_serial_main.txt; C5 the same)
        std::unique_lock<std::mutex> g(R.main_mu, std::defer_lock);
        hipEvent_t mev = nullptr;
        bool mwait = false;
        if (!small && !gb) {
            g.lock();
            if (!R.main_ev && !HIP_CHECK(hipEventCreateWithFlags(&R.main_ev, hipEventDisableTiming))) return false;
            mev = R.main_ev;
            mwait = R.main_rec;
            R.main_rec = true;
        }
        if (!HIP_CHECK(launch_fast(X, P, c.d_norm, d_off, c.d_qm, d_n, d_k, d_s, c.d_list2, gc + 1, c.d_fb, gc + 2,
                                   c.d_fb2, gc + 4, c.d_heavy, gc + 3, c.d_full, gc + 5, c.d_glist, gc, sd, s, side,
                                   side2, c.join, c.join2, c.lists_ev, all_heavy, mev, mwait, gb)))
            return false;
        if (timing) HIP_CHECK(hipEventRecord(c.ev[3], s));
        // the statistics and the path counts in one read-back (the general path adds no statistics)
        if (small) return true;
        if (gb) {
            hipGraphNode_t n = nullptr;
            if (!HIP_CHECK(hipGraphAddMemcpyNode1D(&n, gb->graph, gb->last ? &gb->last : nullptr, gb->last ? 1 : 0,
                                                   c.h_stats, c.d_stats, kSioStats, hipMemcpyDeviceToHost)))
                return false;
            gb->last = n;
            return true;
        }
        return HIP_CHECK(hipMemcpyAsync(c.h_stats, c.d_stats, kSioStats, hipMemcpyDeviceToHost, s));
    };
    // A graph is built node by node (no stream capture, which in this runtime fails other threads'
    // launches while it is open: the threaded test's scoreBatch calls did) and instantiated
    if (capture) {
        GraphBuild gb;
        hipGraphExec_t exec = nullptr;
        bool made = HIP_CHECK(hipGraphCreate(&gb.graph, 0)) && queue_ops(&gb) &&
                    HIP_CHECK(hipGraphInstantiate(&exec, gb.graph, nullptr, nullptr, 0));
        if (gb.graph) hipGraphDestroy(gb.graph);
        (void)hipGetLastError();
        if (made) {
            c.gseen.erase(std::find(c.gseen.begin(), c.gseen.end(), sig));
            if (c.graphs.size() >= Context::kGraphs) {
                hipGraphExecDestroy(c.graphs.front().second);
                c.graphs.erase(c.graphs.begin());
            }
            c.graphs.emplace_back(std::move(sig), exec);
            if (!HIP_CHECK(hipGraphLaunch(exec, s))) return -4;
        } else {  // nothing of the call ran: queue it one by one, and so from now on
            if (exec) hipGraphExecDestroy(exec);
            c.gfail = true;
            if (!queue_ops(nullptr)) return -4;
        }
    } else if (!queue_ops(nullptr)) {
        return -4;
    }
    c.stats_clean = !small && P.waves == 0;  // k_lists queued: it leaves the list counters zero
    return 0;
}

int finish_search(Library& L, Replica& R, Context& c, uint32_t B, const SearchParams& P, const uint64_t* d_off,
                  uint32_t* d_n, uint32_t* d_k, float* d_s, hipStream_t s, bool small = false) {
    if (!HIP_CHECK(hipStreamSynchronize(s))) return -4;
    const DevStats* hst = small ? reinterpret_cast<const DevStats*>(c.h_sio) : c.h_stats;
    const bool timing = L.timing.load();
    ngs_stats st{};
    st.queries = B;
    // general, tier 2, tier 1a hand-overs, heavy, heavy hand-overs, full
    const uint32_t* counts3 = reinterpret_cast<const uint32_t*>(hst + kStatSlots);
    if (counts3[6]) {  // (the rerun resets the path counts with the memset)
        c.stats_clean = false;
        return kRetryQcap;
    }  // a query past the normalised-query buffer: nothing is valid
    const uint32_t ngen = counts3[0];
    if (ngen) {
        std::vector<uint32_t> gl(ngen);
        if (!HIP_CHECK(hipMemcpyAsync(gl.data(), c.d_glist, sizeof(uint32_t) * ngen, hipMemcpyDeviceToHost, s)) ||
            !HIP_CHECK(hipStreamSynchronize(s)))
            return -4;
        std::sort(gl.begin(), gl.end());
        if (!ensure_general(R, c, s)) return -4;
        DevIndex X;
        if (!R.index_for(P.valid, X)) return -4;
        if (timing) HIP_CHECK(hipEventRecord(c.ev[4], s));
        for (uint32_t g0 = 0; g0 < ngen; g0 += c.gen.G) {
            const uint32_t G = std::min(c.gen.G, ngen - g0);
            if (!HIP_CHECK(hipMemcpyAsync(c.d_group, gl.data() + g0, sizeof(uint32_t) * G, hipMemcpyHostToDevice, s)))
                return -4;
            if (!HIP_CHECK(run_general(X, P, c.d_norm, d_off, c.d_qm, c.d_group, gl.data() + g0, G, c.gen, d_n,
                                       d_k, d_s, s)))
                return -4;
        }
        if (timing) HIP_CHECK(hipEventRecord(c.ev[5], s));
        // the last group's k_gen_write still reads c.gen: complete before the context goes back
        // to the pool (and before the call returns, as the ABI promises)
        if (!HIP_CHECK(hipStreamSynchronize(s))) return -4;
    }
    DevStats ds{};
    uint64_t slot_full = 0;
    for (uint32_t i = 0; i < kStatSlots; ++i) {
        const DevStats& x = hst[i];
        ds.postings += x.postings;
        ds.lists += x.lists;
        ds.results += x.results;
        ds.fast += x.fast;
        ds.survivors += x.survivors;
        ds.main_postings += x.main_postings;
        ds.main_lists += x.main_lists;
        ds.errors |= x.errors;
        slot_full += x.slot_full;
    }
    // queries that filled their survivor slots ran again in tier 1b: when that is more than 1/64
    // of the batch, this context's later calls get twice the slots (bounded by emit_cap_max);
    // after kCalmCalls calls in a row that filled none of grown slots, half of them go back
    // the arena's block counter: past its blocks, the arena ran out (those queries went to tier 1b and
    // count as slot_full): later calls get a larger arena, not more slots per query
    // (the queries it ran out for add the blocks they would still need, the next word: the next
    // call's arena is 5/4 of the estimated need, at least 3/2 of this one)
    if (!small) c.heavy_items = counts3[3] * heavy_slices(P, counts3[3], R.dev);  // the next call's heavy grid
    const uint32_t arena_used = small ? 0u : counts3[kArenaCtrWord];
    const bool arena_out = !small && P.at && arena_used > P.ablocks;
    if (arena_out) {
        const uint64_t need = (uint64_t)P.ablocks + counts3[kArenaCtrWord + 1];
        const uint64_t want = std::max<uint64_t>(3ull * P.ablocks / 2, 5ull * need / 4);
        const uint64_t cap = kArenaBudget / ((uint64_t)kArenaBlock * (sizeof(uint32_t) + sizeof(uint8_t)));
        c.arena_grow = (uint32_t)std::min<uint64_t>(want, cap);
        c.arena_calm = 0;
    } else if (!small && P.at && P.ablocks > kArenaInit && (uint64_t)arena_used * 4 < P.ablocks) {
        // a grown arena mostly unused for kCalmCalls calls in a row: halved (as the survivor slots)
        if (++c.arena_calm >= kCalmCalls) {
            c.arena_calm = 0;
            c.arena_shrink_to = std::max<uint32_t>(kArenaInit, P.ablocks / 2);
        }
    } else if (!small) {
        c.arena_calm = 0;
    }
    if (!small && !arena_out) {
        if (slot_full * 64 > B) {
            c.calm = 0;
            if (c.ecap < emit_cap_max(B)) c.ecap_grow = std::max(c.ecap_grow, c.ecap * 2);
        } else if (slot_full == 0 && c.ecap > emit_cap(B) && ++c.calm >= kCalmCalls) {
            c.calm = 0;
            c.ecap_grow = c.ecap / 2 > emit_cap(B) ? c.ecap / 2 : 0u;
            c.shrink = true;
        }
    }
    if (ds.errors) {
        std::fprintf(stderr, "ngram_search: fused kernel reported internal error 0x%x\n", ds.errors);
        t_last_error = kErrInternal;
        return -5;
    }
    if (timing) {
        float ms = 0;
        st.fast_queries = ds.fast;
        st.general_queries = ngen;
        st.tier2_queries = counts3[1];
        // queries tier 1b ran: hand-overs of both lean launches and the full list
        st.handover_queries = counts3[2] + counts3[4] + counts3[5];
        st.heavy_queries = counts3[3];
        st.full_queries = counts3[5];
        st.slot_full_queries = slot_full;
        st.survivor_slots = P.ecap;
        st.survivor_slot_bytes = ((uint64_t)c.ebcap * c.ecap + (uint64_t)c.ablocks * kArenaBlock) *
                                 (sizeof(uint32_t) + sizeof(uint8_t));
        st.arena_blocks = small ? 0u : P.ablocks;
        st.arena_used = arena_used;
        st.postings = ds.postings;
        st.lists = ds.lists;
        st.results = ds.results;
        st.survivors = ds.survivors;
        st.main_postings = ds.main_postings;
        st.main_lists = ds.main_lists;
        if (hipEventElapsedTime(&ms, c.ev[0], c.ev[1]) == hipSuccess) st.prep_kernel_ms = ms;
        if (hipEventElapsedTime(&ms, c.ev[1], c.ev[3]) == hipSuccess) st.fast_kernel_ms = ms;
        if (ngen && hipEventElapsedTime(&ms, c.ev[4], c.ev[5]) == hipSuccess) st.general_ms = ms;
        std::lock_guard<std::mutex> g(L.stats_mu);
        L.last = st;
    }
    return 0;
}

int device_search(Library& L, Replica& R, Context& c, const uint8_t* d_raw, const uint64_t* d_off, uint32_t B,
                  uint64_t qbytes, float thr, uint32_t limit, uint32_t stride, uint32_t* d_n, uint32_t* d_k,
                  float* d_s, hipStream_t s) {
    if (!B) return 0;
    SearchParams P;
    const int rc = queue_search(L, R, c, d_raw, d_off, B, qbytes, thr, limit, stride, d_n, d_k, d_s, s, P, false);
    return rc ? rc : finish_search(L, R, c, B, P, d_off, d_n, d_k, d_s, s);
}

uint32_t effective_limit(const Library& L, uint32_t limit) {
    if (limit == 0) limit = kInt32Max;  // nGramSearch.hpp:420-421
    return std::min<uint32_t>(limit, L.host.n_keys);
}

template <typename CharT>
size_t str_len(const CharT* p) {
    size_t n = 0;
    while (p[n]) ++n;
    return n;
}

// One chunk of a host batch in flight on a context (host_search_one).
struct HostChunk {
    Context* c = nullptr;
    uint32_t q0 = 0, B = 0;
    bool small = false;
    size_t block = 0;
    SearchParams P{};
    const uint8_t* d_raw = nullptr;
    const uint64_t* d_off = nullptr;
    uint32_t *d_n = nullptr, *d_k = nullptr;
    float* d_s = nullptr;
    // pointer mode (pcs != 0): records go out as result pointers pbase + key_off[key] * pcs
    uint64_t pbase = 0;
    uint32_t pcs = 0;
};

// Queues chunk [q0, q0 + B) on context c: the queries packed into pinned staging, one H2D copy
// (two for large chunks), the search kernels. Nothing waits.
template <typename CharT>
bool queue_host_chunk(Library& L, Replica& R, Context& c, const CharT* const* queries, uint32_t q0, uint32_t B,
                      float thr, uint32_t Lm, HostChunk& h, uint64_t pbase) {
    constexpr size_t cs = sizeof(CharT);
    const size_t stride = Lm;
    h = HostChunk{};
    h.pbase = pbase;
    h.pcs = pbase ? (uint32_t)cs : 0u;
    h.c = &c;
    h.q0 = q0;
    h.B = B;
    HostTimer ht;
    // query offsets into pinned staging: lengths on up to 8 threads, one prefix pass
    if (!c.h_off.grow(sizeof(uint64_t) * (B + 1))) return false;
    uint64_t* ho = c.h_off.as<uint64_t>();
    ho[0] = 0;
    parallel_ranges(B, 8192, [&](size_t a, size_t e) {
        for (size_t i = a; i < e; ++i) ho[i + 1] = queries[q0 + i] ? str_len(queries[q0 + i]) * cs : 0;
    });
    for (uint32_t i = 0; i < B; ++i) ho[i + 1] += ho[i];
    const uint64_t qbytes = ho[B];
    // small batches (score()'s latency path): one kernel per tier on one stream, the queries
    // in with one copy and the statistics with the whole output block out with one copy,
    // all through the context's latency block [statistics | results | offsets, bytes]
    h.block = sizeof(uint32_t) * (B + 1 + 2 * (size_t)B * stride);
    const size_t qspace = sizeof(uint64_t) * (B + 1) + qbytes;
    h.small = B <= kSmallBatch && h.block <= kSmallBlock && qspace <= kSmallQ;
    bool ok;
    if (h.small) {
        uint8_t* hq = c.h_sio + kSioStats + kSmallBlock;
        std::memcpy(hq, ho, sizeof(uint64_t) * (B + 1));
        for (uint32_t i = 0; i < B; ++i)
            if (queries[q0 + i])
                std::memcpy(hq + sizeof(uint64_t) * (B + 1) + ho[i], queries[q0 + i], ho[i + 1] - ho[i]);
        uint8_t* dq = c.d_sio + kSioStats + kSmallBlock;
        h.d_off = reinterpret_cast<const uint64_t*>(dq);
        h.d_raw = dq + sizeof(uint64_t) * (B + 1);
        h.d_n = reinterpret_cast<uint32_t*>(c.d_sio + kSioStats);
        h.d_k = h.d_n + B + 1;
        h.d_s = reinterpret_cast<float*>(h.d_k + (size_t)B * stride);
        ok = HIP_CHECK(hipMemcpyAsync(dq, hq, qspace, hipMemcpyHostToDevice, c.stream));
    } else {
        if (!c.h_raw.grow(std::max<uint64_t>(qbytes, 1))) return false;
        uint8_t* hr = c.h_raw.as<uint8_t>();
        parallel_ranges(B, 8192, [&](size_t a, size_t e) {
            for (size_t i = a; i < e; ++i)
                if (queries[q0 + i]) std::memcpy(hr + ho[i], queries[q0 + i], ho[i + 1] - ho[i]);
        });
        ht.mark(kHpPack, "pack queries");
        ok = ensure_queries(c, B, qbytes) && ensure_outputs(c, B, stride) &&
             HIP_CHECK(hipMemcpyAsync(c.d_raw, c.h_raw.p, qbytes, hipMemcpyHostToDevice, c.stream)) &&
             HIP_CHECK(hipMemcpyAsync(c.d_off, ho, sizeof(uint64_t) * (B + 1), hipMemcpyHostToDevice, c.stream));
        h.d_raw = c.d_raw;
        h.d_off = c.d_off;
        h.d_n = c.d_n;
        h.d_k = c.d_k;
        h.d_s = c.d_s;
    }
    if (!ok) return false;
    if (queue_search(L, R, c, h.d_raw, h.d_off, B, qbytes, thr, Lm, (uint32_t)stride, h.d_n, h.d_k, h.d_s, c.stream,
                     h.P, h.small) != 0)
        return false;
    ht.mark(kHpQueue, "copy in + queue kernels");
    return !h.small || HIP_CHECK(hipMemcpyAsync(c.h_sio, c.d_sio, kSioStats + h.block, hipMemcpyDeviceToHost, c.stream));
}

// Completes a queued chunk: waits, runs the general path, reads back exactly the results
// (packed on the device for large chunks), fills the chunk's counts and hands its records to
// `emit(recs, scores, n, last, chunk_total)` (in pieces of the chunk's chunk_total records, in order):
// recs are u32 key ranks, or in pointer mode (h.pcs) u64 result
// pointers.
template <class Emit>
bool finish_host_chunk(Library& L, Replica& R, HostChunk& h, uint32_t Lm, std::vector<uint32_t>& counts, bool last,
                       Emit&& emit) {
    Context& c = *h.c;
    const uint32_t B = h.B, q0 = h.q0;
    const size_t stride = Lm;
    HostTimer ht;
    const int frc = finish_search(L, R, c, B, h.P, h.d_off, h.d_n, h.d_k, h.d_s, c.stream, h.small);
    if (frc == kRetryQcap) t_last_error = kErrQueryBuffer;  // cannot happen: the host path sizes the buffer
    if (frc != 0) return false;
    ht.mark(kHpWait, "wait for kernels");
    if (h.small) {
        const uint32_t* counts3 = reinterpret_cast<const uint32_t*>(c.h_sio) + kStatSlots * 16;
        if (counts3[0]) {  // the general path ran after the read-back: read the results again
            if (!HIP_CHECK(hipMemcpyAsync(c.h_sio + kSioStats, c.d_sio + kSioStats, h.block, hipMemcpyDeviceToHost,
                                          c.stream)) ||
                !HIP_CHECK(hipStreamSynchronize(c.stream)))
                return false;
        }
        const uint32_t* hn = reinterpret_cast<const uint32_t*>(c.h_sio + kSioStats);
        const uint32_t* hk = hn + B + 1;
        const float* hs = reinterpret_cast<const float*>(hk + (size_t)B * stride);
        std::vector<uint32_t> k;
        std::vector<float> sc;
        for (uint32_t i = 0; i < B; ++i) {
            counts[q0 + i] = hn[i];
            k.insert(k.end(), hk + (size_t)i * stride, hk + (size_t)i * stride + hn[i]);
            sc.insert(sc.end(), hs + (size_t)i * stride, hs + (size_t)i * stride + hn[i]);
        }
        if (h.pcs) {  // a few records: their pointers made here
            const uint64_t* koff = L.host.key_off.data();
            std::vector<uint64_t> ptr(k.size());
            for (size_t i = 0; i < k.size(); ++i) ptr[i] = h.pbase + koff[k[i]] * h.pcs;
            emit(static_cast<const void*>(ptr.data()), sc.data(), (uint32_t)k.size(), last, (uint32_t)k.size());
        } else {
            emit(static_cast<const void*>(k.data()), sc.data(), (uint32_t)k.size(), last, (uint32_t)k.size());
        }
        return true;
    }
    // large batches: pack on the device (prefix sum of the counts, one copy per query), read
    // back the offsets, then exactly the packed records
    uint64_t* pp = h.pcs ? reinterpret_cast<uint64_t*>(c.d_pk) : nullptr;
    if (!HIP_CHECK(hipMemsetAsync(c.d_n + B, 0, sizeof(uint32_t), c.stream)) ||
        !HIP_CHECK(launch_pack(c.d_n, c.d_k, c.d_s, B, (uint32_t)stride, c.d_pos, c.d_pk, c.d_ps, c.d_ptemp,
                               c.ptemp_bytes, c.stream, R.dev.key_off, h.pbase, h.pcs, pp)) ||
        !c.h_res.grow(sizeof(uint32_t) * (B + 1)) ||
        !HIP_CHECK(hipMemcpyAsync(c.h_res.p, c.d_pos, sizeof(uint32_t) * (B + 1), hipMemcpyDeviceToHost, c.stream)) ||
        !HIP_CHECK(hipStreamSynchronize(c.stream)))
        return false;
    ht.mark(kHpPackBack, "pack + offsets back");
    const uint32_t total = c.h_res.as<uint32_t>()[B];
    for (uint32_t i = 0; i < B; ++i) counts[q0 + i] = c.h_res.as<uint32_t>()[i + 1] - c.h_res.as<uint32_t>()[i];
    const size_t esz = h.pcs ? sizeof(uint64_t) : sizeof(uint32_t);
    const size_t rb = esz * (size_t)total;  // record bytes
    if (!c.h_res.grow(rb + sizeof(float) * (size_t)total)) return false;
    // the records come back in pieces, each marshalled (straight from the pinned buffer) while the
    // next ones are still on the link: the copy and the host's copy into the caller's arrays overlap
    const uint32_t pieces = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(kBackPieces, total / kBackPieceMin));
    const uint32_t per = (total + pieces - 1) / pieces;
    uint8_t* hr = c.h_res.as<uint8_t>();
    for (uint32_t i = 0; i < pieces; ++i) {
        const size_t a = (size_t)i * per, n = std::min<size_t>(per, total - std::min<size_t>(total, a));
        hipStream_t sp = c.stream;  // (pieces alternating over two streams measured slower: 0.47-0.62 ms)
        if (n && !(HIP_CHECK(hipMemcpyAsync(hr + a * esz, reinterpret_cast<const uint8_t*>(c.d_pk) + a * esz, n * esz,
                                            hipMemcpyDeviceToHost, sp)) &&
                   HIP_CHECK(hipMemcpyAsync(hr + rb + a * sizeof(float), c.d_ps + a, n * sizeof(float),
                                            hipMemcpyDeviceToHost, sp))))
            return false;
        if (!HIP_CHECK(hipEventRecord(c.piece_ev[i], sp))) return false;
    }
    for (uint32_t i = 0; i < pieces; ++i) {
        const size_t a = (size_t)i * per, n = std::min<size_t>(per, total - std::min<size_t>(total, a));
        if (!HIP_CHECK(hipEventSynchronize(c.piece_ev[i]))) {
            (void)hipStreamSynchronize(c.stream);  // nothing may still write the buffer
            return false;
        }
        emit(static_cast<const void*>(hr + a * esz), reinterpret_cast<const float*>(hr + rb) + a, (uint32_t)n, last,
             total);
    }
    ht.mark(kHpRecords, "records back + emit");
    return true;
}

// A large host batch can run as about kPipeChunks chunks (of at least kPipeMinChunk queries) over
// two contexts, one queued ahead, so that chunk k's copies and read-back
// overlap chunk k + 1's kernels. Measured slower than one chunk at C3 (the chunks' read-backs
// waited behind the other chunk's kernels), so one chunk is the default; the batch is still cut
// into chunks where its outputs would exceed kOutBudget / kPartBudget.
constexpr uint32_t kPipeChunks = 1;  // measured: 4 chunks 6.1-6.6 ms against 4.4-4.6 for one at C3
constexpr uint32_t kPipeMinChunk = 8192;

// Queries per chunk of a host batch of nq queries at limit Lm: the outputs within kOutBudget and
// sliced tier 1b's partial results within kPartBudget
size_t host_chunk(uint32_t nq, uint32_t Lm) {
    const size_t stride = std::max<uint32_t>(Lm, 1);
    size_t max_chunk = std::max<size_t>(1, std::min<size_t>(1 << 20, kOutBudget / (stride * 8)));
    if (Lm <= kWaveMaxLimit)  // sliced tier 1b's partial results fit the budget
        max_chunk = std::max<size_t>(1, std::min<size_t>(max_chunk, kPartBudget / (sizeof(uint64_t) * kSlices * stride)));
    const size_t want = std::max<size_t>(kPipeMinChunk, (nq + kPipeChunks - 1) / kPipeChunks);
    return std::min(max_chunk, want);
}

// Scores n queries (characters of the index's width) on one replica; fills counts and hands
// each chunk's records, in query order, to emit(keys, scores, n).
template <typename CharT, class Emit>
bool host_search_chunks(Library& L, Replica& R, const CharT* const* queries, uint32_t nq, float thr, uint32_t Lm,
                        std::vector<uint32_t>& counts, Emit&& emit, uint64_t pbase = 0) {
    counts.assign(nq, 0);
    if (Lm == 0 || nq == 0) return true;
    if (!HIP_CHECK(hipSetDevice(R.device))) return false;
    const size_t chunk = host_chunk(nq, Lm);
    const uint32_t n_chunks = (uint32_t)((nq + chunk - 1) / chunk);
    std::unique_ptr<Context> ctx[2];
    ctx[0] = R.acquire();
    if (!ctx[0]) return false;
    if (n_chunks > 1 && !(ctx[1] = R.acquire())) {
        R.give_back(std::move(ctx[0]));
        return false;
    }
    HostChunk fl[2];
    bool ok = true, pending = false;
    for (uint32_t k = 0; k <= n_chunks && ok; ++k) {
        // queue chunk k, then complete chunk k - 1 while k runs
        if (k < n_chunks) {
            const uint32_t q0 = (uint32_t)(k * chunk), B = (uint32_t)std::min<size_t>(chunk, nq - q0);
            ok = queue_host_chunk(L, R, *ctx[k & 1], queries, q0, B, thr, Lm, fl[k & 1], pbase);
            if (!ok) break;
        }
        if (pending) ok = finish_host_chunk(L, R, fl[(k - 1) & 1], Lm, counts, k == n_chunks, emit);
        pending = k < n_chunks;
    }
    if (!ok)  // a chunk may still be queued: let it drain before its context is reused
        for (auto& c : ctx)
            if (c) hipStreamSynchronize(c->stream);
    for (auto& c : ctx)
        if (c) R.give_back(std::move(c));
    return ok;
}

// ... into flat (key, score) vectors
template <typename CharT>
bool host_search_one(Library& L, Replica& R, const CharT* const* queries, uint32_t nq, float thr, uint32_t Lm,
                     std::vector<uint32_t>& counts, std::vector<uint32_t>& keys, std::vector<float>& scores) {
    keys.clear();
    scores.clear();
    return host_search_chunks(L, R, queries, nq, thr, Lm, counts, [&](const void* recs, const float* sc, uint32_t n,
                                                                       bool, uint32_t) {
        const uint32_t* k = static_cast<const uint32_t*>(recs);
        keys.insert(keys.end(), k, k + n);
        scores.insert(scores.end(), sc, sc + n);
    });
}

// Queries per replica below which a batch is not split (a split costs a host thread and a
// launch sequence per replica). NGS_SPLIT_MIN overrides it (tests split small batches).
uint32_t split_min() {
    static const uint32_t v = [] {
        const char* e = std::getenv("NGS_SPLIT_MIN");
        return e ? std::max<uint32_t>(1, (uint32_t)std::strtoul(e, nullptr, 0)) : 4096u;
    }();
    return v;
}

// Host entry: one replica scores the batch, or (an index on several devices) contiguous slices
// of it go to the replicas, one host thread each, and the slices' results are joined in order.
// Queries are independent, so the joined result is the single-device result.
template <typename CharT>
bool host_search(Library& L, const CharT* const* queries, uint32_t nq, float thr, uint32_t limit,
                 std::vector<uint32_t>& counts, std::vector<uint32_t>& keys, std::vector<float>& scores) {
    const uint32_t Lm = effective_limit(L, limit);
    const size_t nrep = std::max<size_t>(L.split.size(), 1);
    const uint32_t parts = (uint32_t)std::min<uint64_t>(nrep, std::max<uint64_t>(1, nq / split_min()));
    if (parts <= 1) return host_search_one(L, *L.reps.front(), queries, nq, thr, Lm, counts, keys, scores);
    const uint32_t per = (nq + parts - 1) / parts;
    std::vector<std::vector<uint32_t>> pc(parts), pk(parts);
    std::vector<std::vector<float>> ps(parts);
    std::vector<char> pok(parts, 0);
    std::vector<int> perr(parts, 0);  // each worker's ngsLastError, handed to the caller's thread
    const int err0 = t_last_error;
    run_parts(L.workers, parts, [&](size_t i) {
        const uint32_t q0 = (uint32_t)i * per, n = std::min(per, nq - std::min(nq, q0));
        t_last_error = 0;
        pok[i] = host_search_one(L, *L.reps[L.split[i]], queries + q0, n, thr, Lm, pc[i], pk[i], ps[i]);
        perr[i] = pok[i] ? 0 : (t_last_error ? t_last_error : kErrInternal);
    });
    t_last_error = err0;
    for (uint32_t i = 0; i < parts; ++i)
        if (perr[i]) t_last_error = perr[i];
    counts.clear();
    keys.clear();
    scores.clear();
    counts.reserve(nq);
    for (uint32_t i = 0; i < parts; ++i) {
        if (!pok[i]) return false;
        counts.insert(counts.end(), pc[i].begin(), pc[i].end());
        keys.insert(keys.end(), pk[i].begin(), pk[i].end());
        scores.insert(scores.end(), ps[i].begin(), ps[i].end());
    }
    return true;
}

void set_valid(Library& L, const char* chars, int n) {
    uint32_t v[8] = {};
    for (int i = 0; i < n; ++i) {
        const uint8_t c = (uint8_t)chars[i];
        v[c >> 5] |= 1u << (c & 31);
    }
    {
        std::lock_guard<std::mutex> g(L.valid_mu);
        std::memcpy(L.valid, v, sizeof(v));
    }
    // the set's key flags (Replica::index_for) built here, so that the first search under it, an
    // ngsSearchDeviceAsync included, does not build and synchronise them (the caller's device kept)
    int dev = -1;
    (void)hipGetDevice(&dev);
    for (auto& R : L.reps) {
        DevIndex X;
        (void)R->index_for(v, X);
    }
    if (dev >= 0) (void)hipSetDevice(dev);
}

// result strings point into the index's own key storage (valid until dispose, hpp:443-447)
template <typename CharT>
uint32_t marshal(const Library& L, const std::vector<uint32_t>& keys, const std::vector<float>& sc,
                 CharT*** results, float** scores) {
    const size_t n = keys.size();
    if (scores) *scores = new float[n];
    *results = new CharT*[n];
    CharT** res = *results;
    float* out_s = scores ? *scores : nullptr;
    char* base = const_cast<char*>(L.host.key_bytes.data());
    const uint64_t* koff = L.host.key_off.data();
    auto fill = [&](size_t a, size_t b) {  // key_off is gathered at random: memory-latency bound
        for (size_t i = a; i < b; ++i) {
            res[i] = reinterpret_cast<CharT*>(base + koff[keys[i]] * sizeof(CharT));
            if (out_s) out_s[i] = sc[i];
        }
    };
    // a whole batch's records (1.3M at C3) on several host threads
    const size_t nt = n < (size_t(1) << 18) ? 1 : std::min<size_t>(8, std::max(1u, std::thread::hardware_concurrency()));
    if (nt <= 1) {
        fill(0, n);
    } else {
        std::vector<std::thread> th;
        for (size_t t = 0; t < nt; ++t) th.emplace_back(fill, n * t / nt, n * (t + 1) / nt);
        for (auto& x : th) x.join();
    }
    return (uint32_t)n;
}

// The query normalised as k_prep does it (escapeBlank with the index's validChar set, C-locale
// trim, toUpper; nGramSearch.hpp:372-376): its length (kQueryWildcard for "" and "*"), false if
// it does not fit `cap` characters.
bool host_normalise(const uint32_t* valid, const char* q, uint8_t* out, uint32_t cap, uint32_t& m) {
    const size_t n = std::strlen(q);
    if (n == 0 || (n == 1 && q[0] == '*')) {  // nGramSearch.hpp:356
        m = kQueryWildcard;
        return true;
    }
    auto esc = [&](uint8_t c) -> uint8_t { return ((valid[c >> 5] >> (c & 31)) & 1u) ? c : (uint8_t)' '; };
    auto space = [](uint8_t c) { return c == ' ' || (c >= 9 && c <= 13); };
    size_t a = 0, e = n;
    while (a < e && space(esc((uint8_t)q[a]))) ++a;
    while (e > a && space(esc((uint8_t)q[e - 1]))) --e;
    if (e - a > cap) return false;
    m = (uint32_t)(e - a);
    for (size_t i = a; i < e; ++i) {
        const uint8_t c = esc((uint8_t)q[i]);
        out[i - a] = (c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c;
    }
    return true;
}

// score() through the server (ngsServe): false when the call must take the regular path (a
// limit above the wave search's, a library large enough for the sliced latency path, a query
// the server routes to tier 2 or the general path, or a server that cannot be reached).
bool serve_query(Library& L, const char* query, float thr, uint32_t limit, std::vector<uint32_t>& keys,
                 std::vector<float>& sc) {
    // the server's lifetime (shared: requests of other threads run beside this one)
    std::shared_lock<std::shared_mutex> g(L.server_mu);
    if (L.batches.load(std::memory_order_acquire) > 0) return false;
    Server* sv = L.server.get();
    const uint32_t Lm = effective_limit(L, limit);
    Replica& R = *L.reps.front();
    if (!sv || Lm == 0 || Lm > kWaveMaxLimit || R.dev.n_buckets / 8 > 1) return false;
    // a free request slot, tried from one of this thread's own; all busy: try them again (a request
    // holds its slot ~15 us, and a thread put to sleep on a mutex took ~50 us to wake: 8 threads on
    // 4 slots ran at 84k calls/s blocking, against 240k for 4 threads)
    static std::atomic<uint32_t> next_hint{0};
    thread_local const uint32_t hint = next_hint.fetch_add(1, std::memory_order_relaxed);
    uint32_t slot = 0;
    std::unique_lock<std::mutex> sl;
    for (uint32_t i = 0; !sl.owns_lock(); ++i) {
        const uint32_t k = (hint + i) % kServeSlots;
        sl = std::unique_lock<std::mutex>(sv->slot_mu[k], std::try_to_lock);
        if (sl.owns_lock()) slot = k;
        else if (i % kServeSlots == kServeSlots - 1) {
            if (i > 64 * kServeSlots) std::this_thread::yield();
            else __builtin_ia32_pause();
        }
    }
    ServeBlock* b = sv->h + slot;
    uint32_t m = 0;
    {
        std::lock_guard<std::mutex> gv(L.valid_mu);
        if (!host_normalise(L.valid, query, b->q, kServeMaxQuery, m)) return false;
        std::memcpy(b->valid, L.valid, sizeof(b->valid));
    }
    b->thr = thr;
    b->limit = Lm;
    b->m = m;
    b->off[0] = 0;
    b->off[1] = m == kQueryWildcard ? 0 : m;
    const uint64_t seq = ++sv->seq[slot];
    // (re)launch when the kernel has left; a running server reads the key flags of the validChar set
    // it was launched with, so a new set restarts it (the other slots' requests are answered by
    // the new kernel: theirs stay posted)
    auto launch = [&](bool force) -> bool {
        std::lock_guard<std::mutex> gl(sv->launch_mu);
        if (force && R.dev.kt_off && !sv->stopped()) sv->stop();
        if (!sv->stopped()) return true;
        if (!HIP_CHECK(hipSetDevice(sv->device))) return false;
        SearchParams P{};
        P.n_queries = 1;
        P.nslices = 1;
        DevIndex X;
        if (!R.index_for(b->valid, X)) return false;
        std::memcpy(sv->launch_valid, b->valid, sizeof(sv->launch_valid));
        sv->launched = HIP_CHECK(launch_serve(X, P, sv->d, sv->scratch, sv->list2, sv->t_any, kServeIdleMs,
                                              kServeLifeMs, sv->stream));
        return sv->launched;
    };
    {
        bool stale;
        {
            std::lock_guard<std::mutex> gl(sv->launch_mu);
            stale = R.dev.kt_off && std::memcmp(sv->launch_valid, b->valid, sizeof(b->valid)) != 0;
        }
        if ((stale || sv->stopped()) && !launch(stale)) return false;
    }
    __atomic_store_n(&b->req_seq, seq, __ATOMIC_RELEASE);  // the fields above first (x86 stores stay in order)
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t spin = 1; __atomic_load_n(&b->done_seq, __ATOMIC_ACQUIRE) != seq; ++spin) {
        if ((spin & 1023) == 0) {
            // the kernel left (its idle time ran out as the request came in): relaunch, it
            // answers the posted request
            if (sv->stopped() && !launch(false)) return false;
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
                std::lock_guard<std::mutex> gl(sv->launch_mu);
                sv->stop();  // unreachable: leave it to the regular path
                return false;
            }
        }
        __builtin_ia32_pause();
    }
    if (__atomic_load_n(&b->status, __ATOMIC_ACQUIRE) != 0) return false;
    const uint32_t n = std::min(b->n, Lm);
    keys.assign(b->keys, b->keys + n);
    sc.assign(b->scores, b->scores + n);
    return true;
}

// Starts the server for a library it can answer once kAutoServeAfter single-query calls came in
// (unless ngsServe(h, 0) turned it off): score() at the reference's C1 latency with no opt-in.
void maybe_auto_serve(Library& L) {
    if (L.serve_pref.load(std::memory_order_relaxed) != 0 || L.reps.empty() || L.host.csize != 1) return;
    if (L.reps.front()->dev.n_buckets / 8 > 1) return;  // a large library keeps the sliced latency path
    if (L.single_calls.fetch_add(1, std::memory_order_relaxed) + 1 < kAutoServeAfter) return;
    std::unique_lock<std::shared_mutex> g(L.server_mu, std::try_to_lock);
    if (!g.owns_lock() || L.server || L.serve_pref.load() != 0) return;
    auto sv = std::make_unique<Server>();
    if (!sv->init(L.reps.front()->device)) {
        L.serve_pref.store(-1);  // no server on this device: do not try again
        (void)hipGetLastError();
        t_last_error = 0;
        return;
    }
    L.server = std::move(sv);
    L.serving.store(true, std::memory_order_release);
}

// batches of more than kSmallBatch queries count as batch traffic (smaller ones take the latency
// path, like score())
inline Library* batch_mark(Library* L, uint32_t nq) { return nq > kSmallBatch ? L : nullptr; }

// Marks a batch call in flight for its lifetime: a running server kernel is stopped first (its
// stream may share a hardware queue with the batch's streams) and is not relaunched meanwhile.
struct BatchGuard {
    Library* L;
    explicit BatchGuard(Library* l) : L(l) {
        if (!L) return;
        L->batches.fetch_add(1, std::memory_order_acq_rel);
        if (L->serving.load(std::memory_order_acquire)) {
            std::lock_guard<std::shared_mutex> g(L->server_mu);
            if (L->server && !L->server->stopped()) L->server->stop();
        }
    }
    ~BatchGuard() {
        if (L) L->batches.fetch_sub(1, std::memory_order_acq_rel);
    }
    BatchGuard(const BatchGuard&) = delete;
    BatchGuard& operator=(const BatchGuard&) = delete;
};

// A narrow call on a wide index (or the reverse) is answered like an unknown handle.
template <typename CharT>
uint32_t one_query(uint32_t handle, const CharT* query, CharT*** results, float** scores, float thr,
                   uint32_t limit) {
    std::shared_lock<std::shared_mutex> lk(g_lock);
    Library* L = find_lib(handle);
    if (!L || !L->host.indexed || !query || L->host.csize != sizeof(CharT)) return 0;  // dllmain.cpp:69, hpp:417-418
    std::vector<uint32_t> counts, keys;
    std::vector<float> sc;
    if (sizeof(CharT) == 1 && !L->serving.load(std::memory_order_acquire)) maybe_auto_serve(*L);
    if (sizeof(CharT) == 1 && L->serving.load(std::memory_order_acquire) && serve_query(*L, reinterpret_cast<const char*>(query), thr, limit, keys, sc))
        return marshal(*L, keys, sc, results, scores);
    // the regular path's kernels while a server exists (it cannot take this query: a limit past the
    // wave search's, tier 2 or the general path): stop it first, since its stream may share a
    // hardware queue with ours and a resident server would hold our launches until its idle exit
    BatchGuard bg(L->serving.load(std::memory_order_acquire) ? L : nullptr);
    if (!host_search(*L, &query, 1, thr, limit, counts, keys, sc)) return 0;
    return marshal(*L, keys, sc, results, scores);
}

// A batch split over the replicas with the one-replica path's pointer mode (dllmain.cpp:82-90 over
// several devices): each replica's part packs its records on its device as result pointers, the
// parts publish their record counts, the last one allocates the caller's arrays at the exact total,
// and every part copies its records into its own slice of them straight from its pinned read-back.
// kNoDirect: a part would take several chunks (the caller's general path then joins vectors).
constexpr uint32_t kNoDirect = 0xFFFFFFFFu;
template <typename CharT>
uint32_t split_direct(Library& L, const CharT* const* queries, uint32_t nq, float thr, uint32_t Lm, uint32_t* counts,
                      CharT*** results, float** scores) {
    const uint32_t parts = (uint32_t)std::min<uint64_t>(L.split.size(), std::max<uint64_t>(1, nq / split_min()));
    const uint32_t per = (nq + parts - 1) / parts;
    if (parts < 2 || host_chunk(per, Lm) < per || (uint64_t)nq * Lm > kDirectMax) return kNoDirect;
    const uint64_t pbase = (uint64_t)(uintptr_t)L.host.key_bytes.data();
    std::mutex mu;
    std::condition_variable cv;
    std::vector<uint64_t> total(parts, 0), base(parts, 0);
    uint32_t known = 0;
    bool failed = false, ready = false;
    CharT** res = nullptr;
    float* out_s = nullptr;
    // part i knows its record count: the last part to know allocates the arrays for everyone
    auto publish = [&](uint32_t i, uint64_t n, bool fail) {
        std::unique_lock<std::mutex> lk(mu);
        total[i] = n;
        failed |= fail;
        if (++known == parts) {
            uint64_t sum = 0;
            for (uint32_t j = 0; j < parts; ++j) base[j] = sum, sum += total[j];
            if (!failed) {
                res = new CharT*[std::max<uint64_t>(sum, 1)];
                out_s = scores ? new float[std::max<uint64_t>(sum, 1)] : nullptr;
            }
            ready = true;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return ready; });
        }
    };
    std::vector<std::vector<uint32_t>> pc(parts);
    std::vector<int> perr(parts, 0);
    const int err0 = t_last_error;
    run_parts(L.workers, parts, [&](size_t pi) {
        const uint32_t i = (uint32_t)pi, q0 = i * per, n = std::min(per, nq - std::min(nq, q0));
        t_last_error = 0;
        bool seen = false;
        size_t off = 0;
        const bool ok = host_search_chunks(L, *L.reps[L.split[i]], queries + q0, n, thr, Lm, pc[i],
                                           [&](const void* recs, const float* sc, uint32_t m, bool, uint32_t chunk_total) {
            if (!seen) {  // (one chunk: its total is the part's)
                seen = true;
                publish(i, chunk_total, false);
            }
            if (!res) return;  // another part failed
            const uint64_t* p = static_cast<const uint64_t*>(recs);
            CharT** dst = res + base[i] + off;
            float* dsc = out_s ? out_s + base[i] + off : nullptr;
            parallel_ranges(m, size_t(1) << 16, [&](size_t a, size_t e) {
                std::memcpy(dst + a, p + a, (e - a) * sizeof(uint64_t));
                if (dsc) std::memcpy(dsc + a, sc + a, (e - a) * sizeof(float));
            });
            off += m;
        }, pbase);
        if (!seen) publish(i, 0, true);  // (failed before its records: the others must not wait)
        if (!ok) perr[i] = t_last_error ? t_last_error : kErrInternal;
    });
    t_last_error = err0;
    bool bad = failed;
    for (uint32_t i = 0; i < parts; ++i)
        if (perr[i]) bad = true, t_last_error = perr[i];
    if (bad) {
        delete[] res;
        delete[] out_s;
        return 0;
    }
    uint64_t sum = 0;
    for (uint32_t i = 0; i < parts; ++i) {
        std::copy(pc[i].begin(), pc[i].end(), counts + (size_t)i * per);
        sum += total[i];
    }
    *results = res;
    if (scores) *scores = out_s;
    return (uint32_t)sum;
}

template <typename CharT>
uint32_t batch_query(uint32_t handle, const CharT* const* queries, uint32_t nq, float thr, uint32_t limit,
                     uint32_t* counts, CharT*** results, float** scores) {
    if (counts) std::fill(counts, counts + nq, 0u);
    std::shared_lock<std::shared_mutex> lk(g_lock);
    Library* L = find_lib(handle);
    if (!L || !L->host.indexed || !queries || !counts || L->host.csize != sizeof(CharT)) return 0;
    // (a small batch takes the latency path and stops a running server like score()'s fallback)
    BatchGuard bg(L->serving.load(std::memory_order_acquire) ? L : batch_mark(L, nq));
    std::vector<uint32_t> cnt, keys;
    std::vector<float> sc;
    HostTimer ht;
    const uint32_t Lm = effective_limit(*L, limit);
    const bool one_replica = L->split.size() <= 1 || nq / split_min() <= 1;
    if (one_replica && Lm && (uint64_t)nq * Lm <= kDirectMax && nq >= kSmallBatch) {
        // marshalled as the chunks finish, straight into the caller's arrays. One chunk (the
        // common case): the arrays at the exact size, filled from the pinned read-back; several
        // chunks: at the batch's capacity (nq x limit entries; only the pages written are touched)
        CharT** res = nullptr;
        float* out_s = nullptr;
        size_t off = 0, cap = 0;
        // pointer mode: k_pack writes each record as its result pointer into the host key bytes
        // (key_off gathered on the device), so marshalling is two parallel copies
        const uint64_t pbase = (uint64_t)(uintptr_t)L->host.key_bytes.data();
        static_assert(sizeof(CharT*) == sizeof(uint64_t), "result pointers are 64-bit");
        const bool ok = host_search_chunks(*L, *L->reps.front(), queries, nq, thr, Lm, cnt,
                                           [&](const void* recs, const float* sc, uint32_t n, bool last,
                                               uint32_t chunk_total) {
            if (!res) {
                cap = (off == 0 && last) ? std::max<size_t>(chunk_total, 1) : (size_t)nq * Lm;
                res = new CharT*[cap];
                out_s = scores ? new float[cap] : nullptr;
            }
            const uint64_t* p = static_cast<const uint64_t*>(recs);
            parallel_ranges(n, size_t(1) << 16, [&](size_t a, size_t e) {
                std::memcpy(res + off + a, p + a, (e - a) * sizeof(uint64_t));
                if (out_s) std::memcpy(out_s + off + a, sc + a, (e - a) * sizeof(float));
            });
            off += n;
        }, pbase);
        if (ok && !res) {  // no chunk ran (cannot happen with nq >= kSmallBatch): empty arrays
            res = new CharT*[1];
            out_s = scores ? new float[1] : nullptr;
        }
        if (!ok) {
            delete[] res;
            delete[] out_s;
            return 0;
        }
        ht.mark(kHpCall, "search + marshal (chunks)");
        g_host_phase[kHpCalls].fetch_add(1, std::memory_order_relaxed);
        std::copy(cnt.begin(), cnt.end(), counts);
        *results = res;
        if (scores) *scores = out_s;
        return (uint32_t)off;
    }
    if (Lm && nq >= kSmallBatch && !one_replica) {
        const uint32_t n = split_direct(*L, queries, nq, thr, Lm, counts, results, scores);
        if (n != kNoDirect) {
            ht.mark(kHpCall, "search + marshal (replicas)");
            g_host_phase[kHpCalls].fetch_add(1, std::memory_order_relaxed);
            return n;
        }
    }
    if (!host_search(*L, queries, nq, thr, limit, cnt, keys, sc)) return 0;
    std::copy(cnt.begin(), cnt.end(), counts);
    const uint32_t n = marshal(*L, keys, sc, results, scores);
    ht.mark(kHpCall, "search + marshal");
    if (nq >= kSmallBatch) g_host_phase[kHpCalls].fetch_add(1, std::memory_order_relaxed);
    return n;
}

}  // namespace
}  // namespace ngs

using namespace ngs;

namespace ngs {
namespace {
// dllmain.cpp:37-59 for every index flavour: smallest free handle, build, upload.
template <class Build>
uint32_t new_library(Build&& build) {
    std::unique_lock<std::shared_mutex> lk(g_lock);  // dllmain.cpp:39
    uint32_t handle = 1;                             // dllmain.cpp:41-46
    const uint32_t maxVal = std::numeric_limits<uint32_t>::max();
    while (g_libs.count(handle) && handle < maxVal) ++handle;
    if (handle == maxVal) return 0;
    auto L = std::make_unique<Library>();
    set_valid(*L, kDefaultValid, (int)std::strlen(kDefaultValid));
    std::vector<int> devs = t_devices;
    if (devs.empty()) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess) dev = 0;
        devs.push_back(dev);
    }
    (void)hipSetDevice(devs.front());  // the build's device kernels run on the first replica's device
    PhaseTimer pt;
    build(L->host);
    pt.mark("build (intern + layout)");
    if (L->host.indexed && !upload(*L, devs)) {
        std::fprintf(stderr, "ngram_search: indexN could not place the index on a GPU\n");
        return 0;
    }
    if (!L->host.indexed) L->device = devs.front();
    g_libs.emplace(handle, std::move(L));
    return handle;
}
}  // namespace
}  // namespace ngs

extern "C" {

NGS_API uint32_t indexN(char** words, uint64_t size, uint16_t rowSize, float* weight) {
    return new_library([&](HostIndex& H) { build_index(H, words, size, rowSize, weight); });
}

NGS_API uint32_t indexG(char** words, uint64_t size, uint16_t rowSize, float* weight, uint16_t gSize) {
    if (gSize < 1 || gSize > kMaxGramSize) return 0;
    return new_library([&](HostIndex& H) { build_index_g(H, words, size, rowSize, weight, gSize); });
}

NGS_API uint32_t indexW(wchar_t** words, uint64_t size, uint16_t rowSize, float* weight, uint16_t gSize) {
    static_assert(sizeof(wchar_t) == 4, "wide strings are UTF-32");
    if (gSize < 1 || gSize > kMaxGramSize) return 0;
    return new_library([&](HostIndex& H) {
        build_index_w(H, reinterpret_cast<const uint32_t* const*>(words), size, rowSize, weight, gSize);
    });
}

NGS_API uint32_t search(uint32_t handle, const char* query, char*** results, float threshold, uint32_t limit) {
    return one_query(handle, query, results, nullptr, threshold, limit);
}

NGS_API uint32_t score(uint32_t handle, const char* query, char*** results, float** scores, float threshold,
                       uint32_t limit) {
    return one_query(handle, query, results, scores, threshold, limit);
}

NGS_API void release(uint32_t handle, char** results, float* scores) {
    std::shared_lock<std::shared_mutex> lk(g_lock);  // dllmain.cpp:100-103
    if (!find_lib(handle)) return;
    delete[] results;
    delete[] scores;
}

NGS_API void dispose(uint32_t handle) {
    std::unique_lock<std::shared_mutex> lk(g_lock);  // dllmain.cpp:112-113
    g_libs.erase(handle);
}

NGS_API uint64_t getSize(uint32_t handle) {
    std::shared_lock<std::shared_mutex> lk(g_lock);
    Library* L = find_lib(handle);
    return L ? L->host.n_terms : 0;
}

NGS_API uint64_t getLibSize(uint32_t handle) {
    std::shared_lock<std::shared_mutex> lk(g_lock);
    Library* L = find_lib(handle);
    return L ? L->host.n_grams : 0;
}

NGS_API void setValidChar(uint32_t handle, char* characters, int n) {
    std::shared_lock<std::shared_mutex> lk(g_lock);
    Library* L = find_lib(handle);
    if (L && (characters || n == 0)) set_valid(*L, characters, n);
}

NGS_API uint32_t scoreBatch(uint32_t handle, const char* const* queries, uint32_t nQueries, float threshold,
                            uint32_t limit, uint32_t* counts, char*** results, float** scores) {
    return batch_query(handle, queries, nQueries, threshold, limit, counts, results, scores);
}

NGS_API uint32_t searchBatch(uint32_t handle, const char* const* queries, uint32_t nQueries, float threshold,
                             uint32_t limit, uint32_t* counts, char*** results) {
    return batch_query(handle, queries, nQueries, threshold, limit, counts, results, nullptr);
}

// ---- wide (UTF-32 wchar_t) API: Readme.md:91,135,170,190,208,226, keyed by handle like the
// narrow exports (dllmain.cpp). Valid only on indexW handles; narrow calls on a wide handle
// and wide calls on a narrow handle return 0 / nothing.

NGS_API uint32_t searchW(uint32_t handle, const wchar_t* query, wchar_t*** results, float threshold,
                         uint32_t limit) {
    return one_query(handle, query, results, nullptr, threshold, limit);
}

NGS_API uint32_t scoreW(uint32_t handle, const wchar_t* query, wchar_t*** results, float** scores,
                        float threshold, uint32_t limit) {
    return one_query(handle, query, results, scores, threshold, limit);
}

NGS_API uint32_t scoreBatchW(uint32_t handle, const wchar_t* const* queries, uint32_t nQueries, float threshold,
                             uint32_t limit, uint32_t* counts, wchar_t*** results, float** scores) {
    return batch_query(handle, queries, nQueries, threshold, limit, counts, results, scores);
}

NGS_API uint32_t searchBatchW(uint32_t handle, const wchar_t* const* queries, uint32_t nQueries, float threshold,
                              uint32_t limit, uint32_t* counts, wchar_t*** results) {
    return batch_query(handle, queries, nQueries, threshold, limit, counts, results, nullptr);
}

NGS_API void releaseW(uint32_t handle, wchar_t** results, float* scores) {
    std::shared_lock<std::shared_mutex> lk(g_lock);
    if (!find_lib(handle)) return;
    delete[] results;
    delete[] scores;
}

NGS_API void disposeW(uint32_t handle) { dispose(handle); }

NGS_API uint64_t getSizeW(uint32_t handle) { return getSize(handle); }

NGS_API uint64_t getLibSizeW(uint32_t handle) { return getLibSize(handle); }

NGS_API int ngsSetDevices(const int* devices, int n) {
    if (n < 0 || (n > 0 && !devices)) return -(int)hipErrorInvalidValue;
    int nd = 0;
    hipError_t e = hipGetDeviceCount(&nd);
    if (e != hipSuccess) return -(int)e;
    for (int i = 0; i < n; ++i)
        if (devices[i] < 0 || devices[i] >= nd) return -(int)hipErrorInvalidDevice;
    t_devices.assign(devices, devices + n);
    return 0;
}

NGS_API int ngsSetDevice(int device) { return ngsSetDevices(&device, 1); }

NGS_API int ngsReplicaCount(uint32_t handle) {
    std::shared_lock<std::shared_mutex> lk(g_lock);
    Library* L = find_lib(handle);
    return L ? (int)L->reps.size() : -1;
}

NGS_API int ngsDeviceCount(void) {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}

NGS_API uint32_t ngsNumKeys(uint32_t handle) {
    std::shared_lock<std::shared_mutex> lk(g_lock);
    Library* L = find_lib(handle);
    return L ? L->host.n_keys : 0;
}

NGS_API const char* ngsKey(uint32_t handle, uint32_t keyId) {
    std::shared_lock<std::shared_mutex> lk(g_lock);
    Library* L = find_lib(handle);
    if (!L || keyId >= L->host.n_keys || L->host.csize != 1) return nullptr;
    return L->host.key_bytes.data() + L->host.key_off[keyId];
}

NGS_API const wchar_t* ngsKeyW(uint32_t handle, uint32_t keyId) {
    std::shared_lock<std::shared_mutex> lk(g_lock);
    Library* L = find_lib(handle);
    if (!L || keyId >= L->host.n_keys || L->host.csize != sizeof(wchar_t)) return nullptr;
    return reinterpret_cast<const wchar_t*>(L->host.key_bytes.data() + L->host.key_off[keyId] * sizeof(wchar_t));
}

NGS_API uint32_t ngsCharSize(uint32_t handle) {
    std::shared_lock<std::shared_mutex> lk(g_lock);
    Library* L = find_lib(handle);
    return L ? L->host.csize : 0;
}

NGS_API uint32_t ngsGramSize(uint32_t handle) {
    std::shared_lock<std::shared_mutex> lk(g_lock);
    Library* L = find_lib(handle);
    return L ? L->host.gsz : 0;
}

NGS_API int ngsSearchDevice(uint32_t handle, const uint8_t* dQueryBytes, const uint64_t* dQueryOffsets,
                            uint32_t nQueries, float threshold, uint32_t limit, uint32_t outStride, uint32_t* dCounts,
                            uint32_t* dKeys, float* dScores, void* stream) {
    std::shared_lock<std::shared_mutex> lk(g_lock);
    Library* L = find_lib(handle);
    if (!L) return -1;
    if (!L->host.indexed) return -2;
    const uint32_t Lm = effective_limit(*L, limit);
    if (!dQueryOffsets || !dCounts || (nQueries && Lm && (!dKeys || !dScores || outStride < Lm))) return -3;
    // the replica on the caller's current device (the buffers' device)
    int cur = L->device;
    if (!HIP_CHECK(hipGetDevice(&cur))) return -4;
    Replica* Rp = L->replica_at(cur);
    if (!Rp) return -3;  // no replica on the caller's device: its buffers and stream belong there
    Replica& R = *Rp;
    hipStream_t s = (hipStream_t)stream;
    BatchGuard bg(L);
    if (Lm == 0) {
        return HIP_CHECK(hipMemsetAsync(dCounts, 0, sizeof(uint32_t) * nQueries, s)) &&
                       HIP_CHECK(hipStreamSynchronize(s))
                   ? 0
                   : -4;
    }
    std::unique_ptr<Context> c = R.acquire();
    if (!c) return -4;
    // The batch's byte count sizes the normalised-query buffer. A context that has one already
    // launches without reading it back (a sync before any kernel); k_prep flags a batch that
    // does not fit and the call reruns after the read-back.
    int rc = 0;
    auto read_bytes = [&](uint64_t& qb) -> bool {
        return HIP_CHECK(hipMemcpyAsync(&qb, dQueryOffsets + nQueries, sizeof(uint64_t), hipMemcpyDeviceToHost, s)) &&
               HIP_CHECK(hipStreamSynchronize(s));
    };
    uint64_t qbytes = 0;
    if (nQueries && !c->qcap && !read_bytes(qbytes)) rc = -4;
    if (!rc) rc = device_search(*L, R, *c, dQueryBytes, dQueryOffsets, nQueries, qbytes, threshold, Lm, outStride,
                                dCounts, dKeys, dScores, s);
    if (rc == kRetryQcap) {
        rc = read_bytes(qbytes) ? device_search(*L, R, *c, dQueryBytes, dQueryOffsets, nQueries, qbytes, threshold, Lm,
                                                outStride, dCounts, dKeys, dScores, s)
                                : -4;
        if (rc == kRetryQcap) {
            rc = -5;
            t_last_error = kErrQueryBuffer;
        }
    }
    R.give_back(std::move(c));
    return rc;
}

// Asynchronous form (bench.py's pipeline; a server's batches): queue the search on a pooled
// context's own streams, ordered after the work already queued on `stream`, and return. Two
// calls in flight overlap on the GPU: one batch's tail (the last tier-1a waves, k_emit, tier 1b)
// runs beside the next batch's counting.
NGS_API int ngsSearchDeviceAsync(uint32_t handle, const uint8_t* dQueryBytes, const uint64_t* dQueryOffsets,
                                 uint32_t nQueries, float threshold, uint32_t limit, uint32_t outStride,
                                 uint32_t* dCounts, uint32_t* dKeys, float* dScores, void* stream, uint64_t* ticket) {
    std::shared_lock<std::shared_mutex> lk(g_lock);
    Library* L = find_lib(handle);
    if (!L) return -1;
    if (!L->host.indexed) return -2;
    const uint32_t Lm = effective_limit(*L, limit);
    if (!ticket || !dQueryOffsets || !dCounts || (nQueries && Lm && (!dKeys || !dScores || outStride < Lm))) return -3;
    int cur = L->device;
    if (!HIP_CHECK(hipGetDevice(&cur))) return -4;
    Replica* Rp = L->replica_at(cur);
    if (!Rp) return -3;
    hipStream_t s = (hipStream_t)stream;
    BatchGuard bg(L);  // the server stops here; the pending call keeps it stopped until its Wait
    // the batch mark the pending call holds until its Wait; released here on any early return
    struct Mark {
        Library* L;
        bool armed = true;
        explicit Mark(Library* l) : L(l) { L->batches.fetch_add(1, std::memory_order_acq_rel); }
        ~Mark() {
            if (armed) L->batches.fetch_sub(1, std::memory_order_acq_rel);
        }
    } mark(L);
    Library::Pending pd;
    pd.R = Rp;
    pd.dq = dQueryBytes;
    pd.doff = dQueryOffsets;
    pd.B = nQueries;
    pd.Lm = Lm;
    pd.stride = outStride;
    pd.thr = threshold;
    pd.dn = dCounts;
    pd.dk = dKeys;
    pd.ds = dScores;
    if (Lm == 0 || nQueries == 0) {
        if (!HIP_CHECK(hipMemsetAsync(dCounts, 0, sizeof(uint32_t) * nQueries, s))) return -4;
    } else {
        pd.c = Rp->acquire();
        if (!pd.c) return -4;
        Context& c = *pd.c;
        uint64_t qbytes = 0;
        if (!c.qcap && !(HIP_CHECK(hipMemcpyAsync(&qbytes, dQueryOffsets + nQueries, sizeof(uint64_t),
                                                 hipMemcpyDeviceToHost, s)) &&
                         HIP_CHECK(hipStreamSynchronize(s)))) {
            Rp->give_back(std::move(pd.c));
            return -4;
        }
        if (!HIP_CHECK(hipEventRecord(c.in_ev, s)) || !HIP_CHECK(hipStreamWaitEvent(c.stream, c.in_ev, 0))) {
            Rp->give_back(std::move(pd.c));
            return -4;
        }
        pd.rc = queue_search(*L, *Rp, c, dQueryBytes, dQueryOffsets, nQueries, qbytes, threshold, Lm, outStride,
                             dCounts, dKeys, dScores, c.stream, pd.P, false);
    }
    std::lock_guard<std::mutex> g(L->pend_mu);
    *ticket = L->next_ticket++;
    L->pending.emplace(*ticket, std::move(pd));
    mark.armed = false;  // ngsSearchDeviceWait releases it
    return 0;
}

// Completes an ngsSearchDeviceAsync call: waits for its kernels, runs the general path for the
// queries that need it, records the statistics (ngsLastStats). The results are then in place.
// Same return codes as ngsSearchDevice; -3 for an unknown ticket.
NGS_API int ngsSearchDeviceWait(uint32_t handle, uint64_t ticket) {
    std::shared_lock<std::shared_mutex> lk(g_lock);
    Library* L = find_lib(handle);
    if (!L) return -1;
    Library::Pending pd;
    {
        std::lock_guard<std::mutex> g(L->pend_mu);
        auto it = L->pending.find(ticket);
        if (it == L->pending.end()) return -3;
        pd = std::move(it->second);
        L->pending.erase(it);
    }
    struct Done {  // the Async call's batch mark ends with its Wait
        Library* L;
        ~Done() { L->batches.fetch_sub(1, std::memory_order_acq_rel); }
    } done{L};
    if (!pd.c) return 0;  // nothing was queued (limit 0 or no queries): the counts were cleared
    Replica& R = *pd.R;
    Context& c = *pd.c;
    if (!HIP_CHECK(hipSetDevice(R.device))) {
        R.give_back(std::move(pd.c));
        return -4;
    }
    int rc = pd.rc ? pd.rc : finish_search(*L, R, c, pd.B, pd.P, pd.doff, pd.dn, pd.dk, pd.ds, c.stream);
    if (rc == kRetryQcap) {  // the batch outgrew the context's query buffer: rerun with its size
        uint64_t qbytes = 0;
        rc = HIP_CHECK(hipMemcpyAsync(&qbytes, pd.doff + pd.B, sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream)) &&
                     HIP_CHECK(hipStreamSynchronize(c.stream))
                 ? device_search(*L, R, c, pd.dq, pd.doff, pd.B, qbytes, pd.thr, pd.Lm, pd.stride, pd.dn, pd.dk,
                                 pd.ds, c.stream)
                 : -4;
        if (rc == kRetryQcap) {
            rc = -5;
            t_last_error = kErrQueryBuffer;
        }
    }
    R.give_back(std::move(pd.c));
    return rc;
}

NGS_API int ngsServe(uint32_t handle, int enable) {
    std::shared_lock<std::shared_mutex> lk(g_lock);
    Library* L = find_lib(handle);
    if (!L) return -1;
    if (!L->host.indexed || L->reps.empty()) return -2;
    if (L->host.csize != 1) return -3;
    std::lock_guard<std::shared_mutex> g(L->server_mu);
    if (!enable) {
        L->serve_pref.store(-1);  // off, and no automatic start either
        L->serving.store(false, std::memory_order_release);
        L->server.reset();
        return 0;
    }
    L->serve_pref.store(1);
    if (L->server) return 0;
    auto sv = std::make_unique<Server>();
    if (!sv->init(L->reps.front()->device)) return -4;
    L->server = std::move(sv);
    L->serving.store(true, std::memory_order_release);
    return 0;
}

NGS_API int ngsPackResults(const uint32_t* dCounts, const uint32_t* dKeys, const float* dScores, uint32_t n,
                           uint32_t stride, uint32_t* dOffsets, uint32_t* dRecords, void* stream) {
    if (!dCounts || !dOffsets || (n && (!dKeys || !dScores || !dRecords || !stride))) return -3;
    // the scan's scratch: one grow-only buffer per (device, stream), so that calls on different
    // streams never share one while their scans run; a buffer is replaced only after its stream's
    // earlier work has finished with it. (The mutex orders the host-side bookkeeping only.)
    static std::mutex mu;
    static std::map<std::pair<int, hipStream_t>, std::pair<void*, size_t>> temp;
    int dev = 0;
    if (!HIP_CHECK(hipGetDevice(&dev))) return -4;
    std::lock_guard<std::mutex> g(mu);
    auto& t = temp[{dev, (hipStream_t)stream}];
    const size_t need = pack_pairs_temp_bytes(n);
    if (need > t.second) {
        if (t.first && !HIP_CHECK(hipStreamSynchronize((hipStream_t)stream))) return -4;
        if (t.first) (void)hipFree(t.first);
        t = {nullptr, 0};
        if (!HIP_CHECK(hipMalloc(&t.first, std::max<size_t>(need, 1 << 16)))) return -4;
        t.second = std::max<size_t>(need, 1 << 16);
    }
    return HIP_CHECK(launch_pack_pairs(dCounts, dKeys, dScores, n, stride, dOffsets, dRecords, t.first, t.second,
                                       (hipStream_t)stream))
               ? 0
               : -4;
}

NGS_API int ngsServeState(uint32_t handle) {
    std::shared_lock<std::shared_mutex> lk(g_lock);
    Library* L = find_lib(handle);
    if (!L) return -1;
    std::shared_lock<std::shared_mutex> g(L->server_mu);
    if (!L->server) return 0;
    return L->server->stopped() ? 1 : 2;
}

NGS_API int ngsLastError(int clear) {
    const int e = t_last_error;
    if (clear) t_last_error = 0;
    return e;
}

NGS_API int ngsSetTiming(uint32_t handle, int enable) {
    std::shared_lock<std::shared_mutex> lk(g_lock);
    Library* L = find_lib(handle);
    if (!L) return -1;
    L->timing.store(enable != 0);
    return 0;
}

NGS_API int ngsLastStats(uint32_t handle, ngs_stats* out) {
    std::shared_lock<std::shared_mutex> lk(g_lock);
    Library* L = find_lib(handle);
    if (!L || !out) return -1;
    std::lock_guard<std::mutex> g(L->stats_mu);
    *out = L->last;
    return 0;
}

#ifndef NGS_SRC_HASH
#define NGS_SRC_HASH "unknown"
#endif
NGS_API const char* ngsVersion(void) { return "ngram_search 0.2 gfx950 src=" NGS_SRC_HASH; }

NGS_API int ngsIndexDigest(uint32_t handle, uint64_t* out, int n) { return ngsReplicaDigest(handle, 0, out, n); }

NGS_API int ngsReplicaDigest(uint32_t handle, int replica, uint64_t* out, int n) {
    std::shared_lock<std::shared_mutex> lk(g_lock);
    auto it = g_libs.find(handle);
    if (it == g_libs.end() || replica < 0 || (size_t)replica >= it->second->reps.size() || !out) return -1;
    Library& L = *it->second;
    const Replica& R = *L.reps[replica];
    const DevIndex& X = R.dev;
    if (!HIP_CHECK(hipSetDevice(R.device))) return -4;
    // (bytes, FNV-1a) of gram_off, post, gram_row, skip as the kernels read them
    auto digest = [](const void* d, size_t bytes, uint64_t& h) -> bool {
        std::vector<uint8_t> v(bytes);
        if (bytes && !HIP_CHECK(hipMemcpy(v.data(), d, bytes, hipMemcpyDeviceToHost))) return false;
        h = 1469598103934665603ull;
        for (uint8_t c : v) h = (h ^ c) * 1099511628211ull;
        return true;
    };
    uint64_t vals[16] = {};
    if (X.gram_mode == 0) {  // the direct-indexed gram CSR (dictionary indexes: zeros)
        uint64_t n_post = 0;
        const size_t nspace = kGramSpace;
        if (!HIP_CHECK(hipMemcpy(&n_post, X.gram_off + nspace, sizeof(uint64_t), hipMemcpyDeviceToHost))) return -4;
        const size_t rows = L.host.n_grams;
        const size_t sizes[4] = {sizeof(uint64_t) * (nspace + 1), sizeof(uint32_t) * n_post, sizeof(uint32_t) * nspace,
                                 sizeof(uint32_t) * rows * (X.n_buckets + 1)};
        const void* ptrs[4] = {X.gram_off, X.post, X.gram_row, X.skip};
        vals[0] = n_post;
        vals[1] = rows;
        vals[2] = X.n_buckets;
        for (int i = 0; i < 4; ++i)
            if (!digest(ptrs[i], sizes[i], vals[3 + i])) return -4;
        vals[7] = X.bucket_span;
    }
    // the interned library (ngs_intern.hip or the host build): terms, pairs, keys, wildcard answer
    uint64_t tchars = 0;
    uint32_t npairs = 0;
    if (!HIP_CHECK(hipMemcpy(&tchars, X.term_off + X.n_terms, sizeof(uint64_t), hipMemcpyDeviceToHost)) ||
        !HIP_CHECK(hipMemcpy(&npairs, X.tk_off + X.n_terms, sizeof(uint32_t), hipMemcpyDeviceToHost)))
        return -4;
    const uint64_t kchars = L.host.key_off[X.n_keys];
    const size_t tsizes[8] = {sizeof(uint64_t) * (X.n_terms + 1), tchars * X.csize,
                              sizeof(uint32_t) * (X.n_terms + 1), sizeof(uint2) * npairs,
                              sizeof(uint64_t) * (X.n_keys + 1), kchars * X.csize,
                              sizeof(uint32_t) * X.n_keys, sizeof(float) * X.n_keys};
    const void* tptrs[8] = {X.term_off, X.term_bytes, X.tk_off, X.tk, X.key_off, X.key_bytes, X.wild_key, X.wild_score};
    for (int i = 0; i < 8; ++i)
        if (!digest(tptrs[i], tsizes[i], vals[8 + i])) return -4;
    // the shape flags the kernels branch on
    const uint64_t flags = (X.keys_unique ? 1u : 0u) | (X.tk_identity ? 2u : 0u) | (X.tk_monotone ? 4u : 0u) |
                           (X.rank_post ? 8u : 0u);
    const int m = std::min(n, 17);
    for (int i = 0; i < m; ++i) out[i] = i < 16 ? vals[i] : flags;
    return m;
}

// ---- index files: the interned library, the part the build spends its
// time on; the gram CSR and skip table are rebuilt from it on load (GPU, or host for gram
// dictionaries), the keys' wildcard answer too. Little-endian, native widths:
//   "NGSIDX01" | u32 csize, gsz, gram_mode, short_term_len, short_query_len, full_scan_len,
//   n_terms, n_short, n_keys, valid[8] | arrays (u64 element count, then the elements):
//   term_off u64, term_bytes u8, tk_off u32, tk {u32 key, u32 weight bits}, key_off u64,
//   key_bytes u8, wild_w f32
extern "C++" {
namespace ngs {
namespace {
constexpr char kIndexMagic[8] = {'N', 'G', 'S', 'I', 'D', 'X', '0', '1'};

template <class T>
bool put_array(std::FILE* f, const T* p, uint64_t n) {
    return std::fwrite(&n, sizeof n, 1, f) == 1 && (n == 0 || std::fwrite(p, sizeof(T), n, f) == n);
}
template <class T>
bool get_array(std::FILE* f, std::vector<T>& v, uint64_t max_n) {
    uint64_t n = 0;
    if (std::fread(&n, sizeof n, 1, f) != 1 || n > max_n) return false;
    v.resize(n);
    return n == 0 || std::fread(v.data(), sizeof(T), n, f) == n;
}
template <class T>
bool download_vec(std::vector<T>& v, const T* d, uint64_t n) {
    v.resize(n);
    return n == 0 || HIP_CHECK(hipMemcpy(v.data(), d, n * sizeof(T), hipMemcpyDeviceToHost));
}
}  // namespace
}  // namespace ngs
}  // extern "C++"

NGS_API int ngsSaveIndex(uint32_t handle, const char* path) {
    std::shared_lock<std::shared_mutex> lk(g_lock);
    Library* L = find_lib(handle);
    if (!L) return -1;
    if (!L->host.indexed || L->reps.empty()) return -2;
    if (!path) return -3;
    const HostIndex& H = L->host;
    const Replica& R = *L->reps.front();
    if (!HIP_CHECK(hipSetDevice(R.device))) return -4;
    const DevIndex& X = R.dev;
    std::vector<uint64_t> term_off;
    std::vector<uint8_t> term_bytes;
    std::vector<uint32_t> tk_off;
    std::vector<uint2> tk;
    std::vector<float> wild_w;
    if (!download_vec(term_off, X.term_off, (uint64_t)H.n_terms + 1) ||
        !download_vec(term_bytes, X.term_bytes, term_off.back() * H.csize) ||
        !download_vec(tk_off, X.tk_off, (uint64_t)H.n_terms + 1) || !download_vec(tk, X.tk, tk_off.back()) ||
        !download_vec(wild_w, R.wild_w, H.n_keys))
        return -4;
    uint32_t valid[8];
    {
        std::lock_guard<std::mutex> g(L->valid_mu);
        std::memcpy(valid, L->valid, sizeof valid);
    }
    std::FILE* f = std::fopen(path, "wb");
    if (!f) return -3;
    const uint32_t sc[9] = {H.csize,          H.gsz,         H.gram_mode, H.short_term_len, H.short_query_len,
                            H.full_scan_len,  H.n_terms,     H.n_short,   H.n_keys};
    bool ok = std::fwrite(kIndexMagic, 1, 8, f) == 8 && std::fwrite(sc, sizeof sc, 1, f) == 1 &&
              std::fwrite(valid, sizeof valid, 1, f) == 1 && put_array(f, term_off.data(), term_off.size()) &&
              put_array(f, term_bytes.data(), term_bytes.size()) && put_array(f, tk_off.data(), tk_off.size()) &&
              put_array(f, tk.data(), tk.size()) && put_array(f, H.key_off.data(), H.key_off.size()) &&
              put_array(f, H.key_bytes.data(), H.key_bytes.size()) && put_array(f, wild_w.data(), wild_w.size());
    ok = (std::fclose(f) == 0) && ok;
    return ok ? 0 : -3;
}

NGS_API uint32_t ngsLoadIndex(const char* path) {
    if (!path) return 0;
    std::FILE* f = std::fopen(path, "rb");
    if (!f) return 0;
    HostIndex H;
    char magic[8];
    uint32_t sc[9], valid[8];
    constexpr uint64_t kMax = uint64_t(1) << 40;
    bool ok = std::fread(magic, 1, 8, f) == 8 && std::memcmp(magic, kIndexMagic, 8) == 0 &&
              std::fread(sc, sizeof sc, 1, f) == 1 && std::fread(valid, sizeof valid, 1, f) == 1 &&
              get_array(f, H.term_off, kMax) && get_array(f, H.term_bytes, kMax) && get_array(f, H.tk_off, kMax) &&
              get_array(f, H.tk, kMax) && get_array(f, H.key_off, kMax) && get_array(f, H.key_bytes, kMax) &&
              get_array(f, H.wild_w, kMax);
    std::fclose(f);
    if (!ok) return 0;
    H.csize = sc[0];
    H.gsz = sc[1];
    H.gram_mode = sc[2];
    H.short_term_len = sc[3];
    H.short_query_len = sc[4];
    H.full_scan_len = sc[5];
    H.n_terms = sc[6];
    H.n_short = sc[7];
    H.n_keys = sc[8];
    // the arrays must describe the counts (a truncated or foreign file is refused)
    if ((H.csize != 1 && H.csize != 4) || H.gsz < 1 || H.gsz > kMaxGramSize || H.gram_mode > 1 ||
        H.n_short > H.n_terms || H.term_off.size() != (size_t)H.n_terms + 1 ||
        H.tk_off.size() != (size_t)H.n_terms + 1 || H.key_off.size() != (size_t)H.n_keys + 1 ||
        H.wild_w.size() != H.n_keys || H.term_bytes.size() != H.term_off.back() * H.csize ||
        H.tk.size() != H.tk_off.back() || H.key_bytes.size() != H.key_off.back() * H.csize)
        return 0;
    for (const uint2& kw : H.tk)
        if (kw.x >= H.n_keys) return 0;
    // every offset array ascends from 0 to its array's end (a crafted file must not send the
    // kernels or marshal() out of bounds), every key ends in a NUL, the length parameters are the
    // gram size's, and the short / long term split matches the term lengths
    auto ascending = [](const auto& off) {
        if (off.empty() || off.front() != 0) return false;
        for (size_t i = 1; i < off.size(); ++i)
            if (off[i] < off[i - 1]) return false;
        return true;
    };
    if (!ascending(H.term_off) || !ascending(H.tk_off) || !ascending(H.key_off)) return 0;
    if (H.short_term_len != 2 * H.gsz || H.short_query_len != 3 * H.gsz || H.full_scan_len != H.gsz ||
        H.gram_mode != ((H.csize == 1 && H.gsz == 3) ? 0u : 1u))
        return 0;
    for (uint32_t k = 0; k < H.n_keys; ++k) {
        if (H.key_off[k + 1] == H.key_off[k]) return 0;  // not even the NUL
        const uint64_t last = (H.key_off[k + 1] - 1) * H.csize;
        for (uint32_t b = 0; b < H.csize; ++b)
            if (H.key_bytes[last + b] != 0) return 0;
    }
    for (uint32_t t = 0; t < H.n_terms; ++t) {
        const bool is_short = H.term_off[t + 1] - H.term_off[t] < H.short_term_len;
        if (is_short != (t < H.n_short)) return 0;
    }
    H.indexed = true;
    H.grams_built = false;
    const uint32_t handle = new_library([&](HostIndex& dst) {
        dst = std::move(H);  // the gram CSR (and a dictionary index's gram table) built at upload
    });
    if (handle) {
        std::shared_lock<std::shared_mutex> lk(g_lock);
        if (Library* L = find_lib(handle)) {
            std::lock_guard<std::mutex> g(L->valid_mu);
            std::memcpy(L->valid, valid, sizeof valid);
        }
    }
    return handle;
}

NGS_API int ngsHostPhases(uint64_t* out, int n, int reset) {
    const int k = std::min<int>(n, kHpN);
    for (int i = 0; i < k; ++i) out[i] = reset ? g_host_phase[i].exchange(0) : g_host_phase[i].load();
    for (int i = k; reset && i < kHpN; ++i) g_host_phase[i].store(0);
    return kHpN;
}

NGS_API int ngsPhaseStats(uint64_t* out, int n, int reset) {
    return phase_stats((unsigned long long*)out, n, reset != 0);
}

}  // extern "C"
