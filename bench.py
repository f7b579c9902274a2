#!/usr/bin/env python3
"""bench.py — Mqueries/s and achieved HBM GB/s of the batched search() path on MI355X.

Workload (BASELINE.json configs[2], the metric's config): 10M-row ASCII corpus, gSize 3,
per-row float weights, batch of 65,536 queries per GPU, threshold 0.3, limit 100.
Synthetic data (SURVEY.md §8(d) generator, stringsearchlib_amd/csrc/synth.c), built into
the index with indexN and uploaded once; queries are resident in HBM before timing.

A step = one ngsSearchDevice call over the GPU's batch (normalise + fused count/score/top-k
kernel [+ library-wide kernels for the rare queries that need them]); with N > 1 ranks
(one process per GPU, torchrun) each rank scores its own 65,536 queries (weak scaling) and
the step also gathers the compacted top-k records on rank 0 over RCCL.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2]
"""
from __future__ import annotations

import argparse
import collections
import ctypes as C
import json
import os
import sys
import time

import torch  # first: libngram_search.so then binds to torch's HIP runtime (one runtime per process)
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import stringsearchlib_amd as ssl  # noqa: E402
from stringsearchlib_amd import _native, shard  # noqa: E402

METRIC = "Mqueries/sec + achieved HBM GB/s, 10M-row gSize=3 library, batch=65536"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

CONFIGS = {
    # BASELINE.json configs[2]: the metric's configuration
    "c3": dict(rows=10_000_000, batch=65536, threshold=0.3, limit=100, weights=True,
               workload="C3: 10M-row ASCII corpus, gSize=3, rowSize=1, per-row float weights, "
                        "batch=65536/GPU, threshold=0.3, limit=100"),
    # BASELINE.json configs[1]
    # (three batches in flight: a 4,096-query batch is a few waves per CU)
    # (warm-up 40: each context captures its calls as graphs on their second occurrence, one per
    # output buffer it is handed)
    "c2": dict(rows=1_000_000, batch=4096, threshold=0.0, limit=100, weights=False, depth=3, warmup=40,
               workload="C2: 1M-row ASCII corpus, gSize=3, weight=NULL, batch=4096/GPU, threshold=0, limit=100"),
    # BASELINE.json configs[3] (our indexW/gSize extension, parity unpinned). With gSize 2 over the
    # 37-symbol alphabet a list holds ~440k postings and a 12-character query reads ~4.7M (19 MB),
    # 180x a C3 query: one step is ~0.7 s, so run it with a few --steps.
    "c4": dict(rows=10_000_000, batch=65536, threshold=0.3, limit=100, weights=False, row_size=4, gram=2,
               wide=True,
               workload="C4: 10M-row UTF-32 corpus via indexW, gSize=2, rowSize=4 (key + 3 aliases), weight=NULL, "
                        "batch=65536/GPU, threshold=0.3, limit=100"),
    # BASELINE.json configs[4]: 2^20 queries over 8 GPUs = 131,072 per GPU on a 50M-row library
    # (weight=NULL: the config names none). At N=1 this is the per-GPU slice.
    "c5": dict(rows=50_000_000, batch=131072, threshold=0.3, limit=100, weights=False,
               workload="C5: 50M-row ASCII corpus, gSize=3, rowSize=1, weight=NULL, batch=131072/GPU "
                        "(2^20 over 8 GPUs), threshold=0.3, limit=100"),
}


# The reference DLL (nGramSearch/dllmain.cpp, g++ -O2) timed in the survey container on the same
# synthetic spec: BASELINE.md. It cannot run on the GPU box (the reference does not travel), so
# it is quoted beside the oracle port that is timed there.
REFERENCE_DLL = {
    "c3": {"value": 58.5, "unit": "queries/s", "cores": 8, "hardware": "8-vCPU Xeon (survey container)",
           "sample": "4,096 of the 65,536 C3 queries, 8 caller threads", "source": "BASELINE.md"},
    "c2": {"value": 1376.6, "unit": "queries/s", "cores": 8, "hardware": "8-vCPU Xeon (survey container)",
           "sample": "C2 batch of 4,096 queries, 8 caller threads (265.5 q/s on 1)", "source": "BASELINE.md"},
}


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


class Corpus:
    """Synthetic rows + queries in C memory (10M rows would be slow as Python objects)."""

    def __init__(self, rows: int, seed: int = 42, row_size: int = 1, wide: bool = False):
        S = _native.synth()
        self.S, self.rows, self.row_size, self.wide = S, rows, row_size, wide
        self.n_words = rows * row_size
        self.blob, self.words, self.weights, self.state = C.c_void_p(), C.POINTER(C.c_char_p)(), \
            C.POINTER(C.c_float)(), C.c_uint64()
        if S.ngs_synth_corpus(rows, seed, 8, 17, row_size, C.byref(self.blob), C.byref(self.words),
                              C.byref(self.weights), C.byref(self.state)):
            raise MemoryError("synthetic corpus")
        self.wblob, self.wwords = C.POINTER(C.c_uint32)(), C.POINTER(C.POINTER(C.c_uint32))()
        if wide and S.ngs_synth_widen(self.words, self.n_words, C.byref(self.wblob), C.byref(self.wwords)):
            raise MemoryError("synthetic corpus (UTF-32)")

    def queries(self, n: int, skip: int = 0):
        """n queries after `skip` queries of the stream (rank slices of one global stream)."""
        st = C.c_uint64(self.state.value)
        qb, qo = C.c_void_p(), C.POINTER(C.c_uint64)()
        if self.S.ngs_synth_queries(self.words, self.n_words, self.row_size, skip + n, C.byref(st), 12, C.byref(qb),
                                    C.byref(qo)):
            raise MemoryError("synthetic queries")
        lo, hi = qo[skip], qo[skip + n]
        raw = C.string_at(qb.value + lo, hi - lo)
        offs = [qo[skip + i] - lo for i in range(n + 1)]
        self.S.ngs_synth_free(qb)
        self.S.ngs_synth_free(C.cast(qo, C.c_void_p))
        return raw, offs

    def free(self):
        for p in (self.blob, C.cast(self.words, C.c_void_p), C.cast(self.weights, C.c_void_p),
                  C.cast(self.wblob, C.c_void_p), C.cast(self.wwords, C.c_void_p)):
            self.S.ngs_synth_free(p)


def build_index(corpus: Corpus, weights: bool, device: int, gram: int = 3) -> int:
    L = _native.lib()
    if L.ngsSetDevice(device):
        raise RuntimeError(f"ngsSetDevice({device}) failed")
    w = corpus.weights if weights else None
    if corpus.wide:
        h = L.indexW(corpus.wwords, corpus.n_words, corpus.row_size, w, gram)
    elif gram != 3:
        h = L.indexG(corpus.words, corpus.n_words, corpus.row_size, w, gram)
    else:
        h = L.indexN(corpus.words, corpus.n_words, corpus.row_size, w)
    if not h:
        raise RuntimeError("indexN failed")
    return h


def cpu_baseline(corpus: Corpus, cfg: dict, raw: bytes, offs: list, target_s: float = 12.0):
    """Time the oracle (oracle/, the CPU restatement of the reference path) on host cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py
    threads = max(1, min(16, os.cpu_count() or 1))
    w = corpus.weights if cfg["weights"] else None
    qs = [raw[offs[i]:offs[i + 1]] for i in range(len(offs) - 1)]
    cap = cfg["limit"]
    generic = corpus.wide or cfg.get("gram", 3) != 3
    t0 = time.time()
    if generic:  # the gram-size / UTF-32 restatement (oracle/ngs_oracle_g.c)
        O = oracle_py.lib_g()
        U = C.POINTER(C.c_uint32)
        ptrs = corpus.wwords if corpus.wide else C.cast(corpus.words, C.POINTER(U))
        h = O.ngog_build(ptrs, corpus.n_words, corpus.row_size, w, cfg.get("gram", 3), int(corpus.wide))
        qs = [(C.c_uint32 * (len(q) + 1))(*q, 0) if corpus.wide else q for q in qs]
        search_batch, free, name = O.ngog_search_batch, O.ngog_free, "oracle/ngs_oracle_g.c"
    else:
        O = oracle_py.lib()
        h = O.ngo_build(corpus.words, corpus.n_words, corpus.row_size, w)
        search_batch, free, name = O.ngo_search_batch, O.ngo_free, "oracle/ngs_oracle.c"
    build_s = time.time() - t0

    def run(n):
        sample = [qs[i % len(qs)] for i in range(n)]
        if generic:
            arr = (C.POINTER(C.c_uint32) * n)(*[C.cast(q, C.POINTER(C.c_uint32)) for q in sample])
        else:
            arr = (C.c_char_p * n)(*sample)
        counts = (C.c_uint32 * n)()
        keys = (C.c_uint32 * (n * cap))()
        scores = (C.c_float * (n * cap))()
        t = time.time()
        search_batch(h, arr, n, cfg["threshold"], cfg["limit"], counts, keys, scores, cap, threads)
        return time.time() - t

    n = 1024
    dt = run(n)
    while dt < 2.0 and n < 1 << 22:
        n *= 4
        dt = run(n)
    if dt < target_s:
        n = min(1 << 23, int(n * target_s / max(dt, 1e-3)))
        dt = run(n)
    free(h)
    return {"value": n / dt, "unit": "queries/s", "cores": threads, "kind": "port",
            "sample": f"{n} queries of the same stream ({cfg['workload'].split(',')[0]} index, "
                      f"threshold {cfg['threshold']}, limit {cfg['limit']}), {name} on {threads} "
                      f"host threads; index build {build_s:.1f}s not timed"}


HOST_PHASES = ("pack_queries", "copy_in_and_queue", "kernels_wait", "device_pack_and_offsets_back",
               "records_back_and_marshal", "whole_call")


def dropin_path(L, h, cfg: dict, raw: bytes, offs: list, n_batches: int = 20, n_single: int = 300):
    """The reference's own entry points on the bench index: scoreBatch over the whole batch (host
    strings in, new[]'d char** / float* out, released) and single-query score() latency. The host
    phases of the timed scoreBatch calls (ngsHostPhases) come with them, in ms per call."""
    B = len(offs) - 1
    qs = [raw[offs[i]:offs[i + 1]] for i in range(B)]
    arr = (C.c_char_p * B)(*qs)
    counts = (C.c_uint32 * B)()
    res, sc = C.POINTER(C.POINTER(C.c_char))(), C.POINTER(C.c_float)()
    for _ in range(2):  # warm: contexts, pinned staging, the result arrays' heap
        L.scoreBatch(h, arr, B, cfg["threshold"], cfg["limit"], counts, C.byref(res), C.byref(sc))
        L.release(h, res, sc)
    ph = (C.c_uint64 * 8)()
    L.ngsHostPhases(ph, 8, 1)
    per_call = []
    t = time.perf_counter()
    for _ in range(n_batches):
        t1 = time.perf_counter()
        L.scoreBatch(h, arr, B, cfg["threshold"], cfg["limit"], counts, C.byref(res), C.byref(sc))
        L.release(h, res, sc)
        per_call.append(time.perf_counter() - t1)
    batch_s = (time.perf_counter() - t) / n_batches
    L.ngsHostPhases(ph, 8, 1)
    ncalls = max(1, ph[6])
    phases = {name: round(ph[i] / ncalls / 1e6, 4) for i, name in enumerate(HOST_PHASES)}
    per_call.sort()
    lat = []
    for i in range(n_single + 10):
        t = time.perf_counter()
        L.score(h, qs[i % B], C.byref(res), C.byref(sc), cfg["threshold"], cfg["limit"])
        lat.append(time.perf_counter() - t)
        L.release(h, res, sc)
    lat = sorted(lat[10:])
    return {"scorebatch_mqs": round(B / batch_s / 1e6, 4), "scorebatch_ms": round(batch_s * 1e3, 3),
            "scorebatch_calls": n_batches, "scorebatch_ms_min": round(per_call[0] * 1e3, 3),
            "scorebatch_ms_p50": round(per_call[len(per_call) // 2] * 1e3, 3),
            "scorebatch_host_phases_ms": phases,
            "score_us_mean": round(sum(lat) / len(lat) * 1e6, 1), "score_us_p50": round(lat[len(lat) // 2] * 1e6, 1)}


def c1_latency(device: int, n: int = 2000):
    """BASELINE configs[0]: 1k-row ASCII corpus, gSize 3, rowSize 1, no weights, one query per
    score() call at threshold 0 and limit 100 (the reference's SearchTest
    harness measures 14.7 us per query on its CPU DLL). c1_score_us_* are at that
    configuration; c1_thr03_score_us_* repeat them at threshold 0.3."""
    L = _native.lib()
    corpus = Corpus(1000, seed=1)
    h = build_index(corpus, False, device)
    raw, offs = corpus.queries(256)
    qs = [raw[offs[i]:offs[i + 1]] for i in range(256)]
    res, sc = C.POINTER(C.POINTER(C.c_char))(), C.POINTER(C.c_float)()

    def timed(thr):
        lat = []
        for i in range(n + 20):
            t = time.perf_counter()
            L.score(h, qs[i % 256], C.byref(res), C.byref(sc), thr, 100)
            lat.append(time.perf_counter() - t)
            L.release(h, res, sc)
        lat = sorted(lat[20:])
        return round(sum(lat) / len(lat) * 1e6, 1), round(lat[len(lat) // 2] * 1e6, 1)

    # the default path: on a library this small score() starts the persistent server kernel by
    # itself after its 4th call (the 20 untimed calls cover that)
    out = {"c1_config": "1k rows, no weights, threshold 0, limit 100, one query per score() call"}
    out.update(zip(("c1_score_us_mean", "c1_score_us_p50"), timed(0.0)))
    out.update(zip(("c1_thr03_score_us_mean", "c1_thr03_score_us_p50"), timed(0.3)))
    if hasattr(L, "ngsServeState"):
        out["c1_score_served"] = L.ngsServeState(h) == 2
    # the same calls with the server turned off (ngsServe(h, 0)): a kernel launch sequence per call
    if hasattr(L, "ngsServe") and L.ngsServe(h, 0) == 0:
        out.update(zip(("c1_launch_us_mean", "c1_launch_us_p50"), timed(0.0)))
    L.dispose(h)
    corpus.free()
    return out


class StepLoop:
    """The timed loop of one rank: each step scores the rank's batch into a gather buffer
    (shard.GatherBuffer); with depth 1 through a blocking ngsSearchDevice, with depth d through
    ngsSearchDeviceAsync with up to d batches in flight (the oldest waited for with
    ngsSearchDeviceWait), so each batch's tail overlaps the next batch's kernels. With N > 1 ranks
    a finished batch's buffer is gathered to rank 0 (one RCCL collective, in flight beside the
    next batches); a buffer is rewritten only after the batch that last wrote it was waited for
    and its gather ordered before the rewrite (PendingGather.complete). `run` brackets the timed
    steps with a barrier and a device synchronisation on both sides and returns the max over
    ranks of the elapsed time. tests/test_bench_loop.py drives it on CPU (gloo, world size 2)
    with the oracle standing in for the library."""

    def __init__(self, L, h, d_raw, d_off, B, threshold, limit, stride, depth, world, dev, stream,
                 gather_cap=None):
        self.L, self.h, self.d_raw, self.d_off, self.B = L, h, d_raw, d_off, B
        self.threshold, self.limit, self.stride = threshold, limit, stride
        self.depth, self.world, self.dev, self.stream = max(1, depth), world, dev, stream
        self.nbuf = self.depth + 1 if self.depth > 1 else (2 if world > 1 else 1)
        self.gbs = [shard.PackedGather(B, stride, B, dev) for _ in range(self.nbuf)]
        # the record capacity of the packed gathers (N > 1): held by every rank, grown when a retired
        # gather's all-reduced total overflowed it (then gathered again), no host read in the step
        self.cap = shard.GatherCap(B, stride, gather_cap)
        self.st = _native.NgsStats()
        self.pending = {}  # buffer index -> in-flight top-k gather (N > 1)
        self.inflight = collections.deque()  # (ticket, buffer index) of queued batches (depth > 1)
        self.nstep = 0
        self.ktimes = []
        self.gathered = []  # rank 0, N > 1: the PendingGathers of the timed steps (tests decode them)
        self.gather_words = []  # int32 words each gather moved per rank (N > 1)
        self.keep_gathers = False

    def _finished(self, i):  # batch in buffer i is complete: statistics, then its gather (N > 1)
        self.L.ngsLastStats(self.h, C.byref(self.st))
        self.ktimes.append((self.st.fast_kernel_ms, self.st.prep_kernel_ms, self.st.general_ms))
        if self.world > 1:  # packed on the device, gathered up to the largest record count of the ranks
            gb = self.gbs[i].pack(getattr(self.L, "ngsPackResults", None), self.stream)
            pg = shard.gather_packed(gb, async_op=True, cap=self.cap)  # overlaps the next batches
            self.gather_words.append(pg.words)
            self.pending[i] = pg
            if self.keep_gathers:
                self.gathered.append(pg)

    def _wait_one(self):
        t, i = self.inflight.popleft()
        rc = self.L.ngsSearchDeviceWait(self.h, t)
        if rc:
            raise RuntimeError(f"ngsSearchDeviceWait -> {rc}")
        self._finished(i)

    def step(self):
        i = self.nstep % self.nbuf
        self.nstep += 1
        if i in self.pending:  # the gather that last read this buffer: ordered before it is rewritten
            self.pending.pop(i).complete()
        gb = self.gbs[i]
        args_ = (self.h, self.d_raw.data_ptr(), self.d_off.data_ptr(), self.B, self.threshold, self.limit,
                 self.stride, gb.counts.data_ptr(), gb.keys.data_ptr(), gb.scores.data_ptr(), self.stream)
        if self.depth == 1:
            rc = self.L.ngsSearchDevice(*args_)
            if rc:
                raise RuntimeError(f"ngsSearchDevice -> {rc}")
            self._finished(i)
            return
        t = C.c_uint64()
        rc = self.L.ngsSearchDeviceAsync(*args_, C.byref(t))
        if rc:
            raise RuntimeError(f"ngsSearchDeviceAsync -> {rc}")
        self.inflight.append((t.value, i))
        while len(self.inflight) >= self.depth:
            self._wait_one()

    def drain(self):
        while self.inflight:
            self._wait_one()
        for p in self.pending.values():
            p.complete()
        self.pending.clear()

    def _sync(self):
        if self.dev.type == "cuda":
            torch.cuda.synchronize(self.dev)

    def run(self, steps, warmup):
        for _ in range(warmup):
            self.step()
        self.drain()
        self.regathers_warmup = self.cap.regathers
        self.ktimes.clear()
        self.gathered.clear()
        self.gather_words.clear()
        if self.world > 1:
            dist.barrier()
        self._sync()
        t_start = time.perf_counter()
        for _ in range(steps):
            self.step()
        self.drain()  # every batch and gather of the timed steps completes inside the timed region
        self._sync()
        if self.world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t_start
        if self.world > 1:
            e = torch.tensor([elapsed], dtype=torch.float64, device=self.dev)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            elapsed = float(e.item())
        return elapsed, self.ktimes


def serialised_roofline(pmc, st, version):
    """The dominant kernel alone: the main k_wave_lean launch's own algorithmic bytes (4 B per posting
    and 16 B per list opened, of the queries it finished: this run's ngsLastStats) over its mean
    duration with every dispatch serialised (the SQ counter pass in profiles/). With batches in
    flight the launches overlap, so the step-level figure above is the conservative one; this is
    the kernel-level one (None without a committed pass)."""
    if not pmc or not pmc.get("main_kernel_serialised_ns"):
        return None
    ns = pmc["main_kernel_serialised_ns"]
    b = 4 * st.main_postings + 16 * st.main_lists
    return {"kernel": "main k_wave_lean launch (tier 1a over the batch)", "ms": round(ns / 1e6, 4),
            "alg_bytes": int(b), "achieved": round(b / ns, 2), "frac": round(b / ns / HBM_PEAK_GBS, 4),
            "source": pmc.get("sq_pass"), "profiled_library": pmc.get("library"),
            "same_source": pmc.get("library") == version}


def pmc_record(cfg_name: str):
    """The committed rocprofv3 record of this config (tools/pmc_traffic.py): HBM bytes per call from
    the FETCH_SIZE pass, the main k_wave_lean launch's duration under the serialised counter pass, and
    the library stamp they were measured on; None if there is none."""
    p = os.path.join(ROOT, "profiles", f"pmc_{cfg_name}.json")
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    d["file"] = os.path.relpath(p, ROOT)
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps first (default 10; C2 40)")
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--rows", type=int, default=None, help="override corpus rows (debug only)")
    ap.add_argument("--batch", type=int, default=None, help="override per-GPU batch (debug only)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-dropin", action="store_true", help="skip the scoreBatch / score() latency lines")
    ap.add_argument("--depth", type=int, default=None,
                    help="batches in flight (ngsSearchDeviceAsync; default 2, C2 3); 1 = one blocking "
                         "ngsSearchDevice per step")
    args = ap.parse_args()
    cfg = dict(CONFIGS[args.config])
    if args.rows:
        cfg["rows"] = args.rows
    if args.batch:
        cfg["batch"] = args.batch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    t0 = time.time()
    corpus = Corpus(cfg["rows"], row_size=cfg.get("row_size", 1), wide=cfg.get("wide", False))
    corpus_s = time.time() - t0
    t0 = time.time()
    h = build_index(corpus, cfg["weights"], local, cfg.get("gram", 3))
    index_s = time.time() - t0  # indexN / indexW alone (the synthetic corpus is corpus_s)
    L = _native.lib()
    n_keys = L.ngsNumKeys(h)
    log(rank, f"[bench] {cfg['workload']}: index built+uploaded in {index_s:.1f}s, "
              f"{L.getSize(h)} terms, {L.getLibSize(h)} grams")

    B = cfg["batch"]
    raw, offs = corpus.queries(B, skip=rank * B)
    if corpus.wide:  # UTF-32 queries: one 4-byte code point per byte, offsets in bytes
        d_raw = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(torch.int32).to(dev).view(torch.uint8)
        d_off = torch.tensor([4 * o for o in offs], dtype=torch.int64, device=dev)
    else:
        d_raw = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(dev)
        d_off = torch.tensor(offs, dtype=torch.int64, device=dev)
    stride = min(cfg["limit"], n_keys)
    depth = max(1, args.depth if args.depth is not None else cfg.get("depth", 2))
    # HIP-event kernel timing per call (four event records) only where the roofline uses it (depth 1):
    # with batches in flight the step time is the denominator, and a C2 step is ~20 host calls
    L.ngsSetTiming(h, 1 if depth == 1 else 0)
    loop = StepLoop(L, h, d_raw, d_off, B, cfg["threshold"], cfg["limit"], stride, depth, world, dev,
                    torch.cuda.current_stream(dev).cuda_stream)
    warmup = args.warmup if args.warmup is not None else cfg.get("warmup", 10)
    elapsed, ktimes = loop.run(args.steps, warmup)
    if depth > 1:
        # the batch's statistics (postings, lists, paths: the algorithmic bytes) come with the
        # per-call timing, off in the timed steps: one more batch, untimed, with it on
        L.ngsSetTiming(h, 1)
        loop.depth = 1
        loop.step()
        loop.drain()
        L.ngsSetTiming(h, 0)
    st = loop.st

    # per-launch algorithmic bytes of the fused kernel
    qbytes = offs[-1] * (4 if corpus.wide else 1)
    alg_bytes = (4 * st.postings + 16 * st.lists + qbytes + 16 * st.survivors + 8 * st.results + 4 * B)
    fast_ms = sum(k[0] for k in ktimes) / len(ktimes)  # per-batch tier-1 phase (HIP events)
    step_ms = elapsed / args.steps * 1e3
    # with batches pipelined the per-batch phases overlap: the roofline is taken over the whole
    # step instead (every kernel of a batch, per GPU), the conservative figure
    roof_ms = fast_ms if depth == 1 else step_ms
    achieved = alg_bytes / (roof_ms * 1e-3) / 1e9
    pmc = pmc_record(args.config)
    version = L.ngsVersion().decode()
    total_q = B * world * args.steps
    value = total_q / elapsed / 1e6
    out = {
        "metric": METRIC, "value": round(value, 4), "unit": "Mqueries/s", "n_gpus": world, "steps": args.steps,
        "warmup": warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
        "config": {"workload": cfg["workload"], "rows": cfg["rows"], "batch_per_gpu": B,
                   "threshold": cfg["threshold"], "limit": cfg["limit"], "weights": cfg["weights"],
                   "parallelism": f"query-shard x{world}" + (" + RCCL gather of top-k" if world > 1 else "")},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": pmc.get("hbm_bytes_per_launch") if pmc else None,
                     "traffic_source": ({"file": pmc["file"], "fetch_pass": pmc.get("source"),
                                         "profiled_library": pmc.get("library"), "this_library": version,
                                         "same_source": pmc.get("library") == version} if pmc else None),
                     "kernel": ("tier-1 phase: k_wave_lean over the batch + k_emit, beside it k_wave_lean + k_emit on the "
                                "heavy list and k_wave on the full list (side streams), hand-over k_wave, k_fast (HIP "
                                "events on the call stream)" if depth == 1 else
                                f"whole step: every kernel of one batch (k_prep, the tier-1 phase, k_fast), batches "
                                f"pipelined {depth} deep (ngsSearchDeviceAsync); per-GPU step time"),
                     "kernel_ms": round(roof_ms, 4), "alg_bytes_per_launch": alg_bytes,
                     "postings_per_query": round(st.postings / max(1, st.fast_queries), 1),
                     "serialised": serialised_roofline(pmc, st, version)},
        "detail": {"phase_ms": round(fast_ms, 4) if depth == 1 else None, "depth": depth,
                   "prep_ms": round(sum(k[1] for k in ktimes) / len(ktimes), 4) if depth == 1 else None,
                   "general_ms": round(sum(k[2] for k in ktimes) / len(ktimes), 4) if depth == 1 else None,
                   "general_queries": int(st.general_queries), "results_per_query": round(st.results / B, 2),
                   "survivors_per_query": round(st.survivors / B, 2), "index_build_s": round(index_s, 2),
                   "corpus_gen_s": round(corpus_s, 2),
                   "paths": {"tier1a_finished": int(st.fast_queries), "heavy_listed": int(st.heavy_queries),
                             "full_listed": int(st.full_queries), "tier1b_handovers": int(st.handover_queries),
                             "tier2": int(st.tier2_queries), "general": int(st.general_queries),
                             "slot_full": int(st.slot_full_queries)},
                   "survivor_slots": int(st.survivor_slots),
                   "library": L.ngsVersion().decode()},
    }
    if world > 1 and loop.gather_words:  # the packed gather's bytes per rank and step
        out["detail"]["gather"] = {
            "bytes_per_rank_step": round(4 * sum(loop.gather_words) / len(loop.gather_words)),
            "fixed_layout_bytes": 4 * (1 + B * (1 + 2 * stride)),
            "regathers": int(loop.cap.regathers), "cap_records": int(loop.cap.total),
            "note": "packed [batch, total, counts, {key, score} records] up to a record capacity every rank "
                    "holds; an overflowing batch is gathered again whole when its gather is retired"}
    if rank == 0 and world == 1 and not args.no_dropin and not corpus.wide:
        out["detail"]["dropin"] = dropin_path(L, h, cfg, raw, offs)
        out["detail"]["dropin"].update(c1_latency(local))
        out["detail"]["dropin"]["note"] = ("scoreBatch: host strings in, new[]'d char**/float* out (released), "
                                           "PCIe both ways, whole batch; score(): one query per call")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(corpus, cfg, raw, offs)
        if args.config in REFERENCE_DLL:  # the reference itself, measured where it compiles
            out["cpu_baseline"]["reference_dll"] = REFERENCE_DLL[args.config]
    else:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    L.dispose(h)
    corpus.free()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
