// gen_golden — TEST INFRASTRUCTURE ONLY.
//
// Drives the reference StringSearchLib built from /root/reference by oracle/Makefile
// (oracle/_ref/libStringSearchLib.so) through its own C ABI and prints its answers as
// JSON lines. tests/golden/make_golden.py writes the request file, runs this driver
// and stores the answers as fixtures under tests/golden/. Nothing here ships.
//
// Reference entry points exercised (nGramSearch/dllmain.cpp):
//   indexN :37, score :82, release :98, dispose :110, getSize :120, getLibSize :133,
//   setValidChar :142.
//
// Request file (one record per line, strings hex-encoded so any byte can be carried):
//   C <rowSize> <nWords> <hasWeights 0|1>      start a corpus
//   W <hex|-|=> <weight-bits-hex>              one word (- = NULL pointer, = empty string)
//   I                                          call indexN on the words read so far
//   V <hex>                                    setValidChar(handle, bytes)
//   Q <hex|=> <thr-bits-hex> <limit>           score(handle, q, ..., thr, limit)
//   D                                          dispose
//   S <rows> <seed> <minLen> <span> <rowSize> <hasWeights 0|1> <libngs_synth.so>
//                                              generate the synthetic corpus of SURVEY.md §8(d)
//                                              with the bench's own generator (csrc/synth.c,
//                                              dlopen'ed) and call indexN on it: corpora of
//                                              millions of rows without a request file of
//                                              millions of lines
// Answers: {"corpus":..,"size":..,"libSize":..} after I / S; one {"q":..} line per Q.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <dlfcn.h>
#include <string>
#include <vector>

typedef uint32_t (*indexN_t)(char**, uint64_t, uint16_t, float*);
typedef uint32_t (*score_t)(uint32_t, const char*, char***, float**, float, uint32_t);
typedef void (*release_t)(uint32_t, char**, float*);
typedef void (*dispose_t)(uint32_t);
typedef uint64_t (*size_t_fn)(uint32_t);
typedef void (*setvalid_t)(uint32_t, char*, int);
typedef int (*synth_corpus_t)(uint64_t, uint64_t, uint32_t, uint32_t, uint32_t, char**, char***, float**, uint64_t*);
typedef void (*synth_free_t)(void*);

static std::string unhex(const char* h) {
    std::string s;
    size_t n = strlen(h);
    for (size_t i = 0; i + 1 < n; i += 2) {
        unsigned v;
        sscanf(h + i, "%2x", &v);
        s.push_back((char)v);
    }
    return s;
}

static std::string tohex(const char* p) {
    static const char* d = "0123456789abcdef";
    std::string s;
    for (; *p; ++p) {
        unsigned char c = (unsigned char)*p;
        s.push_back(d[c >> 4]);
        s.push_back(d[c & 15]);
    }
    return s;
}

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: gen_golden <libStringSearchLib.so> <requests>\n");
        return 2;
    }
    void* lib = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
    if (!lib) { fprintf(stderr, "dlopen: %s\n", dlerror()); return 2; }
    auto indexN = (indexN_t)dlsym(lib, "indexN");
    auto score = (score_t)dlsym(lib, "score");
    auto release = (release_t)dlsym(lib, "release");
    auto dispose = (dispose_t)dlsym(lib, "dispose");
    auto getSize = (size_t_fn)dlsym(lib, "getSize");
    auto getLibSize = (size_t_fn)dlsym(lib, "getLibSize");
    auto setValidChar = (setvalid_t)dlsym(lib, "setValidChar");
    if (!indexN || !score || !release || !dispose || !getSize || !getLibSize || !setValidChar) {
        fprintf(stderr, "missing export\n");
        return 2;
    }
    FILE* f = fopen(argv[2], "r");
    if (!f) { perror("requests"); return 2; }

    std::vector<std::string> store;
    std::vector<char> isNull;
    std::vector<float> weights;
    int rowSize = 1, hasW = 0;
    uint32_t handle = 0;
    int corpus = -1;
    std::vector<char> line(1 << 22);
    while (fgets(line.data(), (int)line.size(), f)) {
        char* p = line.data();
        size_t L = strlen(p);
        while (L && (p[L - 1] == '\n' || p[L - 1] == '\r')) p[--L] = 0;
        if (!L) continue;
        char tag = p[0];
        char* rest = p + (L > 1 ? 2 : 1);
        if (tag == 'C') {
            int nw;
            sscanf(rest, "%d %d %d", &rowSize, &nw, &hasW);
            store.clear(); isNull.clear(); weights.clear();
            ++corpus;
        } else if (tag == 'W') {
            char hx[1 << 16]; unsigned wb = 0;
            sscanf(rest, "%65535s %x", hx, &wb);
            if (hx[0] == '-') { store.push_back(""); isNull.push_back(1); }
            else if (hx[0] == '=') { store.push_back(""); isNull.push_back(0); }
            else { store.push_back(unhex(hx)); isNull.push_back(0); }
            float w; memcpy(&w, &wb, 4);
            weights.push_back(w);
        } else if (tag == 'I') {
            std::vector<char*> ptrs(store.size());
            for (size_t i = 0; i < store.size(); ++i)
                ptrs[i] = isNull[i] ? nullptr : (char*)store[i].c_str();
            handle = indexN(ptrs.empty() ? nullptr : ptrs.data(), ptrs.size(), (uint16_t)rowSize,
                            hasW ? weights.data() : nullptr);
            printf("{\"corpus\": %d, \"handle\": %u, \"size\": %llu, \"libSize\": %llu}\n", corpus, handle,
                   (unsigned long long)getSize(handle), (unsigned long long)getLibSize(handle));
        } else if (tag == 'S') {
            unsigned long long rows, seed;
            unsigned minLen, span, rs, hw;
            char path[4096];
            sscanf(rest, "%llu %llu %u %u %u %u %4095s", &rows, &seed, &minLen, &span, &rs, &hw, path);
            void* sl = dlopen(path, RTLD_NOW | RTLD_LOCAL);
            if (!sl) { fprintf(stderr, "dlopen: %s\n", dlerror()); return 2; }
            auto gen = (synth_corpus_t)dlsym(sl, "ngs_synth_corpus");
            auto sfree = (synth_free_t)dlsym(sl, "ngs_synth_free");
            if (!gen || !sfree) { fprintf(stderr, "missing synth export\n"); return 2; }
            char* blob = nullptr;
            char** words = nullptr;
            float* w = nullptr;
            uint64_t st = 0;
            if (gen(rows, seed, minLen, span, rs, &blob, &words, &w, &st)) { fprintf(stderr, "synth failed\n"); return 2; }
            ++corpus;
            handle = indexN(words, rows * rs, (uint16_t)rs, hw ? w : nullptr);
            printf("{\"corpus\": %d, \"handle\": %u, \"size\": %llu, \"libSize\": %llu}\n", corpus, handle,
                   (unsigned long long)getSize(handle), (unsigned long long)getLibSize(handle));
            fflush(stdout);
            sfree(blob);  // the reference copied the strings (hpp:120-172)
            sfree(words);
            sfree(w);
        } else if (tag == 'V') {
            std::string v = unhex(rest);
            setValidChar(handle, (char*)v.data(), (int)v.size());
        } else if (tag == 'Q') {
            char hx[1 << 16]; unsigned tb; unsigned limit;
            sscanf(rest, "%65535s %x %u", hx, &tb, &limit);
            std::string q = hx[0] == '=' ? std::string() : unhex(hx);
            float thr; memcpy(&thr, &tb, 4);
            char** res = nullptr; float* sc = nullptr;
            uint32_t n = score(handle, q.c_str(), &res, &sc, thr, limit);
            printf("{\"q\": \"%s\", \"thr\": %u, \"limit\": %u, \"n\": %u, \"keys\": [", tohex(q.c_str()).c_str(),
                   tb, limit, n);
            for (uint32_t i = 0; i < n; ++i) printf("%s\"%s\"", i ? ", " : "", tohex(res[i]).c_str());
            printf("], \"scores\": [");
            for (uint32_t i = 0; i < n; ++i) {
                unsigned b; memcpy(&b, &sc[i], 4);
                printf("%s%u", i ? ", " : "", b);
            }
            printf("]}\n");
            release(handle, res, sc);
        } else if (tag == 'D') {
            dispose(handle);
            handle = 0;
        }
    }
    fclose(f);
    return 0;
}
