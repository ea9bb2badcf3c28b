// oracle/cpu_baseline.cpp — TEST / BASELINE INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).
//
// The reference's per-read CPU algorithms restated in C++ and driven over a whole batch, 1 thread or
// OpenMP over all host cores, so bench.py can time "the reference path on the box's own host cores"
// without running the reference itself there (it never travels to the GPU box).  Same algorithms as
// the reference, not this repo's fast host codec:
//   encode L <= 32   _marshall_bytes_64 (short_seq_64.pyx:96-108): reverse scalar loop, is_base bloom
//                    test per byte (util.pxd:98-99, bloom util.pyx:75), acc = acc << 2 | table_91[c]
//   encode L > 32    _marshall_bytes_array (util.pyx:78-94): full 32-nt blocks by _marshall_full_blocks
//                    (util.pyx:97-119: 8-byte chunks j = 3..0, _bloom_filter_64 util.pxd:116-127,
//                    PEXT 0x0606060606060606) + the tail by _marshall_partial_block (util.pyx:122-140)
//   hamming          __xor__ (short_seq_192.pyx:74-91): per word x = a ^ b, ((x >> 1) | x) & 0x55..,
//                    popcount
//   decode           _unmarshall_bytes_var (short_seq_var.pyx:96-120): charmap[w & 3] per nt
//   counter          _count_sequence (counter.pyx:41-54) as a hash map keyed on the packed word
//                    (one length per batch; std::unordered_map, count += 1, first index kept)
// Calibrated against the reference's own compiled kernels in the container
// (oracle/calibrate_cpu_baseline.py -> profiles/r2/cpu_baseline_calibration.json).
#include <dlfcn.h>
#include <immintrin.h>
#include <omp.h>
#include <stdint.h>
#include <string.h>

#include <mutex>
#include <unordered_map>
#include <utility>
#include <vector>

namespace {

// The reference's compiled _marshall_bytes_array (Cython's exception propagation for util.pyx:88-90)
// calls __Pyx_ErrOccurredWithGIL() -- PyGILState_Ensure, PyErr_Occurred, PyGILState_Release --
// after _divmod and after _marshall_full_blocks, i.e. twice per read of L > 32 (the L <= 32 path,
// _marshall_bytes_64, has no such check).  Inside a Python process (bench.py, the calibration) the
// port makes the same three C-API calls per check, resolved from the process; on the multi-thread
// legs (each core stands for a separate single-threaded reference process with its own GIL) and
// outside Python an uncontended thread-local mutex stands in.
struct PyApi {
    typedef int (*ensure_t)();
    typedef void (*release_t)(int);
    typedef void* (*occurred_t)();
    ensure_t ensure = nullptr;
    release_t release = nullptr;
    occurred_t occurred = nullptr;
    PyApi() {
        ensure = (ensure_t)dlsym(RTLD_DEFAULT, "PyGILState_Ensure");
        release = (release_t)dlsym(RTLD_DEFAULT, "PyGILState_Release");
        occurred = (occurred_t)dlsym(RTLD_DEFAULT, "PyErr_Occurred");
        if (!ensure || !release || !occurred) ensure = nullptr;
    }
};
const PyApi kPy;
int g_gil_checks = 1;   // cb_set_gil_checks(0) turns the emulation off (the pure algorithm)

inline void err_check(bool single) {
    if (!g_gil_checks) return;
    if (single && kPy.ensure) {
        const int st = kPy.ensure();
        (void)kPy.occurred();
        kPy.release(st);
    } else {
        thread_local std::mutex m;
        m.lock();
        m.unlock();
    }
}

constexpr uint64_t kBloom = 0xFFFFFFFFFFEFFF75ull;   // util.pyx:75
constexpr uint64_t kPextMask = 0x0606060606060606ull;  // util.pyx:39
const char kCharmap[4] = {'A', 'C', 'T', 'G'};      // util.pyx:52
// table_91 (util.pyx:44-50): A=0 C=1 G=3 T=2 U=2, everything else 4
struct Table91 {
    uint8_t t[256];
    Table91() {
        for (int i = 0; i < 256; ++i) t[i] = 4;
        t['A'] = 0;
        t['C'] = 1;
        t['G'] = 3;
        t['T'] = 2;
        t['U'] = 2;
    }
};
const Table91 kTable;

inline bool is_base(uint8_t c) { return (kBloom & (1ull << (c & 63))) == 0; }

inline bool bloom64(uint64_t block) {
    const uint64_t s = block & 0x3F3F3F3F3F3F3F3Full;
    uint64_t q = 0;
    for (int k = 0; k < 64; k += 8) q |= 1ull << ((s >> k) & 0xFF);
    return (kBloom & q) == 0;
}

// returns false on an invalid base (the reference raises)
inline bool marshall_64(const uint8_t* seq, uint32_t L, uint64_t& out) {
    uint64_t acc = 0;
    for (int i = (int)L - 1; i >= 0; --i) {
        const uint8_t c = seq[i];
        if (!is_base(c)) return false;
        acc = (acc << 2) | kTable.t[c];
    }
    out = acc;
    return true;
}

inline bool marshall_array(const uint8_t* seq, uint32_t L, uint64_t* dst) {
    const uint32_t full = L / 32, rem = L % 32;
    for (uint32_t b = 0; b < full; ++b) {
        uint64_t block = 0;
        for (int j = 3; j >= 0; --j) {
            uint64_t chunk;
            memcpy(&chunk, seq + 32 * b + 8 * j, 8);
            if (!bloom64(chunk)) return false;
            block = (block << 16) | _pext_u64(chunk, kPextMask);
        }
        dst[b] = block;
    }
    if (rem) return marshall_64(seq + 32 * full, rem, dst[full]);
    return true;
}

inline bool encode_read(const uint8_t* seq, uint32_t L, uint64_t* w, uint32_t wpr, bool single) {
    for (uint32_t k = 0; k < wpr; ++k) w[k] = 0;
    if (L <= 32) return marshall_64(seq, L, w[0]);
    err_check(single);                    // after _divmod (util.pyx:88)
    const bool ok = marshall_array(seq, L, w);
    err_check(single);                    // after _marshall_full_blocks (util.pyx:90)
    return ok;
}

inline uint32_t hamming(const uint64_t* a, const uint64_t* b, uint32_t nw) {
    uint32_t pop = 0;
    for (uint32_t i = 0; i < nw; ++i) {
        uint64_t x = a[i] ^ b[i];
        x = ((x >> 1) | x) & 0x5555555555555555ull;
        pop += (uint32_t)_mm_popcnt_u64(x);
    }
    return pop;
}

inline void decode_read(const uint64_t* w, uint32_t L, uint8_t* out) {
    uint32_t j = 0;
    for (uint32_t b = 0; j < L; ++b) {
        uint64_t block = w[b];
        const uint32_t hi = L - j < 32 ? L - j : 32;
        for (uint32_t k = 0; k < hi; ++k) {
            out[j++] = (uint8_t)kCharmap[block & 3u];
            block >>= 2;
        }
    }
}

inline uint32_t words_for(uint32_t L) { return L <= 32 ? 1u : (L + 31) / 32; }

}  // namespace

extern "C" {

int cb_max_threads(void) { return omp_get_max_threads(); }
void cb_set_gil_checks(int on) { g_gil_checks = on; }
int cb_gil_api(void) { return kPy.ensure != nullptr; }

// encode n reads (row i at ascii + i * L) -> words [n * wpr]; returns the number of invalid reads
uint64_t cb_encode(const uint8_t* ascii, uint64_t n, uint32_t L, uint64_t* words, uint32_t wpr, int threads) {
    uint64_t bad = 0;
#pragma omp parallel for num_threads(threads) schedule(static) reduction(+ : bad)
    for (int64_t i = 0; i < (int64_t)n; ++i)
        bad += encode_read(ascii + (uint64_t)i * L, L, words + (uint64_t)i * wpr, wpr, threads <= 1) ? 0 : 1;
    return bad;
}

// C3: encode + hamming of every read against `ref` (wpr words) -> dist [n]
uint64_t cb_encode_hamming(const uint8_t* ascii, uint64_t n, uint32_t L, uint64_t* words, uint32_t wpr,
                           const uint64_t* ref, uint32_t* dist, int threads) {
    uint64_t bad = 0;
    const uint32_t nw = words_for(L);
#pragma omp parallel for num_threads(threads) schedule(static) reduction(+ : bad)
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        uint64_t* w = words + (uint64_t)i * wpr;
        bad += encode_read(ascii + (uint64_t)i * L, L, w, wpr, threads <= 1) ? 0 : 1;
        dist[i] = hamming(w, ref, nw);
    }
    return bad;
}

// C3': hamming of every pre-packed read (wpr words, the first nw used) against `ref` -> dist [n]
// (the __xor__ kernel of short_seq_64.pyx:77-84 / short_seq_192.pyx:74-91 / short_seq_var.pyx:64-81
// over a batch, without the per-object Python call)
void cb_hamming_ref(const uint64_t* words, uint64_t n, uint32_t L, uint32_t wpr, const uint64_t* ref, uint32_t* dist,
                    int threads) {
    const uint32_t nw = words_for(L);
#pragma omp parallel for num_threads(threads) schedule(static)
    for (int64_t i = 0; i < (int64_t)n; ++i) dist[i] = hamming(words + (uint64_t)i * wpr, ref, nw);
}

// C4: encode + decode round trip -> back [n * L]
uint64_t cb_roundtrip(const uint8_t* ascii, uint64_t n, uint32_t L, uint64_t* words, uint32_t wpr, uint8_t* back,
                      int threads) {
    uint64_t bad = 0;
#pragma omp parallel for num_threads(threads) schedule(static) reduction(+ : bad)
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        uint64_t* w = words + (uint64_t)i * wpr;
        bad += encode_read(ascii + (uint64_t)i * L, L, w, wpr, threads <= 1) ? 0 : 1;
        decode_read(w, L, back + (uint64_t)i * L);
    }
    return bad;
}

// C5: count n reads of one length L <= 32.  threads == 1: one std::unordered_map in read order (the
// reference's loop).  threads > 1: each thread encodes a contiguous chunk and buckets (key, index) by
// hash partition; thread p then folds partition p of every chunk, chunks in order, into its own map
// (first index = first insertion).  Returns the number of distinct keys; *h_total = sum of counts,
// *h_first_sum = sum of first indices (a cheap content check).
uint64_t cb_count(const uint8_t* ascii, uint64_t n, uint32_t L, int threads, uint64_t* h_total, uint64_t* h_first_sum) {
    struct V {
        uint64_t count, first;
    };
    uint64_t uniq = 0, total = 0, fsum = 0;
    if (threads <= 1) {
        std::unordered_map<uint64_t, V> m;
        m.reserve(n);
        for (uint64_t i = 0; i < n; ++i) {
            uint64_t k;
            if (!marshall_64(ascii + i * L, L, k)) continue;
            auto it = m.find(k);
            if (it == m.end()) m.emplace(k, V{1, i});
            else ++it->second.count;
        }
        for (auto& kv : m) {
            total += kv.second.count;
            fsum += kv.second.first;
        }
        *h_total = total;
        *h_first_sum = fsum;
        return m.size();
    }
    const int T = threads;
    std::vector<std::vector<std::vector<std::pair<uint64_t, uint64_t>>>> parts(T, std::vector<std::vector<std::pair<uint64_t, uint64_t>>>(T));
#pragma omp parallel num_threads(T)
    {
        const int t = omp_get_thread_num();
        const uint64_t lo = n * t / T, hi = n * (t + 1) / T;
        auto& mine = parts[t];
        for (auto& v : mine) v.reserve((hi - lo) / T + 16);
        for (uint64_t i = lo; i < hi; ++i) {
            uint64_t k;
            if (!marshall_64(ascii + i * L, L, k)) continue;
            mine[(k * 0x9E3779B97F4A7C15ull >> 32) % T].emplace_back(k, i);
        }
    }
#pragma omp parallel num_threads(T) reduction(+ : uniq, total, fsum)
    {
        const int p = omp_get_thread_num();
        std::unordered_map<uint64_t, V> m;
        m.reserve(1 << 16);
        for (int t = 0; t < T; ++t)
            for (auto& kv : parts[t][p]) {
                auto it = m.find(kv.first);
                if (it == m.end()) m.emplace(kv.first, V{1, kv.second});
                else ++it->second.count;
            }
        uniq += m.size();
        for (auto& kv : m) {
            total += kv.second.count;
            fsum += kv.second.first;
        }
    }
    *h_total = total;
    *h_first_sum = fsum;
    return uniq;
}

}  // extern "C"
