// ss_ingest.hip — ragged read streams counted on the GPU behind the C ABI: the batch side of
// ShortSeqCounter(list) (counter.pyx:22-39) and read_and_count_fastq (counter.pyx:57-70 +
// fast_read.pyx:3-20).  The Cython front calls these entry points directly (no Python or torch in
// between): it stages a list's bytes in the engine's pinned buffer, or names a FASTQ file, and walks
// the returned (length, words, count) rows in first-occurrence order to rebuild the dict.
//
// Per chunk of reads (a staged list, or a FASTQ chunk ending after a newline):
//   1. d_lens (u32 per read; FASTQ: ss_fastq_index_onepass, 0xFFFFFFFF = the reference's strlen
//      underflow) -> stable split into bins: lengths 0..32 one bin each, lengths 33..1024 one bin per
//      length class W = ceil(L/32) (2..32), and the too-long bin.  k_len_count (per-block bin
//      histograms), k_len_binscan (block per bin: offsets inside the bin, its total and first read),
//      k_len_binstart (one block: where each bin starts), k_len_scatter (one wave per block, input
//      order kept: a wave peels its distinct bins with ballots, ranks by popcount) -> d_order = read
//      indices grouped by bin.  One small copy back (totals, first reads, starts).
//   2. a length L in 1..32: ss_gather_rows (dense rows) -> ss_counter_insert_fixed into the table of
//      length L (the length is part of the dict key, short_seq_64.pyx:41-44).  A length class:
//      k_encode_class packs each read straight from the chunk into W words + its length as one more
//      word, and ss_counter_insert_words counts those rows in the class's table (key = (length,
//      words), short_seq_192.pyx:35-41, short_seq_var.pyx:22-28): a 50-150 nt batch is 4 tables, not
//      101.  Each insert's rows get their global read indices appended to the table's row map
//      (k_rowmap).  Length 0 is the empty ShortSeq (counted on the host side of the split); length >
//      1024 is the too-long error.
//   3. first bad read: the inserts' first-bad words come back in one copy (a length's insert reports
//      its row, a class its read); the smallest global index of a rejected read is kept (and its
//      bytes) — the reference raises at the first one in input order, so nothing after the chunk
//      that holds it is read.
// Finish: every table entry marks its global first read in a one-bit-per-read map (k_mark); an
// exclusive scan of the map words' popcounts gives each entry its place in read order (k_rank:
// the words before its bit + the bits below it in its word), and the ordered entries are gathered
// into (length u32, count u64, words u64[ceil(L/32)]) rows (k_gather_host, word offsets by a second
// scan), written straight into engine-owned pinned buffers.  (A per-read 8-B slot array compacted in read
// order cost a 400-MB fill and two passes over it for 50M reads: 0.41 ms against 0.05.)
//
// Tables: one ss_counter per length (1..32) or length class, pooled across calls (reset is lazy).
// Each starts at 2 x the rows its bin brings in the first chunk (a class: scaled by the FASTQ file's
// remaining size) and grows (extract -> merge into a table of twice the needed size) when the rows
// counted could push it past half full (an exact size query decides; the query costs one sync and is
// skipped while rows <= capacity / 2); class tables grow through ss_counter_extract_words +
// ss_counter_merge_words (a length rare in the first chunk and common later).
#include <fcntl.h>
#include <pthread.h>
#include <sched.h>
#include <sys/stat.h>
#include <unistd.h>

#include <string.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "ss_internal.h"

namespace {

// split bins: lengths 0..32 (one table per length), the multi-word length classes W = 2..32 (bins
// 33..63: lengths 32(W-1)+1 .. 32W share one table), 64 = rejected (too long)
constexpr uint32_t kClassBin0 = 31;                 // bin of class W = kClassBin0 + W
constexpr uint32_t kTooLongBin = kClassBin0 + SS_MAX_NT / 32 + 1;
constexpr uint32_t kLenBins = kTooLongBin + 1;
// Lengths 1..31 share ONE table, the short group (kept under bin 1): its keys are the packed word
// with a length marker above it (k_short_keys), so a chunk of small-RNA reads (~15 lengths) is one
// key pass and one insert instead of a gather and an insert per length; Group.L / GDesc.L = kShortL
// (the entry's length and word come back from its key).  Length 32 keeps its own table (all 64 bits).
constexpr uint32_t kShortBin = 1, kShortL = 0xFFFFu;
// k_len_count / k_len_scatter: one wave per block, 8 per SIMD (2048 blocks, 2 per SIMD, left both
// passes latency-bound: 0.21 + 0.49 ms for 50M reads), 8 steps' lengths loaded at once (one a step:
// the f2 count 50 us slower, profiles/r4/f2/libab_lenstep.log)
constexpr uint32_t kSplitBlocks = 8192;
constexpr uint32_t kEmptyGroup = 0xFFFFFFFFu;       // slot marker of the empty read's entry
constexpr uint64_t kNoSlot = ~0ull;

__host__ __device__ __forceinline__ uint32_t len_bin(uint32_t L) {
    return L > SS_MAX_NT ? kTooLongBin : L <= 32 ? L : kClassBin0 + (L + 31) / 32;
}

__global__ __launch_bounds__(64) void k_len_count(const uint32_t* __restrict__ lens, uint64_t n,
                                                  uint32_t* __restrict__ blkhist, uint32_t* __restrict__ blkfirst) {
    __shared__ uint32_t h[kLenBins], f[kLenBins];
    for (uint32_t b = threadIdx.x; b < kLenBins; b += 64) {
        h[b] = 0;
        f[b] = 0xFFFFFFFFu;
    }
    __syncthreads();
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t lo = min(n, (uint64_t)blockIdx.x * per), hi = min(n, lo + per);
    // wave-aggregated: one LDS update per distinct bin of a step (the lanes of a bin counted by a
    // ballot, its first read = the step's lowest lane of that bin), not an LDS atomic pair per read
    // kLenStep steps' lengths loaded before any is binned (one load per step left the pass
    // latency-bound: 130 us for 50M reads)
    constexpr int kLenStep = 8;
    // fast set (a 33-160-nt batch, empty reads too): a step whose reads all fall in the empty bin or
    // the classes W = 2 .. 5 is counted in lane registers -- count and first read per bin, reduced
    // across the wave once at the end -- with no peels and no LDS updates
    constexpr uint32_t kFast = 5;            // bins 0, kClassBin0 + 2 .. kClassBin0 + 5
    uint32_t rc[kFast] = {0, 0, 0, 0, 0}, rf[kFast] = {~0u, ~0u, ~0u, ~0u, ~0u};
    for (uint64_t s0 = lo; s0 < hi; s0 += 64 * kLenStep) {
        uint32_t bs[kLenStep];
#pragma unroll
        for (int k = 0; k < kLenStep; ++k) {
            const uint64_t i = s0 + 64u * k + threadIdx.x;
            bs[k] = i < hi ? len_bin(lens[i]) : 0u;
        }
#pragma unroll
        for (int k = 0; k < kLenStep; ++k) {
            const uint64_t i0 = s0 + 64u * k;
            const bool live = i0 + threadIdx.x < hi;
            const uint32_t b = bs[k];
            const uint32_t fi = b == 0u ? 0u : (b >= kClassBin0 + 2u && b <= kClassBin0 + 5u) ? b - kClassBin0 - 1u : kFast;
            if (__ballot(live && fi == kFast) == 0ull) {
#pragma unroll
                for (uint32_t t = 0; t < kFast; ++t)
                    if (live && fi == t) {
                        ++rc[t];
                        rf[t] = min(rf[t], (uint32_t)(i0 + threadIdx.x));
                    }
                continue;
            }
            uint64_t pending = __ballot(live);
            while (pending) {
                const int leader = __ffsll((long long)pending) - 1;
                const uint32_t b0 = (uint32_t)__shfl((int)b, leader);
                const uint64_t mine = __ballot(live && b == b0);
                if (threadIdx.x == (uint32_t)leader) {
                    h[b0] += (uint32_t)__popcll(mine);
                    if (f[b0] == 0xFFFFFFFFu) f[b0] = (uint32_t)(i0 + (uint64_t)leader);   // steps go in read order
                }
                pending &= ~mine;
            }
        }
    }
#pragma unroll
    for (uint32_t t = 0; t < kFast; ++t) {
        uint32_t c = rc[t], m = rf[t];
        for (int o = 32; o > 0; o >>= 1) {
            c += (uint32_t)__shfl_xor((int)c, o);
            m = min(m, (uint32_t)__shfl_xor((int)m, o));
        }
        if (threadIdx.x == 0 && c) {
            const uint32_t b = t == 0 ? 0u : kClassBin0 + 1u + t;
            h[b] += c;
            f[b] = min(f[b], m);
        }
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < kLenBins; b += 64) {
        blkhist[(uint64_t)b * gridDim.x + blockIdx.x] = h[b];
        blkfirst[(uint64_t)b * gridDim.x + blockIdx.x] = f[b];
    }
}

// one block per length bin: exclusive scan of the bin's per-block counts (bin-major rows of blkhist,
// in place) -> offsets inside the bin; out[b] = bin total, out[kLenBins + b] = first read of the bin
__global__ __launch_bounds__(1024) void k_len_binscan(uint32_t nblk, uint32_t* __restrict__ blkhist,
                                                      const uint32_t* __restrict__ blkfirst, uint64_t* __restrict__ out) {
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t run, fmin;
    const uint32_t b = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t* row = blkhist + (uint64_t)b * nblk;
    const uint32_t* frow = blkfirst + (uint64_t)b * nblk;
    if (threadIdx.x == 0) {
        run = 0;
        fmin = 0xFFFFFFFFu;
    }
    __syncthreads();
    uint32_t f = 0xFFFFFFFFu;
    for (uint32_t k0 = 0; k0 < nblk; k0 += 1024) {
        const uint32_t k = k0 + threadIdx.x;
        const uint32_t v = k < nblk ? row[k] : 0u;
        if (k < nblk) f = min(f, frow[k]);
        uint32_t incl = v;
        for (uint32_t off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(incl, off);
            if (lane >= off) incl += y;
        }
        if (lane == 63) wsum[wave] = incl;
        __syncthreads();
        uint32_t before = run;
        for (uint32_t w = 0; w < wave; ++w) before += wsum[w];
        if (k < nblk) row[k] = before + incl - v;
        __syncthreads();
        if (threadIdx.x == 0)
            for (uint32_t w = 0; w < 16; ++w) run += wsum[w];
        __syncthreads();
    }
    if (f != 0xFFFFFFFFu) atomicMin(&fmin, f);
    __syncthreads();
    if (threadIdx.x == 0) {
        out[b] = run;
        out[kLenBins + b] = fmin == 0xFFFFFFFFu ? kNoSlot : fmin;
    }
}

// one block: out[2 kLenBins + b] = start of bin b in d_order (exclusive scan of the bin totals)
__global__ __launch_bounds__(1024) void k_len_binstart(uint64_t* __restrict__ out) {
    __shared__ uint64_t s[2048];
    for (uint32_t b = threadIdx.x; b < 2048; b += 1024) s[b] = b < kLenBins ? out[b] : 0ull;
    __syncthreads();
    for (uint32_t off = 1; off < 2048; off <<= 1) {
        uint64_t y0 = 0, y1 = 0;
        const uint32_t i0 = threadIdx.x, i1 = threadIdx.x + 1024;
        if (i0 >= off) y0 = s[i0 - off];
        if (i1 >= off) y1 = s[i1 - off];
        __syncthreads();
        s[i0] += y0;
        s[i1] += y1;
        __syncthreads();
    }
    for (uint32_t b = threadIdx.x; b < kLenBins; b += 1024) out[2 * kLenBins + b] = s[b] - out[b];
    // the read-order stride the host will choose (process_chunk's `flat`): every counted read a class
    // read of 2 .. 5 words -> W + 1 of the longest; else 0
    if (threadIdx.x == 0) {
        uint32_t w1 = 0;
        bool ok = true;
        for (uint32_t b = 1; b < kTooLongBin; ++b) {
            if (!out[b]) continue;
            if (b <= 32) ok = false;
            else w1 = max(w1, b - kClassBin0 + 1u);
        }
        out[3 * kLenBins] = ok && w1 >= 3u && w1 <= 6u ? w1 : 0u;
    }
}

// stable scatter: block k walks its range in input order, 64 reads per step; the wave peels the
// distinct lengths of the step (readfirstlane + ballot), ranks lanes by popcount below them and
// advances that length's LDS cursor
__global__ __launch_bounds__(64) void k_len_scatter(const uint32_t* __restrict__ lens, uint64_t n,
                                                    const uint32_t* __restrict__ blkoff, const uint64_t* __restrict__ split,
                                                    uint64_t* __restrict__ order) {
    __shared__ uint32_t cur[kLenBins];
    for (uint32_t b = threadIdx.x; b < kLenBins; b += 64)
        cur[b] = (uint32_t)split[2 * kLenBins + b] + blkoff[(uint64_t)b * gridDim.x + blockIdx.x];
    __syncthreads();
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t lo = min(n, (uint64_t)blockIdx.x * per), hi = min(n, lo + per);
    const uint32_t lane = threadIdx.x;
    const uint64_t lt = (1ull << lane) - 1ull;
    constexpr int kLenStep = 8;         // as k_len_count: the steps' lengths loaded together
    for (uint64_t s0 = lo; s0 < hi; s0 += 64 * kLenStep) {
        uint32_t bs[kLenStep];
#pragma unroll
        for (int k = 0; k < kLenStep; ++k) {
            const uint64_t i = s0 + 64u * k + lane;
            bs[k] = i < hi ? len_bin(lens[i]) : 0u;
        }
#pragma unroll
        for (int k = 0; k < kLenStep; ++k) {
            const uint64_t i = s0 + 64u * k + lane;
            const bool live = i < hi;
            const uint32_t b = bs[k];
            uint64_t pending = __ballot(live);
            while (pending) {
                const int leader = __ffsll((long long)pending) - 1;
                const uint32_t b0 = (uint32_t)__shfl((int)b, leader);
                const uint64_t mine = __ballot(live && b == b0);
                const uint32_t base = cur[b0];
                if (live && b == b0) {
                    const uint32_t pos = base + (uint32_t)__popcll(mine & lt);
                    order[pos] = i;
                }
                __syncthreads();   // one wave: orders the cursor read before the update
                if (lane == (uint32_t)leader) cur[b0] = base + (uint32_t)__popcll(mine);
                __syncthreads();
                pending &= ~mine;
            }
        }
    }
}

// row map of an insert: dst[r] = global index of row r (base + sel[r], or base + r when sel is null)
__global__ __launch_bounds__(256) void k_rowmap(const uint64_t* __restrict__ sel, uint64_t m, uint64_t base,
                                                uint64_t* __restrict__ dst) {
    for (uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x; r < m; r += (uint64_t)gridDim.x * 256)
        dst[r] = base + (sel ? sel[r] : r);
}

// table entry e -> the bit of its global first read (rowmap[first[e]]) in the read map; e == m: the
// empty read's entry at global read `extra` (kNoSlot: none)
// (dm: the entry count on the device instead -- the speculative finish, which runs without a sync)
__global__ __launch_bounds__(256) void k_mark(const uint64_t* __restrict__ first, uint64_t m,
                                              const uint64_t* __restrict__ rowmap, uint64_t extra,
                                              unsigned long long* __restrict__ bits, const uint64_t* dm = nullptr) {
    if (dm) m = min(m, *dm);          // (m: the buffers' capacity then)
    for (uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x; e <= m; e += (uint64_t)gridDim.x * 256) {
        const uint64_t r = e < m ? rowmap[first[e]] : extra;
        if (r != kNoSlot) atomicOr(&bits[r >> 6], 1ull << (r & 63));
    }
}

// entry e of group g -> its place in read order: the marked reads before its first read
// (wpre: exclusive prefix of the map words' popcounts)
__global__ __launch_bounds__(256) void k_rank(const uint64_t* __restrict__ first, uint64_t m,
                                              const uint64_t* __restrict__ rowmap, uint32_t g, uint64_t extra,
                                              const unsigned long long* __restrict__ bits,
                                              const uint64_t* __restrict__ wpre, uint64_t* __restrict__ ordered,
                                              const uint64_t* dm = nullptr, uint64_t ocap = ~0ull) {
    if (dm) m = min(m, *dm);          // (m: the buffers' capacity then; ocap: ordered's)
    for (uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x; e <= m; e += (uint64_t)gridDim.x * 256) {
        const uint64_t r = e < m ? rowmap[first[e]] : extra;
        if (r == kNoSlot) continue;
        const uint64_t pos = wpre[r >> 6] + (uint64_t)__popcll(bits[r >> 6] & ((1ull << (r & 63)) - 1ull));
        if (pos < ocap) ordered[pos] = e < m ? ((uint64_t)g << 32) | e : (uint64_t)kEmptyGroup << 32;
    }
}

// export: entry e's first read (engine-local) = rowmap[first[e]]
// the largest of m counts (atomicMax into *mx): an export's largest count sizes the merge passes.
// Grid-stride with a capped grid and one atomic per block: the single counter takes kMaxBlocks
// atomics, not one per wave of the entries (262k at 2^24 entries, serialised on one address)
constexpr unsigned kCountMaxBlocks = 1024;
__global__ __launch_bounds__(256) void k_count_max(const uint64_t* __restrict__ counts, uint64_t m,
                                                   unsigned long long* mx, const uint64_t* dm = nullptr) {
    if (dm) m = min(m, *dm);
    uint64_t v = 0;
    for (uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x; e < m; e += (uint64_t)gridDim.x * 256)
        v = max(v, counts[e]);
    for (int o = 32; o > 0; o >>= 1) v = max(v, (uint64_t)__shfl_xor((unsigned long long)v, o));
    __shared__ uint64_t wmax[4];
    if ((threadIdx.x & 63u) == 0) wmax[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint64_t b = max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
        if (b) atomicMax(mx, (unsigned long long)b);
    }
}

// one merge pass: take = min(left, room) of every entry's remaining count
__global__ __launch_bounds__(256) void k_count_take(uint64_t* __restrict__ left, uint64_t* __restrict__ take, uint64_t m,
                                                    uint64_t room) {
    for (uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x; e < m; e += (uint64_t)gridDim.x * 256) {
        const uint64_t t = min(left[e], room);
        take[e] = t;
        left[e] -= t;
    }
}

__global__ __launch_bounds__(256) void k_export_reads(const uint64_t* __restrict__ first, uint64_t m,
                                                      const uint64_t* __restrict__ rowmap, uint64_t* __restrict__ out) {
    for (uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x; e < m; e += (uint64_t)gridDim.x * 256)
        out[e] = rowmap[first[e]];
}

// merge: a source group's m entries become rows `rows + e` of the destination group (first index of
// the merged entry), their row map = the source's local first read + the source shard's base
__global__ __launch_bounds__(256) void k_merge_rows(uint64_t m, uint64_t rows, uint64_t base,
                                                    uint64_t* __restrict__ first, uint64_t* __restrict__ rowmap) {
    for (uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x; e < m; e += (uint64_t)gridDim.x * 256) {
        first[e] = rows + e;
        rowmap[rows + e] += base;
    }
}

// spilled counts back onto extracted entries: counts[e] += acc[first[e]] for e < *m (rows < acc_rows)
__global__ __launch_bounds__(256) void k_add_acc(uint64_t* __restrict__ counts, const uint64_t* __restrict__ first,
                                                 const uint64_t* __restrict__ m, const uint64_t* __restrict__ acc,
                                                 uint64_t acc_rows) {
    const uint64_t n = *m;
    for (uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (uint64_t)gridDim.x * 256)
        if (first[e] < acc_rows) counts[e] += acc[first[e]];
}

// re-key with spilled counts: entry e's spilled count moves to its new row e
__global__ __launch_bounds__(256) void k_rekey_acc(const uint64_t* __restrict__ first, uint64_t m,
                                                   const uint64_t* __restrict__ acc, uint64_t acc_rows,
                                                   uint64_t* __restrict__ nacc) {
    for (uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x; e < m; e += (uint64_t)gridDim.x * 256)
        nacc[e] = first[e] < acc_rows ? acc[first[e]] : 0ull;
}

// re-key: entry e of a group's table becomes row e (its first index), the new row map = the entry's
// first read
__global__ __launch_bounds__(256) void k_rekey(const uint64_t* __restrict__ first, uint64_t m,
                                               const uint64_t* __restrict__ rowmap, uint64_t* __restrict__ nmap,
                                               uint64_t* __restrict__ nfirst) {
    for (uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x; e < m; e += (uint64_t)gridDim.x * 256) {
        nmap[e] = rowmap[first[e]];
        nfirst[e] = e;
    }
}

// ---- stable compaction / exclusive scan over n items in 1024 contiguous block ranges -------------
constexpr uint32_t kScanBlocks = 1024;

struct GDesc {
    const uint64_t* words;   // [m * W]
    const uint64_t* counts;  // [m]
    uint32_t W;
    uint32_t L;              // 0: a length class (entry length = its last word, ceil(L/32) words used)
};

__device__ __forceinline__ uint32_t entry_len(const GDesc& d, uint64_t e) {
    if (d.L == kShortL) return (uint32_t)(63 - __clzll((long long)d.words[e])) >> 1;    // marker at 2L + 1
    return d.L ? d.L : (uint32_t)d.words[e * d.W + d.W - 1];
}

// item value for the two scans: MODE 0 = marked reads in read-map word i, MODE 1 = words of ordered
// entry i
template <int MODE>
__device__ __forceinline__ uint32_t item_val(const uint64_t* src, uint64_t i, const GDesc* gd) {
    const uint64_t v = src[i];
    if (MODE == 0) return (uint32_t)__popcll(v);
    const uint32_t g = (uint32_t)(v >> 32);
    if (g == kEmptyGroup) return 0u;
    const GDesc d = gd[g];
    return d.L ? d.W : d.W - 1;      // a class table's entries (W + 1 key words) all have W words
}

template <int MODE>
__global__ __launch_bounds__(256) void k_scan_count(const uint64_t* __restrict__ src, uint64_t n, const GDesc* gd,
                                                    uint64_t* __restrict__ blksum, const uint64_t* dn = nullptr) {
    __shared__ uint64_t s[256];
    if (dn) n = min(n, *dn);
    const uint64_t per = (n + kScanBlocks - 1) / kScanBlocks;
    const uint64_t lo = min(n, (uint64_t)blockIdx.x * per), hi = min(n, lo + per);
    uint64_t c = 0;
    for (uint64_t i = lo + threadIdx.x; i < hi; i += 256) c += item_val<MODE>(src, i, gd);
    s[threadIdx.x] = c;
    __syncthreads();
    for (uint32_t off = 128; off; off >>= 1) {
        if (threadIdx.x < off) s[threadIdx.x] += s[threadIdx.x + off];
        __syncthreads();
    }
    if (threadIdx.x == 0) blksum[blockIdx.x] = s[0];
}

// exclusive scan of kScanBlocks block sums (one block); blksum[kScanBlocks] = total
// 256 threads x 4 sums (not 1024 x 1): on the speculative finish's stream a 16-wave workgroup waits
// for one CU to free 16 wave slots of the verify beside it; four waves find room as soon as one of the
// verify's blocks retires
__global__ __launch_bounds__(256) void k_scan_top(uint64_t* __restrict__ blksum) {
    static_assert(kScanBlocks == 1024, "4 block sums per thread");
    __shared__ uint64_t wsum[4];
    const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
    uint64_t v[4], tot = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        v[k] = blksum[4 * t + k];
        tot += v[k];
    }
    uint64_t incl = tot;
    for (uint32_t off = 1; off < 64; off <<= 1) {
        const uint32_t ylo = (uint32_t)__shfl_up((int)(uint32_t)incl, off), yhi = (uint32_t)__shfl_up((int)(uint32_t)(incl >> 32), off);
        if (lane >= off) incl += (uint64_t)yhi << 32 | ylo;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint64_t run = incl - tot;
    for (uint32_t w = 0; w < wave; ++w) run += wsum[w];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        blksum[4 * t + k] = run;
        run += v[k];
    }
    if (t == 255) blksum[1024] = run;
}

// block-local ordered walk (256 items per step, wave scans + a 4-wave prefix): each item's exclusive
// prefix to dst (MODE 0: read-map word -> marked reads before it; MODE 1: ordered entry -> its word
// offset)
template <int MODE>
__global__ __launch_bounds__(256) void k_scan_apply(const uint64_t* __restrict__ src, uint64_t n, const GDesc* gd,
                                                    const uint64_t* __restrict__ blksum, uint64_t* __restrict__ dst,
                                                    const uint64_t* dn = nullptr) {
    __shared__ uint64_t wsum[4];
    __shared__ uint64_t run;
    if (dn) n = min(n, *dn);
    const uint64_t per = (n + kScanBlocks - 1) / kScanBlocks;
    const uint64_t lo = min(n, (uint64_t)blockIdx.x * per), hi = min(n, lo + per);
    if (threadIdx.x == 0) run = blksum[blockIdx.x];
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint64_t i0 = lo; i0 < hi; i0 += 256) {
        const uint64_t i = i0 + threadIdx.x;
        const uint32_t v = i < hi ? item_val<MODE>(src, i, gd) : 0u;
        // inclusive wave scan of v
        uint32_t incl = v;
        for (uint32_t off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(incl, off);
            if (lane >= off) incl += y;
        }
        if (lane == 63) wsum[wave] = incl;
        __syncthreads();
        uint64_t before = run;
        for (uint32_t w = 0; w < wave; ++w) before += wsum[w];
        const uint64_t pos = before + incl - v;
        if (i < hi) dst[i] = pos;
        __syncthreads();
        if (threadIdx.x == 0) run += wsum[0] + wsum[1] + wsum[2] + wsum[3];
        __syncthreads();
    }
}

// ordered entry k -> (length, count, words at woff[k]) straight into the pinned host result arrays
// (no device copy, no D2H copies after it):
// one block per 256 ordered entries; lengths and counts lane per entry, the block's words (one
// contiguous run of the output) staged in LDS and stored lane per word, so every store to host
// memory is a coalesced run (the device-to-host stores run at the PCIe rate, ~55 GB/s, as the blit
// copies did, with the gather itself hidden under them).
// Where the rows go: the pinned buffer hbase (hcap bytes) laid out as results_layout() says.  dK /
// dNW: the entry and word totals on the device (the speculative finish; K is then the ordered
// buffer's bound) -- a layout past hcap, or more entries than the bound, raises *bad and writes
// nothing.  compact: lengths u16, and counts u32 unless wide (the host's rule: a count can reach
// 2^32 only when the engine has counted that many reads).
struct OutLayout {
    uint8_t* hbase;
    uint64_t hcap;
    const uint64_t* dK;
    const uint64_t* dNW;
    uint64_t NW;
    unsigned long long* bad;
    int compact;
    int wide;               // compact counts as u64 (a count can reach 2^32: the engine's reads can)
};

// byte offsets of the counts and words arrays of K rows (lengths at 0): the plain layout has u32
// lengths and u64 counts; compact, u16 lengths and counts of cw bytes (4 or 8)
__host__ __device__ __forceinline__ void results_layout(uint64_t K, int compact, uint32_t cw, uint64_t& cnt_off,
                                                        uint64_t& word_off) {
    cnt_off = ((compact ? K * 2 : K * 4) + 15) & ~15ull;
    word_off = cnt_off + (((compact ? K * cw : K * 8) + 15) & ~15ull);
}

constexpr uint32_t kOutBuf = 4096;
__global__ __launch_bounds__(256) void k_gather_host(const uint64_t* __restrict__ ordered, uint64_t K,
                                                     const GDesc* __restrict__ gd, const uint64_t* __restrict__ woff,
                                                     uint64_t empty_count, OutLayout o) {
    __shared__ uint64_t buf[kOutBuf];
    __shared__ uint64_t s_lo, s_hi;
    const uint32_t cw = o.wide ? 8u : 4u;
    uint64_t co, wo0;
    if (o.dK) {                     // (K: the ordered buffer's bound then)
        const uint64_t Kd = *o.dK;
        results_layout(Kd, o.compact, cw, co, wo0);
        if (Kd > K || wo0 + *o.dNW * 8 > o.hcap) {
            if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(o.bad, 1ull);
            return;
        }
        K = Kd;
    } else {
        results_layout(K, o.compact, cw, co, wo0);
    }
    uint8_t* h_cnt = o.hbase + co;
    uint64_t* h_words = (uint64_t*)(o.hbase + wo0);
    const uint64_t k0 = (uint64_t)blockIdx.x * 256, k = k0 + threadIdx.x;
    if (k0 >= K) return;
    uint32_t L = 0, nw = 0;
    uint64_t cnt = 0, wo = 0, smask = ~0ull;     // smask: a short-group key's length marker cleared
    const uint64_t* src = nullptr;
    if (k < K) {
        const uint64_t v = ordered[k];
        const uint32_t g = (uint32_t)(v >> 32);
        if (g == kEmptyGroup) {
            cnt = empty_count;
        } else {
            const uint64_t e = (uint32_t)v;
            const GDesc d = gd[g];
            L = entry_len(d, e);
            nw = d.L ? d.W : (L + 31) / 32;
            cnt = d.counts[e];
            src = d.words + e * d.W;
            if (d.L == kShortL) smask = ~(1ull << (2 * L + 1));
        }
        wo = woff[k];
        if (o.compact) {
            ((uint16_t*)o.hbase)[k] = (uint16_t)L;
            if (cw == 4) ((uint32_t*)h_cnt)[k] = (uint32_t)cnt;
            else ((uint64_t*)h_cnt)[k] = cnt;
        } else {
            ((uint32_t*)o.hbase)[k] = L;
            ((uint64_t*)h_cnt)[k] = cnt;
        }
    }
    const uint64_t klast = min(k0 + 255, K - 1);
    if (k == k0) s_lo = wo;
    if (k == klast) s_hi = wo + nw;
    __syncthreads();
    const uint64_t lo = s_lo, hi = s_hi;
    for (uint64_t c0 = lo; c0 < hi; c0 += kOutBuf) {      // one round unless the block's rows are long
        const uint64_t c1 = min(hi, c0 + kOutBuf);
        for (uint32_t q = 0; q < nw; ++q) {
            const uint64_t o = wo + q;
            if (o >= c0 && o < c1) buf[o - c0] = src[q] & smask;
        }
        __syncthreads();
        for (uint64_t o = c0 + threadIdx.x; o < c1; o += 256) h_words[o] = buf[o - c0];
        __syncthreads();
    }
}

// The speculative finish's gather, run beside the verify: kGatherWaves waves in all (a short grid),
// each over chunks of 64 ordered entries on its own (no block barriers; its words staged in its own
// LDS window), the next chunk's entries loaded before the current one's stores.  The rows reach the
// pinned buffer at the PCIe rate from few waves, and the verify keeps the chip: a 50-MB store into
// pinned memory beside a verify-shaped kernel held it 0.94 -> 1.64 ms from 4096 blocks, 1.03 ms from
// 64 at the same ~52 GB/s (tools/probe_overlap.hip).
constexpr uint32_t kGatherBlocks = 64, kGatherWin = 1024;
constexpr uint64_t kGatherWavesMax = 4ull << 20;     // entries (bound) up to which the speculative finish uses it
__global__ __launch_bounds__(256) void k_gather_host_waves(const uint64_t* __restrict__ ordered, uint64_t K,
                                                           const GDesc* __restrict__ gd, const uint64_t* __restrict__ woff,
                                                           uint64_t empty_count, OutLayout o) {
    __shared__ uint64_t buf[4][kGatherWin];
    const uint32_t cw = o.wide ? 8u : 4u, lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint64_t co, wo0;
    const uint64_t Kd = *o.dK;              // (K: the ordered buffer's bound)
    results_layout(Kd, o.compact, cw, co, wo0);
    if (Kd > K || wo0 + *o.dNW * 8 > o.hcap) {
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(o.bad, 1ull);
        return;
    }
    K = Kd;
    uint8_t* h_cnt = o.hbase + co;
    uint64_t* h_words = (uint64_t*)(o.hbase + wo0);
    uint64_t* wb = buf[wave];
    const uint64_t nchunk = (K + 63) / 64, cstride = (uint64_t)gridDim.x * 4;
    uint64_t c = (uint64_t)blockIdx.x * 4 + wave;
    uint64_t v = 0, wo = 0;
    if (c < nchunk) {
        const uint64_t k = min(c * 64 + lane, K - 1);
        v = ordered[k];
        wo = woff[k];
    }
    for (; c < nchunk; c += cstride) {
        const uint64_t k0 = c * 64, k = k0 + lane;
        const bool live = k < K;
        const uint64_t cv = v, cwo = wo;
        if (c + cstride < nchunk) {         // the next chunk's entries in flight behind this one
            const uint64_t kn = min((c + cstride) * 64 + lane, K - 1);
            v = ordered[kn];
            wo = woff[kn];
        }
        uint32_t L = 0, nw = 0;
        uint64_t cnt = 0, smask = ~0ull;
        const uint64_t* src = nullptr;
        if (live) {
            const uint32_t g = (uint32_t)(cv >> 32);
            if (g == kEmptyGroup) {
                cnt = empty_count;
            } else {
                const uint64_t e = (uint32_t)cv;
                const GDesc d = gd[g];
                L = entry_len(d, e);
                nw = d.L ? d.W : (L + 31) / 32;
                cnt = d.counts[e];
                src = d.words + e * d.W;
                if (d.L == kShortL) smask = ~(1ull << (2 * L + 1));
            }
            if (o.compact) {
                ((uint16_t*)o.hbase)[k] = (uint16_t)L;
                if (cw == 4) ((uint32_t*)h_cnt)[k] = (uint32_t)cnt;
                else ((uint64_t*)h_cnt)[k] = cnt;
            } else {
                ((uint32_t*)o.hbase)[k] = L;
                ((uint64_t*)h_cnt)[k] = cnt;
            }
        }
        // the chunk's words are one run of the output: [lane 0's offset, the last live lane's end)
        const uint32_t last = (uint32_t)min((uint64_t)63, K - 1 - k0);
        const uint64_t lo = (uint64_t)__shfl((long long)cwo, 0);
        const uint64_t hi = (uint64_t)__shfl((long long)(cwo + nw), (int)last);
        for (uint64_t c0 = lo; c0 < hi; c0 += kGatherWin) {     // one window unless the chunk's rows are long
            const uint64_t c1 = min(hi, c0 + kGatherWin);
            for (uint32_t q = 0; q < nw; ++q) {
                const uint64_t oo = cwo + q;
                if (oo >= c0 && oo < c1) wb[oo - c0] = src[q] & smask;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            for (uint64_t oo = c0 + lane; oo < c1; oo += 64) h_words[oo] = wb[oo - c0];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
}

// the speculative finish's entry total: the classes' extracted counts (tot[2 .. 5]) + the empty read's
// entry; out[1] = the words total (the word scan's), out[2] = its bad flag folded with the extract's
// capacity overflow -- then one D2H copy of out[0 .. 2]
__global__ void k_spec_total(uint64_t* sd, uint64_t empty, const uint64_t* nw_total, uint64_t empty_count = 0) {
    if (threadIdx.x != 0) return;
    uint64_t K = empty;
    for (int W = 2; W < 6; ++W) K += sd[W];
    sd[6] = K;
    if (nw_total) {
        sd[9] = sd[6];
        sd[10] = *nw_total;
        sd[11] = sd[7] | sd[8];
        sd[12] = max(sd[12], empty_count);   // (the largest count, the empty read's entry too)
    }
}

inline unsigned grid_of(uint64_t items, uint32_t per_block, unsigned cap = 4096) {
    uint64_t b = (items + per_block - 1) / per_block;
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(b, cap));
}

uint64_t pow2_at_least(uint64_t x) {
    uint64_t p = 1024;
    while (p < x) p <<= 1;
    return p;
}

// grow-only device buffer
template <typename T>
struct DBuf {
    T* p = nullptr;
    uint64_t cap = 0;
    int ensure(uint64_t n) {
        if (n <= cap) return SS_OK;
        if (p) {
            (void)hipDeviceSynchronize();   // queued work may still read the old buffer
            (void)hipFree(p);
        }
        p = nullptr;
        cap = 0;
        const uint64_t want = std::max<uint64_t>(n, 1024);
        if (hipMalloc((void**)&p, want * sizeof(T)) != hipSuccess) {
            (void)hipGetLastError();
            return ss_fail(SS_ENOMEM, "ingest: out of device memory");
        }
        cap = want;
        return SS_OK;
    }
    // grow keeping the first `used` elements (geometric: appended-to buffers such as row maps)
    int ensure_keep(uint64_t n, uint64_t used, hipStream_t s) {
        if (n <= cap) return SS_OK;
        T* q = nullptr;
        const uint64_t want = std::max<uint64_t>(n, 2 * cap);
        if (hipMalloc((void**)&q, want * sizeof(T)) != hipSuccess) {
            (void)hipGetLastError();
            return ss_fail(SS_ENOMEM, "ingest: out of device memory");
        }
        int rc = SS_OK;
        if (used) rc = ss_check(hipMemcpyAsync(q, p, used * sizeof(T), hipMemcpyDeviceToDevice, s), "ingest grow copy");
        if (!rc) rc = ss_check(hipStreamSynchronize(s), "ingest grow copy");
        if (p) (void)hipFree(p);
        p = q;
        cap = want;
        return rc;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

// grow-only pinned host buffer
struct HBuf {
    uint8_t* p = nullptr;
    uint64_t cap = 0;
    int ensure(uint64_t n) {
        if (n <= cap) return SS_OK;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        const uint64_t want = std::max<uint64_t>(n, 1 << 20);
        if (hipHostMalloc((void**)&p, want, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            return ss_fail(SS_ENOMEM, "ingest: out of pinned host memory");
        }
        cap = want;
        return SS_OK;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
};

// the FASTQ reader ring (ss_ingest_add_fastq_range): a slot is one chunk, pinned and on the device
constexpr uint64_t kFqPiece = 64ull << 20;           // file read / H2D piece
constexpr uint64_t kFqChunkDefault = 1ull << 30;     // chunk bytes when the caller passes 0
struct FqSlot {
    HBuf h;
    DBuf<uint8_t> d;
    hipEvent_t done = nullptr;    // the slot's H2D pieces are complete (recorded on fq_copy)
    std::vector<hipEvent_t> ev;   // 2 timing events per H2D piece
    uint32_t np = 0;              // pieces of the chunk in the slot
    uint64_t n = 0, use = 0;      // bytes in the slot, bytes up to its last newline (n at the range's end)
    bool at_eof = false;
    int rc = SS_OK;
    std::string err;              // the reader's error message (its last-error string is thread-local)
};

struct Group {
    uint32_t L = 0;               // 1..32: the length of every key; 0: a length class
    uint32_t W1 = 1;              // words per table key: 1, or a class's ceil(L/32) + 1 (length word)
    ss_counter* table = nullptr;
    uint64_t cap = 0;
    uint64_t rows = 0;            // rows inserted (= the table's first index space)
    DBuf<uint64_t> rowmap;        // row -> global read index (the table's first index is the row)
    // finish() / ss_ingest_export(): the extracted entries
    DBuf<uint64_t> fps, words, counts, first;
    DBuf<uint32_t> lens;
    DBuf<uint64_t> xread;         // export: each entry's first read (engine-local index)
    uint64_t m = 0, nw = 0;       // extracted entries, their output words
    DBuf<uint64_t> acc;           // row -> counts spilled out of the table (u64; rows < acc_rows)
    uint64_t acc_rows = 0;
};

}  // namespace

struct ss_ingest {
    int device = 0;
    hipStream_t stream = nullptr;
    // the length classes' table inserts run on up to kSide + 1 streams (independent tables: one
    // class's short partition kernels and aggregate tail overlap another's); forked / joined by events
    static constexpr int kSide = 2;
    hipStream_t side[kSide] = {};
    hipEvent_t ev_fork = nullptr, ev_join[kSide] = {};
    HBuf stage;                    // list bytes / FASTQ chunks (pinned)
    HBuf out_host;                 // results: lens | counts | words (pinned)
    DBuf<uint8_t> dbuf;            // the chunk on the device
    DBuf<uint64_t> offs;           // per read: offset in the chunk
    DBuf<uint32_t> dlens;          // per read: length (0xFFFFFFFF = strlen underflow)
    DBuf<uint64_t> order;          // split output
    DBuf<uint32_t> blkhist, blkfirst;
    DBuf<uint64_t> split_out;      // [3 * kLenBins + 1]: totals, first reads, starts, the read-order stride
    uint64_t* h_split = nullptr;   // pinned copy
    // the previous chunk's read-order stride (0: it took another path): the next chunk's row encode is
    // queued at that stride before its split comes back (process_chunk); flat_streak = how many chunks
    // in a row took the read-order path at that stride
    uint32_t flat_hint = 0, flat_streak = 0;
    // process_chunk: pooled tables taken for new groups have their reset words queued here and set in
    // one dispatch (flush_prep) before any of them is used, not one launch per table
    bool defer_prep = false;
    std::vector<unsigned long long*> prep_p;
    std::vector<unsigned long long> prep_v;
    hipEvent_t ev_split = nullptr;
    DBuf<uint8_t> rows;            // gathered dense rows (lengths <= 32)
    DBuf<uint64_t> cls_words;      // the length classes' packed rows (k_encode_classes / k_encode_class)
    DBuf<uint64_t> cls_fps;        // their fingerprints (k_encode_classes), class after class
    ss_counter* fpt = nullptr;     // the classes' rows counted by fingerprint (single-word scratch table)
    DBuf<uint32_t> cls_flag;       // set by ss_classes_verify_fold: two keys share a fingerprint
    DBuf<uint32_t> hll;            // per class W: 2^kHllLog HyperLogLog registers over the call
    uint32_t* h_hll = nullptr;     // pinned copy
    DBuf<uint64_t> ovf;            // per job: its table's overflow word after the insert
    bool failed = false;           // an add returned SS_EFULL: the counts are void until reset
    int sizing = 0;                // class tables: 0 by their sketch, 1 by their rows, 2 by 1/64 of the
                                   // sketch (tests: forces the SS_EFULL path) -- ss_ingest_set_exact
    DBuf<uint64_t> first_bad;      // [kLenBins + 1]: one u64 per length bin, the class encode's last
    uint64_t* h_bad = nullptr;     // pinned [3 kLenBins + 8]: first-bad and overflow words, a size query
    DBuf<uint64_t> fq_ws, fq_aux, fq_counts;
    std::map<uint32_t, Group> groups;
    std::vector<std::pair<uint64_t, ss_counter*>> pool;    // idle tables (capacity, handle)
    uint64_t nreads = 0;           // global read index of the next read
    uint64_t empty_count = 0, empty_first = kNoSlot;
    // first rejected read (input order)
    uint64_t bad_index = kNoSlot;
    int bad_kind = 0;
    std::string bad_bytes;
    double est_scale = 1.0;        // FASTQ: file bytes / bytes seen (multi-word table sizing)
    bool exported = false;         // ss_ingest_export ran (the groups' m / buffers hold the entries)
    uint64_t xmax = 0;             // the export's largest count (the merge passes it needs)
    // reads counted since the tables' counts were last spilled into the groups' u64 row counts: a
    // slot's u32 count cannot pass it, so the spill before it reaches 2^32 - 1 keeps every count exact
    uint64_t since_spill = 0, spill_limit = 0xFFFFFFFEull;
    uint64_t max_rows = 0xFFFFFFFFull;   // rows a group's table indexes (its first index is u32);
                                         // ss_ingest_set_row_limit lowers it (test hook)
    // A read-order chunk whose class tables held no rows before it (a single-chunk count, the usual
    // case) leaves its verified scratch (fpt and its representatives) unfolded: the next add / export /
    // merge folds it into the class tables first (flush_pending), a finish takes the entries straight
    // from the scratch (ss_classes_flat_extract: no class-table inserts, no table extraction)
    bool pend = false;
    uint32_t pend_S = 0;
    uint64_t pend_base = 0;
    ss_flat_class pend_fc[6] = {};
    DBuf<uint32_t> zero32;         // a device u32 that stays 0
    // The speculative finish: the FIRST chunk of a count (nothing before it), taken by the read-order
    // path with its fold deferred, queues the finish's whole work -- the scratch's entries extracted,
    // read-order ranks, the rows gathered into the pinned result buffer -- on spec_stream right after
    // the scratch's representatives, beside the verify, with every size kept on the device (no sync).
    // ss_ingest_finish then only waits for it; any other call waits for it first (spec_wait) and
    // drops it.  A verify that flags a shared fingerprint, a rejected read, or a result larger than
    // the bound it was given invalidates it (the finish then runs the ordinary way).
    hipStream_t spec_stream = nullptr;
    hipEvent_t ev_reps = nullptr, ev_spec = nullptr;
    bool spec_inflight = false;
    bool spec_valid = false;
    DBuf<uint64_t> spec_dev;       // [12]: class totals [2..5], K [6], gather bad [7], extract overflow [8], K NW bad [9..11]
    uint64_t* h_spec = nullptr;    // pinned [4]: K, NW, bad, the largest count
    int compact = 0;               // ss_ingest_set_results_format: u16 lengths, u32 counts when they fit
    bool wide = false;             // compact results whose counts need u64
    GDesc* h_gdesc = nullptr;      // pinned [8]
    // ss_ingest_merge scratch (this engine as the destination): a source group's entries on this device
    DBuf<uint64_t> mg_words, mg_counts, mg_first, mg_take;
    DBuf<uint32_t> mg_lens;
    // finish() results
    uint64_t nkeys = 0, nwords = 0;
    DBuf<uint64_t> slot, ordered, woff, scan;
    DBuf<GDesc> gdesc;
    // FASTQ stage split since the last ss_ingest_fastq_stages: host ms of the file
    // reads, device ms of the H2D pieces (event pairs, summed), host ms of the index (to its sync), of
    // the chunk counts (process_chunk) and of ss_ingest_finish; the bytes the H2D pieces moved
    double fq_ms[5] = {};
    uint64_t fq_h2d_bytes = 0;
    FqSlot fq[2];
    hipStream_t fq_copy = nullptr;     // the reader thread's H2D pieces
    // the reader thread's CPUs: the GPU's NUMA node's (ss_gpu_numa_cpus; looked up once, fq_node -2
    // until then), so the pinned slots it allocates and the file bytes it copies in are node-local
    std::vector<int> fq_cpus;
    int fq_node = -2;
};

namespace {

// a pooled table of this capacity, preferring one whose key width W1 (its key-word array) and
// partition workspace (rows) already fit: a mismatch reallocates them at the first insert (hipFree +
// hipMalloc, 0.3-0.4 ms per class table on the f2 batch when two classes swapped tables of one size)
int table_get(ss_ingest* g, uint64_t cap, uint32_t W1, uint64_t rows, ss_counter** out) {
    size_t best = g->pool.size();
    int best_score = -1;
    for (size_t i = g->pool.size(); i-- > 0;) {
        if (g->pool[i].first != cap) continue;
        ss_counter* t = g->pool[i].second;
        const int score = (ss_counter_words(t) == (int)W1 ? 2 : 0) + (ss_counter_reserved(t) >= rows ? 1 : 0);
        if (score > best_score) {
            best_score = score;
            best = i;
        }
    }
    if (best < g->pool.size()) {
        *out = g->pool[best].second;
        g->pool.erase(g->pool.begin() + (long)best);
        if (!g->defer_prep) return ss_counter_reset(*out, g->stream);
        unsigned long long* p[3];
        unsigned long long v[3];
        const int rc = ss_counter_reset_host(*out, p, v);
        g->prep_p.insert(g->prep_p.end(), p, p + 3);
        g->prep_v.insert(g->prep_v.end(), v, v + 3);
        return rc;
    }
    return ss_counter_create(cap, out);
}

// the queued reset words in one dispatch on the engine's stream (or several, past kPrepMany words)
int flush_prep(ss_ingest* g) {
    int rc = SS_OK;
    for (size_t i = 0; i < g->prep_p.size() && !rc; i += kPrepMany) {
        const uint32_t k = (uint32_t)std::min<size_t>(kPrepMany, g->prep_p.size() - i);
        rc = ss_prep_words(g->prep_p.data() + i, g->prep_v.data() + i, k, g->stream);
    }
    g->prep_p.clear();
    g->prep_v.clear();
    return rc;
}

// device bytes a pooled table holds: its slots and its partition workspace (~100 B per reserved read)
uint64_t table_bytes(ss_counter* t) { return ss_counter_capacity(t) * 16 + ss_counter_reserved(t) * 100; }

void table_put(ss_ingest* g, ss_counter* t) {
    if (!t) return;
    g->pool.emplace_back(ss_counter_capacity(t), t);   // workspace kept: the next call reuses it
    uint64_t total = 0;
    for (auto& p : g->pool) total += table_bytes(p.second);
    while (!g->pool.empty() && total > (6ull << 30)) {
        total -= table_bytes(g->pool.front().second);
        ss_counter_destroy(g->pool.front().second);
        g->pool.erase(g->pool.begin());
    }
}

// size query (one sync): occupied slots of a table
int table_size(ss_ingest* g, ss_counter* t, uint64_t* out) {
    DBuf<uint64_t>& s = g->scan;
    int rc = s.ensure(kScanBlocks + 8);
    if (rc) return rc;
    rc = ss_counter_size(t, s.p + kScanBlocks + 2, g->stream);
    if (rc) return rc;
    rc = ss_check(hipMemcpyAsync(g->h_bad + 2 * kLenBins + 2, s.p + kScanBlocks + 2, 8, hipMemcpyDeviceToHost, g->stream), "ingest size copy");
    if (!rc) rc = ss_check(hipStreamSynchronize(g->stream), "ingest sync");
    *out = g->h_bad[2 * kLenBins + 2];
    return rc;
}

// HyperLogLog estimate of the distinct keys behind 2^kHllLog registers (Flajolet et al. 2007, with
// linear counting below 2.5 m)
double hll_estimate(const uint32_t* reg) {
    // 2^-k from a table: the estimate sits between the encode and the inserts it sizes, and 2048
    // ldexp calls per class were ~40 us of host time there (a register is <= 64 - kHllLog + 1)
    static const auto pw = [] {
        std::array<double, 66> t{};
        for (int k = 0; k < 66; ++k) t[k] = std::ldexp(1.0, -k);
        return t;
    }();
    const double m = (double)(1u << kHllLog);
    double sum = 0;
    uint32_t zeros = 0;
    for (uint32_t j = 0; j < (1u << kHllLog); ++j) {
        const uint32_t r = std::min<uint32_t>(reg[j], 65u);
        sum += pw[r];
        zeros += r == 0;
    }
    double e = 0.7213 / (1.0 + 1.079 / m) * m * m / sum;
    if (e <= 2.5 * m && zeros) e = m * std::log(m / (double)zeros);
    return e;
}

// key kind of a fresh table: the length (fixed by its first insert) or a class's packed words
int table_kind(const Group& gr, ss_counter* t) {
    // (the short group's keys are whole 64-bit words: a length-32 handle)
    return gr.L ? ss_counter_set_length(t, gr.L == kShortL ? 32u : gr.L) : ss_counter_set_words(t, gr.W1);
}

// A group whose rows would pass the table's u32 first index (max_rows: 2^32 - 1 reads of one length
// or class in one call) is re-keyed: its entries become its rows 0..K-1 (extract, then merge back
// with first index = entry, the row map compacted to the entries' first reads), so one call counts
// any number of reads (the row map holds u64 global read indices).
int group_rekey(ss_ingest* g, Group& gr) {
    hipStream_t s = g->stream;
    const uint64_t cap = gr.cap + 1;
    const uint32_t W = gr.W1;
    int rc = g->scan.ensure(kScanBlocks + 2 + 2 * (uint64_t)kLenBins + 8);
    if (rc || (rc = gr.fps.ensure(cap)) || (rc = gr.words.ensure(cap * W)) || (rc = gr.counts.ensure(cap)) ||
        (rc = gr.first.ensure(cap)) || (rc = gr.lens.ensure(cap)))
        return rc;
    uint64_t* d_cnt = g->scan.p + kScanBlocks + 2;
    rc = ss_counter_extract_words(gr.table, 1, gr.fps.p, gr.lens.p, gr.words.p, gr.counts.p, gr.first.p, cap, d_cnt, s);
    if (!rc) rc = ss_check(hipMemcpyAsync(g->h_bad, d_cnt, 8, hipMemcpyDeviceToHost, s), "ingest rekey count");
    if (!rc) rc = ss_check(hipStreamSynchronize(s), "ingest rekey");
    if (rc) return rc;
    const uint64_t m = g->h_bad[0];
    DBuf<uint64_t> nmap, nacc;
    if ((rc = nmap.ensure(std::max<uint64_t>(m, gr.rows)))) return rc;
    if (gr.acc_rows) {      // spilled counts follow their entries to the new rows
        if ((rc = nacc.ensure(std::max<uint64_t>(m, 1)))) return rc;
        if (m)
            hipLaunchKernelGGL(k_rekey_acc, dim3(grid_of(m, 256)), dim3(256), 0, s, gr.first.p, m, gr.acc.p,
                               gr.acc_rows, nacc.p);
    }
    if (m)
        hipLaunchKernelGGL(k_rekey, dim3(grid_of(m, 256)), dim3(256), 0, s, gr.first.p, m, gr.rowmap.p, nmap.p, gr.fps.p);
    if ((rc = ss_counter_reset(gr.table, s)) || (rc = table_kind(gr, gr.table))) return rc;
    rc = W == 1 ? ss_counter_merge(gr.table, gr.words.p, gr.lens.p, gr.counts.p, gr.fps.p, m, s)
                : ss_counter_merge_words(gr.table, gr.words.p, gr.counts.p, gr.fps.p, m, s);
    if (!rc) rc = ss_check(hipStreamSynchronize(s), "ingest rekey merge");
    if (rc) return rc;
    gr.rowmap.release();
    gr.rowmap = nmap;
    nmap.p = nullptr;
    nmap.cap = 0;
    if (gr.acc_rows) {
        gr.acc.release();
        gr.acc = nacc;
        nacc.p = nullptr;
        nacc.cap = 0;
        gr.acc_rows = m;
    }
    gr.rows = m;
    return SS_OK;
}

// every table's counts into its group's u64 row counts (ss_counter_spill_counts), so the next
// 2^32 - 1 reads cannot wrap a slot's u32 count
int spill_counts(ss_ingest* g) {
    hipStream_t s = g->stream;
    for (auto& kv : g->groups) {
        Group& gr = kv.second;
        if (!gr.table || !gr.rows) continue;
        int rc = gr.acc.ensure_keep(gr.rows, gr.acc_rows, s);
        if (!rc && gr.rows > gr.acc_rows)
            rc = ss_check(hipMemsetAsync(gr.acc.p + gr.acc_rows, 0, (gr.rows - gr.acc_rows) * 8, s), "ingest spill rows");
        if (!rc) rc = ss_counter_spill_counts(gr.table, gr.acc.p, s);
        if (rc) return rc;
        gr.acc_rows = gr.rows;
    }
    g->since_spill = 0;
    return SS_OK;
}

// make room for m more rows in group gr (grow by extract + merge).  need: an upper bound of the
// table's keys after them -- the rows so far (exact), or a class's distinct-key estimate
int group_room(ss_ingest* g, Group& gr, uint64_t m, uint64_t need) {
    if (gr.table && gr.rows + m > g->max_rows) {
        if (m > g->max_rows / 2) return ss_fail(SS_EARG, "ingest: a chunk's rows of one length exceed the row bound");
        const int rc = group_rekey(g, gr);
        if (rc) return rc;
        need = std::min(need, gr.rows + m);
        if (gr.rows + m > g->max_rows) return ss_fail(SS_EFULL, "ingest: a length's distinct keys exceed 2^32 - 1");
    }
    if (gr.table && need <= gr.cap / 2) return SS_OK;
    if (!gr.table) {
        // (a length's table is sized by this chunk's rows: sized for the whole file's rows, est_scale,
        // the tables of the later chunks' small inserts were 2-3x slower -- more regions per insert)
        const double scale = gr.L || need < m ? 1.0 : g->est_scale;
        gr.cap = std::min<uint64_t>(1ull << 32, pow2_at_least((uint64_t)(2.0 * (double)need * scale) + 2));
        int rc = table_get(g, gr.cap, gr.W1, m, &gr.table);
        return rc ? rc : table_kind(gr, gr.table);
    }
    uint64_t size = 0;
    int rc = table_size(g, gr.table, &size);
    if (rc) return rc;
    need = std::min(need, size + m);
    if (need <= gr.cap / 2) return SS_OK;
    const uint64_t ncap = pow2_at_least(2 * need);
    ss_counter* nt = nullptr;
    const bool defer = g->defer_prep;     // (merged into at once: its reset goes out now)
    g->defer_prep = false;
    rc = table_get(g, ncap, gr.W1, m, &nt);
    g->defer_prep = defer;
    if (rc != SS_OK) return rc;
    if ((rc = table_kind(gr, nt)) != SS_OK) return rc;
    const uint64_t cap = gr.cap + 1;
    const uint32_t W = gr.W1;
    DBuf<uint64_t> k, c, f, pc, wd;
    DBuf<uint32_t> l;
    if ((rc = k.ensure(cap)) || (rc = c.ensure(cap)) || (rc = f.ensure(cap)) || (rc = l.ensure(cap)) ||
        (rc = pc.ensure(1)) || (W > 1 && (rc = wd.ensure(cap * W))))
        return rc;
    if (W == 1) {
        rc = ss_counter_extract(gr.table, 1, k.p, l.p, c.p, f.p, cap, pc.p, g->stream);
        if (!rc) rc = ss_counter_merge(nt, k.p, l.p, c.p, f.p, size, g->stream);
    } else {     // packed-word keys: the entries' words travel (equality is decided on them)
        rc = ss_counter_extract_words(gr.table, 1, k.p, l.p, wd.p, c.p, f.p, cap, pc.p, g->stream);
        if (!rc) rc = ss_counter_merge_words(nt, wd.p, c.p, f.p, size, g->stream);
    }
    if (!rc) rc = ss_check(hipStreamSynchronize(g->stream), "ingest grow");
    k.release(), c.release(), f.release(), l.release(), pc.release(), wd.release();
    if (rc) return rc;
    table_put(g, gr.table);
    gr.table = nt;
    gr.cap = ss_counter_capacity(nt);
    return SS_OK;
}

// the deferred fold of a read-order chunk's scratch into its class tables (see ss_ingest::pend); one
// sync for the tables' overflow words (sized from the sketch as for an immediate fold)
int flush_pending(ss_ingest* g) {
    if (!g->pend) return SS_OK;
    g->pend = false;
    hipStream_t s = g->stream;
    int rc = g->ovf.ensure(6);
    if (!rc) rc = ss_check(hipMemsetAsync(g->ovf.p, 0, 6 * 8, s), "ingest overflow reset");
    if (!rc) rc = ss_classes_flat_fold(g->fpt, g->pend_S, g->pend_fc, g->pend_base, g->zero32.p, s);
    for (uint32_t W = 2; W < 6 && !rc; ++W)
        if (g->pend_fc[W].table) rc = ss_counter_overflow(g->pend_fc[W].table, g->ovf.p + W, s);
    if (!rc) rc = ss_check(hipMemcpyAsync(g->h_bad, g->ovf.p, 6 * 8, hipMemcpyDeviceToHost, s), "ingest overflow copy");
    if (!rc) rc = ss_check(hipStreamSynchronize(s), "ingest deferred fold");
    if (rc) return rc;
    for (uint32_t W = 2; W < 6; ++W)
        if (g->h_bad[W]) {
            g->failed = true;
            return ss_fail(SS_EFULL, "ingest: a length class's table ran full (its distinct-key estimate was low); "
                                     "count again with ss_ingest_set_exact");
        }
    return SS_OK;
}

// compact results carry u64 counts only when a count can reach 2^32: no count exceeds the reads
// counted (format 2 forces u64: a test hook)
bool results_wide(const ss_ingest* g) {
    return g->compact == 2 || (g->compact && g->nreads > 0xFFFFFFFFull);
}

// wait for a queued speculative finish (its buffers are about to be reused) and drop it
void spec_wait(ss_ingest* g) {
    if (g->spec_inflight) (void)hipEventSynchronize(g->ev_spec);
    g->spec_inflight = false;
    g->spec_valid = false;
}

// the speculative finish of a first read-order chunk (see ss_ingest::spec_stream); need[W]: the class's
// distinct-key estimate (bounds the result buffer; a larger result invalidates the speculation)
int spec_launch(ss_ingest* g, const uint64_t* need, uint64_t N) {
    hipStream_t ss = g->spec_stream;
    int rc = ss_check(hipStreamWaitEvent(ss, g->ev_reps, 0), "spec wait");
    if (rc) return rc;
    std::vector<Group*> cls;
    ss_flat_out fo[6] = {};
    uint64_t k_ub = 1, nw_ub = 0;
    if ((rc = g->spec_dev.ensure(13))) return rc;
    for (auto& kv : g->groups) {
        Group& gr = kv.second;
        if (!gr.table || gr.L || gr.W1 - 1 >= 6 || g->pend_fc[gr.W1 - 1].table != gr.table) continue;
        const uint32_t W = gr.W1 - 1;
        const uint64_t cap = gr.cap + 1;
        if ((rc = gr.words.ensure(cap * gr.W1)) || (rc = gr.counts.ensure(cap)) || (rc = gr.first.ensure(cap)))
            return rc;
        fo[W] = {gr.words.p, gr.counts.p, gr.first.p, g->spec_dev.p + W, g->spec_dev.p + 8, cap};
        // (sizing mode 5, a test hook: the result bound taken as if the estimate were 0, so a chunk of
        // more than ~1024 distinct keys per class passes it and the finish runs the ordinary way)
        const uint64_t kb = std::min<uint64_t>(cap, (g->sizing == 5 ? 0 : need[W]) + 1024);
        k_ub += kb;
        nw_ub += kb * W;
        cls.push_back(&gr);
    }
    if (cls.empty() || cls.size() > 8) return SS_OK;
    const uint64_t NB = (N + 63) / 64;
    const uint64_t lb = (k_ub * 4 + 15) & ~15ull, out_bytes = lb + k_ub * 8 + nw_ub * 8 + 16;
    if ((rc = g->slot.ensure(NB)) || (rc = g->ordered.ensure(k_ub + 1)) || (rc = g->woff.ensure(std::max(k_ub, NB) + 1)) ||
        (rc = g->gdesc.ensure(8)) || (rc = g->scan.ensure(kScanBlocks + 2 + 3 * (uint64_t)kLenBins + 8)) ||
        (rc = g->out_host.ensure(out_bytes)))
        return rc;
    uint64_t* sd = g->spec_dev.p;
    unsigned long long* bits = (unsigned long long*)g->slot.p;
    if ((rc = ss_check(hipMemsetAsync(sd, 0, 13 * 8, ss), "spec reset")) ||
        (rc = ss_check(hipMemsetAsync(g->slot.p, 0, NB * 8, ss), "spec read map reset")))
        return rc;
    if ((rc = ss_classes_flat_extract(g->fpt, g->pend_S, g->pend_fc, g->pend_base, fo, g->zero32.p, ss))) return rc;
    for (size_t q = 0; q < cls.size(); ++q) {
        Group& gr = *cls[q];
        const uint64_t cap = gr.cap + 1;
        hipLaunchKernelGGL(k_mark, dim3(grid_of(cap, 256)), dim3(256), 0, ss, gr.first.p, cap, gr.rowmap.p, kNoSlot, bits,
                           (const uint64_t*)(sd + gr.W1 - 1));
        g->h_gdesc[q] = {gr.words.p, gr.counts.p, gr.W1, gr.L};
    }
    const uint64_t empty_at = g->empty_count ? g->empty_first : kNoSlot;
    if (g->empty_count)
        hipLaunchKernelGGL(k_mark, dim3(1), dim3(256), 0, ss, (const uint64_t*)nullptr, (uint64_t)0,
                           (const uint64_t*)nullptr, empty_at, bits, (const uint64_t*)nullptr);
    hipLaunchKernelGGL(k_spec_total, dim3(1), dim3(64), 0, ss, sd, g->empty_count ? 1ull : 0ull, (const uint64_t*)nullptr);
    if ((rc = ss_check(hipMemcpyAsync(g->gdesc.p, g->h_gdesc, cls.size() * sizeof(GDesc), hipMemcpyHostToDevice, ss),
                       "spec desc")))
        return rc;
    hipLaunchKernelGGL((k_scan_count<0>), dim3(kScanBlocks), dim3(256), 0, ss, g->slot.p, NB, (const GDesc*)g->gdesc.p,
                       g->scan.p, (const uint64_t*)nullptr);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(256), 0, ss, g->scan.p);
    hipLaunchKernelGGL((k_scan_apply<0>), dim3(kScanBlocks), dim3(256), 0, ss, g->slot.p, NB, (const GDesc*)g->gdesc.p,
                       g->scan.p, g->woff.p, (const uint64_t*)nullptr);
    for (size_t q = 0; q < cls.size(); ++q) {
        Group& gr = *cls[q];
        const uint64_t cap = gr.cap + 1;
        hipLaunchKernelGGL(k_rank, dim3(grid_of(cap, 256)), dim3(256), 0, ss, gr.first.p, cap, gr.rowmap.p, (uint32_t)q,
                           kNoSlot, bits, g->woff.p, g->ordered.p, (const uint64_t*)(sd + gr.W1 - 1), k_ub);
    }
    if (g->empty_count)
        hipLaunchKernelGGL(k_rank, dim3(1), dim3(256), 0, ss, (const uint64_t*)nullptr, (uint64_t)0,
                           (const uint64_t*)nullptr, 0u, empty_at, bits, g->woff.p, g->ordered.p, (const uint64_t*)nullptr,
                           k_ub);
    // word offsets of the ordered entries (K on the device; past the bound the gather refuses)
    hipLaunchKernelGGL((k_scan_count<1>), dim3(kScanBlocks), dim3(256), 0, ss, g->ordered.p, k_ub, (const GDesc*)g->gdesc.p,
                       g->scan.p, (const uint64_t*)(sd + 6));
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(256), 0, ss, g->scan.p);
    hipLaunchKernelGGL((k_scan_apply<1>), dim3(kScanBlocks), dim3(256), 0, ss, g->ordered.p, k_ub, (const GDesc*)g->gdesc.p,
                       g->scan.p, g->woff.p, (const uint64_t*)(sd + 6));
    g->wide = results_wide(g);
    OutLayout ol{g->out_host.p, g->out_host.cap, sd + 6, g->scan.p + kScanBlocks, 0, (unsigned long long*)(sd + 7),
                 g->compact, g->wide ? 1 : 0};
    // up to a few million entries the rows take about as long as the verify beside them: few waves,
    // and the verify keeps the chip; past that the gather is the call's bound and takes the full grid
    if (k_ub <= kGatherWavesMax)
        hipLaunchKernelGGL(k_gather_host_waves, dim3(kGatherBlocks), dim3(256), 0, ss, g->ordered.p, k_ub,
                           (const GDesc*)g->gdesc.p, g->woff.p, g->empty_count, ol);
    else
        hipLaunchKernelGGL(k_gather_host, dim3((unsigned)((k_ub + 255) / 256)), dim3(256), 0, ss, g->ordered.p, k_ub,
                           (const GDesc*)g->gdesc.p, g->woff.p, g->empty_count, ol);
    hipLaunchKernelGGL(k_spec_total, dim3(1), dim3(64), 0, ss, sd, g->empty_count ? 1ull : 0ull,
                       (const uint64_t*)(g->scan.p + kScanBlocks), g->empty_count);
    rc = ss_check(hipMemcpyAsync(g->h_spec, sd + 9, 4 * 8, hipMemcpyDeviceToHost, ss), "spec sizes");
    if (!rc) rc = ss_check(hipEventRecord(g->ev_spec, ss), "spec event");
    if (!rc) rc = ss_check(hipGetLastError(), "spec finish");
    if (!rc) g->spec_inflight = true;
    return rc;
}

// The chunk's reads: d_buf[offs[i], + lens[i]) for i < n (global index base + i).  dense: reads are
// back to back (offs = exclusive prefix of lens) and all have length dense_L (no split, no gather).
// d_buf / d_offs / d_lens: the chunk on the device (the engine's own buffers, or the caller's for
// ss_ingest_add_device); h_chunk / h_offs: the same bytes on the host when there (the first rejected
// read's bytes are then taken from there, else copied back).
int process_chunk(ss_ingest* g, const uint8_t* d_buf, const uint64_t* d_offs, const uint32_t* d_lens, uint64_t nbytes,
                  uint64_t n, uint32_t dense_L, const std::vector<uint64_t>* h_offs, const uint8_t* h_chunk,
                  bool spec_ok = false) {
    spec_wait(g);                    // (its buffers are reused below; the results change)
    if (g->failed) return ss_fail(SS_EFULL, "ingest: an earlier add ran a table full; reset and count again");
    if (n == 0) return SS_OK;
    if (n >= (1ull << 32)) return ss_fail(SS_EARG, "ingest: a chunk holds < 2^32 reads");
    int frc = flush_pending(g);      // the previous chunk's deferred fold (its scratch is reused below)
    if (frc) return frc;
    if (g->since_spill + n > g->spill_limit) {
        const int src = spill_counts(g);
        if (src) return src;
    }
    g->since_spill += n;
    // global read indices are u64 (row maps); a table's first index is a row of its group, u32: a
    // group about to pass kMaxRows rows is re-keyed first (group_room)
    hipStream_t s = g->stream;
    const uint64_t base = g->nreads;
    int rc = SS_OK;
    struct Job {
        uint32_t bin;            // len_bin: a length 1..32 or a length class
        uint64_t m, start, first;
    };
    std::vector<Job> jobs;
    // first-bad words: one per length bin (a length's insert, a class's pass), the class encode's at
    // kLenBins -- all reset here, before anything that may report
    if ((rc = g->first_bad.ensure(kLenBins + 1))) return rc;
    if ((rc = ss_check(hipMemsetAsync(g->first_bad.p, 0xFF, (kLenBins + 1) * 8, s), "ingest first_bad reset"))) return rc;
    uint32_t spec_S = 0;         // the row encode queued behind the split at this stride (gated on the device)
    if (dense_L) {
        if (dense_L > SS_MAX_NT) return ss_fail(SS_EARG, "ingest: dense length > 1024");
        jobs.push_back({dense_L < 32 ? kShortBin : len_bin(dense_L), n, 0, 0});
    } else {
        if ((rc = g->order.ensure(n)) || (rc = g->blkhist.ensure((uint64_t)kLenBins * kSplitBlocks)) ||
            (rc = g->blkfirst.ensure((uint64_t)kLenBins * kSplitBlocks)) || (rc = g->split_out.ensure(3 * kLenBins + 1)))
            return rc;
        // (the side stream's speculative encode below starts behind everything queued so far, not behind the split)
        const bool spec_enc = g->flat_hint != 0 && g->flat_streak >= 2;
        if (spec_enc) rc = ss_check(hipEventRecord(g->ev_fork, s), "ingest fork");
        hipLaunchKernelGGL(k_len_count, dim3(kSplitBlocks), dim3(64), 0, s, d_lens, n, g->blkhist.p, g->blkfirst.p);
        hipLaunchKernelGGL(k_len_binscan, dim3(kLenBins), dim3(1024), 0, s, kSplitBlocks, g->blkhist.p, g->blkfirst.p,
                           g->split_out.p);
        hipLaunchKernelGGL(k_len_binstart, dim3(1), dim3(1024), 0, s, g->split_out.p);
        if (!rc) rc = ss_check(hipMemcpyAsync(g->h_split, g->split_out.p, (3 * kLenBins + 1) * 8, hipMemcpyDeviceToHost, s),
                               "ingest split copy");
        if (!rc) rc = ss_check(hipEventRecord(g->ev_split, s), "ingest split event");
        // The previous chunks took the read-order path: its stride's row encode goes out now.  After two
        // or more chunks at one stride it runs on a side stream beside the split, so the GPU encodes
        // while the split runs and the host waits for it.  When the split then names another path the
        // rows and fingerprints are rewritten by that path (the wasted encode is the price of a wrong
        // guess, hence the streak); the sketch registers and the class first-bad word it touched are
        // harmless: it sketches only class reads of < S words, by the fingerprint every class path
        // sketches them by (a max register: a subset of the same updates), and reports only rejected
        // class reads, which every path reports.  After one chunk it is queued behind the split on the
        // stream, gated on the device by the split's own stride (a wrong guess returns at once).
        if (!rc && g->flat_hint && !spec_enc) {
            const uint32_t S = g->flat_hint;
            if (!(rc = g->cls_words.ensure(n * S + 2)) && !(rc = g->cls_fps.ensure(n))) {
                rc = ss_encode_rows_impl(d_buf, d_offs, d_lens, n, S, g->cls_words.p, g->cls_fps.p, g->hll.p,
                                         g->first_bad.p + kLenBins, s, g->split_out.p + 3 * kLenBins);
                if (!rc) spec_S = S;
            }
        }
        bool joined = false;
        if (!rc && spec_enc) {
            const uint32_t S = g->flat_hint;
            if (!(rc = g->cls_words.ensure(n * S + 2)) && !(rc = g->cls_fps.ensure(n)) &&
                !(rc = ss_check(hipStreamWaitEvent(g->side[0], g->ev_fork, 0), "ingest fork wait"))) {
                rc = ss_encode_rows_impl(d_buf, d_offs, d_lens, n, S, g->cls_words.p, g->cls_fps.p, g->hll.p,
                                         g->first_bad.p + kLenBins, g->side[0], nullptr);
                if (!rc) rc = ss_check(hipEventRecord(g->ev_join[0], g->side[0]), "ingest spec encode join");
                // everything queued on the stream from here on runs behind the encode
                if (!rc) rc = ss_check(hipStreamWaitEvent(s, g->ev_join[0], 0), "ingest spec encode wait");
                joined = !rc;
                if (!rc) spec_S = S;
            }
        }
        if (!rc) rc = ss_check(hipEventSynchronize(g->ev_split), "ingest split");
        if (rc) {
            if (spec_enc && !joined) (void)hipStreamSynchronize(g->side[0]);   // nothing left writing the buffers
            return rc;
        }
        const uint64_t* hh = g->h_split;
        if (spec_S && hh[3 * kLenBins] != spec_S) spec_S = 0;    // the queued encode did nothing (or is rewritten)
        Job shortj{kShortBin, 0, 0, kNoSlot};     // lengths 1..31: contiguous bins of the split, one job
        for (uint32_t b = 0; b < kLenBins; ++b) {
            const uint64_t m = hh[b];
            if (!m) continue;
            const uint64_t f = hh[kLenBins + b];
            if (b >= 1 && b <= 31) {
                if (shortj.m && shortj.start + shortj.m != hh[2 * kLenBins + b])
                    return ss_fail(SS_EARG, "ingest: the split's short-length bins are not contiguous");
                if (!shortj.m) shortj.start = hh[2 * kLenBins + b];
                shortj.m += m;
                shortj.first = std::min(shortj.first, f);
                continue;      // (pushed after the loop, ahead of the others)
            }
            if (b == 0) {
                g->empty_count += m;
                g->empty_first = std::min(g->empty_first, base + f);
            } else if (b == kTooLongBin) {
                if (base + f < g->bad_index) {
                    g->bad_index = base + f;
                    g->bad_kind = SS_ETOO_LONG;
                    g->bad_bytes.clear();
                }
            } else {
                jobs.push_back({b, m, hh[2 * kLenBins + b], f});
            }
        }
        if (shortj.m) jobs.insert(jobs.begin(), shortj);
    }
    const size_t nj = jobs.size();
    if ((rc = g->ovf.ensure(nj + 1))) return rc;
    if (nj && (rc = ss_check(hipMemsetAsync(g->ovf.p, 0, (nj + 1) * 8, s), "ingest overflow reset"))) return rc;
    auto live = [&](const Job& jb) { return base + jb.first <= g->bad_index; };   // may still hold the first error
    // ---- the length classes: rows packed (W words + the length) and their distinct keys sketched ----
    uint64_t woff[33] = {0}, fpoff[33] = {0}, cls_words = 0, cls_rows = 0;
    uint32_t w1max = 0, wlo = 33, whi = 0;
    for (const Job& jb : jobs) {
        if (jb.bin <= 32) continue;
        const uint32_t W = jb.bin - kClassBin0;
        woff[W] = cls_words;
        fpoff[W] = cls_rows;
        cls_words += jb.m * (W + 1);
        cls_rows += jb.m;
        w1max = std::max(w1max, W + 1);
        wlo = std::min(wlo, W);
        whi = std::max(whi, W);
    }
    uint64_t need_cls[33] = {0};
    const bool fused = !dense_L && w1max && w1max <= 16;   // fingerprints and row maps come with the rows
    // every read a class read of <= 5 words (or empty / too long): rows in read order at a stride of
    // w1max words (k_encode_rows), no class ranks and no row maps in the encode
    bool flat = fused && w1max <= 6;
    for (const Job& jb : jobs) flat &= jb.bin > 32;
    if (spec_S && !(flat && w1max == spec_S))
        return ss_fail(SS_EARG, "ingest: the device's read-order stride disagrees with the host's split");
    if (!dense_L) {
        g->flat_streak = flat ? (w1max == g->flat_hint ? g->flat_streak + 1 : 1u) : 0u;
        g->flat_hint = flat ? w1max : 0u;
    }
    // the stable split into d_order: for the lengths 1..32 (row gathers) and the per-class passes; the
    // fused class encode ranks its rows itself from k_len_binscan's per-block offsets
    bool need_order = !dense_L && (!fused && w1max);
    for (const Job& jb : jobs) need_order |= !dense_L && jb.bin <= 32;
    if (need_order)
        hipLaunchKernelGGL(k_len_scatter, dim3(kSplitBlocks), dim3(64), 0, s, d_lens, n, g->blkhist.p,
                           (const uint64_t*)g->split_out.p, g->order.p);
    uint64_t* rmap[33] = {nullptr};
    if (fused) {
        // every class group's rows fit its table's u32 first index (re-keyed first otherwise) and its
        // row map has room for the chunk's rows: the encode writes their read indices there
        for (const Job& jb : jobs) {
            if (jb.bin <= 32) continue;
            Group& gr = g->groups[jb.bin];
            gr.L = 0;
            gr.W1 = jb.bin - kClassBin0 + 1;
            if (gr.table && gr.rows + jb.m > g->max_rows) {
                if (jb.m > g->max_rows / 2) return ss_fail(SS_EARG, "ingest: a chunk's rows of one length exceed the row bound");
                if ((rc = group_rekey(g, gr))) return rc;
            }
            if ((rc = gr.rowmap.ensure_keep(gr.rows + jb.m, gr.rows, s))) return rc;
            rmap[gr.W1 - 1] = gr.rowmap.p + gr.rows;
        }
    }
    if (w1max) {
        if ((rc = g->cls_words.ensure(cls_words))) return rc;
        if (fused && (rc = g->cls_fps.ensure(flat ? n : cls_rows))) return rc;
        if (flat) {
            // (+2: k_flat_verify's quads load a row's last piece as 16 B, one word past an odd stride)
            if ((rc = g->cls_words.ensure(n * w1max + 2))) return rc;
            if (!spec_S)      // (else queued behind the split)
                rc = ss_encode_rows_impl(d_buf, d_offs, d_lens, n, w1max, g->cls_words.p, g->cls_fps.p, g->hll.p,
                                         g->first_bad.p + kLenBins, s);
        } else if (fused) {                 // one read-order pass, the registers updated in it
            rc = ss_encode_classes_impl(d_buf, d_offs, d_lens, n, g->blkhist.p, kSplitBlocks, woff, fpoff, rmap, base,
                                        kClassBin0, w1max, g->cls_words.p, g->cls_fps.p, g->hll.p, g->first_bad.p + kLenBins, s);
        } else {                            // a class per pass (longer reads, or a dense chunk)
            for (size_t j = 0; j < nj && !rc; ++j) {
                const Job& jb = jobs[j];
                if (jb.bin <= 32) continue;
                const uint32_t W = jb.bin - kClassBin0;
                const uint64_t* sel = dense_L ? nullptr : g->order.p + jb.start;
                rc = ss_encode_class_impl(d_buf, d_offs, d_lens, sel, dense_L, jb.m, W, g->cls_words.p + woff[W],
                                          g->first_bad.p + jb.bin, s);
                if (!rc) rc = ss_hll_rows_impl(g->cls_words.p + woff[W], jb.m, W + 1, g->hll.p + ((uint64_t)W << kHllLog), s);
            }
        }
        // the registers come back (one sync): each class table is sized by its distinct keys so far
        // (the sketch covers every chunk of the call), not by its rows
        const uint64_t r0 = (uint64_t)wlo << kHllLog, nr = (uint64_t)(whi - wlo + 1) << kHllLog;
        if (!rc) rc = ss_check(hipMemcpyAsync(g->h_hll + r0, g->hll.p + r0, nr * 4, hipMemcpyDeviceToHost, s), "ingest sketch copy");
        if (!rc) rc = ss_check(hipStreamSynchronize(s), "ingest sketch");
        if (rc) return rc;
        for (const Job& jb : jobs) {
            if (jb.bin <= 32) continue;
            const uint32_t W = jb.bin - kClassBin0;
            const double e = hll_estimate(g->h_hll + ((uint64_t)W << kHllLog));
            need_cls[W] = g->sizing == 1 ? ~0ull                                   // the rows bound
                        : g->sizing == 2 ? (uint64_t)(e / 64.0) + 64                   // test: undersized
                                         : (uint64_t)(1.2 * e) + 256;                  // ~9 sigma above the estimate
        }
    }
    std::vector<size_t> cls_jobs;
    struct FixJob {
        size_t j;
        uint64_t off, stride, row0;   // its rows' byte offset in g->rows and stride, its first table row
    };
    std::vector<FixJob> fix_jobs;
    uint64_t rows_bytes = 0;
    // new groups' pooled tables: their resets queued (table_get) and set in one dispatch below, before
    // the first insert; whatever is still queued goes out when this function returns
    g->defer_prep = true;
    struct PrepScope {
        ss_ingest* g;
        ~PrepScope() {
            g->defer_prep = false;
            if (!g->prep_p.empty()) (void)flush_prep(g);
        }
    } prep_scope{g};
    for (size_t j = 0; j < nj; ++j) {
        const Job& jb = jobs[j];
        const bool cls = jb.bin > 32;
        // (the fused classes are counted together: all of them, the call raises anyway when one lies
        // past the first rejected read)
        if (!live(jb) && !(cls && fused)) continue;
        Group& gr = g->groups[jb.bin];
        gr.L = cls ? 0u : jb.bin == kShortBin ? kShortL : jb.bin;
        gr.W1 = cls ? jb.bin - kClassBin0 + 1 : 1u;
        const uint64_t need = std::min<uint64_t>(gr.rows + jb.m, cls ? need_cls[gr.W1 - 1] : ~0ull);
        if ((rc = group_room(g, gr, jb.m, need))) return rc;
        // (a multi-chunk FASTQ: the first row map holds the whole file's estimated rows, not a doubling per chunk)
        const uint64_t rm = gr.rowmap.cap || g->est_scale <= 1.0 ? gr.rows + jb.m : (uint64_t)((double)(gr.rows + jb.m) * g->est_scale * 1.1);
        if ((rc = gr.rowmap.ensure_keep(std::max(rm, gr.rows + jb.m), gr.rows, s))) return rc;
        const uint64_t* sel = dense_L ? nullptr : g->order.p + jb.start;
        if (cls) {
            cls_jobs.push_back(j);     // inserted below, on the class streams
            continue;
        }
        // length 32: its rows gathered at a 16-B stride into its own run of g->rows; the short group:
        // its keys there (8 B per read); inserted below
        const bool shortg = jb.bin == kShortBin;
        const uint64_t stride = shortg ? 8 : dense_L ? dense_L : (jb.bin + 15) / 16 * 16;
        fix_jobs.push_back({j, rows_bytes, stride, gr.rows});
        if (shortg || !dense_L) rows_bytes += (jb.m * stride + 255) & ~255ull;     // (runs 16-B aligned)
        // (+1/4: the next chunk's slightly larger share of this length reuses the workspace)
        if (jb.m >= (1u << 16) && jb.m < (1ull << 30)) (void)ss_counter_reserve(gr.table, jb.m + jb.m / 4);
        gr.rows += jb.m;
    }
    // The lengths' inserts: every table is sized, its row map grown and its workspace reserved above
    // (host work, syncs), so the gathers, inserts and row maps of up to kSide + 1 lengths now run on
    // as many streams at once -- a small-RNA chunk has ~15 lengths of a few 100k reads each, whose
    // short partition kernels left the GPU mostly idle one length after another.
    if (!fix_jobs.empty()) {
        if (rows_bytes && (rc = g->rows.ensure(rows_bytes))) return rc;
        if ((rc = flush_prep(g))) return rc;
        int used = 0;
        if (fix_jobs.size() > 1) rc = ss_check(hipEventRecord(g->ev_fork, s), "ingest fork");
        for (size_t q = 0; q < fix_jobs.size() && !rc; ++q) {
            const FixJob& fj = fix_jobs[q];
            const Job& jb = jobs[fj.j];
            Group& gr = g->groups[jb.bin];
            const int k = (int)(q % (ss_ingest::kSide + 1));
            hipStream_t cs = s;
            if (k > 0) {
                cs = g->side[k - 1];
                if (k > used) {
                    rc = ss_check(hipStreamWaitEvent(cs, g->ev_fork, 0), "ingest fork wait");
                    used = k;
                }
            }
            const uint64_t* sel = dense_L ? nullptr : g->order.p + jb.start;
            const uint8_t* src = d_buf;
            if (jb.bin == kShortBin) {      // the short group: keys with their length markers, one insert
                uint64_t* keys = (uint64_t*)(g->rows.p + fj.off);
                if (!rc) rc = ss_short_keys_impl(d_buf, d_offs, d_lens, sel, jb.m, dense_L, keys, g->first_bad.p + jb.bin, cs);
                if (!rc) rc = ss_counter_insert_keys(gr.table, keys, jb.m, fj.row0, cs);
            } else {
                if (!rc && !dense_L) {
                    src = g->rows.p + fj.off;
                    rc = ss_gather_rows(d_buf, nbytes, d_offs, sel, jb.m, jb.bin, g->rows.p + fj.off, fj.stride, cs);
                }
                if (!rc) rc = ss_counter_insert_fixed(gr.table, src, jb.m, jb.bin, fj.stride, fj.row0, g->first_bad.p + jb.bin, cs);
            }
            if (!rc)
                hipLaunchKernelGGL(k_rowmap, dim3(grid_of(jb.m, 256)), dim3(256), 0, cs, sel, jb.m, base,
                                   gr.rowmap.p + fj.row0);
        }
        for (int k = 0; k < used; ++k) {     // join (also after an error: nothing may run on past the call)
            const int e = ss_check(hipEventRecord(g->ev_join[k], g->side[k]), "ingest join");
            const int w = e ? e : ss_check(hipStreamWaitEvent(s, g->ev_join[k], 0), "ingest join wait");
            if (!rc) rc = w;
        }
        if (rc) return rc;
    }
    g->defer_prep = false;
    std::vector<uint64_t> cls_base(nj, 0);     // each class job's first table row (the exact redo)
    bool pend_now = false;                     // this chunk's fold deferred (set below)
    if (!(!cls_jobs.empty() && fused) && (rc = flush_prep(g))) return rc;
    if (!cls_jobs.empty() && fused) {
        // the classes' rows counted by fingerprint in one scratch table, checked against their
        // fingerprints' first rows and folded into the class tables (ss_classes_verify_fold); a
        // fingerprint shared by two keys sends the classes to the exact path below, after the sync
        uint64_t need_all = flat ? 1 : 0;     // (the zero rows' entry)
        std::vector<ss_class_rows> cr;
        ss_flat_class fc[6] = {};
        for (size_t j : cls_jobs) {
            const Job& jb = jobs[j];
            Group& gr = g->groups[jb.bin];
            need_all += std::min<uint64_t>(jb.m, need_cls[gr.W1 - 1]);
            cr.push_back({gr.table, g->cls_words.p + woff[gr.W1 - 1], jb.m, gr.rows, gr.W1});
            if (flat) fc[gr.W1 - 1] = {gr.table, gr.rows, gr.rowmap.p + gr.rows};
        }
        // twice the estimate; past 2^24 slots 1.5 times: the per-slot passes (a 64-B representative per
        // slot, the extract) then cost more than a fuller table's longer probes (2^24-pool batch
        // 20.8 -> 19.4 ms; at 2^20 the fuller 2^21 table was 0.4 ms slower, libab_f2_lf15_u2{0,4}.log)
        uint64_t fwant = pow2_at_least(2 * need_all + 2);
        if (fwant > (1ull << 24)) fwant = pow2_at_least(need_all + need_all / 2 + 2);
        const uint64_t fcap = std::min<uint64_t>(1ull << 32, std::max<uint64_t>(1ull << 19, fwant));
        // grow-only with hysteresis: a stream whose per-chunk estimates cross a power of
        // two keeps its table; only a table 8x too large (its per-slot passes, reps and fold, scale
        // with the capacity) is replaced by a smaller one
        if (g->fpt && (ss_counter_capacity(g->fpt) < fcap || ss_counter_capacity(g->fpt) >= 8 * fcap)) {
            (void)hipStreamSynchronize(s);
            ss_counter_destroy(g->fpt);
            g->fpt = nullptr;
        }
        if (!g->fpt && (rc = ss_counter_create(fcap, &g->fpt))) return rc;
        {   // the scratch table's reset with the class tables' queued ones, one dispatch
            unsigned long long* p[3];
            unsigned long long v[3];
            if ((rc = ss_counter_reset_host(g->fpt, p, v))) return rc;
            g->prep_p.insert(g->prep_p.end(), p, p + 3);
            g->prep_v.insert(g->prep_v.end(), v, v + 3);
            if ((rc = flush_prep(g))) return rc;
        }
        if ((rc = g->cls_flag.ensure(1))) return rc;
        // (sizing modes 3 / 4, test hooks: the flag starts raised, as if two keys shared a fingerprint;
        // 4 keeps the deferred fold and the speculative finish, so the flag is found after they were queued)
        rc = ss_check(hipMemsetAsync(g->cls_flag.p, g->sizing == 3 || g->sizing == 4 ? 1 : 0, 4, s),
                      "ingest class flag reset");
        if (!rc && !flat) rc = ss_counter_insert_keys(g->fpt, g->cls_fps.p, cls_rows, 0, s);
        if (!rc && !flat) rc = ss_classes_verify_fold(g->fpt, g->cls_fps.p, cr.data(), (uint32_t)cr.size(), g->cls_flag.p, s);
        // the fold is deferred when every class of the chunk starts from an empty table (see pend)
        bool defer = flat && (g->sizing == 0 || g->sizing >= 4);
        for (uint32_t W = 2; W < 6; ++W) defer &= !fc[W].table || fc[W].base == 0;
        if (!rc && flat) rc = ss_counter_insert_keys(g->fpt, g->cls_fps.p, n, 0, s);
        if (!rc && flat && defer) {
            // a first chunk of an add_device / add_blob also queues the speculative finish beside the verify
            const bool spec = spec_ok && base == 0 && g->bad_index == kNoSlot;
            rc = ss_classes_flat_verify(g->fpt, g->cls_words.p, w1max, n, g->cls_fps.p, g->cls_flag.p, s,
                                        spec ? (void*)g->ev_reps : nullptr);
            if (!rc) {      // pending once the flag comes back clear (checked after the sync below)
                g->pend_S = w1max;
                g->pend_base = base;
                for (uint32_t W = 0; W < 6; ++W) g->pend_fc[W] = fc[W];
            }
            if (!rc && spec) rc = spec_launch(g, need_cls, base + n);
        } else if (!rc && flat) {
            rc = ss_classes_flat_verify_fold(g->fpt, g->cls_words.p, w1max, n, g->cls_fps.p, fc, base, g->cls_flag.p, s);
        }
        pend_now = !rc && flat && defer;
        if (!rc) rc = ss_counter_overflow(g->fpt, g->ovf.p + nj, s);
        for (size_t q = 0; q < cls_jobs.size() && !rc; ++q) {
            const size_t j = cls_jobs[q];
            const Job& jb = jobs[j];
            Group& gr = g->groups[jb.bin];
            cls_base[j] = gr.rows;
            rc = ss_counter_overflow(gr.table, g->ovf.p + j, s);
            gr.rows += jb.m;           // (their row map: written by the encode, or by the fold for new keys)
        }
        if (rc) return rc;
    } else if (!cls_jobs.empty()) {
        // every table of a class job is sized, reset and its row map grown on the main stream above
        int used = 0;
        if (cls_jobs.size() > 1) rc = ss_check(hipEventRecord(g->ev_fork, s), "ingest fork");
        for (size_t q = 0; q < cls_jobs.size() && !rc; ++q) {
            const size_t j = cls_jobs[q];
            const Job& jb = jobs[j];
            Group& gr = g->groups[jb.bin];
            const int k = (int)(q % (ss_ingest::kSide + 1));
            hipStream_t cs = s;
            if (k > 0) {
                cs = g->side[k - 1];
                if (k > used) {
                    rc = ss_check(hipStreamWaitEvent(cs, g->ev_fork, 0), "ingest fork wait");
                    used = k;
                }
            }
            if (!rc) rc = ss_counter_insert_words(gr.table, g->cls_words.p + woff[gr.W1 - 1], jb.m, gr.rows, cs);
            if (!rc) rc = ss_counter_overflow(gr.table, g->ovf.p + j, cs);
            if (rc) break;
            const uint64_t* sel = dense_L ? nullptr : g->order.p + jb.start;
            hipLaunchKernelGGL(k_rowmap, dim3(grid_of(jb.m, 256)), dim3(256), 0, cs, sel, jb.m, base,
                               gr.rowmap.p + gr.rows);
            gr.rows += jb.m;
        }
        for (int k = 0; k < used; ++k) {     // join (also after an error: nothing may run on past the call)
            const int e = ss_check(hipEventRecord(g->ev_join[k], g->side[k]), "ingest join");
            const int w = e ? e : ss_check(hipStreamWaitEvent(s, g->ev_join[k], 0), "ingest join wait");
            if (!rc) rc = w;
        }
        if (rc) return rc;
    }
    if (jobs.empty()) {
        g->nreads += n;
        return SS_OK;
    }
    // first-bad words, the class tables' overflow words (the scratch table's last) and the class
    // fingerprint flag back in one sync
    // (hb: the kLenBins + 1 first-bad words, then ho: the nj + 1 overflow words and the flag)
    uint64_t* hb = g->h_bad;
    uint64_t* ho = hb + kLenBins + 1;
    rc = ss_check(hipMemcpyAsync(hb, g->first_bad.p, (kLenBins + 1) * 8, hipMemcpyDeviceToHost, s), "ingest bad copy");
    if (!rc) rc = ss_check(hipMemcpyAsync(ho, g->ovf.p, (nj + 1) * 8, hipMemcpyDeviceToHost, s), "ingest overflow copy");
    if (!rc && fused && !cls_jobs.empty())
        rc = ss_check(hipMemcpyAsync(ho + nj + 1, g->cls_flag.p, 4, hipMemcpyDeviceToHost, s), "ingest flag copy");
    if (!rc) rc = ss_check(hipStreamSynchronize(s), "ingest chunk");
    if (rc) return rc;
    for (size_t j = 0; j <= nj; ++j) {
        if (!ho[j] || (j == nj && !(fused && !cls_jobs.empty()))) continue;
        g->failed = true;
        return ss_fail(SS_EFULL, "ingest: a length class's table ran full (its distinct-key estimate was low); "
                                     "count again with ss_ingest_set_exact");
    }
    g->pend = pend_now && !(uint32_t)ho[nj + 1];
    if (fused && !cls_jobs.empty() && (uint32_t)ho[nj + 1]) {
        spec_wait(g);                  // (it reads the class tables the exact path now fills)
        // two keys share a fingerprint: the class tables were left untouched, count them exactly
        if (flat) {     // class-ordered rows and their row maps first (the one-pass class encode)
            uint64_t* cmap[33] = {nullptr};
            for (size_t j : cls_jobs) {
                Group& gr = g->groups[jobs[j].bin];
                cmap[gr.W1 - 1] = gr.rowmap.p + cls_base[j];
            }
            rc = ss_encode_classes_impl(d_buf, d_offs, d_lens, n, g->blkhist.p, kSplitBlocks, woff, fpoff, cmap, base,
                                        kClassBin0, w1max, g->cls_words.p, g->cls_fps.p, g->hll.p, g->first_bad.p + kLenBins, s);
            if (rc) return rc;
        }
        for (size_t j : cls_jobs) {
            Group& gr = g->groups[jobs[j].bin];
            if ((rc = ss_counter_insert_words(gr.table, g->cls_words.p + woff[gr.W1 - 1], jobs[j].m, cls_base[j], s)) ||
                (rc = ss_counter_overflow(gr.table, g->ovf.p + j, s)))
                return rc;
        }
        rc = ss_check(hipMemcpyAsync(ho, g->ovf.p, nj * 8, hipMemcpyDeviceToHost, s), "ingest overflow copy");
        if (!rc) rc = ss_check(hipStreamSynchronize(s), "ingest exact classes");
        if (rc) return rc;
        for (size_t j = 0; j < nj; ++j)
            if (ho[j]) {
                g->failed = true;
                return ss_fail(SS_EFULL, "ingest: a length class's table ran full; count again with ss_ingest_set_exact");
            }
    }
    for (size_t j = 0; j <= nj; ++j) {
        const uint64_t fb = hb[j < nj ? jobs[j].bin : kLenBins];
        if (fb == kNoSlot || (j < nj && base + jobs[j].first > g->bad_index)) continue;
        // a length's insert reports its row (rows are in read order); the class encodes and the short
        // group's keys report the read
        const bool by_row = j < nj && !dense_L && jobs[j].bin <= 32 && jobs[j].bin != kShortBin;
        uint64_t idx = fb;
        if (by_row) {
            rc = ss_check(hipMemcpy(&idx, g->order.p + jobs[j].start + fb, 8, hipMemcpyDeviceToHost), "ingest bad row");
            if (rc) return rc;
        }
        if (base + idx < g->bad_index) {
            g->bad_index = base + idx;
            g->bad_kind = SS_EINVALID_BASE;
            uint32_t L = dense_L ? dense_L : (by_row ? jobs[j].bin : 0u);
            if (!L && (rc = ss_check(hipMemcpy(&L, d_lens + idx, 4, hipMemcpyDeviceToHost), "ingest bad len")))
                return rc;
            uint64_t off = dense_L ? idx * dense_L : 0;
            if (h_offs) {
                off = (*h_offs)[idx];
            } else if (!dense_L &&
                       (rc = ss_check(hipMemcpy(&off, d_offs + idx, 8, hipMemcpyDeviceToHost), "ingest bad off"))) {
                return rc;
            }
            if (h_chunk) {
                g->bad_bytes.assign((const char*)h_chunk + off, L);
            } else {
                g->bad_bytes.assign(L, '\0');
                rc = ss_check(hipMemcpy(&g->bad_bytes[0], d_buf + off, L, hipMemcpyDeviceToHost), "ingest bad read");
                if (rc) return rc;
            }
        }
    }
    // a too-long read's bytes (the message does not quote them) are not needed
    g->nreads += n;
    // the queued finish stands for this count unless a read was rejected (the finish is then not asked for)
    g->spec_valid = g->spec_inflight && g->pend && g->bad_index == kNoSlot;
    return SS_OK;
}

// Every table of the engine extracted (entries of group q into its fps / words / counts / first /
// lens buffers, gr.m entries), then their entry counts and overflow words back in one sync; the
// output word total gr.nw follows from the count (one word per entry for a length 1..32, W1 - 1 for
// a class table).
// flat: the pending scratch's classes are taken from the scratch (ss_classes_flat_extract) instead of
// their (empty) tables -- the finish; export and merge flush the scratch into the tables first.
int extract_groups(ss_ingest* g, std::vector<Group*>& placed, bool flat = false) {
    hipStream_t s = g->stream;
    int rc = g->scan.ensure(kScanBlocks + 2 + 3 * (uint64_t)kLenBins + 8);
    if (rc) return rc;
    uint64_t* d_cnt = g->scan.p + kScanBlocks + 2;
    rc = ss_check(hipMemsetAsync(d_cnt, 0, 3 * (uint64_t)kLenBins * 8, s), "ingest word totals reset");
    if (rc) return rc;
    ss_flat_out fo[6] = {};
    bool any_flat = false;
    for (auto& kv : g->groups) {
        Group& gr = kv.second;
        gr.m = 0;
        if (!gr.table) continue;      // a length of an earlier call
        const uint32_t W = gr.W1;
        const uint64_t cap = gr.cap + 1;
        const uint64_t q = placed.size();
        if ((rc = gr.fps.ensure(cap)) || (rc = gr.words.ensure(cap * W)) || (rc = gr.counts.ensure(cap)) ||
            (rc = gr.first.ensure(cap)) || (rc = gr.lens.ensure(cap)))
            return rc;
        if (flat && !gr.L && W - 1 < 6 && g->pend_fc[W - 1].table == gr.table) {
            // at most cap entries (the extract raises the overflow word past it, as the fold would)
            fo[W - 1] = {gr.words.p, gr.counts.p, gr.first.p, d_cnt + 3 * q, d_cnt + 3 * q + 1, cap};
            any_flat = true;
            placed.push_back(&gr);
            continue;
        }
        rc = ss_counter_extract_words(gr.table, 1, gr.fps.p, gr.lens.p, gr.words.p, gr.counts.p, gr.first.p, cap,
                                      d_cnt + 3 * q, s);
        if (!rc) rc = ss_counter_overflow(gr.table, d_cnt + 3 * q + 1, s);
        if (rc) return rc;
        if (gr.acc_rows)    // the counts spilled out of the table (u64) back onto its entries
            hipLaunchKernelGGL(k_add_acc, dim3(grid_of(cap, 256)), dim3(256), 0, s, gr.counts.p, gr.first.p,
                               (const uint64_t*)(d_cnt + 3 * q), gr.acc.p, gr.acc_rows);
        placed.push_back(&gr);
    }
    if (any_flat && (rc = ss_classes_flat_extract(g->fpt, g->pend_S, g->pend_fc, g->pend_base, fo, g->zero32.p, s)))
        return rc;
    if (!placed.empty()) {
        rc = ss_check(hipMemcpyAsync(g->h_bad, d_cnt, 3 * placed.size() * 8, hipMemcpyDeviceToHost, s), "ingest");
        if (!rc) rc = ss_check(hipStreamSynchronize(s), "ingest extract");
        if (rc) return rc;
    }
    for (size_t q = 0; q < placed.size(); ++q) {
        if (g->h_bad[3 * q + 1]) return ss_fail(SS_EFULL, "ingest: a length's counter table overflowed");
        placed[q]->m = g->h_bad[3 * q];
        // a class table keys W = W1 - 1 words for every entry (its lengths are 32(W-1)+1 .. 32W)
        placed[q]->nw = placed[q]->L ? placed[q]->m : placed[q]->m * (placed[q]->W1 - 1);
    }
    return SS_OK;
}

// ---- FASTQ file reading (parallel preads into the pinned staging buffer) ---------------------------
uint64_t pread_full(int fd, uint8_t* dst, uint64_t len, uint64_t pos) {
    uint64_t got = 0;
    while (got < len) {
        const ssize_t k = pread(fd, dst + got, len - got, (off_t)(pos + got));
        if (k <= 0) break;
        got += (uint64_t)k;
    }
    return got;
}

uint64_t read_parallel(int fd, uint8_t* dst, uint64_t len, uint64_t pos, unsigned threads) {
    if (len < (32ull << 20) || threads <= 1) return pread_full(fd, dst, len, pos);
    const uint64_t per = ((len + threads - 1) / threads + (1 << 20) - 1) & ~((uint64_t)(1 << 20) - 1);
    std::vector<std::thread> ts;
    std::vector<uint64_t> got(threads, 0);
    for (unsigned t = 0; t < threads; ++t) {
        const uint64_t a = (uint64_t)t * per;
        if (a >= len) break;
        const uint64_t b = std::min(len, a + per);
        ts.emplace_back([&, t, a, b] { got[t] = pread_full(fd, dst + a, b - a, pos + a); });
    }
    uint64_t sum = 0;
    for (size_t t = 0; t < ts.size(); ++t) {
        ts[t].join();
        sum += got[t];
    }
    return sum;
}

}  // namespace

extern "C" {

int ss_ingest_create(int device, ss_ingest** h_out) {
    if (!h_out) return ss_fail(SS_EARG, "null h_out");
    int rc = ss_check(hipSetDevice(device), "ingest hipSetDevice");
    if (rc) return rc;
    ss_ingest* g = new ss_ingest();
    g->device = device;
    rc = ss_check(hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking), "ingest stream");
    for (int k = 0; k < ss_ingest::kSide && !rc; ++k) {
        rc = ss_check(hipStreamCreateWithFlags(&g->side[k], hipStreamNonBlocking), "ingest side stream");
        if (!rc) rc = ss_check(hipEventCreateWithFlags(&g->ev_join[k], hipEventDisableTiming), "ingest event");
    }
    if (!rc) rc = ss_check(hipEventCreateWithFlags(&g->ev_fork, hipEventDisableTiming), "ingest event");
    if (!rc) rc = ss_check(hipHostMalloc((void**)&g->h_split, (3 * kLenBins + 1) * 8, hipHostMallocDefault), "ingest pinned");
    if (!rc) rc = ss_check(hipHostMalloc((void**)&g->h_bad, (3 * kLenBins + 8) * 8, hipHostMallocDefault), "ingest pinned");
    if (!rc) rc = ss_check(hipHostMalloc((void**)&g->h_hll, (33ull << kHllLog) * 4, hipHostMallocDefault), "ingest pinned");
    if (!rc) rc = g->hll.ensure(33ull << kHllLog);
    if (!rc) rc = ss_check(hipMemsetAsync(g->hll.p, 0, (33ull << kHllLog) * 4, g->stream), "ingest sketch reset");
    if (!rc) {       // the speculative finish runs beside the verify: it gets the CU slots first
        int lo = 0, hi = 0;
        (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
        rc = ss_check(hipStreamCreateWithPriority(&g->spec_stream, hipStreamNonBlocking, hi), "ingest spec stream");
    }
    if (!rc) rc = ss_check(hipEventCreateWithFlags(&g->ev_reps, hipEventDisableTiming), "ingest event");
    if (!rc) rc = ss_check(hipEventCreateWithFlags(&g->ev_split, hipEventDisableTiming), "ingest event");
    if (!rc) rc = ss_check(hipEventCreateWithFlags(&g->ev_spec, hipEventDisableTiming), "ingest event");
    if (!rc) rc = ss_check(hipHostMalloc((void**)&g->h_spec, 4 * 8, hipHostMallocDefault), "ingest pinned");
    if (!rc) rc = ss_check(hipHostMalloc((void**)&g->h_gdesc, 8 * sizeof(GDesc), hipHostMallocDefault), "ingest pinned");
    if (!rc) rc = g->zero32.ensure(1);
    if (!rc) rc = ss_check(hipMemsetAsync(g->zero32.p, 0, 4, g->stream), "ingest zero word");
    if (rc) {
        ss_ingest_destroy(g);
        return rc;
    }
    *h_out = g;
    return SS_OK;
}

int ss_ingest_reset(ss_ingest* g) {
    if (!g) return ss_fail(SS_EARG, "null ingest");
    (void)hipSetDevice(g->device);
    spec_wait(g);
    // tables go back to the pool; a length's row map and extraction buffers stay (grow-only) for the
    // next call (a fresh hipMalloc per call and length costs more than the counting)
    for (auto& kv : g->groups) {
        table_put(g, kv.second.table);
        kv.second.table = nullptr;
        kv.second.cap = 0;
        kv.second.rows = 0;
        kv.second.m = 0;
        kv.second.acc_rows = 0;
    }
    g->nreads = 0;
    g->since_spill = 0;
    g->empty_count = 0;
    g->empty_first = kNoSlot;
    g->bad_index = kNoSlot;
    g->bad_kind = 0;
    g->bad_bytes.clear();
    g->est_scale = 1.0;
    g->nkeys = g->nwords = 0;
    g->failed = false;
    g->exported = false;
    g->pend = false;
    if (!g->hll.p) return SS_OK;
    return ss_check(hipMemsetAsync(g->hll.p, 0, (33ull << kHllLog) * 4, g->stream), "ingest sketch reset");
}

int ss_ingest_set_count_limit(ss_ingest* g, uint64_t reads) {
    if (!g) return ss_fail(SS_EARG, "null ingest");
    if (reads < 1 || reads > 0xFFFFFFFEull) return ss_fail(SS_EARG, "count limit in 1 .. 2^32 - 2");
    g->spill_limit = reads;
    return SS_OK;
}

int ss_ingest_set_row_limit(ss_ingest* g, uint64_t rows) {
    if (!g) return ss_fail(SS_EARG, "null ingest");
    if (rows < 1024 || rows > 0xFFFFFFFFull) return ss_fail(SS_EARG, "row limit in 1024 .. 2^32 - 1");
    g->max_rows = rows;
    return SS_OK;
}

int ss_ingest_set_exact(ss_ingest* g, int exact) {
    if (!g) return ss_fail(SS_EARG, "null ingest");
    if (exact < 0 || exact > 5) return ss_fail(SS_EARG, "sizing mode 0 .. 5");
    g->sizing = exact;
    return SS_OK;
}

int ss_ingest_destroy(ss_ingest* g) {
    if (!g) return SS_OK;
    ss_ingest_reset(g);
    for (auto& kv : g->groups) {
        kv.second.rowmap.release();
        kv.second.fps.release(), kv.second.words.release(), kv.second.counts.release(), kv.second.first.release();
        kv.second.lens.release(), kv.second.xread.release();
    }
    g->groups.clear();
    for (auto& p : g->pool) ss_counter_destroy(p.second);
    g->pool.clear();
    for (FqSlot& sl : g->fq) {
        for (hipEvent_t e : sl.ev) (void)hipEventDestroy(e);
        sl.ev.clear();
        if (sl.done) (void)hipEventDestroy(sl.done);
        sl.done = nullptr;
        sl.h.release(), sl.d.release();
    }
    if (g->fq_copy) (void)hipStreamDestroy(g->fq_copy);
    g->fq_copy = nullptr;
    g->stage.release();
    g->out_host.release();
    g->dbuf.release(), g->offs.release(), g->dlens.release(), g->order.release(), g->blkhist.release();
    g->blkfirst.release(), g->split_out.release(), g->rows.release(), g->first_bad.release();
    g->fq_ws.release(), g->fq_aux.release(), g->fq_counts.release();
    g->slot.release(), g->ordered.release(), g->woff.release(), g->scan.release(), g->gdesc.release();
    g->cls_words.release(), g->cls_fps.release(), g->hll.release(), g->ovf.release();
    g->cls_flag.release(), g->zero32.release();
    if (g->fpt) ss_counter_destroy(g->fpt);
    g->fpt = nullptr;
    g->mg_words.release(), g->mg_counts.release(), g->mg_first.release(), g->mg_lens.release(), g->mg_take.release();
    if (g->h_hll) (void)hipHostFree(g->h_hll);
    if (g->h_split) (void)hipHostFree(g->h_split);
    if (g->h_bad) (void)hipHostFree(g->h_bad);
    if (g->h_spec) (void)hipHostFree(g->h_spec);
    if (g->h_gdesc) (void)hipHostFree(g->h_gdesc);
    g->spec_dev.release();
    if (g->ev_reps) (void)hipEventDestroy(g->ev_reps);
    if (g->ev_split) (void)hipEventDestroy(g->ev_split);
    if (g->ev_spec) (void)hipEventDestroy(g->ev_spec);
    if (g->spec_stream) (void)hipStreamDestroy(g->spec_stream);
    for (int k = 0; k < ss_ingest::kSide; ++k) {
        if (g->side[k]) (void)hipStreamDestroy(g->side[k]);
        if (g->ev_join[k]) (void)hipEventDestroy(g->ev_join[k]);
    }
    if (g->ev_fork) (void)hipEventDestroy(g->ev_fork);
    if (g->stream) (void)hipStreamDestroy(g->stream);
    delete g;
    return SS_OK;
}

int ss_ingest_staging(ss_ingest* g, uint64_t nbytes, uint8_t** h_ptr) {
    if (!g || !h_ptr) return ss_fail(SS_EARG, "null argument");
    int rc = g->stage.ensure(nbytes + 16);
    *h_ptr = rc ? nullptr : g->stage.p;
    return rc;
}

int ss_ingest_add_blob(ss_ingest* g, const uint8_t* h_blob, const uint32_t* h_lens, uint64_t n) {
    if (!g || (n && (!h_blob || !h_lens))) return ss_fail(SS_EARG, "null argument");
    if (n == 0 || g->bad_index != kNoSlot) return SS_OK;
    (void)hipSetDevice(g->device);
    std::vector<uint64_t> offs(n);
    uint64_t total = 0;
    bool same = true;
    for (uint64_t i = 0; i < n; ++i) {
        offs[i] = total;
        total += h_lens[i];
        same &= h_lens[i] == h_lens[0];
    }
    hipStream_t s = g->stream;
    int rc;
    if ((rc = g->dbuf.ensure(total + 16)) || (rc = g->offs.ensure(n)) || (rc = g->dlens.ensure(n))) return rc;
    rc = ss_check(hipMemcpyAsync(g->dbuf.p, h_blob, total ? total : 1, hipMemcpyHostToDevice, s), "ingest H2D");
    const uint32_t dense = (same && h_lens[0] > 0 && h_lens[0] <= SS_MAX_NT) ? h_lens[0] : 0u;
    if (!rc && !dense) {
        rc = ss_check(hipMemcpyAsync(g->offs.p, offs.data(), n * 8, hipMemcpyHostToDevice, s), "ingest H2D");
        if (!rc) rc = ss_check(hipMemcpyAsync(g->dlens.p, h_lens, n * 4, hipMemcpyHostToDevice, s), "ingest H2D");
    }
    if (!rc) rc = process_chunk(g, g->dbuf.p, g->offs.p, g->dlens.p, total, n, dense, &offs, h_blob, true);
    if (!rc) rc = ss_check(hipStreamSynchronize(s), "ingest blob");   // staging reusable after return
    return rc;
}

int ss_ingest_add_device(ss_ingest* g, const uint8_t* d_blob, uint64_t nbytes, const uint64_t* d_offsets,
                         const uint32_t* d_lens, uint64_t n) {
    if (!g || (n && (!d_blob || !d_offsets || !d_lens))) return ss_fail(SS_EARG, "null argument");
    if (n == 0 || g->bad_index != kNoSlot) return SS_OK;
    (void)hipSetDevice(g->device);
    int rc = process_chunk(g, d_blob, d_offsets, d_lens, nbytes, n, 0, nullptr, nullptr, true);
    if (!rc) rc = ss_check(hipStreamSynchronize(g->stream), "ingest device blob");
    return rc;
}

int ss_ingest_add_fastq(ss_ingest* g, const char* path, uint64_t chunk_bytes, uint64_t* h_nseqs) {
    return ss_ingest_add_fastq_range(g, path, 0, ~0ull, 0, chunk_bytes, h_nseqs);
}

int ss_fastq_split(const char* path, uint32_t nparts, uint64_t* h_begin, uint64_t* h_line0) {
    if (!path || !nparts || !h_begin || !h_line0) return ss_fail(SS_EARG, "null argument");
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return ss_fail(SS_EARG, "cannot open the FASTQ file");
    struct stat st;
    if (fstat(fd, &st) != 0) {
        close(fd);
        return ss_fail(SS_EARG, "cannot stat the FASTQ file");
    }
    const uint64_t size = (uint64_t)st.st_size;
    // part p starts right after the first newline at or past p * size / nparts (part 0 at 0); parts
    // may come out empty (begin[p] == begin[p + 1]) when lines are long
    std::vector<uint64_t> b(nparts + 1, size);
    b[0] = 0;
    std::vector<uint8_t> buf(1 << 16);
    for (uint32_t p = 1; p < nparts; ++p) {
        uint64_t pos = std::max(b[p - 1], size * p / nparts), at = size;
        while (pos < size && at == size) {
            const uint64_t got = pread_full(fd, buf.data(), std::min<uint64_t>(buf.size(), size - pos), pos);
            if (got == 0) break;
            const void* nl = memchr(buf.data(), '\n', got);
            if (nl) at = pos + (uint64_t)((const uint8_t*)nl - buf.data()) + 1;
            pos += got;
        }
        b[p] = at;
    }
    // newlines before each part: the parts' newline counts (one thread per part), prefix-summed
    std::vector<uint64_t> nl(nparts, 0);
    std::vector<std::thread> ts;
    for (uint32_t p = 0; p + 1 < nparts; ++p)
        ts.emplace_back([&, p] {
            std::vector<uint8_t> tb(1 << 20);
            uint64_t cnt = 0;
            for (uint64_t pos = b[p]; pos < b[p + 1];) {
                const uint64_t got = pread_full(fd, tb.data(), std::min<uint64_t>(tb.size(), b[p + 1] - pos), pos);
                if (got == 0) break;
                for (uint64_t k = 0; k < got; ++k) cnt += tb[k] == '\n';
                pos += got;
            }
            nl[p] = cnt;
        });
    for (auto& t : ts) t.join();
    close(fd);
    uint64_t run = 0;
    for (uint32_t p = 0; p < nparts; ++p) {
        h_begin[p] = b[p];
        h_line0[p] = run;
        run += nl[p];
    }
    h_begin[nparts] = size;
    return SS_OK;
}

int ss_ingest_add_fastq_range(ss_ingest* g, const char* path, uint64_t begin, uint64_t end, uint64_t line0,
                              uint64_t chunk_bytes, uint64_t* h_nseqs) {
    if (!g || !path) return ss_fail(SS_EARG, "null argument");
    (void)hipSetDevice(g->device);
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return ss_fail(SS_EARG, "cannot open the FASTQ file");
    struct stat st;
    if (fstat(fd, &st) != 0) {
        close(fd);
        return ss_fail(SS_EARG, "cannot stat the FASTQ file");
    }
    // the range [begin, end) of the file: it starts at a line boundary and ends at the file's end or
    // right after a newline, so its last line is complete (the strlen - 1 rule of a final line with no
    // newline applies only at the file's end)
    const uint64_t size = std::min<uint64_t>((uint64_t)st.st_size, end);
    if (h_nseqs) *h_nseqs = 0;
    if (begin >= size) {
        close(fd);
        return SS_OK;
    }
    if (chunk_bytes == 0) chunk_bytes = kFqChunkDefault;
    const uint64_t cap0 = std::max<uint64_t>(16, std::min<uint64_t>(chunk_bytes, size - begin + 16));
    hipStream_t s = g->stream;
    int rc = SS_OK;
    if (!g->fq_copy) rc = ss_check(hipStreamCreateWithFlags(&g->fq_copy, hipStreamNonBlocking), "ingest fastq stream");
    for (int i = 0; i < 2 && !rc; ++i)
        if (!g->fq[i].done) rc = ss_check(hipEventCreateWithFlags(&g->fq[i].done, hipEventDisableTiming), "ingest fastq event");
    if (rc) {
        close(fd);
        return rc;
    }
    const uint64_t seqs0 = g->nreads;
    const unsigned threads = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
    using Clock = std::chrono::steady_clock;
    auto since = [](Clock::time_point t0) { return std::chrono::duration<double, std::milli>(Clock::now() - t0).count(); };
    // The reader ring: a reader thread fills chunk k + 1 into slot (k + 1) & 1 -- the previous chunk's
    // tail (bytes after its last newline) first, then file reads in pieces of kFqPiece, each piece's
    // H2D queued on fq_copy as soon as it is read -- while this thread indexes and counts chunk k
    // from slot k & 1 on the engine's stream.  A slot goes back to the reader once the engine's
    // stream has finished with it.  state[i]: 0 the reader's, 1 filled (this thread's).
    std::mutex mu;
    std::condition_variable cv;
    int state[2] = {0, 0};
    bool stop = false;
    if (g->fq_node == -2) {
        int allowed = 0;
        g->fq_cpus = ss_gpu_numa_cpus(g->device, &g->fq_node, &allowed);
        const char* env = getenv("SHORTSEQ_FQ_PIN");
        if (env && env[0] == '0') g->fq_cpus.clear();
    }
    auto reader = [&]() {
        (void)hipSetDevice(g->device);
        if (!g->fq_cpus.empty()) {     // (read_parallel's threads inherit the mask)
            cpu_set_t set;
            CPU_ZERO(&set);
            for (int c : g->fq_cpus) CPU_SET(c, &set);
            (void)pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
        }
        uint64_t pos = begin, cap = cap0, carry = 0;
        const uint8_t* csrc = nullptr;
        for (uint64_t k = 0;; ++k) {
            FqSlot& sl = g->fq[k & 1];
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop || state[k & 1] == 0; });
                if (stop) return;
            }
            int r = SS_OK;
            sl.np = 0;
            try {
                for (;;) {
                    if (cap >= (1ull << 32)) {
                        r = ss_fail(SS_EARG, "a FASTQ line is longer than 2 GiB");
                        break;
                    }
                    if ((r = sl.h.ensure(cap)) || (r = sl.d.ensure(cap + 16))) break;
                    if (carry && csrc != sl.h.p) memcpy(sl.h.p, csrc, carry);
                    uint8_t* hv = sl.h.p;
                    const uint64_t want = std::min(cap - carry, size - std::min(size, pos));
                    const uint64_t npieces = (want + kFqPiece - 1) / kFqPiece + 1;
                    while (sl.ev.size() < 2 * (sl.np + npieces) && !r) {
                        hipEvent_t e = nullptr;
                        r = ss_check(hipEventCreate(&e), "ingest fastq event");
                        if (!r) sl.ev.push_back(e);
                    }
                    if (r) break;
                    auto h2d = [&](uint64_t off, uint64_t len) {
                        int q = ss_check(hipEventRecord(sl.ev[2 * sl.np], g->fq_copy), "ingest fastq event");
                        if (!q) q = ss_check(hipMemcpyAsync(sl.d.p + off, hv + off, len, hipMemcpyHostToDevice, g->fq_copy), "ingest H2D");
                        if (!q) q = ss_check(hipEventRecord(sl.ev[2 * sl.np + 1], g->fq_copy), "ingest fastq event");
                        ++sl.np;
                        g->fq_h2d_bytes += len;
                        return q;
                    };
                    if (carry) r = h2d(0, carry);
                    uint64_t got = 0;
                    for (uint64_t off = 0; off < want && !r; off += kFqPiece) {
                        const uint64_t len = std::min(kFqPiece, want - off);
                        const auto t0 = Clock::now();
                        const uint64_t n = read_parallel(fd, hv + carry + off, len, pos + off, threads);
                        g->fq_ms[0] += since(t0);
                        got += n;
                        if (n != len) break;
                        r = h2d(carry + off, len);
                    }
                    if (r) break;
                    if (got != want) {
                        r = ss_fail(SS_EHIP, "short read of the FASTQ file");
                        break;
                    }
                    pos += got;
                    sl.n = carry + got;
                    sl.at_eof = pos >= size;
                    sl.use = sl.n;
                    if (sl.at_eof || sl.n == 0) break;
                    sl.use = 0;
                    for (uint64_t q = sl.n; q > 0; --q)
                        if (hv[q - 1] == '\n') {
                            sl.use = q;
                            break;
                        }
                    if (sl.use) break;
                    // one line fills the chunk: grow this slot (its bytes kept, sent again as the carry)
                    if ((r = ss_check(hipStreamSynchronize(g->fq_copy), "ingest fastq grow"))) break;
                    HBuf grown;
                    if ((r = grown.ensure(2 * cap))) break;
                    memcpy(grown.p, hv, sl.n);
                    sl.h.release();
                    sl.h = grown;
                    cap *= 2;
                    carry = sl.n;
                    csrc = sl.h.p;
                }
            } catch (...) {     // (the event vector, read_parallel's threads)
                r = ss_fail(SS_ENOMEM, "FASTQ reader: out of host memory");
            }
            if (!r) r = ss_check(hipEventRecord(sl.done, g->fq_copy), "ingest fastq event");
            sl.rc = r;
            if (r) sl.err = ss_last_error_string();
            {
                std::lock_guard<std::mutex> lk(mu);
                state[k & 1] = 1;
            }
            cv.notify_all();
            if (r || sl.at_eof || sl.n == 0) return;
            csrc = sl.h.p + sl.use;
            carry = sl.n - sl.use;
        }
    };
    // a range that fits one chunk has nothing to overlap: it is read on this thread (no thread start)
    // unless the reader is to run on the GPU's NUMA node (the caller's affinity is left alone)
    std::thread rd;
    if (size - begin <= cap0 && g->fq_cpus.empty()) {
        reader();
    } else {
        try {
            rd = std::thread(reader);
        } catch (...) {
            close(fd);
            return ss_fail(SS_EHIP, "cannot start the FASTQ reader thread");
        }
    }
    for (uint64_t k = 0; !rc; ++k) {
        FqSlot& sl = g->fq[k & 1];
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return state[k & 1] == 1; });
        }
        if (sl.rc) {
            rc = ss_fail(sl.rc, sl.err.c_str());     // (raised again on this thread: the message is thread-local)
            break;
        }
        if (sl.n == 0) break;
        const uint64_t use = sl.use;
        const bool at_eof = sl.at_eof;
        // index the chunk on the device once its H2D pieces are done (the engine's stream waits for them)
        const auto ti = Clock::now();
        rc = ss_check(hipStreamWaitEvent(s, sl.done, 0), "ingest fastq wait");
        uint64_t maxr = use / 16 + 2;
        uint64_t nl = 0, nrec = 0;
        while (!rc) {
            const uint64_t wsb = ss_fastq_onepass_ws_bytes(use, maxr);
            if ((rc = g->fq_ws.ensure(wsb / 8 + 1)) || (rc = g->offs.ensure(maxr)) || (rc = g->dlens.ensure(maxr)) ||
                (rc = g->fq_aux.ensure(maxr)) || (rc = g->fq_counts.ensure(3)))
                break;
            rc = ss_fastq_index_onepass(sl.d.p, use, line0, at_eof ? 1 : 0, g->fq_ws.p, wsb, g->offs.p, g->dlens.p,
                                        g->fq_aux.p, maxr, g->fq_counts.p, s);
            if (!rc) rc = ss_check(hipMemcpyAsync(g->h_bad, g->fq_counts.p, 24, hipMemcpyDeviceToHost, s), "ingest fq");
            if (!rc) rc = ss_check(hipStreamSynchronize(s), "ingest fq");
            if (rc) break;
            nl = g->h_bad[0];
            nrec = g->h_bad[1];
            if (g->h_bad[2]) {
                maxr *= 2;
                continue;
            }
            if (nrec <= maxr) break;
            maxr = nrec;
        }
        if (rc) break;
        g->fq_ms[2] += since(ti);
        for (uint32_t q = 0; q < sl.np; ++q) {     // the pieces' H2D times (all complete: the index synced)
            float ms = 0;
            if (hipEventElapsedTime(&ms, sl.ev[2 * q], sl.ev[2 * q + 1]) == hipSuccess) g->fq_ms[1] += ms;
            else (void)hipGetLastError();
        }
        if (!at_eof && g->est_scale == 1.0 && use) g->est_scale = (double)(size - begin) / (double)use;
        const auto tc = Clock::now();
        rc = process_chunk(g, sl.d.p, g->offs.p, g->dlens.p, use, nrec, 0, nullptr, sl.h.p);
        g->fq_ms[3] += since(tc);
        if (rc) break;
        line0 += nl;
        if (at_eof || g->bad_index != kNoSlot) break;
        if ((rc = ss_check(hipStreamSynchronize(s), "ingest chunk"))) break;
        {
            std::lock_guard<std::mutex> lk(mu);
            state[k & 1] = 0;
        }
        cv.notify_all();
    }
    {
        std::lock_guard<std::mutex> lk(mu);
        stop = true;
    }
    cv.notify_all();
    if (rd.joinable()) rd.join();
    const int rc2 = ss_check(hipStreamSynchronize(g->fq_copy), "ingest fastq copies");
    if (!rc) rc = rc2;
    close(fd);
    if (!rc) rc = ss_check(hipStreamSynchronize(s), "ingest fastq");
    if (h_nseqs) *h_nseqs = g->nreads - seqs0;
    return rc;
}

int ss_ingest_error(ss_ingest* g, uint64_t* h_index, int* h_kind, uint8_t* h_read, uint64_t cap, uint64_t* h_len) {
    if (!g || !h_index || !h_kind) return ss_fail(SS_EARG, "null argument");
    *h_index = g->bad_index;
    *h_kind = g->bad_kind;
    if (h_len) *h_len = g->bad_bytes.size();
    if (h_read && cap) memcpy(h_read, g->bad_bytes.data(), std::min<uint64_t>(cap, g->bad_bytes.size()));
    return SS_OK;
}

static int finish_impl(ss_ingest* g, uint64_t* h_nkeys, uint64_t* h_nwords);

int ss_ingest_finish(ss_ingest* g, uint64_t* h_nkeys, uint64_t* h_nwords) {
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = finish_impl(g, h_nkeys, h_nwords);
    if (g) g->fq_ms[4] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

int ss_ingest_fastq_stages(ss_ingest* g, double* h_ms, uint64_t* h_h2d_bytes) {
    if (!g || !h_ms || !h_h2d_bytes) return ss_fail(SS_EARG, "null argument");
    for (int i = 0; i < 5; ++i) {
        h_ms[i] = g->fq_ms[i];
        g->fq_ms[i] = 0;
    }
    *h_h2d_bytes = g->fq_h2d_bytes;
    g->fq_h2d_bytes = 0;
    return SS_OK;
}

static int finish_impl(ss_ingest* g, uint64_t* h_nkeys, uint64_t* h_nwords) {
    if (!g || !h_nkeys || !h_nwords) return ss_fail(SS_EARG, "null argument");
    if (g->failed) return ss_fail(SS_EFULL, "ingest: an earlier add ran a table full; reset and count again");
    (void)hipSetDevice(g->device);
    hipStream_t s = g->stream;
    const uint64_t N = g->nreads;
    int rc = SS_OK;
    *h_nkeys = *h_nwords = 0;
    if (g->spec_valid) {            // the speculative finish queued by the add: wait for it
        const int e = ss_check(hipEventSynchronize(g->ev_spec), "ingest spec finish");
        g->spec_inflight = false;
        if (e) return e;
        if (!g->h_spec[2]) {        // (stays valid: a second finish returns the same rows)
            g->nkeys = g->h_spec[0];
            g->nwords = g->h_spec[1];
            *h_nkeys = g->nkeys;
            *h_nwords = g->nwords;
            return SS_OK;
        }
    }
    spec_wait(g);
    if (N == 0) return SS_OK;
    const uint64_t NB = (N + 63) / 64;      // read-map words
    if ((rc = g->slot.ensure(NB))) return rc;
    rc = ss_check(hipMemsetAsync(g->slot.p, 0, NB * 8, s), "ingest read map reset");
    unsigned long long* bits = (unsigned long long*)g->slot.p;
    std::vector<GDesc> desc;
    std::vector<Group*> placed;
    // a deferred fold's classes come straight from the scratch (they stay pending: a later add folds them)
    if ((rc = extract_groups(g, placed, g->pend))) return rc;
    for (size_t q = 0; q < placed.size(); ++q) {
        Group& gr = *placed[q];
        hipLaunchKernelGGL(k_mark, dim3(grid_of(gr.m + 1, 256)), dim3(256), 0, s, gr.first.p, gr.m, gr.rowmap.p,
                           kNoSlot, bits);
        desc.push_back({gr.words.p, gr.counts.p, gr.W1, gr.L});
    }
    const uint64_t empty_at = g->empty_count ? g->empty_first : kNoSlot;
    if (g->empty_count)
        hipLaunchKernelGGL(k_mark, dim3(1), dim3(256), 0, s, (const uint64_t*)nullptr, (uint64_t)0,
                           (const uint64_t*)nullptr, empty_at, bits);
    // the entry and word totals came back with the extraction's sync: no sync until the results
    uint64_t K = g->empty_count ? 1 : 0, NW = 0;
    for (Group* gr : placed) {
        K += gr->m;
        NW += gr->nw;
    }
    // results -> pinned host (results_layout: lens | counts | words), written by the gather
    uint64_t co = 0, wo0 = 0;
    results_layout(K, 0, 8, co, wo0);      // (the plain layout bounds the compact one)
    if ((rc = g->gdesc.ensure(desc.size() + 1)) || (rc = g->ordered.ensure(K + 1)) ||
        (rc = g->woff.ensure(std::max(K, NB) + 1)) || (rc = g->out_host.ensure(wo0 + NW * 8 + 16)) ||
        (rc = g->spec_dev.ensure(13)))
        return rc;

    if (!desc.empty())
        rc = ss_check(hipMemcpyAsync(g->gdesc.p, desc.data(), desc.size() * sizeof(GDesc), hipMemcpyHostToDevice, s),
                      "ingest desc");
    if (rc) return rc;
    // marked reads before each read-map word (read order = dict order); woff holds that prefix first
    // (it becomes the word offsets below)
    hipLaunchKernelGGL((k_scan_count<0>), dim3(kScanBlocks), dim3(256), 0, s, g->slot.p, NB, (const GDesc*)g->gdesc.p,
                       g->scan.p);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(256), 0, s, g->scan.p);
    hipLaunchKernelGGL((k_scan_apply<0>), dim3(kScanBlocks), dim3(256), 0, s, g->slot.p, NB, (const GDesc*)g->gdesc.p,
                       g->scan.p, g->woff.p);
    for (size_t q = 0; q < placed.size(); ++q)
        hipLaunchKernelGGL(k_rank, dim3(grid_of(placed[q]->m + 1, 256)), dim3(256), 0, s, placed[q]->first.p,
                           placed[q]->m, placed[q]->rowmap.p, (uint32_t)q, kNoSlot, bits, g->woff.p, g->ordered.p);
    if (g->empty_count)
        hipLaunchKernelGGL(k_rank, dim3(1), dim3(256), 0, s, (const uint64_t*)nullptr, (uint64_t)0,
                           (const uint64_t*)nullptr, 0u, empty_at, bits, g->woff.p, g->ordered.p);
    // word offsets of the ordered entries
    hipLaunchKernelGGL((k_scan_count<1>), dim3(kScanBlocks), dim3(256), 0, s, g->ordered.p, K, (const GDesc*)g->gdesc.p,
                       g->scan.p);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(256), 0, s, g->scan.p);
    hipLaunchKernelGGL((k_scan_apply<1>), dim3(kScanBlocks), dim3(256), 0, s, g->ordered.p, K, (const GDesc*)g->gdesc.p,
                       g->scan.p, g->woff.p);
    if (K >= (1ull << 31) * 256) return ss_fail(SS_EARG, "ingest: too many distinct keys for one gather");
    g->wide = results_wide(g);
    OutLayout ol{g->out_host.p, g->out_host.cap, nullptr, nullptr, NW, nullptr, g->compact, g->wide ? 1 : 0};
    hipLaunchKernelGGL(k_gather_host, dim3((unsigned)((K + 255) / 256)), dim3(256), 0, s, g->ordered.p, K,
                       (const GDesc*)g->gdesc.p, g->woff.p, g->empty_count, ol);
    rc = ss_check(hipGetLastError(), "k_gather_host");
    if (!rc) rc = ss_check(hipStreamSynchronize(s), "ingest out");
    if (rc) return rc;
    g->nkeys = K;
    g->nwords = NW;
    *h_nkeys = K;
    *h_nwords = NW;
    return SS_OK;
}

int ss_ingest_export(ss_ingest* g, uint64_t* h_nkeys) {
    if (!g) return ss_fail(SS_EARG, "null ingest");
    if (g->failed) return ss_fail(SS_EFULL, "ingest: an earlier add ran a table full; reset and count again");
    (void)hipSetDevice(g->device);
    std::vector<Group*> placed;
    spec_wait(g);
    int rc = flush_pending(g);
    if (!rc) rc = extract_groups(g, placed);
    if (rc) return rc;
    uint64_t keys = 0;
    for (Group* gr : placed) {
        if (!gr->m) continue;
        if ((rc = gr->xread.ensure(gr->m))) return rc;
        hipLaunchKernelGGL(k_export_reads, dim3(grid_of(gr->m, 256)), dim3(256), 0, g->stream, gr->first.p, gr->m,
                           gr->rowmap.p, gr->xread.p);
        keys += gr->m;
    }
    // the largest exported count: a merge takes it in passes of what a u32 slot can hold
    if ((rc = g->mg_take.ensure(1)) ||
        (rc = ss_check(hipMemsetAsync(g->mg_take.p, 0, 8, g->stream), "ingest export max")))
        return rc;
    for (Group* gr : placed)
        if (gr->m)
            hipLaunchKernelGGL(k_count_max, dim3(std::min<unsigned>(grid_of(gr->m, 256), kCountMaxBlocks)), dim3(256), 0,
                               g->stream, gr->counts.p, gr->m,
                               (unsigned long long*)g->mg_take.p);
    rc = ss_check(hipMemcpyAsync(g->h_bad + 3 * kLenBins + 4, g->mg_take.p, 8, hipMemcpyDeviceToHost, g->stream), "ingest export max");
    if (!rc) rc = ss_check(hipStreamSynchronize(g->stream), "ingest export");
    if (rc) return rc;
    g->xmax = g->h_bad[3 * kLenBins + 4];
    g->exported = true;
    if (h_nkeys) *h_nkeys = keys + (g->empty_count ? 1 : 0);
    return SS_OK;
}

int ss_ingest_reserve_merge(ss_ingest* dst, ss_ingest* const* srcs, uint32_t nsrc) {
    if (!dst || (nsrc && !srcs)) return ss_fail(SS_EARG, "ingest reserve merge: null argument");
    if (dst->failed) return ss_fail(SS_EFULL, "ingest: an earlier add ran a table full; reset and count again");
    std::map<uint32_t, std::pair<uint64_t, const Group*>> total;      // bin -> (entries, a source group)
    for (uint32_t k = 0; k < nsrc; ++k) {
        ss_ingest* src = srcs[k];
        if (!src || src == dst) return ss_fail(SS_EARG, "ingest reserve merge: sources distinct from the destination");
        if (!src->exported) return ss_fail(SS_EARG, "ingest reserve merge: ss_ingest_export the sources first");
        for (auto& kv : src->groups)
            if (kv.second.table && kv.second.m) {
                auto& t = total[kv.first];
                t.first += kv.second.m;
                t.second = &kv.second;
            }
    }
    if (total.empty()) return SS_OK;
    spec_wait(dst);
    int rc = ss_check(hipSetDevice(dst->device), "ingest reserve merge device");
    if (!rc) rc = flush_pending(dst);
    if (rc) return rc;
    hipStream_t s = dst->stream;
    const double scale = dst->est_scale;
    dst->est_scale = 1.0;
    for (auto& kv : total) {
        const uint64_t m = kv.second.first;
        Group& gr = dst->groups[kv.first];
        gr.L = kv.second.second->L;
        gr.W1 = kv.second.second->W1;
        // one table growth (at most) for the union of every source's entries, and the row map's
        // room, instead of a growth -- every existing entry re-inserted -- at each merge
        if ((rc = group_room(dst, gr, m, gr.rows + m)) || (rc = gr.rowmap.ensure_keep(gr.rows + m, gr.rows, s))) break;
    }
    dst->est_scale = scale;
    return rc;
}

int ss_ingest_merge(ss_ingest* dst, ss_ingest* src, uint64_t src_base) {
    if (!dst || !src || dst == src) return ss_fail(SS_EARG, "ingest merge: two distinct engines");
    if (!src->exported) return ss_fail(SS_EARG, "ingest merge: ss_ingest_export the source first");
    if (dst->failed) return ss_fail(SS_EFULL, "ingest: an earlier add ran a table full; reset and count again");
    if (src_base < dst->nreads) return ss_fail(SS_EARG, "ingest merge: sources follow the destination's reads, in order");
    spec_wait(dst);
    spec_wait(src);
    int rc = ss_check(hipSetDevice(dst->device), "ingest merge device");
    if (!rc) rc = flush_pending(dst);
    if (rc) return rc;
    const bool peer = src->device != dst->device;
    if (peer) {
        int can = 0;
        (void)hipDeviceCanAccessPeer(&can, dst->device, src->device);
        if (can) {
            const hipError_t e = hipDeviceEnablePeerAccess(src->device, 0);
            if (e != hipSuccess) (void)hipGetLastError();     // already enabled, or unsupported: copies stage
        }
    }
    hipStream_t s = dst->stream;
    auto copy = [&](void* d, const void* p, uint64_t bytes) -> int {
        if (!bytes) return SS_OK;
        return ss_check(peer ? hipMemcpyPeerAsync(d, dst->device, p, src->device, bytes, s)
                             : hipMemcpyAsync(d, p, bytes, hipMemcpyDeviceToDevice, s),
                        "ingest merge copy");
    };
    // the source's reads count toward the destination's spill: its slots stay below 2^32 after the merge
    // (one source's key past 2^32 - 1 copies still raises SS_EFULL)
    if (dst->since_spill + src->nreads > dst->spill_limit && (rc = spill_counts(dst))) return rc;
    // what a slot can still take before the next spill (no fewer than the source's reads unless the
    // source itself spilled: then its counts go in passes)
    const uint64_t room0 = std::max<uint64_t>(1, std::min<uint64_t>(dst->spill_limit, 0xFFFFFFFEull) - dst->since_spill);
    const double scale = dst->est_scale;
    dst->est_scale = 1.0;            // a new group is sized by the entries it receives
    for (auto& kv : src->groups) {
        const Group& sg = kv.second;
        if (!sg.table || !sg.m) continue;
        const uint64_t m = sg.m;
        const uint32_t bin = kv.first;
        Group& gr = dst->groups[bin];
        gr.L = sg.L;
        gr.W1 = sg.W1;
        if ((rc = group_room(dst, gr, m, gr.rows + m))) break;
        if ((rc = gr.rowmap.ensure_keep(gr.rows + m, gr.rows, s))) break;
        if ((rc = dst->mg_words.ensure(m * gr.W1)) || (rc = dst->mg_counts.ensure(m)) || (rc = dst->mg_first.ensure(m)) ||
            (rc = dst->mg_lens.ensure(m)))
            break;
        // the source's entries cross to this device (xGMI peer copies; a plain copy on one device)
        if ((rc = copy(dst->mg_words.p, sg.words.p, m * gr.W1 * 8)) || (rc = copy(dst->mg_counts.p, sg.counts.p, m * 8)) ||
            (rc = copy(dst->mg_lens.p, sg.lens.p, m * 4)) || (rc = copy(gr.rowmap.p + gr.rows, sg.xread.p, m * 8)))
            break;
        hipLaunchKernelGGL(k_merge_rows, dim3(grid_of(m, 256)), dim3(256), 0, s, m, gr.rows, src_base,
                           dst->mg_first.p, gr.rowmap.p);
        // appended as one block after every earlier row: a key already here keeps its (smaller) first
        // row, a key also in a later source gets that source's larger rows -> min = first occurrence.
        // Counts a u32 slot cannot take at once go in passes of `room`, the destination's counts
        // spilled to its u64 row counts between passes.
        const uint64_t* cnt = dst->mg_counts.p;
        uint64_t left = src->xmax, room = room0;
        const bool passes = left > room;
        if (passes && (rc = dst->mg_take.ensure(m))) break;
        gr.rows += m;               // the appended rows (the spill between passes sizes the row counts by them)
        do {
            if (passes) {           // every pass takes min(remaining, room), the last one the rest
                hipLaunchKernelGGL(k_count_take, dim3(grid_of(m, 256)), dim3(256), 0, s, dst->mg_counts.p, dst->mg_take.p,
                                   m, room);
                cnt = dst->mg_take.p;
            }
            rc = gr.W1 == 1 ? ss_counter_merge(gr.table, dst->mg_words.p, dst->mg_lens.p, cnt, dst->mg_first.p, m, s)
                            : ss_counter_merge_words(gr.table, dst->mg_words.p, cnt, dst->mg_first.p, m, s);
            if (rc) break;
            left = left > room ? left - room : 0;
            if (left) {
                if ((rc = spill_counts(dst))) break;
                room = std::min<uint64_t>(dst->spill_limit, 0xFFFFFFFEull);
            }
        } while (left);
        if (rc) break;
    }
    dst->est_scale = scale;
    dst->since_spill = std::min<uint64_t>(dst->spill_limit, dst->since_spill + src->nreads);
    if (rc) return rc;
    if (src->empty_count) {
        dst->empty_count += src->empty_count;
        dst->empty_first = std::min(dst->empty_first, src_base + src->empty_first);
    }
    dst->nreads = std::max(dst->nreads, src_base + src->nreads);
    dst->exported = false;           // its tables changed: a later merge out of it exports them again
    return ss_check(hipStreamSynchronize(s), "ingest merge");    // the source may be reset after return
}

int ss_ingest_results(ss_ingest* g, const uint32_t** h_lens, const uint64_t** h_counts, const uint64_t** h_words) {
    if (!g || !h_lens || !h_counts || !h_words) return ss_fail(SS_EARG, "null argument");
    if (g->compact) return ss_fail(SS_EARG, "ingest results: compact format set (ss_ingest_results_compact)");
    uint64_t co = 0, wo = 0;
    results_layout(g->nkeys, 0, 8, co, wo);
    *h_lens = (const uint32_t*)g->out_host.p;
    *h_counts = (const uint64_t*)(g->out_host.p + co);
    *h_words = (const uint64_t*)(g->out_host.p + wo);
    return SS_OK;
}

int ss_ingest_set_results_format(ss_ingest* g, int compact) {
    if (!g) return ss_fail(SS_EARG, "null ingest");
    // (2: compact with u64 counts whatever they hold -- a test hook for the wide branch)
    if (compact < 0 || compact > 2) return ss_fail(SS_EARG, "results format 0 (plain), 1 (compact) or 2");
    spec_wait(g);                  // (a queued finish wrote the other layout)
    g->compact = compact;
    return SS_OK;
}

int ss_ingest_results_compact(ss_ingest* g, const uint16_t** h_lens, const void** h_counts, uint32_t* h_count_bytes,
                              const uint64_t** h_words) {
    if (!g || !h_lens || !h_counts || !h_count_bytes || !h_words) return ss_fail(SS_EARG, "null argument");
    if (!g->compact) return ss_fail(SS_EARG, "ingest results: plain format (ss_ingest_results)");
    const uint32_t cw = g->wide ? 8u : 4u;
    uint64_t co = 0, wo = 0;
    results_layout(g->nkeys, 1, cw, co, wo);
    *h_lens = (const uint16_t*)g->out_host.p;
    *h_counts = (const void*)(g->out_host.p + co);
    *h_count_bytes = cw;
    *h_words = (const uint64_t*)(g->out_host.p + wo);
    return SS_OK;
}

}  // extern "C"
