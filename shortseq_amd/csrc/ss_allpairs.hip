// ss_allpairs.hip — all-pairs thresholded hamming (UMI-style dedup; the reference
// benchmark compares its __xor__ against UMI-tools' edit_distance, benchmark.py:11,153).
//
// Distance = the reference's ShortSeq.__xor__ (short_seq_64.pyx:77-84, short_seq_192.pyx:74-91,
// short_seq_var.pyx:64-81): over W words, popcount(((x >> 1) | x) & 0x5555...), x = a ^ b, i.e. the
// number of nucleotide positions whose 2-bit codes differ.
//
// This is the one compute-bound piece of the path (O(n^2) pairs over O(n) bytes).  Each packed word
// (32 nt) is split once into two bit-planes (lo = even bits, hi = odd bits, 32 bits each), so a
// pair costs, per word: lo_a^lo_b, hi_a^hi_b, OR, v_bcnt (accumulating) — then one compare and
// one add for the row count: ~6 VALU ops per pair per word instead of ~10 on the interleaved form.
// Tiling: a block owns a row tile of S = 256 * R reads held in registers (R per lane, converted to
// planes on load) and a column tile of S reads, staged through LDS in chunks (planes), read by
// every lane with broadcast LDS reads.  Only tile pairs bj >= bi run (unordered pairs once; the
// diagonal tile masks j <= i).  Hits are rare for UMI thresholds, so they leave the inner loop
// through a wave ballot: row counts stay in registers, column counts go to LDS counters, pairs
// are appended with one global atomic per wave.
#include <mutex>

#include "ss_device.h"
#include "ss_internal.h"

namespace {

using namespace ssd;

// even bits of x (nt codes' low bits) -> 32-bit plane; odd bits -> the other plane
__device__ __forceinline__ uint32_t even_bits(uint64_t x) {
    x &= 0x5555555555555555ull;
    x = (x | (x >> 1)) & 0x3333333333333333ull;
    x = (x | (x >> 2)) & 0x0F0F0F0F0F0F0F0Full;
    x = (x | (x >> 4)) & 0x00FF00FF00FF00FFull;
    x = (x | (x >> 8)) & 0x0000FFFF0000FFFFull;
    x = (x | (x >> 16)) & 0x00000000FFFFFFFFull;
    return (uint32_t)x;
}

struct AllPairsArgs {
    const uint64_t* words;
    uint64_t n;
    uint32_t wpr;       // words per read in memory
    uint32_t W;         // words compared (ham_words(L)); words W..WT-1 of the template are zero
    uint32_t k;         // max distance
    uint32_t ntiles;
    uint32_t* counts;   // nullable
    uint32_t* pairs;    // nullable: (i, j) u32 pairs
    uint64_t max_pairs;
    unsigned long long* npairs;
};

template <int WT, int R>
struct Tile {
    static constexpr int S = 256 * R;                        // reads per tile
    static constexpr int C0 = (WT <= 4) ? 1024 : (4096 / WT);
    static constexpr int C = C0 < S ? C0 : S;               // columns per LDS chunk (divides S)
};

template <int WT>
__device__ __forceinline__ void load_planes(const AllPairsArgs& a, uint64_t r, uint32_t* lo, uint32_t* hi) {
#pragma unroll
    for (int w = 0; w < WT; ++w) {
        uint64_t x = 0;
        if (r < a.n && (uint32_t)w < a.W) x = a.words[r * a.wpr + w];
        lo[w] = even_bits(x);
        hi[w] = even_bits(x >> 1);
    }
}

template <int WT, int R>
__global__ __launch_bounds__(256) void k_allpairs(AllPairsArgs a) {
    constexpr int S = Tile<WT, R>::S, C = Tile<WT, R>::C;
    const uint32_t bi = blockIdx.y, bj = blockIdx.x;
    if (bj < bi) return;                                    // unordered pairs: upper triangle only
    __shared__ uint2 pl[C * WT];                             // {lo, hi} planes per column word
    __shared__ uint32_t colcnt[C];
    __shared__ unsigned long long blkhits;   // count-only calls: the block's hits, one global atomic
    if (threadIdx.x == 0) blkhits = 0;
    const bool diag = bi == bj;
    // rows of this lane: i = bi*S + r*256 + tid
    uint32_t alo[R][WT], ahi[R][WT];
    uint32_t rowcnt[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint64_t i = (uint64_t)bi * S + r * 256 + threadIdx.x;
        load_planes<WT>(a, i, alo[r], ahi[r]);
        rowcnt[r] = 0;
    }
    const uint64_t nrow_lim = a.n;
    for (int c0 = 0; c0 < S; c0 += C) {
        const uint64_t j0 = (uint64_t)bj * S + c0;
        if (j0 >= a.n) break;
        __syncthreads();
        for (int c = threadIdx.x; c < C; c += 256) {
            uint32_t lo[WT], hi[WT];
            load_planes<WT>(a, j0 + c, lo, hi);
#pragma unroll
            for (int w = 0; w < WT; ++w) pl[c * WT + w] = make_uint2(lo[w], hi[w]);
            colcnt[c] = 0;
        }
        __syncthreads();
        const uint32_t ncols = (uint32_t)min<uint64_t>(C, a.n - j0);

        for (uint32_t c = 0; c < ncols; ++c) {
            uint32_t blo[WT], bhi[WT];
#pragma unroll
            for (int w = 0; w < WT; ++w) {
                const uint2 p = pl[c * WT + w];
                blo[w] = p.x;
                bhi[w] = p.y;
            }
            const uint64_t j = j0 + c;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint64_t i = (uint64_t)bi * S + r * 256 + threadIdx.x;
                uint32_t d = 0;
#pragma unroll
                for (int w = 0; w < WT; ++w) d += __popc((alo[r][w] ^ blo[w]) | (ahi[r][w] ^ bhi[w]));
                bool hit = d <= a.k && i < nrow_lim;
                if (diag) hit = hit && j > i;
                rowcnt[r] += hit ? 1u : 0u;
                if (__ballot(hit)) {                        // rare: column count + pair output
                    if (hit && a.counts) atomicAdd(&colcnt[c], 1u);
                    if (a.pairs) {
                        const uint64_t mask = __ballot(hit);
                        const uint32_t lane = threadIdx.x & 63u;
                        const uint32_t rank = __popcll(mask & ((1ull << lane) - 1ull));
                        unsigned long long base = 0;
                        if (lane == (uint32_t)__ffsll((unsigned long long)mask) - 1u)
                            base = atomicAdd(a.npairs, (unsigned long long)__popcll(mask));
                        base = __shfl(base, __ffsll((unsigned long long)mask) - 1);
                        const uint64_t slot = base + rank;
                        if (hit && slot < a.max_pairs) {
                            a.pairs[2 * slot] = (uint32_t)i;
                            a.pairs[2 * slot + 1] = (uint32_t)j;
                        }
                    } else {
                        const uint64_t mask = __ballot(hit);   // all lanes, before the leader's branch
                        if ((threadIdx.x & 63u) == (uint32_t)__ffsll((unsigned long long)mask) - 1u)
                            atomicAdd(&blkhits, (unsigned long long)__popcll(mask));
                    }
                }
            }
        }
        __syncthreads();
        if (a.counts) {
            for (int c = threadIdx.x; c < (int)ncols; c += 256)
                if (colcnt[c]) atomicAdd(&a.counts[j0 + c], colcnt[c]);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0 && blkhits) atomicAdd(a.npairs, blkhits);
    if (a.counts) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint64_t i = (uint64_t)bi * S + r * 256 + threadIdx.x;
            if (i < a.n && rowcnt[r]) atomicAdd(&a.counts[i], rowcnt[r]);
        }
    }
}

// ------------------------------------------------------------------------------------------------
// MFMA form for one-word reads (L <= 32, the UMI case).  Matching positions are a dot product of
// one-hot codes: position p of a read -> 4 int8 lanes with a 1 at its code, so for reads i, j
// D[i][j] = sum_k A[i][k] B[k][j] = number of positions with equal codes, and distance = P - D.
// P = min(L + 1, 32) positions: positions > L are code 0 in every packed word, position L can
// carry the table-path alias bit, which the reference's whole-word __xor__ counts.
// v_mfma_i32_32x32x32_i8 takes 8 positions per k-step: lane l (r = l & 31, h = l >> 5) holds
// row / column r and positions 8s + 4h + q (q = 0..3) in its 4 VGPRs, VGPR q = 1 << (8 * code);
// D: col = l & 31, row = (reg & 3) + 8 (reg >> 2) + 4 h (tools/probe_mfma_i8.hip checks the maps).
// Block: 4 waves x RB row blocks of 32 rows = S rows (A fragments in registers), the S columns
// of the paired tile staged in LDS as packed words; per 32-column block each wave builds its B
// fragments once and runs RB x KS MFMAs.  A hit needs D >= P - k; the 16 results of a tile are
// OR-reduced (bit 7 after a 128 - thr bias) and tested with one ballot, so the (rare) hit path runs
// only for tiles that have one.
// Rows / columns past n get zero fragments (D = 0); the hit path checks indices.
// ------------------------------------------------------------------------------------------------
typedef int v4i32 __attribute__((ext_vector_type(4)));
typedef int v16i32 __attribute__((ext_vector_type(16)));

template <int KS>
__device__ __forceinline__ void onehot_frag(uint64_t word, bool valid, uint32_t P, uint32_t h, v4i32* f) {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
        v4i32 v;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t p = 8u * s + 4u * h + q;
            const uint32_t code = (uint32_t)(word >> (2u * p)) & 3u;
            v[q] = (valid && p < P) ? (int)(1u << (8u * code)) : 0;
        }
        f[s] = v;
    }
}

// Hit path of one 32 x 32 result tile (st = its 16 result registers per lane, [reg][lane], hit =
// bit 7): index checks, LDS row / column counts, wave-aggregated pair append.
__device__ __noinline__ void ap_hits(const AllPairsArgs& a, const int* st, uint32_t rl0, uint32_t cl, uint64_t row0,
                                     uint64_t col0, bool diag, uint32_t* rowcnt, uint32_t* colcnt,
                                     unsigned long long* blkhits) {
    const uint32_t lane = threadIdx.x & 63u, h = lane >> 5;
#pragma unroll 1
    for (int q = 0; q < 16; ++q) {
        const uint32_t rl = rl0 + (q & 3) + 8 * (q >> 2) + 4 * h;
        const uint64_t i = row0 + rl, j = col0 + cl;
        bool hit = (st[q * 64 + lane] & 128) && i < a.n && j < a.n;
        if (diag) hit = hit && j > i;
        const uint64_t mask = __ballot(hit);
        if (!mask) continue;
        if (hit && a.counts) {
            atomicAdd(&rowcnt[rl], 1u);
            atomicAdd(&colcnt[cl], 1u);
        }
        const int leader = __ffsll((unsigned long long)mask) - 1;
        if (!a.pairs) {         // count only: the block's LDS total, one global atomic per block
            if ((int)lane == leader) atomicAdd(blkhits, (unsigned long long)__popcll(mask));
            continue;
        }
        unsigned long long base = 0;
        if ((int)lane == leader) base = atomicAdd(a.npairs, (unsigned long long)__popcll(mask));
        base = __shfl(base, leader);
        if (hit) {
            const uint64_t slot = base + __popcll(mask & ((1ull << lane) - 1ull));
            if (slot < a.max_pairs) {
                a.pairs[2 * slot] = (uint32_t)i;
                a.pairs[2 * slot + 1] = (uint32_t)j;
            }
        }
    }
}

// Upper-triangle tile pair (bi <= bj) of linear block k over t tiles, row-major: row bi holds
// t - bi pairs.  A float estimate of bi, corrected by integer steps.
__device__ __forceinline__ void tri_pair(uint64_t k, uint64_t t, uint32_t& bi, uint32_t& bj) {
    const double b = 2.0 * (double)t + 1.0;
    int64_t i = (int64_t)((b - sqrt(b * b - 8.0 * (double)k)) / 2.0);
    auto before = [&](int64_t r) { return (uint64_t)(r * (int64_t)t - r * (r - 1) / 2); };   // pairs in rows < r
    if (i < 0) i = 0;
    while (i > 0 && before(i) > k) --i;
    while (before(i + 1) <= k) ++i;
    bi = (uint32_t)i;
    bj = (uint32_t)(i + (int64_t)(k - before(i)));
}

// TAB: fragments from a 256-entry LDS table (4 codes of a byte -> the 4 one-hot VGPRs of a k-step
// half, one ds_read_b128) instead of per-VGPR bit arithmetic.  Positions P .. 8 KS - 1 are then
// code 0 on both sides and add the constant 8 KS - P to every result, folded into the threshold.
// TRI: the launch may be a 1-D grid over upper-triangle tile pairs (kept out of the RB >= 4
// instantiations: its registers cost them a wave per SIMD)
template <int KS, int RB, bool TAB, bool TRI>
__global__ __launch_bounds__(256) void k_allpairs_mfma(AllPairsArgs a, uint32_t P) {
    constexpr int S = 4 * RB * 32;
    constexpr int NW = (KS + 3) / 4;                       // packed words per read (32 positions each)
    // one block per upper-triangle tile pair (a 1-D grid while its work-item count fits 32 bits;
    // beyond that the square 2-D grid, lower-triangle blocks exiting at once)
    uint32_t bi = blockIdx.y, bj = blockIdx.x;
    if (TRI && gridDim.y == 1) tri_pair(blockIdx.x, (a.n + S - 1) / S, bi, bj);
    if (bj < bi) return;
    __shared__ uint64_t cw[S * NW];
    __shared__ uint32_t rowcnt[S], colcnt[S];
    __shared__ int stash[4 * 1024];                        // hit path: [wave][result reg][lane]
    __shared__ v4i32 ohtab[TAB ? 256 : 1];
    __shared__ unsigned long long blkhits;
    const bool diag = bi == bj;
    if (threadIdx.x == 0) blkhits = 0;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, h = lane >> 5, r = lane & 31u;
    const uint64_t row0 = (uint64_t)bi * S, col0 = (uint64_t)bj * S;
    if (TAB) {
        v4i32 e;
#pragma unroll
        for (int q = 0; q < 4; ++q) e[q] = (int)(1u << (8u * ((threadIdx.x >> (2 * q)) & 3u)));
        ohtab[threadIdx.x] = e;
    }
    for (int c = threadIdx.x; c < S; c += 256) {
        const uint64_t j = col0 + c;
#pragma unroll
        for (int w = 0; w < NW; ++w) cw[c * NW + w] = (j < a.n && (uint32_t)w < a.W) ? a.words[j * a.wpr + w] : 0ull;
        rowcnt[c] = 0;
        colcnt[c] = 0;
    }
    if (TAB) __syncthreads();
    // k-step s covers positions 8s .. 8s+7 = byte 2(s % 4) + h of word s / 4 (4 codes per byte)
    auto frag = [&](const uint64_t* word, bool valid, v4i32* f) {
        if constexpr (TAB) {
#pragma unroll
            for (int s2 = 0; s2 < KS; ++s2) {
                const v4i32 z = {0, 0, 0, 0};
                const uint32_t byte = (uint32_t)(word[s2 / 4] >> (16 * (s2 % 4) + 8 * h)) & 0xFFu;
                f[s2] = valid ? ohtab[byte] : z;
            }
        } else {
            static_assert(TAB || NW == 1, "the arithmetic one-hot build is one-word only");
            onehot_frag<KS>(word[0], valid, P, h, f);
        }
    };
    v4i32 A[RB][KS];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
        const uint64_t i = row0 + (wave * RB + rb) * 32 + r;
        uint64_t rw[NW];
#pragma unroll
        for (int w = 0; w < NW; ++w) rw[w] = (i < a.n && (uint32_t)w < a.W) ? a.words[i * a.wpr + w] : 0ull;
        frag(rw, i < a.n, A[rb]);
    }
    __syncthreads();
    // hit iff matches >= thr.  The accumulators start at 128 - thr, so a hit is bit 7 of the
    // result (results stay in [96, 160]) and one OR-reduction of the 16 registers tests a tile.
    // thr <= 0 (max distance >= P): every pair hits; thr = 0 flags them all.
    const int thr = max(0, (int)P - (int)a.k) + (TAB ? 8 * KS - (int)P : 0);
    v16i32 Cinit;
#pragma unroll
    for (int q = 0; q < 16; ++q) Cinit[q] = 128 - thr;
    const uint32_t ncb = (uint32_t)min<uint64_t>(S / 32, (a.n - col0 + 31) / 32);
    for (uint32_t cb = 0; cb < ncb; ++cb) {
        const uint32_t cl = cb * 32 + r;                 // this lane's column (local)
        v4i32 B[KS];
        frag(&cw[cl * NW], TAB ? true : col0 + cl < a.n, B);   // TAB: a padding column is "A..A" (filtered)
        // RB >= 4 (short reads): all RB tiles of the column block first, one ballot for all of
        // them: no branch between the tiles' MFMA chains, so they interleave; a hit (rare)
        // recomputes the tiles below.  (100k x 12 nt: 14.7 -> 15.6 T pairs/s; at RB <= 2 the
        // per-tile form measured faster.  Two tiles' chains explicitly interleaved with independent
        // accumulators measured level at RB 8, slower at RB 4: profiles/r2/r2f/tune_ap_pair.log.)
        if constexpr (RB >= 4) {
            int any_all = 0;
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) {
                v16i32 D = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[rb][0], B[0], Cinit, 0, 0, 0);
#pragma unroll
                for (int s2 = 1; s2 < KS; ++s2) D = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[rb][s2], B[s2], D, 0, 0, 0);
#pragma unroll
                for (int q = 0; q < 16; ++q) any_all |= D[q];
            }
            if (!__ballot(any_all & 128)) continue;
        }
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
            v16i32 D = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[rb][0], B[0], Cinit, 0, 0, 0);
#pragma unroll
            for (int s2 = 1; s2 < KS; ++s2) D = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[rb][s2], B[s2], D, 0, 0, 0);
            int any = D[0];
#pragma unroll
            for (int q = 1; q < 16; ++q) any |= D[q];
            if (!__ballot(any & 128)) continue;
            // hit path (rare): the 16 results go through a per-wave LDS stash into an out-of-line
            // loop, so the common path keeps its registers
            int* st = stash + wave * 1024;
#pragma unroll
            for (int q = 0; q < 16; ++q) st[q * 64 + lane] = D[q];
            ap_hits(a, st, (wave * RB + rb) * 32, cl, row0, col0, diag, rowcnt, colcnt, &blkhits);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0 && blkhits) atomicAdd(a.npairs, blkhits);
    if (a.counts) {
        for (int c = threadIdx.x; c < S; c += 256) {
            if (rowcnt[c]) atomicAdd(&a.counts[row0 + c], rowcnt[c]);
            if (colcnt[c]) atomicAdd(&a.counts[col0 + c], colcnt[c]);
        }
    }
}

// row blocks per wave: more A reuse for short reads, fewer registers for long ones
// (tools/tune_allpairs.hip: KS 2 -> RB 8, KS 4 -> RB 2)
template <int KS, int RB = (KS <= 2 ? 8 : (KS == 3 ? 4 : (KS == 4 ? 2 : 1))), bool TAB = true>
int launch_allpairs_mfma(AllPairsArgs a, uint32_t P, hipStream_t s) {
    constexpr int S = 4 * RB * 32;
    const uint64_t t = (a.n + S - 1) / S;
    if (t > 65535) return ss_fail(SS_EARG, "all-pairs: n too large for one launch (split the batch)");
    const uint64_t tri = t * (t + 1) / 2;
    // measured: the 1-D triangle is faster at RB <= 2 (50k x 32 nt 7.45 -> 8.16 T pairs/s, 20k x 96 nt
    // 1.80 -> 1.92), slower at RB 8 (100k x 12 nt 15.6 -> 13.3), where the square grid stays
    constexpr bool TRI = RB <= 2;
    const dim3 grid = (TRI && t > 1 && tri * 256 < (1ull << 32)) ? dim3((unsigned)tri) : dim3((unsigned)t, (unsigned)t);
    hipLaunchKernelGGL((k_allpairs_mfma<KS, RB, TAB, TRI>), grid, dim3(256), 0, s, a, P);
    return ss_check(hipGetLastError(), "k_allpairs_mfma");
}

template <int WT, int R>
int launch_allpairs(AllPairsArgs a, hipStream_t s) {
    constexpr int S = Tile<WT, R>::S;
    const uint64_t t = (a.n + S - 1) / S;
    if (t > 65535) return ss_fail(SS_EARG, "all-pairs: n too large for one launch (split the batch)");
    a.ntiles = (uint32_t)t;
    hipLaunchKernelGGL((k_allpairs<WT, R>), dim3((unsigned)t, (unsigned)t), dim3(256), 0, s, a);
    return ss_check(hipGetLastError(), "k_allpairs");
}

// ------------------------------------------------------------------------------------------------
// Pigeonhole form (one-word reads, small max_dist k): split the P compared positions into G = k + 1
// contiguous segments.  Two reads within distance k differ in at most k positions, so at least one
// segment is equal in both.  Per segment g the reads are bucketed by that segment's value (counting
// sort: histogram -> tile sums -> scan -> scatter of {word, index}); only pairs sharing a bucket are
// candidates, and a candidate (i, j) is reported by segment g only when segment g is equal and
// every segment g' < g differs (the pair's first equal segment), so each pair is reported once.
// Work is sum over buckets of c (c - 1) / 2 per segment instead of n (n - 1) / 2: for n random UMIs
// of 12 nt and k = 1, 2 segments of 6 nt (the alias position L joins the last), ~n^2 / 4096
// candidates.  Skewed batches (one UMI repeated many times, low-complexity segments) make buckets
// large; AUTO reads the candidate totals back after the histogram and hands such batches to the
// tiled MFMA form.  Kernels: k_pig_hist (bucket counts, each read's rank), k_pig_tile (tile sums;
// its last block scans them), k_pig_apply (bucket starts), k_pig_scatter, k_pig_pairs.
// Buckets: the segment value itself when it has <= nbmax bits, else a 64-bit multiplicative hash of
// it (colliding values only add candidates: the equality test is on the segment value).
// ------------------------------------------------------------------------------------------------
constexpr int kPigMaxG = 16;
constexpr uint32_t kPigTile = 4096;      // buckets per scan tile: 256 threads x 16
constexpr uint32_t kPigMaxBits = 22;     // <= 1024 tiles per segment (4 per thread of the scanning block)
constexpr uint64_t kPigRatio = 16;       // auto: pigeonhole when candidates < all pairs / kPigRatio

struct PigArgs {
    const uint64_t* words;
    uint64_t n;
    uint32_t wpr, k, G, nbmax, maxtiles, exact;   // exact: bit g = segment g buckets by value
    uint32_t shift[kPigMaxG], nb[kPigMaxG];
    uint64_t mask[kPigMaxG];
    // multi-word reads (W = 2 .. 4, L 33 .. 128; k_pigw_*): segment g = positions [seg[g], seg[g + 1])
    // of the row's 32 W positions (it may cross a word boundary)
    uint32_t W;
    uint32_t seg[kPigMaxG + 1];
    uint32_t* hist;       // G << nbmax: counts, then bucket starts (k_pig_apply)
    uint32_t* tile_cnt;   // G * maxtiles: bucket sums, then tile bases
    uint64_t* tile_cand;  // G * maxtiles
    uint64_t* cand;       // G: candidate pairs per segment
    uint32_t* done;       // k_pig_tile's finished-block count (zeroed with hist)
    uint32_t zero_out;    // k_pig_hist zeroes counts and *npairs (the entry point left them)
    uint64_t* sw;         // G * n words in bucket order
    uint32_t* sid;        // G * n read indices in bucket order
    uint32_t* rank;       // G * n: read i's rank in its bucket of segment g (k_pig_hist's atomics)
    uint32_t* counts;
    uint32_t* pairs;
    uint64_t max_pairs;
    unsigned long long* npairs;
};

__device__ __forceinline__ uint64_t shfl64x(uint64_t v, int o) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, o), hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), o);
    return (uint64_t)hi << 32 | lo;
}
__device__ __forceinline__ uint64_t pig_key(const PigArgs& a, uint32_t g, uint64_t w) {
    return (w >> a.shift[g]) & a.mask[g];
}
__device__ __forceinline__ uint32_t pig_bucket(const PigArgs& a, uint32_t g, uint64_t w) {
    const uint64_t key = pig_key(a, g, w);
    return (a.exact >> g) & 1u ? (uint32_t)key : (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> (64 - a.nb[g]));
}

__global__ __launch_bounds__(256) void k_pig_hist(PigArgs a) {
    if (a.zero_out && blockIdx.x == 0 && threadIdx.x == 0) *a.npairs = 0ull;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < a.n; i += (uint64_t)gridDim.x * 256) {
        if (a.zero_out && a.counts) a.counts[i] = 0u;
        const uint64_t w = a.words[i * a.wpr];
        for (uint32_t g = 0; g < a.G; ++g)
            a.rank[g * a.n + i] = atomicAdd(&a.hist[((uint64_t)g << a.nbmax) + pig_bucket(a, g, w)], 1u);
    }
}

// block sums of a 256-thread block: returns the total to every thread
template <typename T>
__device__ __forceinline__ T block_sum256(T v, T* red) {
    for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63u) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    const T t = red[0] + red[1] + red[2] + red[3];
    __syncthreads();
    return t;
}

// per tile of 4096 buckets: number of reads and candidate pairs; the grid's last block to finish
// then scans every segment's tile sums (<= 1024 tiles: 4 per thread) into tile bases and the
// segment's candidate total -- no separate scan launch
__global__ __launch_bounds__(256) void k_pig_tile(PigArgs a) {
    const uint32_t g = blockIdx.y, t0 = blockIdx.x * kPigTile, nbk = 1u << a.nb[g];
    __shared__ uint32_t r32[4];
    __shared__ uint64_t r64[4];
    __shared__ uint32_t s_last;
    if (t0 < nbk) {
        const uint32_t* h = a.hist + ((uint64_t)g << a.nbmax) + t0;
        uint32_t c = 0;
        uint64_t cand = 0;
        for (uint32_t j = threadIdx.x; j < kPigTile && t0 + j < nbk; j += 256) {
            const uint64_t v = h[j];
            c += (uint32_t)v;
            cand += v * (v - (v ? 1 : 0)) / 2;
        }
        c = block_sum256(c, r32);
        cand = block_sum256(cand, r64);
        if (threadIdx.x == 0) {
            a.tile_cnt[g * a.maxtiles + blockIdx.x] = c;
            a.tile_cand[g * a.maxtiles + blockIdx.x] = cand;
        }
    }
    if (threadIdx.x == 0) {
        __threadfence();                                          // this block's sums before its count
        s_last = atomicAdd(a.done, 1u) + 1u == gridDim.x * gridDim.y;
    }
    __syncthreads();
    if (!s_last) return;
    __threadfence();                                              // every block's sums visible
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    for (uint32_t gg = 0; gg < a.G; ++gg) {
        const uint32_t nt = ((1u << a.nb[gg]) + kPigTile - 1) / kPigTile;
        uint32_t* tc = a.tile_cnt + gg * a.maxtiles;
        uint64_t* td = a.tile_cand + gg * a.maxtiles;
        uint32_t v[4], sum = 0;
        uint64_t cand = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t t = 4 * threadIdx.x + k;
            // device-scope loads (other blocks wrote them): past this CU's cache
            v[k] = t < nt ? __hip_atomic_load(&tc[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
            cand += t < nt ? __hip_atomic_load(&td[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
            sum += v[k];
        }
        uint32_t inc = sum;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(inc, o);
            if (lane >= (uint32_t)o) inc += y;
        }
        if (lane == 63) r32[wv] = inc;
        const uint64_t ctot = block_sum256(cand, r64);              // (its barriers order r32 too)
        uint32_t run = inc - sum;
        for (uint32_t i = 0; i < wv; ++i) run += r32[i];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t t = 4 * threadIdx.x + k;
            if (t < nt) tc[t] = run;
            run += v[k];
        }
        if (threadIdx.x == 0) a.cand[gg] = ctot;
        __syncthreads();                                          // r32 of the next segment
    }
}

// bucket starts: each thread owns 16 consecutive buckets of the tile
__global__ __launch_bounds__(256) void k_pig_apply(PigArgs a) {
    const uint32_t g = blockIdx.y, t0 = blockIdx.x * kPigTile, nbk = 1u << a.nb[g];
    if (t0 >= nbk) return;
    uint32_t* h = a.hist + ((uint64_t)g << a.nbmax) + t0;
    const uint32_t b0 = threadIdx.x * 16u;
    const uint32_t m = b0 < nbk - t0 ? min(16u, nbk - t0 - b0) : 0u;
    uint32_t v[16];
    uint32_t s = 0;
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
        v[j] = j < m ? h[b0 + j] : 0u;
        s += v[j];
    }
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    uint32_t inc = s;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o);
        if (lane >= (uint32_t)o) inc += y;
    }
    __shared__ uint32_t ws[4];
    if (lane == 63) ws[wv] = inc;
    __syncthreads();
    uint32_t run = a.tile_cnt[g * a.maxtiles + blockIdx.x] + inc - s;
    for (uint32_t i = 0; i < wv; ++i) run += ws[i];
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
        if (j < m) h[b0 + j] = run;
        run += v[j];
    }
}

__global__ __launch_bounds__(256) void k_pig_scatter(PigArgs a) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < a.n; i += (uint64_t)gridDim.x * 256) {
        const uint64_t w = a.words[i * a.wpr];
        for (uint32_t g = 0; g < a.G; ++g) {
            const uint32_t pos = a.hist[((uint64_t)g << a.nbmax) + pig_bucket(a, g, w)] + a.rank[g * a.n + i];
            a.sw[g * a.n + pos] = w;
            a.sid[g * a.n + pos] = (uint32_t)i;
        }
    }
}

// Hit output of a wave without one global atomic per hit ballot: pairs gather in a per-wave LDS
// buffer and leave in runs (one pair-counter atomic per run of up to kPairBuf); count-only calls keep
// the wave's hit count in a register and add it once.
constexpr uint32_t kPairBuf = 512;
constexpr uint64_t kPigTileWalk = 256;     // a wave's entry run past this: walked as broadcast tiles
struct WaveHits {
    uint2* buf;          // this wave's kPairBuf LDS entries
    uint32_t fill = 0;   // wave-uniform
    uint64_t nh = 0;     // wave-uniform (count-only)
};
__device__ __forceinline__ void lds_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ void hits_flush(const PigArgs& a, WaveHits& wh) {
    if (!wh.fill) return;
    lds_wave_sync();
    const uint32_t lane = threadIdx.x & 63u;
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(a.npairs, (unsigned long long)wh.fill);
    base = __shfl(base, 0);
    for (uint32_t e = lane; e < wh.fill; e += 64) {
        const uint64_t slot = base + e;
        if (slot < a.max_pairs) {
            const uint2 pr = wh.buf[e];
            a.pairs[2 * slot] = pr.x;
            a.pairs[2 * slot + 1] = pr.y;
        }
    }
    lds_wave_sync();
    wh.fill = 0;
}
__device__ __forceinline__ void hits_add(const PigArgs& a, WaveHits& wh, bool hit, uint64_t mask, uint32_t i, uint32_t j) {
    const uint32_t c = (uint32_t)__popcll(mask);
    if (!a.pairs) {
        wh.nh += c;
        return;
    }
    if (wh.fill + c > kPairBuf) hits_flush(a, wh);
    const uint32_t lane = threadIdx.x & 63u;
    if (hit) wh.buf[wh.fill + __popcll(mask & ((1ull << lane) - 1ull))] = make_uint2(min(i, j), max(i, j));
    wh.fill += c;
}

// one lane per read in bucket order of segment g = blockIdx.y, compared with the reads after it in its
// bucket (see the walk below).  Hits leave through wave ballots into the wave's hit buffer; a
// count-only call sums the block's hits in LDS and adds them with one atomic per block (one per
// wave on the single pair counter measured a third of the kernel).
template <int GM>   // G <= GM segments: the first-equal-segment test unrolled over GM - 1 masks
__global__ __launch_bounds__(256) void k_pig_pairs(PigArgs a) {
    __shared__ uint2 pbuf[4][kPairBuf];
    __shared__ unsigned long long s_hits;
    if (threadIdx.x == 0) s_hits = 0;
    __syncthreads();
    const uint32_t g = blockIdx.y, lane = threadIdx.x & 63u;
    // the wave's first position, made scalar (threadIdx.x & ~63 is wave-uniform)
    const uint64_t p0 = (uint64_t)blockIdx.x * 256 + (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x & ~63u));
    const uint64_t p = p0 + lane;
    const bool valid = p < a.n;                              // (a wave past the batch walks nothing)
    const uint64_t* sw = a.sw + g * a.n;
    const uint32_t* sid = a.sid + g * a.n;
    const uint32_t* start = a.hist + ((uint64_t)g << a.nbmax);
    const uint32_t nbk = 1u << a.nb[g];
    const uint64_t w = valid ? sw[p] : 0ull;
    const uint32_t id = valid ? sid[p] : 0u;
    const uint32_t b = pig_bucket(a, g, w);
    uint64_t end = valid ? (b + 1 < nbk ? start[b + 1] : a.n) : 0ull;
    // segment h's positions as one bit per position (the low bit of its 2-bit code): with
    // d = the positions where two words differ, the pair is segment g's iff d misses segment g and
    // meets every segment before it (g is the pair's first equal segment) and popcount(d) <= k
    constexpr uint64_t kLo = 0x5555555555555555ull;
    uint64_t segm[GM];
#pragma unroll
    for (int h = 0; h < GM; ++h) segm[h] = (uint32_t)h < g ? (a.mask[h] << a.shift[h]) & kLo : 0ull;
    const uint64_t mg = (a.mask[g] << a.shift[g]) & kLo;
    const uint32_t kmax = (uint32_t)__builtin_amdgcn_readfirstlane((int)a.k);
    WaveHits wh;
    wh.buf = pbuf[threadIdx.x >> 6];
    uint32_t row = 0;
    // the wave's run of entries, [p0 + 1, its largest bucket end): long (large buckets: heavy
    // duplicates, short segments) -> the wave walks it in 64-entry tiles, one coalesced load per tile
    // and each entry broadcast to the wave by v_readlane (the 64 compares of a tile wait on no
    // memory); short (the UMI case) -> each lane walks its own run (below)
    uint64_t wend = end;
    for (int o = 32; o; o >>= 1) {
        const uint64_t y = shfl64x(wend, o);
        wend = y > wend ? y : wend;
    }
    wend = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(wend >> 32)) << 32 |
           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)wend);   // uniform: scalar loop bounds
    if (wend > p0 + kPigTileWalk) {
        for (uint64_t t0 = p0 + 1; t0 < wend; t0 += 64) {
            const uint64_t qt = t0 + lane;
            const uint64_t tw = qt < a.n ? sw[qt] : 0ull;
            const uint32_t tid = qt < a.n ? sid[qt] : 0u;
            const uint32_t twl = (uint32_t)tw, twh = (uint32_t)(tw >> 32);
            const uint32_t ne = (uint32_t)((wend - t0) < 64 ? (wend - t0) : 64);
            for (uint32_t e = 0; e < ne; ++e) {
                const uint64_t q = t0 + e;
                const uint64_t w2 = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)twh, (int)e) << 32 |
                                    (uint32_t)__builtin_amdgcn_readlane((int)twl, (int)e);
                const uint64_t x = w ^ w2, d = (x | (x >> 1)) & kLo;
                bool hit = (q > p) & (q < end) & ((uint32_t)__popcll(d) <= kmax) & !(d & mg);
#pragma unroll
                for (int h = 0; h < GM - 1; ++h) hit = hit && ((uint32_t)h >= g || (d & segm[h]) != 0ull);
                const uint64_t mask = __ballot(hit);
                if (!mask) continue;
                const uint32_t jd = (uint32_t)__builtin_amdgcn_readlane((int)tid, (int)e);
                row += hit ? 1u : 0u;
                if (a.counts && lane == (uint32_t)__ffsll((unsigned long long)mask) - 1u)
                    atomicAdd(&a.counts[jd], (uint32_t)__popcll(mask));
                hits_add(a, wh, hit, mask, id, jd);
            }
        }
        end = 0;                                           // (the lane walk below has nothing left)
    }
    // each lane walks its own bucket run (p, end): consecutive lanes read consecutive entries, so a
    // step's 64 loads are one coalesced run; kPigStep entries per step, the next step's in flight
    constexpr int kPigStep = 4;
    uint64_t nx[kPigStep];
#pragma unroll
    for (int u = 0; u < kPigStep; ++u) nx[u] = p + 1 + u < end ? sw[p + 1 + u] : 0ull;
    for (uint64_t q0 = p + 1;; q0 += kPigStep) {
        if (!__ballot(q0 < end)) break;
        uint64_t cur[kPigStep];
#pragma unroll
        for (int u = 0; u < kPigStep; ++u) {
            cur[u] = nx[u];
            const uint64_t qn = q0 + kPigStep + u;
            nx[u] = qn < end ? sw[qn] : 0ull;
        }
#pragma unroll
        for (int u = 0; u < kPigStep; ++u) {
            const uint64_t q = q0 + u;
            const uint64_t x = w ^ cur[u], d = (x | (x >> 1)) & kLo;
            bool hit = (q < end) & ((uint32_t)__popcll(d) <= kmax) & !(d & mg);
#pragma unroll
            for (int h = 0; h < GM - 1; ++h) hit = hit && ((uint32_t)h >= g || (d & segm[h]) != 0ull);
            const uint64_t mask = __ballot(hit);
            if (!mask) continue;
            const uint32_t jd = hit ? sid[q] : 0u;
            row += hit ? 1u : 0u;
            if (hit && a.counts) atomicAdd(&a.counts[jd], 1u);
            hits_add(a, wh, hit, mask, id, jd);
        }
    }
    if (a.pairs) hits_flush(a, wh);
    else if (lane == 0 && wh.nh) atomicAdd(&s_hits, (unsigned long long)wh.nh);
    if (a.counts && row) atomicAdd(&a.counts[id], row);
    __syncthreads();
    if (threadIdx.x == 0 && s_hits) atomicAdd(a.npairs, s_hits);
}

// ---- Multi-word reads (W = 2 .. 4 words: 33 .. 128 nt).  The same pigeonhole
// argument over the P = min(L + 1, 32 W) compared positions of the row: G = k + 1 contiguous segments
// (a segment may cross a word boundary and be longer than 32 positions).  A segment's bucket is its
// value when it has <= nbmax bits, else a hash of its (up to 128-bit) value; equality, the distance
// and the first-equal-segment rule are decided on the words of both rows, so a hash collision only
// adds candidates.  Rows live W words apiece in the bucket-ordered arrays (sw: G x n x W words).
template <int W>
__device__ __forceinline__ void pig_row(const PigArgs& a, uint64_t i, uint64_t (&w)[W]) {
#pragma unroll
    for (int q = 0; q < W; ++q) w[q] = a.words[i * a.wpr + q];
}
// bits [2 b0, 2 b0 + 64) of a row (b0 in positions, < 32 W)
template <int W>
__device__ __forceinline__ uint64_t row_bits64(const uint64_t (&w)[W], uint32_t b0) {
    const uint32_t q = b0 >> 5, sh = 2u * (b0 & 31u);
    uint64_t lo = 0, hi = 0;
#pragma unroll
    for (int k = 0; k < W; ++k) {
        if ((uint32_t)k == q) lo = w[k];
        if ((uint32_t)k == q + 1u) hi = w[k];
    }
    return sh ? (lo >> sh) | (hi << (64u - sh)) : lo;
}
template <int W>
__device__ __forceinline__ uint32_t pigw_bucket(const PigArgs& a, uint32_t g, const uint64_t (&w)[W]) {
    const uint32_t p0 = a.seg[g], len = a.seg[g + 1] - p0;
    if ((a.exact >> g) & 1u) return (uint32_t)(row_bits64<W>(w, p0) & ((1ull << (2u * len)) - 1ull));
    uint64_t h = 0x243F6A8885A308D3ull ^ len;
    for (uint32_t b = 0; b < len; b += 32) {          // the segment's 64-bit pieces, the last masked
        const uint32_t m = len - b < 32u ? len - b : 32u;
        uint64_t v = row_bits64<W>(w, p0 + b);
        if (m < 32u) v &= (1ull << (2u * m)) - 1ull;
        h = (h ^ v) * 0x9E3779B97F4A7C15ull;
        h ^= h >> 29;
    }
    return (uint32_t)(h >> (64 - a.nb[g]));
}

template <int W>
__global__ __launch_bounds__(256) void k_pigw_hist(PigArgs a) {
    if (a.zero_out && blockIdx.x == 0 && threadIdx.x == 0) *a.npairs = 0ull;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < a.n; i += (uint64_t)gridDim.x * 256) {
        if (a.zero_out && a.counts) a.counts[i] = 0u;
        uint64_t w[W];
        pig_row<W>(a, i, w);
        for (uint32_t g = 0; g < a.G; ++g)
            a.rank[g * a.n + i] = atomicAdd(&a.hist[((uint64_t)g << a.nbmax) + pigw_bucket<W>(a, g, w)], 1u);
    }
}

template <int W>
__global__ __launch_bounds__(256) void k_pigw_scatter(PigArgs a) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < a.n; i += (uint64_t)gridDim.x * 256) {
        uint64_t w[W];
        pig_row<W>(a, i, w);
        for (uint32_t g = 0; g < a.G; ++g) {
            const uint64_t pos = a.hist[((uint64_t)g << a.nbmax) + pigw_bucket<W>(a, g, w)] + a.rank[g * a.n + i];
            uint64_t* dst = a.sw + ((uint64_t)g * a.n + pos) * W;
#pragma unroll
            for (int q = 0; q < W; ++q) dst[q] = w[q];
            a.sid[g * a.n + pos] = (uint32_t)i;
        }
    }
}

// one lane per row in bucket order of segment g = blockIdx.y, each walking its own bucket run (p, end)
// with kPigStep rows in flight (consecutive lanes on consecutive rows: coalesced).  A candidate is a
// hit when its distance is <= k and g is the first segment the rows agree on: the <= k differing
// positions are walked and their segments marked (segment of a position: the boundaries in a.seg).
template <int W>
__global__ __launch_bounds__(256) void k_pigw_pairs(PigArgs a) {
    __shared__ uint2 pbuf[4][kPairBuf];
    __shared__ unsigned long long s_hits;
    if (threadIdx.x == 0) s_hits = 0;
    __syncthreads();
    const uint32_t g = blockIdx.y, lane = threadIdx.x & 63u;
    const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const bool valid = p < a.n;
    const uint64_t* sw = a.sw + (uint64_t)g * a.n * W;
    const uint32_t* sid = a.sid + g * a.n;
    const uint32_t* start = a.hist + ((uint64_t)g << a.nbmax);
    const uint32_t nbk = 1u << a.nb[g];
    uint64_t w[W];
#pragma unroll
    for (int q = 0; q < W; ++q) w[q] = valid ? sw[p * W + q] : 0ull;
    const uint32_t id = valid ? sid[p] : 0u;
    const uint32_t b = pigw_bucket<W>(a, g, w);
    const uint64_t end = valid ? (b + 1 < nbk ? start[b + 1] : a.n) : 0ull;
    constexpr uint64_t kLo = 0x5555555555555555ull;
    const uint32_t kmax = (uint32_t)__builtin_amdgcn_readfirstlane((int)a.k);
    const uint32_t want = (1u << g) - 1u;             // segments 0 .. g - 1 differ, g agrees
    WaveHits wh;
    wh.buf = pbuf[threadIdx.x >> 6];
    uint32_t row = 0;
    constexpr int kPigStep = 4;
    uint64_t nx[kPigStep][W];
#pragma unroll
    for (int u = 0; u < kPigStep; ++u)
#pragma unroll
        for (int q = 0; q < W; ++q) nx[u][q] = p + 1 + u < end ? sw[(p + 1 + u) * W + q] : 0ull;
    for (uint64_t q0 = p + 1;; q0 += kPigStep) {
        if (!__ballot(q0 < end)) break;
        uint64_t cur[kPigStep][W];
#pragma unroll
        for (int u = 0; u < kPigStep; ++u) {
            const uint64_t qn = q0 + kPigStep + u;
#pragma unroll
            for (int q = 0; q < W; ++q) {
                cur[u][q] = nx[u][q];
                nx[u][q] = qn < end ? sw[qn * W + q] : 0ull;
            }
        }
#pragma unroll
        for (int u = 0; u < kPigStep; ++u) {
            const uint64_t qq = q0 + u;
            uint64_t d[W];
            uint32_t dd = 0;
#pragma unroll
            for (int q = 0; q < W; ++q) {
                const uint64_t x = w[q] ^ cur[u][q];
                d[q] = (x | (x >> 1)) & kLo;
                dd += (uint32_t)__popcll(d[q]);
            }
            bool hit = (qq < end) & (dd <= kmax);
            if (hit) {     // the segments the differing positions fall in
                uint32_t segs = 0;
#pragma unroll
                for (int q = 0; q < W; ++q) {
                    uint64_t m = d[q];
                    while (m) {
                        const uint32_t pos = 32u * q + ((uint32_t)__ffsll((long long)m) - 1u) / 2u;
                        uint32_t sgi = 0;
                        while (sgi + 1 < a.G && pos >= a.seg[sgi + 1]) ++sgi;
                        segs |= 1u << sgi;
                        m &= m - 1ull;
                    }
                }
                hit = (segs & (want | (1u << g))) == want;
            }
            const uint64_t mask = __ballot(hit);
            if (!mask) continue;
            const uint32_t jd = hit ? sid[qq] : 0u;
            row += hit ? 1u : 0u;
            if (hit && a.counts) atomicAdd(&a.counts[jd], 1u);
            hits_add(a, wh, hit, mask, id, jd);
        }
    }
    if (a.pairs) hits_flush(a, wh);
    else if (lane == 0 && wh.nh) atomicAdd(&s_hits, (unsigned long long)wh.nh);
    if (a.counts && row) atomicAdd(&a.counts[id], row);
    __syncthreads();
    if (threadIdx.x == 0 && s_hits) atomicAdd(a.npairs, s_hits);
}

// Per-device scratch of the pigeonhole form, grow-only and stream-ordered: a call holds the device's
// lock, waits (on its stream) for the previous call's kernels before reusing the buffer, and records
// its own end.
struct PigScratch {
    std::mutex mu;
    void* p = nullptr;
    size_t bytes = 0;
    hipEvent_t done = nullptr;
    uint64_t* h_cand = nullptr;   // pinned: the candidate totals read back
};
PigScratch g_pig[64];

// returns 0 with *done = false when the auto choice hands the batch to the tiled form
int pig_all_pairs(const AllPairsArgs& b, uint32_t L, uint32_t P, bool forced, hipStream_t s, bool* done) {
    *done = false;
    PigArgs a{};
    a.words = b.words;
    a.n = b.n;
    a.wpr = b.wpr;
    a.k = b.k;
    a.G = b.k + 1;
    a.counts = b.counts;
    a.pairs = b.pairs;
    a.max_pairs = b.max_pairs;
    a.npairs = b.npairs;
    a.zero_out = 1;
    a.W = b.W;
    uint32_t lg = 0;
    while ((1ull << lg) < a.n) ++lg;
    a.nbmax = lg < 10 ? 10 : (lg > kPigMaxBits ? kPigMaxBits : lg);
    a.maxtiles = ((1u << a.nbmax) + kPigTile - 1) / kPigTile;
    // the L read positions split evenly (the first L % G segments one longer); the alias position L
    // (P = L + 1: nearly always code 0, so no bucketing entropy) joins the last segment
    const uint32_t Lr = P < L ? P : L;
    for (uint32_t g = 0, pos = 0; g < a.G; ++g) {
        uint32_t len = Lr / a.G + (g < Lr % a.G ? 1u : 0u);
        if (g + 1 == a.G) len = P - pos;
        a.shift[g] = 2 * pos;
        a.mask[g] = len >= 32 ? ~0ull : ((1ull << (2 * len)) - 1ull);
        a.nb[g] = 2 * len < a.nbmax ? 2 * len : a.nbmax;
        if (2 * len <= a.nbmax) a.exact |= 1u << g;
        a.seg[g] = pos;
        pos += len;
    }
    a.seg[a.G] = P;
    // the scratch, its event and the pinned totals belong to the device that holds the words (the
    // kernels run there, on the caller's stream), not to whichever device is current
    int cur = 0, dev = 0;
    int rc = ss_check(hipGetDevice(&cur), "hipGetDevice");
    if (rc) return rc;
    hipPointerAttribute_t pa{};
    rc = ss_check(hipPointerGetAttributes(&pa, b.words), "all-pairs: words pointer attributes");
    if (rc) return rc;
    dev = pa.device;
    if (dev < 0 || dev >= 64) return ss_fail(SS_EARG, "all-pairs: device index past 63");
    struct DevGuard {
        int prev, now;
        ~DevGuard() {
            if (prev != now) (void)hipSetDevice(prev);
        }
    } guard{cur, dev};
    if (dev != cur) {
        rc = ss_check(hipSetDevice(dev), "all-pairs: hipSetDevice");
        if (rc) return rc;
    }
    PigScratch& ps = g_pig[dev];
    std::lock_guard<std::mutex> lock(ps.mu);
    const size_t hist_n = (size_t)a.G << a.nbmax, tiles_n = (size_t)a.G * a.maxtiles;
    const size_t need = tiles_n * 8 + a.G * 8 + (hist_n + 2) * 4 + tiles_n * 4 + 64 + (size_t)a.G * a.n * (8 * a.W + 8);
    if (!ps.done) rc = ss_check(hipEventCreateWithFlags(&ps.done, hipEventDisableTiming), "pig event");
    if (!rc && !ps.h_cand) rc = ss_check(hipHostMalloc((void**)&ps.h_cand, kPigMaxG * 8, hipHostMallocDefault), "pinned totals");
    if (!rc && ps.bytes < need) {
        if (ps.p) {
            rc = ss_check(hipEventSynchronize(ps.done), "pig scratch idle");
            if (!rc) rc = ss_check(hipFree(ps.p), "pig scratch free");
            ps.p = nullptr;
            ps.bytes = 0;
        }
        const size_t want = need + need / 4;
        if (!rc && hipMalloc(&ps.p, want) != hipSuccess) {
            (void)hipGetLastError();
            ps.p = nullptr;
            if (forced) return ss_fail(SS_ENOMEM, "pigeonhole all-pairs scratch: out of device memory");
            // auto: the tiled form needs no scratch; it gets the outputs zeroed as the entry skipped that
            rc = ss_check(hipMemsetAsync(a.npairs, 0, sizeof(uint64_t), s), "npairs reset");
            if (!rc && a.counts) rc = ss_check(hipMemsetAsync(a.counts, 0, a.n * sizeof(uint32_t), s), "counts reset");
            return rc;
        }
        if (!rc) ps.bytes = want;
    } else if (!rc) {
        rc = ss_check(hipStreamWaitEvent(s, ps.done, 0), "pig scratch wait");
    }
    if (rc) return rc;
    char* q = (char*)ps.p;
    a.tile_cand = (uint64_t*)q;
    a.cand = a.tile_cand + tiles_n;
    a.sw = a.cand + a.G;
    a.hist = (uint32_t*)(a.sw + (size_t)a.G * a.n * a.W);
    a.done = a.hist + hist_n;                 // zeroed with hist
    a.tile_cnt = a.done + 2;
    a.sid = a.tile_cnt + tiles_n;
    a.rank = a.sid + (size_t)a.G * a.n;
    const unsigned rgrid = (unsigned)std::min<uint64_t>((a.n + 255) / 256, 2048);
    const dim3 tgrid(a.maxtiles, a.G);
    rc = ss_check(hipMemsetAsync(a.hist, 0, (hist_n + 2) * 4, s), "pig hist reset");
    if (!rc) {
        if (a.W == 1) hipLaunchKernelGGL(k_pig_hist, dim3(rgrid), dim3(256), 0, s, a);
        else if (a.W == 2) hipLaunchKernelGGL(k_pigw_hist<2>, dim3(rgrid), dim3(256), 0, s, a);
        else if (a.W == 3) hipLaunchKernelGGL(k_pigw_hist<3>, dim3(rgrid), dim3(256), 0, s, a);
        else hipLaunchKernelGGL(k_pigw_hist<4>, dim3(rgrid), dim3(256), 0, s, a);
        hipLaunchKernelGGL(k_pig_tile, tgrid, dim3(256), 0, s, a);
        rc = ss_check(hipGetLastError(), "k_pig_hist/tile");
    }
    bool use = forced;
    if (!rc && !forced) {
        rc = ss_check(hipMemcpyAsync(ps.h_cand, a.cand, a.G * 8, hipMemcpyDeviceToHost, s), "pig totals");
        if (!rc) rc = ss_check(hipStreamSynchronize(s), "pig totals sync");
        uint64_t cand = 0;
        for (uint32_t g = 0; !rc && g < a.G; ++g) cand += ps.h_cand[g];
        // measured (tools/probe_f4.py, profiles/r5/probe_f4_*.log): see kPigRatio
        use = cand < a.n * (a.n - 1) / 2 / kPigRatio;
    }
    if (!rc && use) {
        hipLaunchKernelGGL(k_pig_apply, tgrid, dim3(256), 0, s, a);
        if (a.W == 1) hipLaunchKernelGGL(k_pig_scatter, dim3(rgrid), dim3(256), 0, s, a);
        else if (a.W == 2) hipLaunchKernelGGL(k_pigw_scatter<2>, dim3(rgrid), dim3(256), 0, s, a);
        else if (a.W == 3) hipLaunchKernelGGL(k_pigw_scatter<3>, dim3(rgrid), dim3(256), 0, s, a);
        else hipLaunchKernelGGL(k_pigw_scatter<4>, dim3(rgrid), dim3(256), 0, s, a);
        const uint64_t pb = (a.n + 255) / 256;
        if (pb > 0x7FFFFFFFull) rc = ss_fail(SS_EARG, "all-pairs: n too large");
        else if (a.W == 2) hipLaunchKernelGGL(k_pigw_pairs<2>, dim3((unsigned)pb, a.G), dim3(256), 0, s, a);
        else if (a.W == 3) hipLaunchKernelGGL(k_pigw_pairs<3>, dim3((unsigned)pb, a.G), dim3(256), 0, s, a);
        else if (a.W == 4) hipLaunchKernelGGL(k_pigw_pairs<4>, dim3((unsigned)pb, a.G), dim3(256), 0, s, a);
        else if (a.G <= 2) hipLaunchKernelGGL(k_pig_pairs<2>, dim3((unsigned)pb, a.G), dim3(256), 0, s, a);
        else if (a.G <= 4) hipLaunchKernelGGL(k_pig_pairs<4>, dim3((unsigned)pb, a.G), dim3(256), 0, s, a);
        else if (a.G <= 8) hipLaunchKernelGGL(k_pig_pairs<8>, dim3((unsigned)pb, a.G), dim3(256), 0, s, a);
        else hipLaunchKernelGGL(k_pig_pairs<kPigMaxG>, dim3((unsigned)pb, a.G), dim3(256), 0, s, a);
        if (!rc) rc = ss_check(hipGetLastError(), "k_pig_apply/scatter/pairs");
        if (!rc) *done = true;
    }
    const int r2 = ss_check(hipEventRecord(ps.done, s), "pig scratch event");
    return rc ? rc : r2;
}

}  // namespace

extern "C" {

int ss_hamming_all_pairs(const uint64_t* d_words, uint64_t n, uint32_t L, uint32_t wpr, uint32_t max_dist,
                         uint32_t* d_counts, uint32_t* d_pairs, uint64_t max_pairs, uint64_t* d_npairs,
                         void* stream) {
    return ss_hamming_all_pairs_ex(d_words, n, L, wpr, max_dist, d_counts, d_pairs, max_pairs, d_npairs,
                                   SS_ALLPAIRS_AUTO, stream);
}

int ss_hamming_all_pairs_ex(const uint64_t* d_words, uint64_t n, uint32_t L, uint32_t wpr, uint32_t max_dist,
                            uint32_t* d_counts, uint32_t* d_pairs, uint64_t max_pairs, uint64_t* d_npairs,
                            uint32_t method, void* stream) {
    if (method > SS_ALLPAIRS_PIGEONHOLE) return ss_fail(SS_EARG, "unknown all-pairs method");
    if (L > SS_MAX_NT) return ss_fail(SS_EARG, "L must be <= 1024");
    const uint32_t W = L <= 32u ? 1u : (L + 31u) / 32u;
    if (wpr < W || wpr > 32) return ss_fail(SS_EARG, "bad wpr");
    if (!d_npairs) return ss_fail(SS_EARG, "d_npairs is required");
    if (n >= (1ull << 32)) return ss_fail(SS_EARG, "n must be < 2^32");
    hipStream_t s = (hipStream_t)stream;
    // the pigeonhole form (tried first when it may apply) zeroes the outputs in its first kernel
    const uint32_t Pw = L + 1 < 32u * W ? L + 1 : 32u * W, Gw = max_dist + 1;
    // AUTO on a stream being captured into a hipGraph stays on the tiles: the pigeonhole decision
    // allocates and reads the candidate totals back (a host sync), neither of which a capture allows
    // (the entry point was capturable before AUTO existed)
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (method == SS_ALLPAIRS_AUTO && hipStreamIsCapturing((hipStream_t)stream, &cap) != hipSuccess) {
        (void)hipGetLastError();
        cap = hipStreamCaptureStatusNone;
    }
    const bool capturing = cap != hipStreamCaptureStatusNone;
    const bool pig_try = n >= 2 && W <= 4 && method != SS_ALLPAIRS_TILES && !(capturing && method == SS_ALLPAIRS_AUTO) &&
                         wpr >= W && d_words &&
                         (method == SS_ALLPAIRS_PIGEONHOLE ? Gw <= (uint32_t)kPigMaxG
                                                           : Gw <= (uint32_t)kPigMaxG && Pw / Gw >= 3 && n >= (1u << 15));
    int rc = SS_OK;
    if (!pig_try) {
        rc = ss_check(hipMemsetAsync(d_npairs, 0, sizeof(uint64_t), s), "npairs reset");
        if (!rc && d_counts && n) rc = ss_check(hipMemsetAsync(d_counts, 0, n * sizeof(uint32_t), s), "counts reset");
    }
    if (rc || n < 2) return rc;
    if (!d_words || (d_pairs && max_pairs == 0)) return ss_fail(SS_EARG, "null buffer");
    AllPairsArgs a;
    a.words = d_words;
    a.n = n;
    a.wpr = wpr;
    a.W = W;
    a.k = max_dist;
    a.ntiles = 0;
    a.counts = d_counts;
    a.pairs = d_pairs;
    a.max_pairs = d_pairs ? max_pairs : 0;
    a.npairs = (unsigned long long*)d_npairs;
    if (method == SS_ALLPAIRS_PIGEONHOLE && (W > 4 || max_dist + 1 > (uint32_t)kPigMaxG))
        return ss_fail(SS_EARG, "pigeonhole all-pairs needs L <= 128 and max_dist < 16");
    // auto: segments of >= 3 nt and a batch large enough to pay the host read of the totals
    if (pig_try) {
        bool done = false;
        rc = pig_all_pairs(a, L, Pw, method == SS_ALLPAIRS_PIGEONHOLE, s, &done);
        if (rc || done) return rc;
    }
    if (W <= 4) {
        // MFMA form: P = min(L + 1, 32 W) positions (the alias bit of the tail block can sit at
        // position L), 8 per k-step; k-steps rounded up to an instantiated count (the padding
        // positions are code 0 on both sides and shift every result by the same constant)
        const uint32_t P = L + 1 < 32u * W ? L + 1 : 32u * W;
        const uint32_t ks = (P + 7) / 8;
        if (ks <= 1) return launch_allpairs_mfma<1>(a, P, s);
        if (ks <= 2) return launch_allpairs_mfma<2>(a, P, s);
        if (ks <= 3) return launch_allpairs_mfma<3>(a, P, s);
        if (ks <= 4) return launch_allpairs_mfma<4>(a, P, s);
        if (ks <= 6) return launch_allpairs_mfma<6>(a, P, s);
        if (ks <= 8) return launch_allpairs_mfma<8>(a, P, s);
        if (ks <= 12) return launch_allpairs_mfma<12>(a, P, s);
        return launch_allpairs_mfma<16>(a, P, s);
    }
    if (W <= 8) return launch_allpairs<8, 1>(a, s);
    if (W <= 16) return launch_allpairs<16, 1>(a, s);
    return launch_allpairs<32, 1>(a, s);
}

}  // extern "C"
