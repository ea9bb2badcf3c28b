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
                    } else if (hit) {
                        atomicAdd(a.npairs, 1ull);
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
                                     uint64_t col0, bool diag, uint32_t* rowcnt, uint32_t* colcnt) {
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
        unsigned long long base = 0;
        if ((int)lane == leader) base = atomicAdd(a.npairs, (unsigned long long)__popcll(mask));
        base = __shfl(base, leader);
        if (hit && a.pairs) {
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
    const bool diag = bi == bj;
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
            ap_hits(a, st, (wave * RB + rb) * 32, cl, row0, col0, diag, rowcnt, colcnt);
        }
    }
    __syncthreads();
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

}  // namespace

extern "C" {

int ss_hamming_all_pairs(const uint64_t* d_words, uint64_t n, uint32_t L, uint32_t wpr, uint32_t max_dist,
                         uint32_t* d_counts, uint32_t* d_pairs, uint64_t max_pairs, uint64_t* d_npairs,
                         void* stream) {
    if (L > SS_MAX_NT) return ss_fail(SS_EARG, "L must be <= 1024");
    const uint32_t W = L <= 32u ? 1u : (L + 31u) / 32u;
    if (wpr < W || wpr > 32) return ss_fail(SS_EARG, "bad wpr");
    if (!d_npairs) return ss_fail(SS_EARG, "d_npairs is required");
    if (n >= (1ull << 32)) return ss_fail(SS_EARG, "n must be < 2^32");
    hipStream_t s = (hipStream_t)stream;
    int rc = ss_check(hipMemsetAsync(d_npairs, 0, sizeof(uint64_t), s), "npairs reset");
    if (!rc && d_counts && n) rc = ss_check(hipMemsetAsync(d_counts, 0, n * sizeof(uint32_t), s), "counts reset");
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
