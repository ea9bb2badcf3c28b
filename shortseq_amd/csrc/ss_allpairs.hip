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
    if (W == 1) return launch_allpairs<1, 4>(a, s);
    if (W == 2) return launch_allpairs<2, 4>(a, s);
    if (W <= 4) return launch_allpairs<4, 2>(a, s);
    if (W <= 8) return launch_allpairs<8, 1>(a, s);
    if (W <= 16) return launch_allpairs<16, 1>(a, s);
    return launch_allpairs<32, 1>(a, s);
}

}  // extern "C"
