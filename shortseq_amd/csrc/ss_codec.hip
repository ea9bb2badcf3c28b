// ss_codec.hip — batch 2-bit encode / decode / hamming / synthetic-read kernels for gfx950.
//
// Kernel families:
//   k_encode_g16   fast path, L % 16 == 0: one lane per 16-byte ASCII chunk (one dwordx4 load,
//                  fully coalesced), one u32 half-word out per lane.  Lanes are grouped per read in
//                  power-of-two groups of G >= 2*wpr lanes so carries (table path) move by one
//                  __shfl_xor and per-read sums (fused hamming) reduce inside the group.
//   k_encode_gen   any L / stride / variable lengths: one lane per output word, aligned dword
//                  loads + v_alignbyte; the general and ragged path.
//   k_ham_dense / k_ham_dense3x hamming on dense packed rows (dwordx4 streams; k_ham_group otherwise)
//   k_decode_g16 / k_decode_gen, k_ham_group, k_synth_*.
#include "ss_device.h"
#include "ss_internal.h"

namespace {

using namespace ssd;

constexpr int kThreads = 256;        // general / grid-stride kernels

__host__ __device__ inline uint32_t words_for(uint32_t L) { return (L + 31u) / 32u; }
__host__ __device__ inline uint32_t ham_words(uint32_t L) { return L <= 32u ? 1u : words_for(L); }

inline uint32_t log2_ceil(uint32_t x) {
    uint32_t l = 0;
    while ((1u << l) < x) ++l;
    return l;
}

// ------------------------------------------------------------------------------------------------
// Fast path.  Lane slot g -> read r = g >> logG, chunk k = g & (G-1).  Chunks k < cpr carry data;
// lanes cpr <= k < wpr2 produce the zero (or carry-only) padding half-words.
//   table path for chunk k iff L <= 32 (short_seq.pyx:57) or k >= full2 (tail block, util.pyx:92)
// ------------------------------------------------------------------------------------------------
struct G16Args {
    const uint4* in;          // 16-B aligned
    uint64_t in_stride16;     // read stride in 16-B chunks
    uint32_t* out32;          // packed words viewed as u32 half-words (may be null: no store)
    uint32_t wpr2;            // 2 * words per read
    uint64_t n;
    uint32_t cpr;             // L / 16
    uint32_t full2;           // 2 * (L / 32): chunks that belong to full PEXT blocks
    uint32_t all_table;       // L <= 32
    uint32_t logG;
    const uint32_t* ref32;    // fused hamming: reference half-words (wpr2 of them)
    uint32_t ham2;            // 2 * ham_words(L)
    uint32_t* counts;
    unsigned long long* first_bad;
};

// Compile-time path of every chunk of a launch (the launcher picks it from L):
//   kPathTable: L <= 32, every chunk on the table path (short_seq_64.pyx:96-108)
//   kPathPext:  L % 32 == 0 and L >= 64, every chunk a full PEXT block chunk (util.pyx:100-119):
//               no alias carries at all, so no neighbour exchange
//   kPathMixed: per chunk, k >= full2 -> table path (the L % 32 tail block, util.pyx:92-94)
enum { kPathMixed = 0, kPathTable = 1, kPathPext = 2 };

template <int PATH>
__device__ __forceinline__ uint32_t encode_chunk(const uint4& x, uint32_t k, const G16Args& a, uint32_t& bad) {
    const bool table = PATH == kPathTable ? true : (PATH == kPathPext ? false : (a.all_table || k >= a.full2));
    const Enc32 e = encode16(x.x, x.y, x.z, x.w, table);
    bad = e.bad;
    if constexpr (PATH == kPathPext) return e.v;
    const uint32_t cin = swap_pair(e.cout);            // carry from the neighbouring (lower) half
    return e.v | ((k & 1u) ? cin : 0u);
}

// XCD-contiguous block order: the dispatcher deals blocks round-robin over the 8 XCDs (observed,
// MI355X_MICROARCH.md §Workgroup dispatch; speed only, never correctness), so block b runs on XCD
// b % 8; remapping gives each XCD one contiguous eighth of the stream.
template <bool XCD>
__device__ __forceinline__ uint64_t block_order() {
    if constexpr (!XCD) return blockIdx.x;
    const uint32_t per = (gridDim.x + 7u) / 8u;
    const uint64_t b = (uint64_t)(blockIdx.x % 8u) * per + blockIdx.x / 8u;
    return b;
}

// DENSE: stride == L, wpr == L/32, L % 32 == 0 -> lane slot g IS the chunk index and the u32
// output index (no per-lane read/chunk arithmetic, a pure 16 B -> 4 B stream).
// Otherwise lane slot g -> read r = g >> logG, chunk k = g & (G-1) (G = next_pow2(2*wpr)).
template <bool HAM, bool DENSE, int PATH, int T, int U, bool XCD, bool NTST>
__global__ __launch_bounds__(T) void k_encode_g16(G16Args a) {
    const uint32_t G = 1u << a.logG;
    const uint64_t base = block_order<XCD>() * (U * T) + threadIdx.x;
    const uint64_t nslots = DENSE ? a.n * a.cpr : 0;
    uint4 x[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint64_t g = base + (uint64_t)j * T;
        if constexpr (DENSE) {
            x[j] = g < nslots ? ld_stream(&a.in[g]) : make_uint4(0x41414141u, 0x41414141u, 0x41414141u, 0x41414141u);
        } else {
            const uint64_t r = g >> a.logG;
            const uint32_t k = (uint32_t)g & (G - 1u);
            if (r < a.n && k < a.cpr)
                x[j] = ld_stream(&a.in[r * a.in_stride16 + k]);
            else
                x[j] = make_uint4(0x41414141u, 0x41414141u, 0x41414141u, 0x41414141u);  // "AAAA": code 0, valid
        }
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint64_t g = base + (uint64_t)j * T;
        const uint64_t r = g >> a.logG;
        const uint32_t k = (uint32_t)g & (G - 1u);
        uint32_t bad;
        const uint32_t v = encode_chunk<PATH>(x[j], k, a, bad);
        const bool live = DENSE ? g < nslots : r < a.n;
        if constexpr (DENSE) report_bad_div(live && bad != 0u, g, a.cpr, a.first_bad);
        else report_bad(live && bad != 0u, r, a.first_bad);
        uint32_t* dst = nullptr;
        if constexpr (DENSE) {
            if (a.out32 && live) dst = &a.out32[g];
        } else {
            if (a.out32 && live && k < a.wpr2) dst = &a.out32[r * a.wpr2 + k];
        }
        if (dst) {
            if constexpr (NTST) st_stream(dst, v);
            else *dst = v;
        }
        if constexpr (HAM) {
            uint32_t part = (k < a.ham2) ? ham32(v ^ a.ref32[k]) : 0u;
            for (uint32_t s = 1; s < G; s <<= 1) part += __shfl_xor(part, s);
            if (live && k == 0) a.counts[r] = part;
        }
    }
}

// Dense fused encode + hamming for any even chunks-per-read (e.g. 96 nt: 6 chunks = 3 words): the
// block owns rpb whole reads = rpb*cpr consecutive chunks (dense, coalesced loads/stores as in the
// DENSE encode); per-chunk distances (<= 16) go to LDS bytes, then one thread per read sums them and
// stores the read's distance (the reads of a block are contiguous: coalesced u32 stores).
// PAD8 (cpr <= 8): a read's bytes are padded to 8 (byte 8 rl + k; the unwritten bytes cpr..7 are
// masked off), so the sum is one 8-B LDS read and two v_sad_u8 instead of cpr byte reads (96 nt:
// 0.775-0.784 -> 0.790-0.795 of peak, same box, tools/tune_c3.hip); otherwise byte cl of the block's
// chunk order.
// Local read index = floor((cl + 0.5) * (1/cpr)) in f32 (exact for cl < 4096, cpr <= 64; checked
// exhaustively, and written with _rn intrinsics so no FMA contraction changes the rounding).
template <int PATH, int T, int U, bool NTST, bool PAD8>
__global__ __launch_bounds__(T) void k_encode_ham_dense(G16Args a, uint32_t rpb, float inv_cpr) {
    constexpr int kPartWords = PAD8 ? T * U / 2 : T * U / 8;   // PAD8: rpb <= T U / 2 reads (cpr >= 2)
    __shared__ uint64_t part8[kPartWords];
    uint8_t* part = (uint8_t*)part8;
    const uint64_t r0 = (uint64_t)blockIdx.x * rpb;
    const uint32_t nr = (uint32_t)min((uint64_t)rpb, a.n - r0);
    const uint32_t nloc = nr * a.cpr;
    const uint64_t c0 = r0 * a.cpr;
    uint4 x[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint32_t cl = j * T + threadIdx.x;
        x[j] = cl < nloc ? ld_stream(&a.in[c0 + cl]) : make_uint4(0x41414141u, 0x41414141u, 0x41414141u, 0x41414141u);
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint32_t cl = j * T + threadIdx.x;
        const uint32_t rl = (uint32_t)__fmul_rn(__fadd_rn((float)cl, 0.5f), inv_cpr);
        const uint32_t k = cl - rl * a.cpr;
        uint32_t bad;
        const uint32_t v = encode_chunk<PATH>(x[j], k, a, bad);
        const bool live = cl < nloc;
        report_bad(live && bad != 0u, r0 + rl, a.first_bad);
        if (live && a.out32) {
            if constexpr (NTST) st_stream(&a.out32[c0 + cl], v);
            else a.out32[c0 + cl] = v;
        }
        const uint8_t d = (uint8_t)((live && k < a.ham2) ? ham32(v ^ a.ref32[k]) : 0u);
        if constexpr (PAD8) {
            if (live) part[8 * rl + k] = d;
        } else {
            part[cl] = d;
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nr; i += T) {
        uint32_t sum = 0;
        if constexpr (PAD8) {
            const uint64_t p = part8[i] & (~0ull >> (64 - 8 * a.cpr));   // bytes cpr..7 are never written
            sum = __builtin_amdgcn_sad_u8((uint32_t)p, 0u, 0u) + __builtin_amdgcn_sad_u8((uint32_t)(p >> 32), 0u, 0u);
        } else {
            for (uint32_t k = 0; k < a.cpr; ++k) sum += part[i * a.cpr + k];
        }
        st_stream(&a.counts[r0 + i], sum);
    }
}

// ------------------------------------------------------------------------------------------------
// General path: one lane per (read, word).  Bytes come from aligned dword loads (only dwords that
// hold at least one byte of the read) realigned with v_alignbyte; bytes past the read are replaced
// by 'A' (code 0, no carry), so the tail word's Q1 carry lands at bit 2*nb exactly as the reference.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t encode_word_at(const uint8_t* p, uint32_t nb, bool table, uint32_t& bad) {
    const uintptr_t addr = (uintptr_t)p;
    const uint32_t* d = (const uint32_t*)(addr & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(addr & 3);
    const uint32_t nd = (sh + nb + 3u) >> 2;
    uint32_t dw[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) dw[i] = ((uint32_t)i < nd) ? d[i] : 0x41414141u;
    uint32_t xw[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint32_t v = __builtin_amdgcn_alignbyte(dw[i + 1], dw[i], sh);
        const int m = (int)nb - 4 * i;
        if (m <= 0) {
            v = 0x41414141u;
        } else if (m < 4) {
            const uint32_t keep = (1u << (8 * m)) - 1u;
            v = (v & keep) | (0x41414141u & ~keep);
        }
        xw[i] = v;
    }
    Enc32 lo = encode16(xw[0], xw[1], xw[2], xw[3], table);
    Enc32 hi = encode16(xw[4], xw[5], xw[6], xw[7], table);
    bad |= lo.bad | hi.bad;
    return (uint64_t)lo.v | ((uint64_t)(hi.v | lo.cout) << 32);
}

// The drop-in engine's short reads (lengths 1..31) as ONE table's keys (ss_ingest's short group):
// key = the read's packed word | 1 << (2L + 1).  The marker sits above the word's 2L code bits and
// above bit 2L, where the table path's carry of an aliased last nucleotide lands, so it
// is the key's highest set bit: keys of different lengths never meet, and the length and the word
// come back from the key alone.  Row i = read sel[i] (sel null: read i); dense_L > 0: the reads lie
// back to back, each dense_L bytes.  A rejected read's chunk index goes to *first_bad (atomicMin).
__global__ __launch_bounds__(256) void k_short_keys(const uint8_t* __restrict__ in, const uint64_t* __restrict__ offs,
                                                    const uint32_t* __restrict__ lens, const uint64_t* __restrict__ sel,
                                                    uint64_t m, uint32_t dense_L, uint64_t* __restrict__ keys,
                                                    unsigned long long* first_bad) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < m; i += (uint64_t)gridDim.x * 256) {
        const uint64_t r = sel ? sel[i] : i;
        const uint32_t L = dense_L ? dense_L : lens[r];
        const uint64_t off = dense_L ? r * dense_L : offs[r];
        uint32_t bad = 0;
        const uint64_t word = encode_word_at(in + off, L, true, bad);
        keys[i] = word | (1ull << (2u * L + 1u));
        if (bad) atomicMin(first_bad, (unsigned long long)r);
    }
}

// The ragged kernel's word loader: the 16-B-aligned chunks that hold the word's bytes (three
// dwordx4 loads, the third clamped to the last chunk holding a byte of the word, so every load stays
// inside chunks the read touches: no fault past the buffer's last 16-B chunk) realigned by a
// funnel shift; bytes past nb become 'A'.  Against nine dword loads per lane: a third of the load
// instructions, each touching half the cache lines.
struct Chunks3 {
    uint4 c0, c1, c2;
    uint32_t sh;
};

__device__ __forceinline__ Chunks3 load_word_q(const uint8_t* p, uint32_t nb) {
    const uintptr_t addr = (uintptr_t)p;
    const uint4* q = (const uint4*)(addr & ~(uintptr_t)15);
    Chunks3 c;
    c.sh = (uint32_t)(addr & 15);
    const uint32_t last = (c.sh + nb - 1u) >> 4;    // 0..2: the chunk holding the word's last byte
    c.c0 = q[0];
    c.c1 = q[min(1u, last)];
    c.c2 = q[min(2u, last)];
    return c;
}

__device__ __forceinline__ uint64_t pack_word_q(const Chunks3& c, uint32_t nb, bool table, uint32_t& bad) {
    const uint32_t d[12] = {c.c0.x, c.c0.y, c.c0.z, c.c0.w, c.c1.x, c.c1.y, c.c1.z, c.c1.w, c.c2.x, c.c2.y, c.c2.z, c.c2.w};
    const uint32_t s4 = c.sh >> 2, sb = c.sh & 3u;
    // e[k] = d[k + s4] (s4 < 4) by two masked selects on constant indices: written as a ternary on
    // the index, the compiler turns the 12 dwords into a scratch array indexed at run time
    const uint32_t m1 = 0u - (s4 & 1u), m2 = 0u - ((s4 >> 1) & 1u);
    uint32_t a[11], e[9];
#pragma unroll
    for (int k = 0; k < 11; ++k) a[k] = d[k] ^ ((d[k] ^ d[k + 1]) & m1);
#pragma unroll
    for (int k = 0; k < 9; ++k) e[k] = a[k] ^ ((a[k] ^ a[min(k + 2, 10)]) & m2);
    uint32_t xw[8];
    // bytes at or past nb read as 'A', branch-free: dword i keeps k = clamp(nb - 4i, 0, 4) bytes, the
    // 'A' mask being ~0 << 8k as two shifts of 4k (a single shift by 32 would keep the word whole).
    // (Per-dword branches on nb - 4i cost ~9 VALU plus exec-mask changes per dword, this 6.)
    const int nb4 = 4 * (int)nb;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t v = __builtin_amdgcn_alignbyte(e[i + 1], e[i], sb);
        const uint32_t k4 = (uint32_t)min(max(nb4 - 16 * i, 0), 16);   // 4k (v_med3_i32)
        const uint32_t pad = (~0u << k4) << k4;
        xw[i] = (v & ~pad) | (0x41414141u & pad);
    }
    Enc32 lo = encode16(xw[0], xw[1], xw[2], xw[3], table);
    Enc32 hi = encode16(xw[4], xw[5], xw[6], xw[7], table);
    bad |= lo.bad | hi.bad;
    return (uint64_t)lo.v | ((uint64_t)(hi.v | lo.cout) << 32);
}

__device__ __forceinline__ uint64_t encode_word_q(const uint8_t* p, uint32_t nb, bool table, uint32_t& bad) {
    return pack_word_q(load_word_q(p, nb), nb, table, bad);
}

// Ragged batches (ss_encode_var): one lane per output word, dense -- lane g writes out[g], word
// w = g mod wpr of read r = g / wpr (a double reciprocal, corrected by one step), so no lane idles on
// power-of-two padding and every wave stores 512 contiguous bytes.  Words at or past a read's length
// are written as 0 (the row padding).  The blob's 16-B chunks are read whole (encode_word_q): the
// blob must be readable to the end of its last 16-B chunk (any hipMalloc / torch allocation is).
// Two words per lane (words base + lane and base + 64 + lane of its wave's 128-word span): both
// words' offset / length loads, then both words' chunk loads, go out before either is packed
// (tools/tune_encvar.hip on the F2 batch: 1 word 0.514, 2 words 0.561, 4 words 0.533 of 8 TB/s).
constexpr int kVarK = 2;
__global__ __launch_bounds__(kThreads) void k_encode_var_dense(const uint8_t* in, const uint64_t* __restrict__ offs,
                                                               const uint32_t* __restrict__ lens, uint64_t n,
                                                               uint64_t* __restrict__ out, uint32_t wpr,
                                                               double inv_wpr, unsigned long long* first_bad) {
    const uint64_t total = n * wpr;
    const uint64_t base = ((uint64_t)blockIdx.x * kThreads + (threadIdx.x & ~63u)) * kVarK + (threadIdx.x & 63u);
    uint64_t r[kVarK], off[kVarK];
    uint32_t w[kVarK], L[kVarK], nb[kVarK];
#pragma unroll
    for (int k = 0; k < kVarK; ++k) {
        const uint64_t g = base + 64u * k;
        uint64_t rr = (uint64_t)((double)g * inv_wpr);
        if (rr * wpr > g) --rr;
        else if ((rr + 1) * wpr <= g) ++rr;
        r[k] = g < total ? rr : 0;
        w[k] = (uint32_t)(g - rr * wpr);
        L[k] = g < total ? lens[r[k]] : 0u;
        off[k] = g < total ? offs[r[k]] : 0u;
    }
    Chunks3 c[kVarK];
#pragma unroll
    for (int k = 0; k < kVarK; ++k) {
        nb[k] = (L[k] <= SS_MAX_NT && 32u * w[k] < L[k]) ? min(32u, L[k] - 32u * w[k]) : 0u;
        if (nb[k]) c[k] = load_word_q(in + off[k] + 32u * w[k], nb[k]);
    }
#pragma unroll
    for (int k = 0; k < kVarK; ++k) {
        const uint64_t g = base + 64u * k;
        if (g >= total) continue;
        uint32_t bad = 0;
        uint64_t word = 0;
        if (L[k] > SS_MAX_NT) bad = (w[k] == 0);          // short_seq.pyx:74 (too long), reported per read
        else if (nb[k]) word = pack_word_q(c[k], nb[k], (L[k] <= 32u) || (nb[k] < 32u), bad);
        out[g] = word;
        report_bad(bad != 0u, r[k], first_bad);
    }
}

// Drop-in engine, one multi-word length class (ss_ingest): row i = read sel[i] of the chunk (read i
// of a dense chunk of fixed length dense_L when sel is null), W words (ss_encode_var's rule) then
// its length as word W, one lane per output word.  first_bad: the smallest chunk read index that
// holds a rejected byte (rows are ordered by length, so the row would not give input order).
__global__ __launch_bounds__(kThreads) void k_encode_class(const uint8_t* in, const uint64_t* __restrict__ offs,
                                                           const uint32_t* __restrict__ lens,
                                                           const uint64_t* __restrict__ sel, uint32_t dense_L,
                                                           uint64_t m, uint32_t W, double inv_w1,
                                                           uint64_t* __restrict__ out, unsigned long long* first_bad) {
    const uint32_t W1 = W + 1;
    const uint64_t total = m * W1;
    for (uint64_t g = (uint64_t)blockIdx.x * kThreads + threadIdx.x; g < total; g += (uint64_t)gridDim.x * kThreads) {
        uint64_t i = (uint64_t)((double)g * inv_w1);
        if (i * W1 > g) --i;
        else if ((i + 1) * W1 <= g) ++i;
        const uint32_t w = (uint32_t)(g - i * W1);
        const uint64_t r = sel ? sel[i] : i;
        const uint32_t L = dense_L ? dense_L : lens[r];
        uint32_t bad = 0;
        uint64_t word = L;
        if (w < W) {
            word = 0;
            if (32u * w < L) {
                const uint64_t off = dense_L ? r * dense_L : offs[r];
                const uint32_t nb = min(32u, L - 32u * w);
                word = encode_word_q(in + off + 32u * w, nb, nb < 32u, bad);
            }
        }
        out[g] = word;
        report_bad(bad != 0u, r, first_bad);
    }
}

// Drop-in engine, every multi-word length class of a chunk in one pass, in read order (the blob is
// read once; per class, k_encode_class re-reads the lines its rows share with other classes').  A
// block takes kClsTile consecutive reads.  Within the tile the reads of class W hold consecutive rows
// of W's block (k_len_scatter is stable), so the tile's rows of a class are one contiguous span:
//   a. per read: class W = ceil(L/32) (L 33..1024), its row (posof[r] - binstart[bin0 + W]); per
//      class the tile's first row and count (LDS atomics); a scan of W + 1 over the reads
//   b. lane per word slot in read order (k_encode_var_dense's access pattern: consecutive lanes,
//      consecutive words of consecutive reads).  A read starting at byte sh = off % 16 has word w at
//      byte sh of its 16-B-aligned chunk 2w, so each of the three aligned chunks holding the word is
//      encoded where it lies (encode16 without the alias carry: 16 codes) and the word is a funnel
//      shift of the three code words by 2 sh bits, tail codes past the read masked to 'A' = 0 --
//      no byte realignment (encode_word_q's selects and v_alignbyte: ~210 VALU per word, which
//      left the former form VALU-bound at 2.1 ms on the f2 batch).  Rejected bytes: a chunk with
//      any gives its byte mask, windowed the same way (FASTQ neighbours are newlines and quality
//      bytes: only a read's first and last chunks); a partial tail word holding a bit-6-clear byte
//      (the table path's alias carry) is re-encoded exactly (encode_word_q).  w == W is
//      the length.  Into the tile's LDS class spans, the class beside it (a byte)
//   c. the spans out with dense stores (a per-class run of whole rows); each read's row fingerprint
//      (words_fp over its LDS row, the class table's slot key) to fps[fpoff[W] + row] when fps is
//      given, and into class W's HyperLogLog registers (2^kHllLog per class, max of the rank), which
//      the engine reads to size each class's table by its distinct keys rather than by its reads.
// (A lane-per-read-slot form with the rows stored straight from registers measured 3.6 ms against
// 2.75 for the four per-class passes on the f2 batch: its row stores land 24-48 B at a time.  The
// chunks staged once in LDS as codes + masks (each chunk encoded once) measured 3.08 ms: 46 KB of
// LDS per 256 reads left 3 waves per SIMD for a kernel of three dependent load phases.)
struct ClassOut {
    uint64_t woff[33];
    uint64_t fpoff[33];
    uint64_t* rmap[33];     // class W's row map at its first row of this chunk (null: not written)
    uint64_t base;          // global read index of the chunk's read 0
    uint32_t bin0;
};
constexpr uint32_t kClsTile = 256;

// the class's sketch register from the fingerprint's own bits (words_fp ends in a full mix; the
// class width is in its seed)
__device__ __forceinline__ void hll_add(uint32_t* reg_base, uint64_t fp, uint32_t W1) {
    (void)W1;
    const uint64_t h = fp;
    uint32_t* reg = reg_base + (uint32_t)(h >> (64 - kHllLog));
    const uint32_t rho = (uint32_t)__clzll((h << kHllLog) | (1ull << (kHllLog - 1))) + 1u;
    if (*reg < rho) atomicMax(reg, rho);    // registers settle early: most reads only load
}

// bit b of the result: byte b of m is nonzero (b < 4)
__device__ __forceinline__ uint32_t nz_bytes(uint32_t m) {
    const uint32_t t = ((m & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | m;
    return ((t >> 7) & 1u) | ((t >> 14) & 2u) | ((t >> 21) & 4u) | ((t >> 28) & 8u);
}

// 16 aligned bytes -> their 16 codes (no alias carry); *odd != 0 when some byte is rejected or has
// bit 6 clear (the rare path: chunk_masks then says which)
__device__ __forceinline__ uint32_t code_chunk(const uint4& c, uint32_t& odd) {
    const uint32_t p0 = c.x & 0x06060606u, p1 = c.y & 0x06060606u, p2 = c.z & 0x06060606u, p3 = c.w & 0x06060606u;
    odd |= ((c.x & 0x3F3F3F3Fu) ^ __builtin_amdgcn_perm(0x00070014u, 0x00030001u, p0)) |
           ((c.y & 0x3F3F3F3Fu) ^ __builtin_amdgcn_perm(0x00070014u, 0x00030001u, p1)) |
           ((c.z & 0x3F3F3F3Fu) ^ __builtin_amdgcn_perm(0x00070014u, 0x00030001u, p2)) |
           ((c.w & 0x3F3F3F3Fu) ^ __builtin_amdgcn_perm(0x00070014u, 0x00030001u, p3)) |
           (~(c.x & c.y & c.z & c.w) & 0x40404040u);
    return transpose2x4((p0 >> 1) | (p1 << 1) | (p2 << 3) | (p3 << 5));
}

// rejected-byte mask | bit-6-clear byte mask << 16 of 16 aligned bytes
__device__ __forceinline__ uint32_t chunk_masks(const uint4& c) {
    const uint32_t x[4] = {c.x, c.y, c.z, c.w};
    uint32_t bad = 0, al = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t m = (x[i] & 0x3F3F3F3Fu) ^ __builtin_amdgcn_perm(0x00070014u, 0x00030001u, x[i] & 0x06060606u);
        bad |= nz_bytes(m) << (4 * i);
        al |= nz_bytes(~x[i] & 0x40404040u) << (4 * i);
    }
    return bad | al << 16;
}

// 6 waves per SIMD: left to itself the compiler spent 117-151 VGPRs (4 or 3 waves) on a kernel that
// waits on memory two thirds of its cycles (SQ_WAIT_ANY / SQ_WAVE_CYCLES)
__global__ __launch_bounds__(kClsTile) __attribute__((amdgpu_waves_per_eu(6))) void k_encode_classes(const uint8_t* in, const uint64_t* __restrict__ offs,
                                                             const uint32_t* __restrict__ lens, uint64_t n,
                                                             const uint32_t* __restrict__ blkoff, uint32_t nblk,
                                                             ClassOut co, uint32_t w1max, uint64_t* __restrict__ out,
                                                             uint64_t* __restrict__ fps, uint32_t* hll,
                                                             unsigned long long* first_bad) {
    extern __shared__ __attribute__((aligned(16))) unsigned char dyn[];
    constexpr uint32_t kWaves = kClsTile / 64;
    const uint32_t nslot = kClsTile * w1max;
    uint64_t* sw = (uint64_t*)dyn;                          // [nslot] the tile's class spans, class after class
    uint8_t* scls = (uint8_t*)(sw + nslot);                 // [nslot] span slot -> its class
    uint8_t* smap = scls + nslot;                           // [nslot] word slot -> read of the tile
    uint16_t* sodd = (uint16_t*)(smap + nslot);             // [nslot] word slots left to the exact re-encode
    __shared__ uint64_t soff[kClsTile];
    __shared__ uint32_t srow[kClsTile];                     // row within the tile's span of its class
    __shared__ uint16_t sqoff[kClsTile + 1], sL[kClsTile];
    __shared__ uint32_t wcnt[kWaves][33], tcnt[33], cur[33], cbase[34], wsum[kWaves], nodd;
    const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
    const uint64_t lt = (1ull << lane) - 1ull;
    // this block's read range: k_len_count's (its class rows start at the binscan's offsets)
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t lo = min(n, (uint64_t)blockIdx.x * per), hi = min(n, lo + per);
    if (t < 33) cur[t] = t >= 2 ? blkoff[(uint64_t)(co.bin0 + t) * nblk + blockIdx.x] : 0u;
    // loads carried across tiles, off the tile's chain of round trips: the next tile's length and
    // offset (issued in phase c), and the previous tile's sketch register (checked one tile later)
    uint32_t nL0 = 0;
    uint64_t noff = 0;
    if (lo < hi) {
        const uint64_t rc = min(lo + t, n - 1);
        nL0 = lens[rc];
        noff = offs[rc];
    }
    uint32_t* hreg = nullptr;
    uint32_t hrho = 0, hval = 0;
    for (uint64_t r0 = lo; r0 < hi; r0 += kClsTile) {
        const uint64_t r = r0 + t;
        // a. classes, rows (stable: the wave's lanes ranked by ballot, the waves in order), word slots
        const uint32_t L0 = nL0;
        const uint64_t off = noff;
        for (uint32_t i = t; i < kWaves * 33; i += kClsTile) (&wcnt[0][0])[i] = 0;
        if (t == 0) nodd = 0;
        __syncthreads();
        const uint32_t L = r < hi ? L0 : 0u;
        const bool cls = L > 32u && L <= SS_MAX_NT;
        const uint32_t W = cls ? (L + 31u) / 32u : 0u, w1 = cls ? W + 1u : 0u;
        uint32_t rk = 0;
        uint64_t pending = __ballot(cls);
        while (pending) {
            const int leader = __ffsll((long long)pending) - 1;
            const uint32_t Wl = (uint32_t)__shfl((int)W, leader);
            const uint64_t mine = __ballot(cls && W == Wl);
            if (cls && W == Wl) rk = (uint32_t)__popcll(mine & lt);
            if (lane == (uint32_t)leader) wcnt[wave][Wl] = (uint32_t)__popcll(mine);
            pending &= ~mine;
        }
        if (cls) soff[t] = off;
        sL[t] = (uint16_t)(cls ? L : 0u);
        uint32_t inc = w1;
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(inc, d);
            if (lane >= d) inc += y;
        }
        if (lane == 63) wsum[wave] = inc;
        __syncthreads();
        uint32_t before = 0;
        for (uint32_t u = 0; u < wave; ++u) before += wsum[u];
        const uint32_t q0 = before + inc - w1;
        sqoff[t] = (uint16_t)q0;
        if (t == kClsTile - 1) sqoff[kClsTile] = (uint16_t)(q0 + w1);
        for (uint32_t k = 0; k < w1; ++k) smap[q0 + k] = (uint8_t)t;
        if (cls) {
            uint32_t pre = rk;
            for (uint32_t u = 0; u < wave; ++u) pre += wcnt[u][W];
            srow[t] = pre;
        }
        if (t == 0) {
            uint32_t c = 0;
            for (uint32_t u = 0; u < 33; ++u) {
                uint32_t m = 0;
                for (uint32_t v = 0; v < kWaves; ++v) m += wcnt[v][u];
                tcnt[u] = u >= 2 ? m : 0u;
                cbase[u] = c;
                c += tcnt[u] * (u + 1u);
            }
            cbase[33] = c;
        }
        __syncthreads();
        // b. lane per word slot, read order: the word's three aligned chunks encoded where they lie,
        //    the three loads issued together.  A word whose chunks hold a rejected or bit-6-clear byte
        //    anywhere (an invalid base, an alias, or -- in a FASTQ chunk -- the newline and quality
        //    bytes around a read) goes to a list and is re-encoded exactly after the pass
        //    (encode_word_q: the byte-realigning form, table semantics for a partial tail word); kept
        //    out of this loop, its registers would set the kernel's occupancy
        const uint32_t Q = sqoff[kClsTile];
        const uint4* in16 = (const uint4*)in;
        for (uint32_t q = t; q < Q; q += kClsTile) {
            const uint32_t tt = smap[q];
            const uint32_t LL = sL[tt], WW = (LL + 31u) / 32u, w = q - sqoff[tt];
            const uint32_t at = cbase[WW] + srow[tt] * (WW + 1u) + w;
            uint64_t word = LL;
            if (w < WW) {
                const uint64_t ro = soff[tt];
                const uint32_t nb = min(32u, LL - 32u * w), sh = (uint32_t)(ro & 15u);
                const uint32_t last = (sh + nb - 1u) >> 4;       // 0..2: the chunk holding the word's last byte
                const uint64_t c0 = (ro >> 4) + 2u * w;
                const uint4 xa = in16[c0], xb = in16[c0 + min(1u, last)], xc = in16[c0 + min(2u, last)];
                uint32_t odd = 0;
                const uint32_t ca = code_chunk(xa, odd), cb = code_chunk(xb, odd), cc = code_chunk(xc, odd);
                const uint64_t lo64 = (uint64_t)cb << 32 | ca;
                word = sh ? (lo64 >> (2u * sh)) | ((uint64_t)cc << (64u - 2u * sh)) : lo64;
                if (nb < 32u) word &= (1ull << (2u * nb)) - 1ull;
                if (odd) sodd[atomicAdd(&nodd, 1u)] = (uint16_t)q;
            }
            sw[at] = word;
            scls[at] = (uint8_t)WW;
        }
        __syncthreads();
        if (nodd) {     // block-uniform
            for (uint32_t k = t; k < nodd; k += kClsTile) {
                const uint32_t q = sodd[k], tt = smap[q];
                const uint32_t LL = sL[tt], WW = (LL + 31u) / 32u, w = q - sqoff[tt];
                const uint32_t nb = min(32u, LL - 32u * w);
                uint32_t bad = 0;
                sw[cbase[WW] + srow[tt] * (WW + 1u) + w] = encode_word_q(in + soff[tt] + 32u * w, nb, nb < 32u, bad);
                if (bad) atomicMin(first_bad, (unsigned long long)(r0 + tt));
            }
            __syncthreads();
        }
        // c. the class spans out (dense), fingerprints, sketches, the rows' read indices
        for (uint32_t q = t; q < Q; q += kClsTile) {
            const uint32_t c = scls[q];
            out[co.woff[c] + (uint64_t)cur[c] * (c + 1u) + (q - cbase[c])] = sw[q];
        }
        if (r0 + kClsTile < hi) {
            const uint64_t rc = min(r + kClsTile, n - 1);
            nL0 = lens[rc];
            noff = offs[rc];
        }
        if (hreg && hval < hrho) atomicMax(hreg, hrho);     // registers settle early: most reads only load
        hreg = nullptr;
        if (cls) {
            const uint32_t row = cur[W] + srow[t];
            const uint64_t fp = words_fp(sw + cbase[W] + srow[t] * w1, w1);
            if (fps) fps[co.fpoff[W] + row] = fp;
            if (co.rmap[W]) co.rmap[W][row] = co.base + r;
            const uint64_t h = fp;                         // hll_add's register and rank
            hreg = hll + ((uint64_t)W << kHllLog) + (uint32_t)(h >> (64 - kHllLog));
            hrho = (uint32_t)__clzll((h << kHllLog) | (1ull << (kHllLog - 1))) + 1u;
            hval = *hreg;
        }
        __syncthreads();
        if (t < 33) cur[t] += tcnt[t];
    }
    if (hreg && hval < hrho) atomicMax(hreg, hrho);
}

// Drop-in engine, a chunk whose reads are all class reads of at most S - 1 words (S <= 6): every
// read's row in READ order at a fixed stride of S words -- its W words, its length, zeros -- so no
// class ranks, no LDS staging, no barriers and no row map (the row of read r is r).  A wave holds
// R = 64 / S reads per group, S lanes each (lane w: word w, the length at w == W, 0 past it), and
// kRowsK groups per tile: the groups' length / offset loads, then their chunk loads, go out together
// (one group per wave measured 3.35 ms on the f2 batch: three dependent round trips for 1 KB of
// input; 1 / 2 / 4 / 5 / 6 groups as persistent waves 2.35 / 2.04 / 1.91 / 1.93 / 1.89 ms,
// profiles/r4/f2/libab_encrows_occupancy.log, libab_encrows_k56.log).  The words are
// k_encode_classes' phase b (16-B chunks, funnel shift, the rare odd word re-encoded exactly), each
// chunk of a read loaded by one lane only.  The row goes through the wave's LDS to one lane per read,
// which runs its fingerprint (words_fp over the W + 1 words) and its class's sketch update.  Reads
// that are not class reads (empty: the length split counts those) get a zero row and the
// fingerprint of one zero word, an entry the fold skips.  A tile holds R kRowsK <= 128 reads (the
// fingerprint lanes take two each at most: S = 3, R = 21).
constexpr int kRowsK = 6;
static_assert(21 * kRowsK <= 128, "a tile's reads: two per fingerprint lane at most");
// the tile's lengths / offsets (reads rb .. rb + R kRowsK - 1): loaded coalesced, a lane per read (two
// rounds past 64 reads; rows_meta_load, issued a tile ahead), then handed to the S lanes of each read
// by shuffles (rows_meta_split, when the tile starts) -- not loaded by every lane of the read
struct RowsMeta {
    uint32_t la, lb;
    uint64_t oa, ob;
};
__device__ __forceinline__ RowsMeta rows_meta_load(const uint64_t* __restrict__ offs, const uint32_t* __restrict__ lens,
                                                   uint64_t n, uint64_t rb, uint32_t per, uint32_t lane) {
    RowsMeta m;
    const uint64_t ra = rb + lane, rbb = rb + 64u + lane;
    m.la = (lane < per && ra < n) ? lens[ra] : 0u;
    m.oa = (lane < per && ra < n) ? offs[ra] : 0ull;
    m.lb = 0;
    m.ob = 0;
    if (per > 64u) {            // wave-uniform (S <= 5)
        m.lb = (64u + lane < per && rbb < n) ? lens[rbb] : 0u;
        m.ob = (64u + lane < per && rbb < n) ? offs[rbb] : 0ull;
    }
    return m;
}

__device__ __forceinline__ void rows_meta_split(const RowsMeta& m, uint32_t R, uint32_t i, uint32_t* L, uint64_t* off) {
    const bool two = R * kRowsK > 64u;
#pragma unroll
    for (int k = 0; k < kRowsK; ++k) {
        const uint32_t jj = (uint32_t)k * R + i;            // this lane's read in the tile
        const int src = (int)(jj & 63u);
        const uint32_t l0 = (uint32_t)__shfl((int)m.la, src), o0l = (uint32_t)__shfl((int)(uint32_t)m.oa, src),
                       o0h = (uint32_t)__shfl((int)(uint32_t)(m.oa >> 32), src);
        uint32_t l1 = 0, o1l = 0, o1h = 0;
        if (two) {
            l1 = (uint32_t)__shfl((int)m.lb, src);
            o1l = (uint32_t)__shfl((int)(uint32_t)m.ob, src);
            o1h = (uint32_t)__shfl((int)(uint32_t)(m.ob >> 32), src);
        }
        const bool hi = jj >= 64u, live = i < R;
        L[k] = live ? (hi ? l1 : l0) : 0u;
        off[k] = live ? ((uint64_t)(hi ? o1h : o0h) << 32 | (hi ? o1l : o0l)) : 0ull;
    }
}

__global__ __launch_bounds__(256) void k_encode_rows(const uint8_t* in, const uint64_t* __restrict__ offs,
                                                     const uint32_t* __restrict__ lens, uint64_t n, uint32_t S,
                                                     uint64_t* __restrict__ out, uint64_t* __restrict__ fps,
                                                     uint32_t* hll, unsigned long long* first_bad,
                                                     const uint64_t* __restrict__ gate) {
    if (gate && *gate != S) return;       // queued before the split came back: the split chose another path
    const uint32_t lane = threadIdx.x & 63u, R = 64u / S, wave = threadIdx.x >> 6;
    const uint32_t i = lane / S, w = lane - i * S;
    const uint64_t per = (uint64_t)R * kRowsK, tiles = (n + per - 1) / per, stride = (uint64_t)gridDim.x * 4;
    const uint4* in16 = (const uint4*)in;
    __shared__ uint64_t srow[4][kRowsK * 64];     // the wave's rows (group k: lanes k * 64 ..)
    __shared__ uint16_t slen[4][kRowsK * 24];     // the wave's reads' lengths (read j = k * R + i; R <= 21)
    uint64_t tile = (uint64_t)blockIdx.x * 4 + wave;
    RowsMeta meta = rows_meta_load(offs, lens, n, tile * per, (uint32_t)per, lane);
    uint32_t* hreg[2] = {nullptr, nullptr};       // the previous tile's sketch updates (<= 2 reads a lane)
    uint32_t hval[2] = {0, 0}, hrho[2] = {0, 0};
    for (; tile < tiles; tile += stride) {
        const uint64_t r0 = tile * per + i;
        uint32_t L[kRowsK];
        uint64_t off[kRowsK];
        rows_meta_split(meta, R, i, L, off);
        // the read's 16-B chunks once each: lane w loads chunks 2w and 2w + 1 of its read (relative to
        // the read's first chunk, clamped to its last), the length lane W only chunk 2W when the read
        // reaches it; word w's third chunk 2w + 2 is lane w + 1's first (a shuffle).  Lanes past W load
        // nothing.
        uint4 xa[kRowsK], xb[kRowsK];
#pragma unroll
        for (int k = 0; k < kRowsK; ++k) {
            const uint32_t W = (L[k] + 31u) / 32u;
            const uint64_t cb = off[k] >> 4;
            const uint32_t lastc = L[k] ? (uint32_t)(((off[k] + L[k] - 1u) >> 4) - cb) : 0u;
            xa[k] = make_uint4(0u, 0u, 0u, 0u);
            xb[k] = xa[k];
            if (L[k] && w <= W && 2u * w <= lastc) xa[k] = in16[cb + 2u * w];
            if (L[k] && w < W) xb[k] = in16[cb + min(2u * w + 1u, lastc)];
        }
        uint64_t badr = ~0ull;              // the tile's first rejected read of this lane (one report)
        // the next tile's lengths / offsets go out behind the chunks
        meta = rows_meta_load(offs, lens, n, (tile + stride) * per, (uint32_t)per, lane);
#pragma unroll
        for (int k = 0; k < kRowsK; ++k) {
            const uint64_t r = r0 + (uint64_t)k * R;
            const bool live = i < R && r < n;
            const uint32_t W = (L[k] + 31u) / 32u;
            const bool cls = L[k] > 32u && W < S;
            // every lane codes its first chunk; lane w + 1's code (and its odd flag) is word w's
            // third chunk, one shuffle each instead of coding the shuffled chunk again
            uint32_t oa = 0;
            const uint32_t ca = code_chunk(xa[k], oa);
            const uint32_t cn = (uint32_t)__shfl_down((int)ca, 1), on = (uint32_t)__shfl_down((int)oa, 1);
            uint64_t word = 0;
            uint32_t bad = 0;
            if (cls && w < W) {
                const uint32_t nb = min(32u, L[k] - 32u * w), sh = (uint32_t)(off[k] & 15u);
                const uint32_t last = (sh + nb - 1u) >> 4;
                uint32_t odd = oa;
                const uint32_t cb = code_chunk(xb[k], odd);
                const uint32_t cc = last == 2u ? cn : cb;
                odd |= last == 2u ? on : 0u;
                // bits 2 sh .. 2 sh + 63 of cc:cb:ca by two 32-bit funnel shifts, then the 2 nb bits kept
                const uint32_t s2 = 2u * sh, b2 = 2u * nb;
                const uint32_t lo = __builtin_amdgcn_alignbit(cb, ca, s2), hi = __builtin_amdgcn_alignbit(cc, cb, s2);
                const uint32_t mlo = b2 >= 32u ? ~0u : (1u << b2) - 1u;
                const uint32_t mhi = b2 >= 64u ? ~0u : b2 <= 32u ? 0u : (1u << (b2 - 32u)) - 1u;
                word = (uint64_t)(hi & mhi) << 32 | (lo & mlo);
                if (odd) word = encode_word_q(in + off[k] + 32u * w, nb, nb < 32u, bad);   // rare: exact semantics
            } else if (cls && w == W) {
                word = L[k];
            }
            if (live) out[r * S + w] = word;
            if (bad) badr = min(badr, r);
            srow[wave][k * 64 + lane] = word;
            if (w == 0 && i < R) slen[wave][k * R + i] = (uint16_t)(cls ? L[k] : 0u);
        }
        report_bad(badr != ~0ull, badr, first_bad);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");     // srow / slen are the wave's own
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // the previous tile's sketch registers (loaded a tile ago) settle now
#pragma unroll
        for (int p = 0; p < 2; ++p)
            if (hreg[p] && hval[p] < hrho[p]) atomicMax(hreg[p], hrho[p]);
        // lane per read: its row's fingerprint (words_fp over W + 1 words; one zero word for a read
        // that is no class read) and its class's sketch register -- one chain per read
        const uint64_t rb = tile * per;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const uint32_t j = lane + 64u * p;
            hreg[p] = nullptr;
            if (j >= per || rb + j >= n) continue;
            const uint32_t k = j / R, ii = j - k * R;
            const uint32_t LL = slen[wave][j];
            const uint32_t W1 = LL ? (LL + 31u) / 32u + 1u : 1u;
            const uint64_t* row = &srow[wave][k * 64 + ii * S];
            uint64_t rw[6];                     // all LDS reads issued before the chain (S <= 6)
#pragma unroll
            for (uint32_t q = 0; q < 6; ++q) rw[q] = row[min(q, S - 1)];
            uint64_t h = fp_seed(W1);
#pragma unroll
            for (uint32_t q = 0; q < 6; ++q)
                if (q < W1) h = fp_step(h, rw[q]);
            h = fp_final(h);
            fps[rb + j] = h;
            if (LL) {       // hll_add, its register's load left in flight until the next tile
                const uint64_t hh = h;
                hreg[p] = hll + ((uint64_t)(W1 - 1) << kHllLog) + (uint32_t)(hh >> (64 - kHllLog));
                hrho[p] = (uint32_t)__clzll((hh << kHllLog) | (1ull << (kHllLog - 1))) + 1u;
                hval[p] = *hreg[p];
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");     // this tile's LDS reads before the next's writes
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
#pragma unroll
    for (int p = 0; p < 2; ++p)
        if (hreg[p] && hval[p] < hrho[p]) atomicMax(hreg[p], hrho[p]);
}

// The same registers from rows already packed (k_encode_class's paths): lane per row, the same hash.
__global__ __launch_bounds__(kThreads) void k_hll_rows(const uint64_t* __restrict__ rows, uint64_t m, uint32_t W1,
                                                       uint32_t* hll) {
    for (uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x; i < m; i += (uint64_t)gridDim.x * kThreads)
        hll_add(hll, words_fp(rows + i * W1, W1), W1);
}

// Lane slot g -> read r = g >> logG, word w = g & (G-1) (G = next_pow2(wpr)); lanes w >= wpr idle.
// The grid-stride loop has a uniform trip count so the hamming reduction's shuffles see whole waves.
template <bool VAR, bool HAM>
__global__ __launch_bounds__(kThreads) void k_encode_gen(const uint8_t* in, uint64_t stride,
                                                         const uint64_t* offs, const uint32_t* lens,
                                                         uint32_t Lfix, uint64_t n, uint64_t* out,
                                                         uint32_t wpr, uint32_t logG, const uint64_t* ref,
                                                         uint32_t hamw, uint32_t* counts,
                                                         unsigned long long* first_bad) {
    const uint32_t G = 1u << logG;
    const uint64_t total = n << logG;
    const uint64_t gstride = (uint64_t)gridDim.x * kThreads;
    for (uint64_t g0 = (uint64_t)blockIdx.x * kThreads; g0 < total; g0 += gstride) {
        const uint64_t g = g0 + threadIdx.x;
        const uint64_t r = g >> logG;
        const uint32_t w = (uint32_t)g & (G - 1u);
        const bool live = r < n;
        uint32_t bad = 0;
        uint64_t word = 0;
        if (live && w < wpr) {
            const uint32_t L = VAR ? lens[r] : Lfix;
            const uint64_t off = VAR ? offs[r] : r * stride;
            if (L > SS_MAX_NT) {
                bad = (w == 0);                     // short_seq.pyx:74 (too long), reported per read
            } else if (32u * w < L) {
                const uint32_t nb = min(32u, L - 32u * w);
                const bool table = (L <= 32u) || (nb < 32u);
                word = encode_word_at(in + off + 32u * w, nb, table, bad);
            }
            if (out) out[r * wpr + w] = word;
        }
        if (bad) atomicMin(first_bad, (unsigned long long)r);
        if constexpr (HAM) {
            uint32_t part = (live && w < hamw) ? ham64(word ^ ref[w]) : 0u;
            for (uint32_t sft = 1; sft < G; sft <<= 1) part += __shfl_xor(part, sft);
            if (live && w == 0) counts[r] = part;
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Decode
// ------------------------------------------------------------------------------------------------
template <int T, int U, bool NTLD, bool NTST>
__global__ __launch_bounds__(T) void k_decode_g16(const uint32_t* __restrict__ w32, uint32_t wpr2,
                                                  uint64_t n, uint32_t cpr, uint32_t logG,
                                                  uint4* __restrict__ out, uint64_t out_stride16) {
    const uint32_t G = 1u << logG;
    const uint64_t base = (uint64_t)blockIdx.x * (U * T) + threadIdx.x;
    uint32_t v[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint64_t g = base + (uint64_t)j * T;
        const uint64_t r = g >> logG;
        const uint32_t k = (uint32_t)g & (G - 1u);
        const bool ok = r < n && k < cpr;
        if constexpr (NTLD) v[j] = ok ? __builtin_nontemporal_load(&w32[r * wpr2 + k]) : 0u;
        else v[j] = ok ? w32[r * wpr2 + k] : 0u;
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint64_t g = base + (uint64_t)j * T;
        const uint64_t r = g >> logG;
        const uint32_t k = (uint32_t)g & (G - 1u);
        if (r < n && k < cpr) {
            if constexpr (NTST) st_stream(&out[r * out_stride16 + k], decode16(v[j]));
            else out[r * out_stride16 + k] = decode16(v[j]);
        }
    }
}

__device__ __forceinline__ void store_chars(uint8_t* dst, uint64_t word, uint32_t nb) {
    const uint32_t lo = (uint32_t)word, hi = (uint32_t)(word >> 32);
    const uint4 a = decode16(lo), b = decode16(hi);
    const uint32_t c[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    if ((((uintptr_t)dst) & 3) == 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int m = (int)nb - 4 * i;
            if (m >= 4) {
                *(uint32_t*)(dst + 4 * i) = c[i];
            } else if (m > 0) {
                for (int b2 = 0; b2 < m; ++b2) dst[4 * i + b2] = (uint8_t)(c[i] >> (8 * b2));
            }
        }
    } else {
        for (uint32_t i = 0; i < nb; ++i) dst[i] = (uint8_t)(c[i >> 2] >> (8 * (i & 3)));
    }
}

template <bool VAR>
__global__ __launch_bounds__(kThreads) void k_decode_gen(const uint64_t* words, const uint32_t* lens,
                                                         uint32_t Lfix, uint64_t n, uint32_t wpr,
                                                         uint8_t* out, uint64_t stride, const uint64_t* offs) {
    const uint64_t total = n * wpr;
    for (uint64_t g = (uint64_t)blockIdx.x * kThreads + threadIdx.x; g < total;
         g += (uint64_t)gridDim.x * kThreads) {
        const uint64_t r = g / wpr;
        const uint32_t w = (uint32_t)(g - r * wpr);
        const uint32_t L = VAR ? lens[r] : Lfix;
        if (L > SS_MAX_NT || 32u * w >= L) continue;
        const uint32_t nb = min(32u, L - 32u * w);
        const uint64_t off = VAR ? offs[r] : r * stride;
        store_chars(out + off + 32u * w, words[g], nb);
    }
}

// ------------------------------------------------------------------------------------------------
// Hamming on packed words: lane per word, power-of-two lane groups per read, shfl_xor reduction.
// ------------------------------------------------------------------------------------------------
template <bool PAIR>
__global__ __launch_bounds__(kThreads) void k_ham_group(const uint64_t* __restrict__ a,
                                                        const uint64_t* __restrict__ b, uint64_t n,
                                                        uint32_t W, uint32_t wpr, uint32_t logG,
                                                        uint32_t* __restrict__ out) {
    const uint32_t G = 1u << logG;
    const uint64_t g = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    const uint64_t r = g >> logG;
    const uint32_t k = (uint32_t)g & (G - 1u);
    uint32_t part = 0;
    if (r < n && k < W) {
        const uint64_t x = a[r * wpr + k] ^ (PAIR ? b[r * wpr + k] : b[k]);
        part = ham64(x);
    }
    for (uint32_t s = 1; s < G; s <<= 1) part += __shfl_xor(part, s);
    if (r < n && k == 0) out[r] = part;
}

// distance stores of the dense hamming kernels (streamed once: nontemporal; same-box A/B against
// plain stores, C3' 32 / 96 nt: 0.73 -> 0.78, 0.69 -> 0.72 of peak, 512 nt unchanged)
__device__ __forceinline__ void ham_store(uint32_t* p, uint32_t v) {
    __builtin_nontemporal_store(v, p);
}
__device__ __forceinline__ void ham_store2(uint32_t* p, uint32_t lo, uint32_t hi) {
    const uint64_t v = ((uint64_t)hi << 32) | lo;
    __builtin_nontemporal_store(v, (uint64_t*)p);
}

// Dense hamming for W = 3 (96 nt, C3'): a read's 24 B are two dwordx3 halves held by a lane pair
// (lane 2k: dwords 0-2 = word 0 and the low half of word 1; lane 2k+1: dwords 3-5), so a
// wave-instruction loads 768 contiguous bytes (32 reads, six whole lines) with no shuffle needed to
// assemble a read.  The split at bit 32 of word 1 falls on a 2-bit boundary, so each lane's three
// 32-bit XOR-collapse-popcounts plus one DPP pair swap give the read's distance.  A wave takes U
// groups of 32 reads; their U x 32 distances go through LDS (one 4-B write per even lane and group)
// and leave as ONE dwordx4 store from U x 8 lanes.  Lanes past n load the last read again (clamped,
// branch-free); the wave holding the batch end (or an output that is not 16-B aligned) stores its
// distances one by one.  Same box (tools/tune_ham3.hip, profiles/r3/ham3_x3s.log): 0.826-0.835 of the
// 8-TB/s peak in 128-thread blocks at U = 2 (256 threads 0.819-0.829), against 0.793-0.796 for the same lanes storing
// 4 B from every even lane (U = 4, one-wave blocks), 0.776-0.786 for the former lane-triple form
// over 1-KiB chunks, 0.73 with the chunks DMA'd into LDS (global_load_lds) and read back per lane.
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
template <bool PAIR, int T, int U>
__global__ __launch_bounds__(T) void k_ham_dense3x(const uint32_t* __restrict__ a, const uint32_t* __restrict__ b,
                                                   const uint64_t* __restrict__ ref, uint64_t n,
                                                   uint32_t* __restrict__ out) {
    constexpr uint32_t NWV = T / 64;
    static_assert(U * 8 <= 64, "one dwordx4 store per wave");
    __shared__ __attribute__((aligned(16))) uint32_t sd[NWV][U * 32];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6, h = lane & 1u;
    const uint64_t g0 = ((uint64_t)blockIdx.x * NWV + wv) * U;     // the wave's first group of 32 reads
    u32x3 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t rc = min((g0 + u) * 32 + (lane >> 1), n - 1);
        x[u] = __builtin_nontemporal_load((const u32x3*)(a + rc * 6 + 3 * h));
        if constexpr (PAIR) y[u] = __builtin_nontemporal_load((const u32x3*)(b + rc * 6 + 3 * h));
    }
    uint32_t c0 = 0, c1 = 0, c2 = 0;
    if constexpr (!PAIR) {   // the reference's dwords this lane's half meets
        const uint64_t r0 = ref[0], r1 = ref[1], r2 = ref[2];
        c0 = h ? (uint32_t)(r1 >> 32) : (uint32_t)r0;
        c1 = h ? (uint32_t)r2 : (uint32_t)(r0 >> 32);
        c2 = h ? (uint32_t)(r2 >> 32) : (uint32_t)r1;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        uint32_t d;
        if constexpr (PAIR) d = ham32(x[u].x ^ y[u].x) + ham32(x[u].y ^ y[u].y) + ham32(x[u].z ^ y[u].z);
        else d = ham32(x[u].x ^ c0) + ham32(x[u].y ^ c1) + ham32(x[u].z ^ c2);
        d += swap_pair(d);
        if (!h) sd[wv][u * 32 + (lane >> 1)] = d;
    }
    __syncthreads();
    const uint64_t rb = g0 * 32;
    if (rb + U * 32 <= n && (((uintptr_t)out) & 15u) == 0) {
        if (lane < U * 8) {
            const uint4 v = *(const uint4*)&sd[wv][4 * lane];
            st_stream((uint4*)(out + rb + 4 * lane), v);
        }
    } else {
        for (uint32_t k = lane; k < U * 32; k += 64)
            if (rb + k < n) ham_store(&out[rb + k], sd[wv][k]);
    }
}

// Dense hamming on packed rows (wpr == W, 16-B aligned): the block owns RPB whole reads = RPB*W
// consecutive words (RPB even, so every block starts on a 16-B boundary) and streams them as
// dwordx4 pairs of words, U per lane, all loads issued before any use.
//   W = 1:        a lane's pair of words is two reads -> one 8-B store of two distances
//   W = 2^k >= 2: a read is W/2 consecutive lanes -> shfl_xor sum, the group's first lane stores
//   other W:      per-word distances (<= 32) as bytes in LDS, then one thread per read sums its W
//                 bytes and the block stores its distances coalesced (W <= 8: bytes padded to 8
//                 per read, one 8-B LDS read + v_sad_u8)
// PAD8 (other W <= 8): a read's distance bytes sit at 8 rl + k and one 8-B LDS read + two v_sad_u8
// sum them (the fused C3 kernel's tail); otherwise byte w of the block's word order
template <bool PAIR, bool POW2, int T, int U, bool PAD8 = false>
__global__ __launch_bounds__(T) void k_ham_dense(const uint4* __restrict__ a, const uint4* __restrict__ b,
                                                 const uint64_t* __restrict__ ref, uint64_t n, uint32_t W,
                                                 uint32_t rpb, float inv_w, uint32_t* __restrict__ out) {
    __shared__ uint64_t part8[POW2 ? 1 : (PAD8 ? (2 * T * U) / 3 + 1 : (2 * T * U) / 8)];   // PAD8: W >= 3
    uint8_t* part = (uint8_t*)part8;
    __shared__ uint64_t sref[PAIR || POW2 ? 1 : 32];   // the reference read (W <= 32 words)
    if constexpr (!PAIR && !POW2) {
        if (threadIdx.x < W) sref[threadIdx.x] = ref[threadIdx.x];
    }
    // power-of-two W: lane ql's words sit at positions (2 ql) % W and (2 ql + 1) % W of their read,
    // the same for every j (W divides 2T), so the reference words are fetched once per lane
    uint64_t pref_lo = 0, pref_hi = 0;
    if constexpr (!PAIR && POW2) {
        pref_lo = ref[W == 1 ? 0u : ((2u * threadIdx.x) & (W - 1u))];
        pref_hi = ref[W == 1 ? 0u : ((2u * threadIdx.x + 1u) & (W - 1u))];
    }
    const uint64_t r0 = (uint64_t)blockIdx.x * rpb;
    const uint32_t nr = (uint32_t)min((uint64_t)rpb, n - r0);
    const uint32_t nw = nr * W, nfull = nw / 2;    // live words; whole dwordx4 of the block
    const uint64_t q0 = r0 * W / 2;
    // an odd word count ends on a half pair: that word is read alone (no over-read past the rows)
    auto load = [&](const uint4* p, uint32_t ql) -> uint4 {
        if (ql < nfull) return ld_stream(&p[q0 + ql]);
        if (ql * 2 < nw) {
            const uint64_t v = ((const uint64_t*)p)[2 * (q0 + ql)];
            return make_uint4((uint32_t)v, (uint32_t)(v >> 32), 0u, 0u);
        }
        return make_uint4(0u, 0u, 0u, 0u);
    };
    uint4 x[U], y[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint32_t ql = j * T + threadIdx.x;
        x[j] = load(a, ql);
        if constexpr (PAIR) y[j] = load(b, ql);
    }
    if constexpr (!PAIR && !POW2) __syncthreads();   // sref
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint32_t ql = j * T + threadIdx.x;
        const uint32_t wl = 2 * ql;                 // block-local index of the lane's first word
        uint64_t r_lo, r_hi;
        if constexpr (PAIR) {
            r_lo = ((uint64_t)y[j].y << 32) | y[j].x;
            r_hi = ((uint64_t)y[j].w << 32) | y[j].z;
        } else if (POW2) {
            r_lo = pref_lo;
            r_hi = pref_hi;
        }
        if constexpr (POW2) {
            const uint32_t d_lo = ham64((((uint64_t)x[j].y << 32) | x[j].x) ^ r_lo);
            const uint32_t d_hi = ham64((((uint64_t)x[j].w << 32) | x[j].z) ^ r_hi);
            if (W == 1) {
                const uint32_t r = 2 * ql;          // reads r, r + 1 of the block (nr is even or the tail)
                if (r + 1 < nr) ham_store2(&out[r0 + r], d_lo, d_hi);
                else if (r < nr) ham_store(&out[r0 + r], d_lo);
            } else {
                const uint32_t G = W / 2;           // lanes per read (a power of two, <= 16)
                uint32_t s = d_lo + d_hi;
                for (uint32_t m = 1; m < G; m <<= 1) s += __shfl_xor(s, m);
                const uint32_t r = ql / G;
                if ((ql & (G - 1u)) == 0 && r < nr) ham_store(&out[r0 + r], s);
            }
        } else {
            // word -> read: floor((wl + 0.5) / W) in f32, exact for wl < 4096 and W <= 64 (the same
            // rule k_encode_ham_dense uses); the pair's two words may belong to two reads
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint32_t w = wl + h;
                const uint32_t rl = (uint32_t)__fmul_rn(__fadd_rn((float)w, 0.5f), inv_w);
                const uint32_t k = w - rl * W;
                const uint64_t v = h ? (((uint64_t)x[j].w << 32) | x[j].z) : (((uint64_t)x[j].y << 32) | x[j].x);
                uint64_t rv;
                if constexpr (PAIR) rv = h ? r_hi : r_lo;
                else rv = sref[k];
                if constexpr (PAD8) {
                    if (w < nw) part[8 * rl + k] = (uint8_t)ham64(v ^ rv);
                } else {
                    part[w] = (uint8_t)(w < nw ? ham64(v ^ rv) : 0u);
                }
            }
        }
    }
    if constexpr (!POW2) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < nr; i += T) {
            uint32_t sum = 0;
            if constexpr (PAD8) {
                const uint64_t p = part8[i] & (~0ull >> (64 - 8 * W));        // bytes W..7 never written
                sum = __builtin_amdgcn_sad_u8((uint32_t)p, 0u, 0u) + __builtin_amdgcn_sad_u8((uint32_t)(p >> 32), 0u, 0u);
            } else {
                for (uint32_t k = 0; k < W; ++k) sum += part[i * W + k];
            }
            ham_store(&out[r0 + i], sum);
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Slice / subscript on packed words (short_seq.pyx:78-238: _slice -> _slice_to_ShortSeq64 /
// _shift_copy_trim; _subscript = a 1-nt slice): output word i of read r is the 64-bit funnel shift
// of source words w, w+1 at bit 2*start + 64*i, the last word trimmed to the slice (_bzhi_u64),
// words past the slice zero.  Lane per (read, output word), power-of-two lane groups per read.
// RLEN: per-read lengths clamp (start, len) to the read (start' = min(start, L), len' = min(len,
// L - start')), Python slice semantics for trimming ragged reads.
// ------------------------------------------------------------------------------------------------
template <bool VAR>
__global__ __launch_bounds__(kThreads) void k_slice(const uint64_t* __restrict__ src, uint64_t n, uint32_t wpr,
                                                    uint32_t start_fix, uint32_t len_fix,
                                                    const uint32_t* __restrict__ starts,
                                                    const uint32_t* __restrict__ slens,
                                                    const uint32_t* __restrict__ rlens, uint64_t* __restrict__ out,
                                                    uint32_t out_wpr, uint32_t logG) {
    const uint32_t G = 1u << logG;
    const uint64_t total = n << logG;
    for (uint64_t g = (uint64_t)blockIdx.x * kThreads + threadIdx.x; g < total;
         g += (uint64_t)gridDim.x * kThreads) {
        const uint64_t r = g >> logG;
        const uint32_t i = (uint32_t)g & (G - 1u);
        if (i >= out_wpr) continue;
        uint32_t st = VAR ? starts[r] : start_fix;
        uint32_t ln = VAR ? slens[r] : len_fix;
        if (rlens) {
            const uint32_t L = rlens[r];
            st = min(st, L);
            ln = min(ln, L - st);
        }
        const uint32_t bits = 2u * ln;
        uint64_t v = 0;
        if (64u * i < bits) {
            const uint32_t bit = 2u * st + 64u * i, w = bit >> 6, o = bit & 63u;
            const uint64_t* s = src + r * wpr;
            v = (w < wpr ? s[w] : 0ull) >> o;
            if (o && w + 1 < wpr) v |= s[w + 1] << (64u - o);
            const uint32_t rem = bits - 64u * i;
            if (rem < 64u) v &= (1ull << rem) - 1ull;
        }
        out[r * out_wpr + i] = v;
    }
}

// ------------------------------------------------------------------------------------------------
// Synthetic reads; lane per (read, word).
// ------------------------------------------------------------------------------------------------
// Zipf pool draw: rank = #{k : cdf[k] <= u63} for the read's 63-bit uniform u63 (cdf[U-1] = 2^63,
// so the rank is < U); pool id = rank (id 0 the most frequent).
__device__ __forceinline__ uint64_t zipf_rank(const uint64_t* __restrict__ cdf, uint64_t U, uint64_t u63) {
    uint64_t lo = 0, hi = U;           // first k with cdf[k] > u63 lies in [lo, hi]
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (cdf[mid] <= u63) lo = mid + 1; else hi = mid;
    }
    return lo < U ? lo : U - 1;
}

// POOL: 0 = read i is generator read i; 1 = pool read drawn uniformly from U; 2 = Zipf draw (cdf)
template <int POOL>
__global__ __launch_bounds__(kThreads) void k_synth(uint8_t* out, uint64_t seed, uint64_t pool_seed,
                                                    uint64_t U, uint64_t i0, uint64_t n, uint32_t L,
                                                    uint64_t stride, const uint64_t* __restrict__ cdf = nullptr) {
    const uint32_t W = words_for(L);
    const uint64_t total = n * W;
    for (uint64_t g = (uint64_t)blockIdx.x * kThreads + threadIdx.x; g < total;
         g += (uint64_t)gridDim.x * kThreads) {
        const uint64_t k = g / W;
        const uint32_t w = (uint32_t)(g - k * W);
        uint64_t id = i0 + k;
        if (POOL == 1) id = splitmix64(pool_seed ^ (id * 0xD1B54A32D192ED03ull)) % U;
        if (POOL == 2) id = zipf_rank(cdf, U, splitmix64(pool_seed ^ (id * 0xD1B54A32D192ED03ull)) >> 1);
        const uint32_t nb = min(32u, L - 32u * w);
        uint64_t r = splitmix64(seed + id * W + w);
        if (nb < 32u) r &= (1ull << (2 * nb)) - 1ull;
        uint8_t* dst = out + k * stride + 32u * w;
        if ((((uintptr_t)dst) & 15) == 0 && (nb & 15u) == 0) {
            ((uint4*)dst)[0] = decode16((uint32_t)r);
            if (nb == 32u) ((uint4*)dst)[1] = decode16((uint32_t)(r >> 32));
        } else {
            store_chars(dst, r, nb);
        }
    }
}

// Ragged pool reads (the f2 workload): read i draws pool item
// p = splitmix64(pool_seed ^ i * 0xD1B54A32D192ED03) % U (the uniform pool draw of k_synth<1>); item
// p has length Lmin + splitmix64(seed ^ kLenSalt ^ p) % (Lmax - Lmin + 1) and word w
// splitmix64(seed + 32 p + w), masked to its nucleotides.  Mirrored by oracle.ragged_pool_*.
constexpr uint64_t kLenSalt = 0x6A09E667F3BCC909ull;

__device__ __forceinline__ uint64_t ragged_item(uint64_t pool_seed, uint64_t i, uint64_t U) {
    return splitmix64(pool_seed ^ (i * 0xD1B54A32D192ED03ull)) % U;
}

__device__ __forceinline__ uint32_t ragged_len(uint64_t seed, uint64_t p, uint32_t Lmin, uint32_t span) {
    return Lmin + (uint32_t)(splitmix64(seed ^ kLenSalt ^ p) % span);
}

__global__ __launch_bounds__(kThreads) void k_synth_ragged_lens(uint32_t* __restrict__ lens, uint64_t seed,
                                                                uint64_t pool_seed, uint64_t U, uint64_t i0,
                                                                uint64_t n, uint32_t Lmin, uint32_t span) {
    for (uint64_t k = (uint64_t)blockIdx.x * kThreads + threadIdx.x; k < n; k += (uint64_t)gridDim.x * kThreads)
        lens[k] = ragged_len(seed, ragged_item(pool_seed, i0 + k, U), Lmin, span);
}

// one lane per (read, 32-nt word slot); slots past a read's length idle
__global__ __launch_bounds__(kThreads) void k_synth_ragged(uint8_t* __restrict__ out, const uint64_t* __restrict__ offs,
                                                           uint64_t seed, uint64_t pool_seed, uint64_t U, uint64_t i0,
                                                           uint64_t n, uint32_t Lmin, uint32_t span, uint32_t wmax) {
    for (uint64_t g = (uint64_t)blockIdx.x * kThreads + threadIdx.x; g < n * wmax; g += (uint64_t)gridDim.x * kThreads) {
        const uint64_t k = g / wmax;
        const uint32_t w = (uint32_t)(g - k * wmax);
        const uint64_t p = ragged_item(pool_seed, i0 + k, U);
        const uint32_t L = ragged_len(seed, p, Lmin, span);
        if (32u * w >= L) continue;
        const uint32_t nb = min(32u, L - 32u * w);
        uint64_t r = splitmix64(seed + 32ull * p + w);
        if (nb < 32u) r &= (1ull << (2 * nb)) - 1ull;
        store_chars(out + offs[k] + 32u * w, r, nb);
    }
}

inline unsigned grid_for(uint64_t items, uint64_t per_block, unsigned cap = 0) {
    uint64_t b = (items + per_block - 1) / per_block;
    if (b == 0) b = 1;
    if (cap && b > cap) b = cap;
    return (unsigned)b;
}

constexpr unsigned kGenGridCap = 256u * 16u;   // grid-stride general kernels: 16 blocks per CU

}  // namespace

// ==================================================================================================
// Launch configurations.  Streaming kernels: T threads x U chunks of 16 B per thread, NT loads;
// shapes picked by tools/tune_kernels.hip sweeps of these exact kernels on MI355X (profiles/r1/).
// ==================================================================================================
namespace {

template <bool HAM, bool DENSE, int PATH, int T, int U, bool XCD, bool NTST>
void launch_g16(const G16Args& a, hipStream_t s) {
    const uint64_t slots = DENSE ? a.n * a.cpr : (a.n << a.logG);
    unsigned grid = grid_for(slots, (uint64_t)T * U);
    if (XCD) grid = (grid + 7u) / 8u * 8u;
    hipLaunchKernelGGL((k_encode_g16<HAM, DENSE, PATH, T, U, XCD, NTST>), dim3(grid), dim3(T), 0, s, a);
}

template <int PATH, int T, int U, bool NTST>
void launch_ham_dense(const G16Args& a, hipStream_t s) {
    const uint32_t rpb = (U * T) / a.cpr;
    if (a.cpr <= 8)
        hipLaunchKernelGGL((k_encode_ham_dense<PATH, T, U, NTST, true>), dim3(grid_for(a.n, rpb)), dim3(T), 0, s, a,
                           rpb, 1.0f / (float)a.cpr);
    else
        hipLaunchKernelGGL((k_encode_ham_dense<PATH, T, U, NTST, false>), dim3(grid_for(a.n, rpb)), dim3(T), 0, s, a,
                           rpb, 1.0f / (float)a.cpr);
}

template <int T, int U, bool NTLD, bool NTST>
void launch_decode_g16(const uint32_t* w32, uint32_t wpr2, uint64_t n, uint32_t cpr, uint32_t logG, uint4* out,
                       uint64_t out_stride16, hipStream_t s) {
    const unsigned grid = grid_for(n << logG, (uint64_t)U * T);
    hipLaunchKernelGGL((k_decode_g16<T, U, NTLD, NTST>), dim3(grid), dim3(T), 0, s, w32, wpr2, n, cpr, logG, out,
                       out_stride16);
}

// Production shapes
// dense encode: table path (L <= 32) 384 x 2, PEXT path (L % 32 == 0, L >= 64) 128 x 2 (same box,
// three interleaved rounds: 32 nt 0.6018 -> 0.5978 ms, 512 nt 4.975 -> 4.819 ms against 768 x 2;
// tools/tune_kernels.hip, profiles/r2/r2f/tune_encode_shapes.log)
constexpr int kEncT = 384, kEncU = 2, kEncTP = 128;
constexpr bool kEncXcd = false, kEncNtSt = true;
constexpr int kHamT = 192, kHamU = 4;        // fused encode + hamming (dense, LDS reduction): 768-chunk
                                             // blocks, 128 whole 96-nt reads (tools/tune_stream.hip)
constexpr int kDecT = 256, kDecU = 2;        // decode
constexpr int kHamDT = 256, kHamDU = 4;      // dense hamming on packed rows: 2048 words per block

template <int T, int U>
void launch_ham_dense_k(const uint64_t* a, const uint64_t* b, uint64_t n, uint32_t W, uint32_t* out,
                               bool pair, hipStream_t s) {
    static_assert(2 * T * U <= 4096, "block-local word index must stay < 4096 (f32 read index)");
    const uint32_t rpb = ((2u * T * U) / W) & ~1u;
    const unsigned grid = grid_for(n, rpb);
    const bool pow2 = (W & (W - 1u)) == 0;
    const float inv_w = 1.0f / (float)W;
    const uint4 *a4 = (const uint4*)a, *b4 = (const uint4*)b;
    const bool pad8 = !pow2 && W <= 8;
    if (pair && pow2)
        hipLaunchKernelGGL((k_ham_dense<true, true, T, U>), dim3(grid), dim3(T), 0, s, a4, b4, b, n, W, rpb, inv_w, out);
    else if (pair && pad8)
        hipLaunchKernelGGL((k_ham_dense<true, false, T, U, true>), dim3(grid), dim3(T), 0, s, a4, b4, b, n, W, rpb, inv_w, out);
    else if (pair)
        hipLaunchKernelGGL((k_ham_dense<true, false, T, U>), dim3(grid), dim3(T), 0, s, a4, b4, b, n, W, rpb, inv_w, out);
    else if (pow2)
        hipLaunchKernelGGL((k_ham_dense<false, true, T, U>), dim3(grid), dim3(T), 0, s, a4, b4, b, n, W, rpb, inv_w, out);
    else if (pad8)
        hipLaunchKernelGGL((k_ham_dense<false, false, T, U, true>), dim3(grid), dim3(T), 0, s, a4, b4, b, n, W, rpb, inv_w, out);
    else
        hipLaunchKernelGGL((k_ham_dense<false, false, T, U>), dim3(grid), dim3(T), 0, s, a4, b4, b, n, W, rpb, inv_w, out);
}

constexpr bool kDecNtLd = false, kDecNtSt = false;

void launch_encode_fast(const G16Args& a, bool dense, bool ham, uint32_t L, hipStream_t s) {
    const int path = L <= 32 ? kPathTable : (L % 32 == 0 ? kPathPext : kPathMixed);
    if (ham && dense) {
        if (path == kPathTable) launch_ham_dense<kPathTable, kHamT, kHamU, true>(a, s);
        else launch_ham_dense<kPathPext, kHamT, kHamU, true>(a, s);
    } else if (ham) {
        launch_g16<true, false, kPathMixed, 256, 4, false, true>(a, s);
    } else if (dense) {
        if (path == kPathTable) launch_g16<false, true, kPathTable, kEncT, kEncU, kEncXcd, kEncNtSt>(a, s);
        else launch_g16<false, true, kPathPext, kEncTP, kEncU, kEncXcd, kEncNtSt>(a, s);
    } else {
        launch_g16<false, false, kPathMixed, 256, 4, false, true>(a, s);
    }
}

}  // namespace

// ==================================================================================================
// C ABI
// ==================================================================================================
extern "C" {

// The first-bad slot is reset by a stream write packet (no fill-kernel dispatch in front of every
// encode); hipMemsetAsync only where the runtime refuses the write packet.
static int reset_first_bad(uint64_t* d_first_bad, hipStream_t s) {
    if (!d_first_bad) return SS_OK;
    if (hipStreamWriteValue64(s, d_first_bad, ~0ull, 0) == hipSuccess) return SS_OK;
    (void)hipGetLastError();
    return ss_check(hipMemsetAsync(d_first_bad, 0xFF, sizeof(uint64_t), s), "reset first_bad");
}

int ss_encode_fixed_impl(const uint8_t* d_ascii, uint64_t n, uint32_t L, uint64_t stride,
                         uint64_t* d_words, uint32_t wpr, uint64_t* d_first_bad,
                         const uint64_t* d_ref_words, uint32_t* d_out, void* stream) {
    if (L == 0 || L > SS_MAX_NT) return ss_fail(SS_EARG, "L must be in 1..1024");
    if (wpr < words_for(L) || wpr > 32) return ss_fail(SS_EARG, "wpr must be in ceil(L/32)..32");
    if (stride < L) return ss_fail(SS_EARG, "stride < L");
    if (!d_first_bad) return ss_fail(SS_EARG, "d_first_bad is required");
    if (n && (!d_ascii || (!d_words && !d_out))) return ss_fail(SS_EARG, "null buffer");
    hipStream_t s = (hipStream_t)stream;
    int rc = reset_first_bad(d_first_bad, s);
    if (rc || n == 0) return rc;
    const bool ham = d_out != nullptr;
    if (ham && !d_ref_words) return ss_fail(SS_EARG, "d_ref_words is required for hamming");
    const bool fast = (L % 16u == 0) && (stride % 16u == 0) && ((((uintptr_t)d_ascii) & 15) == 0) &&
                      (d_words == nullptr || (((uintptr_t)d_words) & 7) == 0);
    if (fast) {
        G16Args a;
        a.in = (const uint4*)d_ascii;
        a.in_stride16 = stride / 16;
        a.out32 = (uint32_t*)d_words;
        a.wpr2 = 2 * wpr;
        a.n = n;
        a.cpr = L / 16;
        a.full2 = 2 * (L / 32);
        a.all_table = L <= 32;
        a.logG = log2_ceil(a.wpr2);
        a.ref32 = (const uint32_t*)d_ref_words;
        a.ham2 = 2 * ham_words(L);
        a.counts = d_out;
        a.first_bad = (unsigned long long*)d_first_bad;
        const bool dense = stride == L && L % 32u == 0 && a.wpr2 == a.cpr;
        launch_encode_fast(a, dense, ham, L, s);
        return ss_check(hipGetLastError(), "k_encode_g16");
    }
    const uint32_t logG = log2_ceil(wpr);
    const unsigned grid = grid_for(n << logG, kThreads, kGenGridCap);
    if (ham)
        hipLaunchKernelGGL((k_encode_gen<false, true>), dim3(grid), dim3(kThreads), 0, s, d_ascii, stride,
                           (const uint64_t*)nullptr, (const uint32_t*)nullptr, L, n, d_words, wpr, logG,
                           d_ref_words, ham_words(L), d_out, (unsigned long long*)d_first_bad);
    else
        hipLaunchKernelGGL((k_encode_gen<false, false>), dim3(grid), dim3(kThreads), 0, s, d_ascii, stride,
                           (const uint64_t*)nullptr, (const uint32_t*)nullptr, L, n, d_words, wpr, logG,
                           (const uint64_t*)nullptr, 0u, (uint32_t*)nullptr, (unsigned long long*)d_first_bad);
    return ss_check(hipGetLastError(), "k_encode_gen");
}

int ss_encode_fixed(const uint8_t* d_ascii, uint64_t n, uint32_t L, uint64_t stride,
                    uint64_t* d_words, uint32_t wpr, uint64_t* d_first_bad, void* stream) {
    if (!d_words && n) return ss_fail(SS_EARG, "d_words is null");
    return ss_encode_fixed_impl(d_ascii, n, L, stride, d_words, wpr, d_first_bad, nullptr, nullptr, stream);
}

int ss_encode_hamming_ref(const uint8_t* d_ascii, uint64_t n, uint32_t L, uint64_t stride,
                          uint64_t* d_words, uint32_t wpr, const uint64_t* d_ref_words,
                          uint32_t* d_out, uint64_t* d_first_bad, void* stream) {
    if (!d_out && n) return ss_fail(SS_EARG, "d_out is null");
    return ss_encode_fixed_impl(d_ascii, n, L, stride, d_words, wpr, d_first_bad, d_ref_words, d_out, stream);
}

int ss_encode_var(const uint8_t* d_ascii, const uint64_t* d_offsets, const uint32_t* d_lens,
                  uint64_t n, uint64_t* d_words, uint32_t wpr, uint64_t* d_first_bad, void* stream) {
    if (wpr == 0 || wpr > 32) return ss_fail(SS_EARG, "wpr must be in 1..32");
    if (!d_first_bad) return ss_fail(SS_EARG, "d_first_bad is required");
    if (n && (!d_ascii || !d_offsets || !d_lens || !d_words)) return ss_fail(SS_EARG, "null buffer");
    hipStream_t s = (hipStream_t)stream;
    int rc = reset_first_bad(d_first_bad, s);
    if (rc || n == 0) return rc;
    // kVarK words per lane, no grid-stride round: every lane's dependent loads (offset / length,
    // then the bytes) overlap across many resident waves
    const unsigned grid = grid_for((n * wpr + kVarK - 1) / kVarK, kThreads, 0x7FFFFFFFu);
    if ((uint64_t)grid * kThreads * kVarK < n * wpr) return ss_fail(SS_EARG, "ss_encode_var: batch too large");
    hipLaunchKernelGGL(k_encode_var_dense, dim3(grid), dim3(kThreads), 0, s, d_ascii, d_offsets, d_lens, n, d_words,
                       wpr, 1.0 / (double)wpr, (unsigned long long*)d_first_bad);
    return ss_check(hipGetLastError(), "k_encode_var_dense");
}

int ss_short_keys_impl(const uint8_t* d_buf, const uint64_t* d_offs, const uint32_t* d_lens, const uint64_t* d_sel,
                       uint64_t m, uint32_t dense_L, uint64_t* d_keys, uint64_t* d_first_bad, void* stream) {
    if (dense_L > 31) return ss_fail(SS_EARG, "k_short_keys: reads of 1 to 31 nt");
    if (m == 0) return SS_OK;
    const unsigned grid = grid_for(m, 256, 8192);
    hipLaunchKernelGGL(k_short_keys, dim3(grid), dim3(256), 0, (hipStream_t)stream, d_buf, d_offs, d_lens, d_sel, m,
                       dense_L, d_keys, (unsigned long long*)d_first_bad);
    return ss_check(hipGetLastError(), "k_short_keys");
}

int ss_encode_rows_impl(const uint8_t* d_buf, const uint64_t* d_offs, const uint32_t* d_lens, uint64_t n, uint32_t S,
                        uint64_t* d_out, uint64_t* d_fps, uint32_t* d_hll, uint64_t* d_first_bad, void* stream,
                        const uint64_t* d_gate) {
    if (S < 3 || S > 6) return ss_fail(SS_EARG, "k_encode_rows: rows of 3 to 6 words");
    if (n == 0) return SS_OK;
    // persistent waves (the occupancy's worth of blocks), each over tiles of R * kRowsK reads with the
    // next tile's lengths / offsets and the last tile's sketch registers in flight
    static const int resident = [] {         // thread-safe one-time init (every device is a gfx950)
        int dev = 0, cus = 0, occ = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)k_encode_rows, 256, 0);
        return std::max(1, cus) * std::max(1, occ);
    }();
    const uint64_t per = (uint64_t)(64 / S) * kRowsK, tiles = (n + per - 1) / per;
    const uint64_t blocks = std::min<uint64_t>((tiles + 3) / 4, (uint64_t)resident);
    hipLaunchKernelGGL(k_encode_rows, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, d_buf, d_offs, d_lens,
                       n, S, d_out, d_fps, d_hll, (unsigned long long*)d_first_bad, d_gate);
    return ss_check(hipGetLastError(), "k_encode_rows");
}

int ss_encode_classes_impl(const uint8_t* d_buf, const uint64_t* d_offs, const uint32_t* d_lens, uint64_t n,
                           const uint32_t* d_blkoff, uint32_t nblk, const uint64_t* h_woff, const uint64_t* h_fpoff,
                           uint64_t* const* h_rmap, uint64_t base, uint32_t bin0, uint32_t w1max, uint64_t* d_out,
                           uint64_t* d_fps, uint32_t* d_hll, uint64_t* d_first_bad, void* stream) {
    if (n == 0) return SS_OK;
    if (w1max < 3 || w1max > 16) return ss_fail(SS_EARG, "k_encode_classes: classes of 2 to 15 words");
    ClassOut co;
    for (int W = 0; W < 33; ++W) {
        co.woff[W] = h_woff[W];
        co.fpoff[W] = h_fpoff ? h_fpoff[W] : 0;
        co.rmap[W] = h_rmap ? h_rmap[W] : nullptr;
    }
    co.base = base;
    co.bin0 = bin0;
    const size_t lds = (size_t)kClsTile * w1max * 12;
    hipLaunchKernelGGL(k_encode_classes, dim3(nblk), dim3(kClsTile), lds, (hipStream_t)stream, d_buf, d_offs, d_lens, n,
                       d_blkoff, nblk, co, w1max, d_out, d_fps, d_hll, (unsigned long long*)d_first_bad);
    return ss_check(hipGetLastError(), "k_encode_classes");
}

int ss_hll_rows_impl(const uint64_t* d_rows, uint64_t m, uint32_t W1, uint32_t* d_hll, void* stream) {
    if (m == 0) return SS_OK;
    hipLaunchKernelGGL(k_hll_rows, dim3(grid_for(m, kThreads, 4096)), dim3(kThreads), 0, (hipStream_t)stream, d_rows, m,
                       W1, d_hll);
    return ss_check(hipGetLastError(), "k_hll_rows");
}

int ss_encode_class_impl(const uint8_t* d_buf, const uint64_t* d_offs, const uint32_t* d_lens, const uint64_t* d_sel,
                         uint32_t dense_L, uint64_t m, uint32_t W, uint64_t* d_out, uint64_t* d_first_bad,
                         void* stream) {
    if (m == 0) return SS_OK;
    if (W < 2 || W > 32) return ss_fail(SS_EARG, "class words must be in 2..32");
    const unsigned grid = grid_for(m * (W + 1), kThreads, 0x7FFFFFFFu);
    hipLaunchKernelGGL(k_encode_class, dim3(grid), dim3(kThreads), 0, (hipStream_t)stream, d_buf, d_offs, d_lens, d_sel,
                       dense_L, m, W, 1.0 / (double)(W + 1), d_out, (unsigned long long*)d_first_bad);
    return ss_check(hipGetLastError(), "k_encode_class");
}

int ss_decode_fixed(const uint64_t* d_words, uint64_t n, uint32_t L, uint32_t wpr,
                    uint8_t* d_ascii, uint64_t stride, void* stream) {
    if (L > SS_MAX_NT) return ss_fail(SS_EARG, "L must be <= 1024");
    if (wpr < words_for(L) || wpr == 0 || wpr > 32) return ss_fail(SS_EARG, "bad wpr");
    if (stride < L) return ss_fail(SS_EARG, "stride < L");
    if (n == 0 || L == 0) return SS_OK;
    if (!d_words || !d_ascii) return ss_fail(SS_EARG, "null buffer");
    hipStream_t s = (hipStream_t)stream;
    const bool fast = (L % 16u == 0) && (stride % 16u == 0) && ((((uintptr_t)d_ascii) & 15) == 0) &&
                      ((((uintptr_t)d_words) & 7) == 0);
    if (fast) {
        const uint32_t cpr = L / 16, wpr2 = 2 * wpr, logG = log2_ceil(cpr);
        launch_decode_g16<kDecT, kDecU, kDecNtLd, kDecNtSt>((const uint32_t*)d_words, wpr2, n, cpr, logG,
                                                            (uint4*)d_ascii, stride / 16, s);
        return ss_check(hipGetLastError(), "k_decode_g16");
    }
    const unsigned grid = grid_for(n * wpr, kThreads, kGenGridCap);
    hipLaunchKernelGGL((k_decode_gen<false>), dim3(grid), dim3(kThreads), 0, s, d_words,
                       (const uint32_t*)nullptr, L, n, wpr, d_ascii, stride, (const uint64_t*)nullptr);
    return ss_check(hipGetLastError(), "k_decode_gen");
}

int ss_decode_var(const uint64_t* d_words, const uint32_t* d_lens, uint64_t n, uint32_t wpr,
                  uint8_t* d_ascii, const uint64_t* d_offsets, void* stream) {
    if (wpr == 0 || wpr > 32) return ss_fail(SS_EARG, "bad wpr");
    if (n == 0) return SS_OK;
    if (!d_words || !d_lens || !d_ascii || !d_offsets) return ss_fail(SS_EARG, "null buffer");
    const unsigned grid = grid_for(n * wpr, kThreads, kGenGridCap);
    hipLaunchKernelGGL((k_decode_gen<true>), dim3(grid), dim3(kThreads), 0, (hipStream_t)stream, d_words,
                       d_lens, 0u, n, wpr, d_ascii, (uint64_t)0, d_offsets);
    return ss_check(hipGetLastError(), "k_decode_gen<var>");
}

static int launch_ham(const uint64_t* a, const uint64_t* b, uint64_t n, uint32_t L, uint32_t wpr,
                      uint32_t* out, void* stream, bool pair) {
    if (L > SS_MAX_NT) return ss_fail(SS_EARG, "L must be <= 1024");
    const uint32_t W = ham_words(L);
    if (wpr < W || wpr > 32) return ss_fail(SS_EARG, "bad wpr");
    if (n == 0) return SS_OK;
    if (!a || !b || !out) return ss_fail(SS_EARG, "null buffer");
    const bool aligned = (((uintptr_t)a | (uintptr_t)(pair ? b : a)) & 15u) == 0 && (((uintptr_t)out) & 7u) == 0;
    if (wpr == W && aligned && W <= 32) {   // dense rows: the streaming kernel (W <= 32 keeps wl < 4096 exact)
        hipStream_t s = (hipStream_t)stream;
        if (W == 3) {   // 96 nt (C3'): lane pairs of dwordx3 halves, 2 x 32 reads per wave, 2 waves per block
            constexpr int T = 128, U = 2;
            const unsigned grid = grid_for(n, (uint64_t)32 * (T / 64) * U);
            const uint32_t *a32 = (const uint32_t*)a, *b32 = (const uint32_t*)b;
            if (pair) hipLaunchKernelGGL((k_ham_dense3x<true, T, U>), dim3(grid), dim3(T), 0, s, a32, b32, b, n, out);
            else hipLaunchKernelGGL((k_ham_dense3x<false, T, U>), dim3(grid), dim3(T), 0, s, a32, b32, b, n, out);
            return ss_check(hipGetLastError(), "k_ham_dense3x");
        }
        // hamming vs one read on power-of-two W: small blocks (4-8 KiB of rows each) stream best
        // (tools/tune_ham.hip, same box: W 1 0.786 -> 0.850, 2 0.779 -> 0.844, 4 0.775 -> 0.801,
        // 8 0.756 -> 0.789, 16 0.747 -> 0.777 of 8 TB/s; W 32 level)
        const bool pow2 = (W & (W - 1u)) == 0;
        if (!pair && pow2 && W <= 2) launch_ham_dense_k<128, 2>(a, b, n, W, out, pair, s);
        else if (!pair && pow2 && (W == 8 || W == 16)) launch_ham_dense_k<64, 4>(a, b, n, W, out, pair, s);
        else if (!pair && pow2) launch_ham_dense_k<128, 4>(a, b, n, W, out, pair, s);
        else launch_ham_dense_k<kHamDT, kHamDU>(a, b, n, W, out, pair, s);
        return ss_check(hipGetLastError(), "k_ham_dense");
    }
    const uint32_t logG = log2_ceil(W);
    const unsigned grid = grid_for(n << logG, kThreads);
    if (pair)
        hipLaunchKernelGGL((k_ham_group<true>), dim3(grid), dim3(kThreads), 0, (hipStream_t)stream, a, b,
                           n, W, wpr, logG, out);
    else
        hipLaunchKernelGGL((k_ham_group<false>), dim3(grid), dim3(kThreads), 0, (hipStream_t)stream, a, b,
                           n, W, wpr, logG, out);
    return ss_check(hipGetLastError(), "k_ham_group");
}

int ss_hamming_ref(const uint64_t* d_words, uint64_t n, uint32_t L, uint32_t wpr,
                   const uint64_t* d_ref, uint32_t* d_out, void* stream) {
    return launch_ham(d_words, d_ref, n, L, wpr, d_out, stream, false);
}

int ss_hamming_pair(const uint64_t* d_a, const uint64_t* d_b, uint64_t n, uint32_t L, uint32_t wpr,
                    uint32_t* d_out, void* stream) {
    return launch_ham(d_a, d_b, n, L, wpr, d_out, stream, true);
}

int ss_slice_fixed(const uint64_t* d_words, uint64_t n, uint32_t L, uint32_t wpr, uint32_t start, uint32_t len,
                   uint64_t* d_out, uint32_t out_wpr, void* stream) {
    if (L > SS_MAX_NT || wpr < words_for(L) || wpr == 0 || wpr > 32) return ss_fail(SS_EARG, "bad L / wpr");
    if ((uint64_t)start + len > L) return ss_fail(SS_EARG, "slice past the read");
    if (out_wpr < (words_for(len) ? words_for(len) : 1u) || out_wpr > 32) return ss_fail(SS_EARG, "bad out_wpr");
    if (n == 0) return SS_OK;
    if (!d_words || !d_out) return ss_fail(SS_EARG, "null buffer");
    const uint32_t logG = log2_ceil(out_wpr);
    const unsigned grid = grid_for(n << logG, kThreads, kGenGridCap);
    hipLaunchKernelGGL((k_slice<false>), dim3(grid), dim3(kThreads), 0, (hipStream_t)stream, d_words, n, wpr, start,
                       len, (const uint32_t*)nullptr, (const uint32_t*)nullptr, (const uint32_t*)nullptr, d_out,
                       out_wpr, logG);
    return ss_check(hipGetLastError(), "k_slice");
}

int ss_slice_var(const uint64_t* d_words, uint64_t n, uint32_t wpr, const uint32_t* d_read_lens,
                 const uint32_t* d_starts, const uint32_t* d_lens, uint64_t* d_out, uint32_t out_wpr, void* stream) {
    if (wpr == 0 || wpr > 32 || out_wpr == 0 || out_wpr > 32) return ss_fail(SS_EARG, "bad wpr / out_wpr");
    if (n == 0) return SS_OK;
    if (!d_words || !d_starts || !d_lens || !d_out) return ss_fail(SS_EARG, "null buffer");
    const uint32_t logG = log2_ceil(out_wpr);
    const unsigned grid = grid_for(n << logG, kThreads, kGenGridCap);
    hipLaunchKernelGGL((k_slice<true>), dim3(grid), dim3(kThreads), 0, (hipStream_t)stream, d_words, n, wpr, 0u, 0u,
                       d_starts, d_lens, d_read_lens, d_out, out_wpr, logG);
    return ss_check(hipGetLastError(), "k_slice<var>");
}

int ss_synth_reads(uint8_t* d_ascii, uint64_t seed, uint64_t i0, uint64_t n, uint32_t L,
                   uint64_t stride, void* stream) {
    if (L == 0 || L > SS_MAX_NT || stride < L) return ss_fail(SS_EARG, "bad L/stride");
    if (n == 0) return SS_OK;
    if (!d_ascii) return ss_fail(SS_EARG, "null buffer");
    const unsigned grid = grid_for(n * words_for(L), kThreads, kGenGridCap);
    hipLaunchKernelGGL((k_synth<0>), dim3(grid), dim3(kThreads), 0, (hipStream_t)stream, d_ascii, seed,
                       (uint64_t)0, (uint64_t)1, i0, n, L, stride);
    return ss_check(hipGetLastError(), "k_synth");
}

int ss_synth_pool_reads(uint8_t* d_ascii, uint64_t seed, uint64_t pool_seed, uint64_t U,
                        uint64_t i0, uint64_t n, uint32_t L, uint64_t stride, void* stream) {
    if (L == 0 || L > SS_MAX_NT || stride < L || U == 0) return ss_fail(SS_EARG, "bad L/stride/U");
    if (n == 0) return SS_OK;
    if (!d_ascii) return ss_fail(SS_EARG, "null buffer");
    const unsigned grid = grid_for(n * words_for(L), kThreads, kGenGridCap);
    hipLaunchKernelGGL((k_synth<1>), dim3(grid), dim3(kThreads), 0, (hipStream_t)stream, d_ascii, seed,
                       pool_seed, U, i0, n, L, stride, (const uint64_t*)nullptr);
    return ss_check(hipGetLastError(), "k_synth<pool>");
}

int ss_synth_ragged_lens(uint32_t* d_lens, uint64_t seed, uint64_t pool_seed, uint64_t U, uint64_t i0, uint64_t n,
                         uint32_t Lmin, uint32_t Lmax, void* stream) {
    if (Lmin > Lmax || Lmax > SS_MAX_NT || U == 0) return ss_fail(SS_EARG, "bad Lmin/Lmax/U");
    if (n == 0) return SS_OK;
    if (!d_lens) return ss_fail(SS_EARG, "null buffer");
    hipLaunchKernelGGL(k_synth_ragged_lens, dim3(grid_for(n, kThreads, kGenGridCap)), dim3(kThreads), 0,
                       (hipStream_t)stream, d_lens, seed, pool_seed, U, i0, n, Lmin, Lmax - Lmin + 1);
    return ss_check(hipGetLastError(), "k_synth_ragged_lens");
}

int ss_synth_ragged_reads(uint8_t* d_blob, const uint64_t* d_offsets, uint64_t seed, uint64_t pool_seed, uint64_t U,
                          uint64_t i0, uint64_t n, uint32_t Lmin, uint32_t Lmax, void* stream) {
    if (Lmin > Lmax || Lmax > SS_MAX_NT || U == 0) return ss_fail(SS_EARG, "bad Lmin/Lmax/U");
    if (n == 0) return SS_OK;
    if (!d_blob || !d_offsets) return ss_fail(SS_EARG, "null buffer");
    const uint32_t wmax = words_for(Lmax ? Lmax : 1);
    hipLaunchKernelGGL(k_synth_ragged, dim3(grid_for(n * wmax, kThreads, kGenGridCap)), dim3(kThreads), 0,
                       (hipStream_t)stream, d_blob, d_offsets, seed, pool_seed, U, i0, n, Lmin, Lmax - Lmin + 1, wmax);
    return ss_check(hipGetLastError(), "k_synth_ragged");
}

int ss_synth_zipf_reads(uint8_t* d_ascii, uint64_t seed, uint64_t pool_seed, const uint64_t* d_cdf, uint64_t U,
                        uint64_t i0, uint64_t n, uint32_t L, uint64_t stride, void* stream) {
    if (L == 0 || L > SS_MAX_NT || stride < L || U == 0) return ss_fail(SS_EARG, "bad L/stride/U");
    if (n == 0) return SS_OK;
    if (!d_ascii || !d_cdf) return ss_fail(SS_EARG, "null buffer");
    const unsigned grid = grid_for(n * words_for(L), kThreads, kGenGridCap);
    hipLaunchKernelGGL((k_synth<2>), dim3(grid), dim3(kThreads), 0, (hipStream_t)stream, d_ascii, seed,
                       pool_seed, U, i0, n, L, stride, d_cdf);
    return ss_check(hipGetLastError(), "k_synth<zipf>");
}

}  // extern "C"
