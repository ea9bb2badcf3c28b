// ss_fastq.hip — FASTQ ingest on the device: sequence-line index + row gather.
//
// Reference rule (fast_read.pyx:3-20, _read_fastq_short_seqs): getline() splits the file at '\n',
// the line counter starts at 1 and lines with count % 4 == 2 are kept (0-based line j: j % 4 == 1);
// each kept line goes through _from_chars (short_seq.pyx:49-52): length = strlen(line) - 1.  So the
// trailing '\n' is dropped, a last line without '\n' loses its last character, an embedded NUL
// ends the line early, and strlen 0 (a NUL first) underflows into the too-long error
// (short_seq.pyx:74).
//
// Device passes over one chunk of the file (a chunk < 4 GiB that ends right after a '\n', or at
// EOF); the caller owns every buffer, nothing is allocated here:
//   ss_fastq_scan : k_fq_count (newlines per 16-KiB tile, dwordx4 loads + SWAR byte compare)
//                   k_fq_scan_local / k_fq_scan_groups (two-level exclusive scan -> tile bases)
//   ss_fastq_index: k_fq_emit  (re-reads the tile; the block scan gives every 16-B chunk its line
//                               number; each '\n' closes a sequence line (end) or opens one (start),
//                               each NUL inside a sequence line is folded in with atomicMin)
//                   k_fq_lens  (thread per sequence line: the strlen - 1 rule -> lens)
// Output: d_offsets[i] / d_lens[i] of sequence line i, exactly the ragged layout ss_encode_var and
// ss_gather_rows take.  HBM traffic: the chunk is read twice (count + emit), ~2 B per file byte.
#include "ss_device.h"
#include "ss_internal.h"

namespace {

using namespace ssd;

constexpr int kFqT = 256;                                   // threads per block
constexpr int kFqU = 4;                                     // 16-B chunks per thread
constexpr uint64_t kFqTile = (uint64_t)kFqT * kFqU * 16;    // 16 KiB per block
constexpr uint32_t kNone32 = 0xFFFFFFFFu;

// 0x80 in every byte of x equal to the byte replicated in pat, 0 elsewhere (exact, no false hits).
__device__ __forceinline__ uint32_t eq_bytes(uint32_t x, uint32_t pat) {
    const uint32_t v = x ^ pat;
    return ~(((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v | 0x7F7F7F7Fu);
}

// 16 bytes of the chunk at byte offset `off` (< nbytes); bytes past nbytes read as ' ' (neither
// '\n' nor NUL).  d_buf is 16-B aligned, so only the last chunk can be partial.
__device__ __forceinline__ uint4 load_chunk(const uint8_t* buf, uint64_t off, uint64_t nbytes) {
    if (off + 16 <= nbytes) return ld_stream((const uint4*)(buf + off));
    uint32_t w[4] = {0x20202020u, 0x20202020u, 0x20202020u, 0x20202020u};
    for (uint32_t b = 0; b < 16 && off + b < nbytes; ++b) {
        const uint32_t sh = 8 * (b & 3);
        w[b >> 2] = (w[b >> 2] & ~(0xFFu << sh)) | ((uint32_t)buf[off + b] << sh);
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ uint32_t count_nl(const uint4& x) {
    return __popc(eq_bytes(x.x, 0x0A0A0A0Au)) + __popc(eq_bytes(x.y, 0x0A0A0A0Au)) +
           __popc(eq_bytes(x.z, 0x0A0A0A0Au)) + __popc(eq_bytes(x.w, 0x0A0A0A0Au));
}

__global__ __launch_bounds__(kFqT) void k_fq_count(const uint8_t* __restrict__ buf, uint64_t nbytes,
                                                   uint32_t* __restrict__ tile_cnt) {
    __shared__ uint32_t part[kFqT / 64];
    const uint64_t t0 = (uint64_t)blockIdx.x * kFqTile;
    uint4 x[kFqU];
#pragma unroll
    for (int j = 0; j < kFqU; ++j) {
        const uint64_t off = t0 + 16ull * (j * kFqT + threadIdx.x);
        x[j] = off < nbytes ? load_chunk(buf, off, nbytes) : make_uint4(0x20202020u, 0x20202020u, 0x20202020u, 0x20202020u);
    }
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < kFqU; ++j) c += count_nl(x[j]);
    for (int s = 32; s > 0; s >>= 1) c += __shfl_xor(c, s);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int i = 0; i < kFqT / 64; ++i) t += part[i];
        tile_cnt[blockIdx.x] = t;
    }
}

// Tile bases in two levels: group g = tiles [1024 g, 1024 g + 1024) is scanned by one block of
// 1024 (one coalesced load per thread), which writes the tiles' group-local exclusive prefixes and
// the group total; k_fq_scan_groups (one block) turns the group totals into group bases.  (The
// former one-block scan looped over ntiles / 1024 dependent loads per thread: 0.24 ms for 2 GB.)
__device__ __forceinline__ uint64_t block_excl_scan_1024(uint64_t v, uint64_t* wsum, uint64_t& total) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint64_t inc = v;
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t o = __shfl_up(inc, d);
        if (lane >= (uint32_t)d) inc += o;
    }
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    uint64_t before = 0;
    total = 0;
    for (uint32_t w = 0; w < 16; ++w) {
        if (w < wave) before += wsum[w];
        total += wsum[w];
    }
    return before + inc - v;
}

__global__ __launch_bounds__(1024) void k_fq_scan_local(const uint32_t* __restrict__ tile_cnt, uint64_t ntiles,
                                                        uint64_t* __restrict__ tile_base,
                                                        uint64_t* __restrict__ group_tot) {
    __shared__ uint64_t wsum[16];
    const uint64_t i = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
    const uint64_t v = i < ntiles ? tile_cnt[i] : 0;
    uint64_t total;
    const uint64_t ex = block_excl_scan_1024(v, wsum, total);
    if (i < ntiles) tile_base[i] = ex;
    if (threadIdx.x == 0) group_tot[blockIdx.x] = total;
}

// one block: exclusive scan of the group totals in place (any number of groups, 1024 per round) ->
// group bases (k_fq_emit adds its tile's group base); tile_base[ntiles] = *d_nl = all newlines
__global__ __launch_bounds__(1024) void k_fq_scan_groups(uint64_t* __restrict__ group_tot, uint64_t ngroups,
                                                         uint64_t ntiles, uint64_t* __restrict__ tile_base,
                                                         uint64_t* d_nl) {
    __shared__ uint64_t wsum[16];
    __shared__ uint64_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (uint64_t g0 = 0; g0 < ngroups; g0 += 1024) {
        const uint64_t g = g0 + threadIdx.x;
        const uint64_t v = g < ngroups ? group_tot[g] : 0;
        uint64_t total;
        const uint64_t ex = block_excl_scan_1024(v, wsum, total);
        const uint64_t c = carry;
        if (g < ngroups) group_tot[g] = c + ex;       // group base
        __syncthreads();
        if (threadIdx.x == 0) carry = c + total;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        tile_base[ntiles] = carry;
        *d_nl = carry;
    }
}

struct FqOut {
    uint64_t* offsets;
    uint64_t* ends;      // aux: '\n' position closing sequence line i (~0: none)
    uint32_t* nul;       // NUL position (chunk-relative u32) inside sequence line i (~0u: none)
    uint64_t max_reads;
    uint64_t sel0;       // (line0 + 2) / 4 = sequence lines before the chunk
    uint64_t nbytes;
};

// '\n' at p closes line j (global index)
__device__ __forceinline__ void on_newline(const FqOut& o, uint64_t p, uint64_t j) {
    const uint32_t m = (uint32_t)(j & 3u);
    if (m == 1u) {
        const uint64_t i = (j + 2) / 4 - o.sel0;
        if (i < o.max_reads) o.ends[i] = p;
    } else if (m == 0u && p + 1 < o.nbytes) {
        const uint64_t i = (j + 3) / 4 - o.sel0;        // line j + 1 is a sequence line
        if (i < o.max_reads) o.offsets[i] = p + 1;
    }
}

__global__ __launch_bounds__(kFqT) void k_fq_emit(const uint8_t* __restrict__ buf, FqOut o, uint64_t line0,
                                                  const uint64_t* __restrict__ tile_base,
                                                  const uint64_t* __restrict__ group_base) {
    __shared__ uint64_t wtot[kFqT / 64];
    const uint64_t t0 = (uint64_t)blockIdx.x * kFqTile;
    uint4 x[kFqU];
    uint64_t packed = 0;                   // 16-bit newline count of chunk j at bits 16j
#pragma unroll
    for (int j = 0; j < kFqU; ++j) {
        const uint64_t off = t0 + 16ull * (j * kFqT + threadIdx.x);
        x[j] = off < o.nbytes ? load_chunk(buf, off, o.nbytes) : make_uint4(0x20202020u, 0x20202020u, 0x20202020u, 0x20202020u);
        packed |= (uint64_t)count_nl(x[j]) << (16 * j);
    }
    // block-wide inclusive scan of the four 16-bit lanes at once (each field's total <= 4096)
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint64_t v = packed;
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t u = __shfl_up(v, d);
        if (lane >= (uint32_t)d) v += u;
    }
    if (lane == 63) wtot[wave] = v;
    __syncthreads();
    uint64_t before = 0, total = 0;
#pragma unroll
    for (int w = 0; w < kFqT / 64; ++w) {
        if ((uint32_t)w < wave) before += wtot[w];
        total += wtot[w];
    }
    const uint64_t excl = before + v - packed;
    uint64_t rows_before = 0;              // newlines in the rows j' < j (whole block)
    const uint64_t lbase = line0 + group_base[blockIdx.x >> 10] + tile_base[blockIdx.x];
#pragma unroll
    for (int j = 0; j < kFqU; ++j) {
        const uint64_t off = t0 + 16ull * (j * kFqT + threadIdx.x);
        uint64_t li = lbase + rows_before + ((excl >> (16 * j)) & 0xFFFFu);
        rows_before += (total >> (16 * j)) & 0xFFFFu;
        if (off >= o.nbytes) continue;
        const uint32_t xw[4] = {x[j].x, x[j].y, x[j].z, x[j].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t mnl = eq_bytes(xw[q], 0x0A0A0A0Au), mnul = eq_bytes(xw[q], 0u);
            uint32_t m = mnl | mnul;
            while (m) {
                const uint32_t bit = __builtin_ctz(m);
                m &= m - 1;
                const uint64_t p = off + 4 * q + (bit >> 3);
                if (p >= o.nbytes) break;
                if ((mnl >> bit) & 1u) {
                    on_newline(o, p, li);
                    ++li;
                } else if ((li & 3u) == 1u) {
                    const uint64_t i = (li + 2) / 4 - o.sel0;
                    if (i < o.max_reads) atomicMin(&o.nul[i], (uint32_t)p);
                }
            }
        }
    }
}

__global__ __launch_bounds__(256) void k_fq_lens(const uint8_t* __restrict__ buf, FqOut o, uint64_t line0,
                                                 int at_eof, uint64_t ntiles, const uint64_t* __restrict__ tile_base,
                                                 uint32_t* __restrict__ lens, uint64_t* d_nreads) {
    const uint64_t nl = tile_base[ntiles];
    const bool partial = at_eof && o.nbytes > 0 && buf[o.nbytes - 1] != '\n';
    const uint64_t nlines = nl + (partial ? 1u : 0u);
    const uint64_t nsel = (line0 + nlines + 2) / 4 - o.sel0;
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i == 0) *d_nreads = nsel;
    if (i >= nsel || i >= o.max_reads) return;
    uint64_t start = o.offsets[i];
    if (i == 0 && (line0 & 3u) == 1u) {
        start = 0;                          // the chunk opens with a sequence line
        o.offsets[0] = 0;
    }
    const uint64_t e = o.ends[i];
    const bool has_nl = e != ~0ull;
    const uint64_t end = has_nl ? e : o.nbytes;
    const uint32_t nul = o.nul[i];
    const uint64_t slen = nul != kNone32 ? (uint64_t)nul - start : end - start + (has_nl ? 1u : 0u);
    lens[i] = slen == 0 ? kNone32 : (uint32_t)min<uint64_t>(slen - 1, 0xFFFFFFFEull);
}

// Gather rows: dst row r (r < m) = src[offsets[sel ? sel[r] : r] ..  + L), L <= 1024, into a dense
// 16-B aligned layout (dst_stride % 16 == 0); bytes of the last 16-B chunk past L are 'A'.
// Lane per 16-B output chunk: aligned dword loads (only dwords entirely inside src_bytes; the rest
// bytewise) + v_alignbyte, one dwordx4 store.
__global__ __launch_bounds__(256) void k_gather_rows(const uint8_t* __restrict__ src, uint64_t src_bytes,
                                                     const uint64_t* __restrict__ offs,
                                                     const uint64_t* __restrict__ sel, uint64_t m, uint32_t L,
                                                     uint32_t cpo, uint8_t* __restrict__ dst, uint64_t dst_stride) {
    const uint64_t total = m * cpo;
    for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g < total; g += (uint64_t)gridDim.x * 256) {
        const uint64_t r = g / cpo;
        const uint32_t k = (uint32_t)(g - r * cpo);
        const uint64_t row = sel ? sel[r] : r;
        const uint64_t off = offs[row] + 16ull * k;
        const uint32_t nb = min(16u, L - 16u * k);
        const uint64_t a0 = off & ~3ull;
        const uint32_t sh = (uint32_t)(off & 3u);
        uint32_t d[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const uint64_t a = a0 + 4ull * i;
            if (a + 4 <= src_bytes) {
                d[i] = *(const uint32_t*)(src + a);
            } else {
                uint32_t v = 0x41414141u;
                for (uint32_t b = 0; b < 4; ++b)
                    if (a + b < src_bytes) v = (v & ~(0xFFu << (8 * b))) | ((uint32_t)src[a + b] << (8 * b));
                d[i] = v;
            }
        }
        uint32_t o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            uint32_t v = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh);
            const int rem = (int)nb - 4 * i;
            if (rem <= 0) {
                v = 0x41414141u;
            } else if (rem < 4) {
                const uint32_t keep = (1u << (8 * rem)) - 1u;
                v = (v & keep) | (0x41414141u & ~keep);
            }
            o[i] = v;
        }
        *(uint4*)(dst + r * dst_stride + 16ull * k) = make_uint4(o[0], o[1], o[2], o[3]);
    }
}

inline uint64_t fq_tiles(uint64_t nbytes) { return (nbytes + kFqTile - 1) / kFqTile; }

inline uint64_t fq_groups(uint64_t t) { return (t + 1023) / 1024; }

}  // namespace

extern "C" {

// workspace: tile_base u64 [t + 1] | group_base u64 [g + 1] | tile_cnt u32 [t]
uint64_t ss_fastq_scan_ws_bytes(uint64_t nbytes) {
    const uint64_t t = fq_tiles(nbytes);
    return 8 * (t + 1) + 8 * (fq_groups(t) + 1) + 4 * t + 16;
}

int ss_fastq_scan(const uint8_t* d_buf, uint64_t nbytes, void* d_ws, uint64_t ws_bytes, uint64_t* d_nlines,
                  void* stream) {
    if (nbytes >= (1ull << 32)) return ss_fail(SS_EARG, "FASTQ chunk must be < 4 GiB");
    if (!d_ws || !d_nlines || (nbytes && !d_buf)) return ss_fail(SS_EARG, "null buffer");
    if ((((uintptr_t)d_buf) & 15) || (((uintptr_t)d_ws) & 7)) return ss_fail(SS_EARG, "d_buf must be 16-B aligned, d_ws 8-B");
    if (ws_bytes < ss_fastq_scan_ws_bytes(nbytes)) return ss_fail(SS_EARG, "workspace too small");
    hipStream_t s = (hipStream_t)stream;
    const uint64_t t = fq_tiles(nbytes);
    uint64_t* tile_base = (uint64_t*)d_ws;
    uint64_t* group_base = tile_base + t + 1;
    const uint64_t g = fq_groups(t);
    uint32_t* tile_cnt = (uint32_t*)(group_base + g + 1);
    if (t) {
        hipLaunchKernelGGL(k_fq_count, dim3((unsigned)t), dim3(kFqT), 0, s, d_buf, nbytes, tile_cnt);
        hipLaunchKernelGGL(k_fq_scan_local, dim3((unsigned)g), dim3(1024), 0, s, (const uint32_t*)tile_cnt, t,
                           tile_base, group_base);
    }
    hipLaunchKernelGGL(k_fq_scan_groups, dim3(1), dim3(1024), 0, s, group_base, g, t, tile_base, d_nlines);
    return ss_check(hipGetLastError(), "k_fq_count/k_fq_scan");
}

int ss_fastq_index(const uint8_t* d_buf, uint64_t nbytes, uint64_t line0, int at_eof, const void* d_ws,
                   uint64_t* d_offsets, uint32_t* d_lens, uint64_t* d_aux, uint64_t max_reads,
                   uint64_t* d_nreads, void* stream) {
    if (nbytes >= (1ull << 32)) return ss_fail(SS_EARG, "FASTQ chunk must be < 4 GiB");
    if (!d_ws || !d_nreads || (nbytes && !d_buf)) return ss_fail(SS_EARG, "null buffer");
    if (max_reads && (!d_offsets || !d_lens || !d_aux)) return ss_fail(SS_EARG, "null output buffer");
    if ((((uintptr_t)d_buf) & 15) || (((uintptr_t)d_ws) & 7)) return ss_fail(SS_EARG, "d_buf must be 16-B aligned, d_ws 8-B");
    hipStream_t s = (hipStream_t)stream;
    const uint64_t t = fq_tiles(nbytes);
    const uint64_t* tile_base = (const uint64_t*)d_ws;
    const uint64_t* group_base = tile_base + t + 1;
    int rc = SS_OK;
    if (max_reads) {
        rc = ss_check(hipMemsetAsync(d_aux, 0xFF, max_reads * sizeof(uint64_t), s), "fastq aux reset");
        if (!rc) rc = ss_check(hipMemsetAsync(d_lens, 0xFF, max_reads * sizeof(uint32_t), s), "fastq lens reset");
        if (rc) return rc;
    }
    FqOut o;
    o.offsets = d_offsets;
    o.ends = d_aux;
    o.nul = d_lens;               // NUL positions live in the lens array until k_fq_lens replaces them
    o.max_reads = max_reads;
    o.sel0 = (line0 + 2) / 4;
    o.nbytes = nbytes;
    if (t) hipLaunchKernelGGL(k_fq_emit, dim3((unsigned)t), dim3(kFqT), 0, s, d_buf, o, line0, tile_base, group_base);
    const uint64_t g = max_reads ? (max_reads + 255) / 256 : 1;
    hipLaunchKernelGGL(k_fq_lens, dim3((unsigned)(g < 0x7FFFFFFFull ? g : 0x7FFFFFFFull)), dim3(256), 0, s, d_buf, o, line0,
                       at_eof, t, tile_base, d_lens, d_nreads);
    return ss_check(hipGetLastError(), "k_fq_emit/k_fq_lens");
}

int ss_gather_rows(const uint8_t* d_src, uint64_t src_bytes, const uint64_t* d_offsets, const uint64_t* d_sel,
                   uint64_t m, uint32_t L, uint8_t* d_dst, uint64_t dst_stride, void* stream) {
    if (L == 0 || L > SS_MAX_NT) return ss_fail(SS_EARG, "L must be in 1..1024");
    if (dst_stride % 16 || dst_stride < ((L + 15u) & ~15u)) return ss_fail(SS_EARG, "dst_stride must be a multiple of 16 >= L");
    if (m == 0) return SS_OK;
    if (!d_src || !d_offsets || !d_dst) return ss_fail(SS_EARG, "null buffer");
    if (((uintptr_t)d_dst) & 15) return ss_fail(SS_EARG, "d_dst must be 16-B aligned");
    const uint32_t cpo = (L + 15u) / 16u;
    uint64_t blocks = (m * cpo + 255) / 256;
    if (blocks > 256ull * 64) blocks = 256ull * 64;
    hipLaunchKernelGGL(k_gather_rows, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, d_src, src_bytes,
                       d_offsets, d_sel, m, L, cpo, d_dst, dst_stride);
    return ss_check(hipGetLastError(), "k_gather_rows");
}

}  // extern "C"
