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
//                               each NUL inside a sequence line is listed)
//                   k_fq_lens  (thread per sequence line: the strlen - 1 rule -> lens)
//                   k_fq_nulfix (the listed lines re-measured)
//   HBM traffic: the chunk is read twice (count + emit), ~2 B per file byte.
//   ss_fastq_index_onepass: the chunk read once (k_fq_nlpos stages newline positions per tile,
//                   k_fq_place resolves line numbers from the tile counts): see below.
// Output: d_offsets[i] / d_lens[i] of sequence line i, exactly the ragged layout ss_encode_var and
// ss_gather_rows take.
#include "ss_device.h"
#include "ss_internal.h"

namespace {

using namespace ssd;

// 512 x 4 / 512 x 8 / 128 x 8 / 128 x 16 measured slower or level (profiles/r2/r2f/tune_f1_t.log)
constexpr int kFqT = 256;                                   // threads per block
constexpr int kFqU = 4;                                     // 16-B chunks per thread
constexpr uint64_t kFqTile = (uint64_t)kFqT * kFqU * 16;    // 16 KiB per block
constexpr uint32_t kNone32 = 0xFFFFFFFFu;
constexpr uint64_t kNone64 = ~0ull;

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

// U chunks per thread of the tile at t0 (chunk j of thread t at t0 + 16 (j kFqT + t)).  A whole tile
// (block-uniform test) loads unconditionally, so the U loads go out back to back; a guarded load per
// chunk (the tile holding the end of the chunk) puts each load in its own branch, and the compiler
// then waits for each one before issuing the next.
template <int U>
__device__ __forceinline__ void load_chunks(const uint8_t* buf, uint64_t nbytes, uint64_t t0, uint4 (&x)[U]) {
    if (t0 + 16ull * U * kFqT <= nbytes) {
#pragma unroll
        for (int j = 0; j < U; ++j) x[j] = ld_stream((const uint4*)(buf + t0 + 16ull * (j * kFqT + threadIdx.x)));
    } else {
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint64_t off = t0 + 16ull * (j * kFqT + threadIdx.x);
            x[j] = off < nbytes ? load_chunk(buf, off, nbytes)
                                : make_uint4(0x20202020u, 0x20202020u, 0x20202020u, 0x20202020u);
        }
    }
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
    load_chunks<kFqU>(buf, nbytes, t0, x);
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

// One-pass path: k_fq_scan_local and k_fq_scan_groups in one launch.  The group blocks scan as
// above; the last one to finish (a ticket among the per-call reset words) then turns the group
// totals into group bases and writes the newline count (one launch and its gap fewer per chunk).
__global__ __launch_bounds__(1024) void k_fq_scan_last(const uint32_t* __restrict__ tile_cnt, uint64_t ntiles,
                                                       uint64_t* __restrict__ tile_base, uint64_t* group_tot,
                                                       uint64_t ngroups, uint32_t* ticket, uint64_t* d_nl) {
    __shared__ uint64_t wsum[16];
    __shared__ uint64_t carry;
    __shared__ uint32_t last;
    const uint64_t i = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
    const uint64_t v = i < ntiles ? tile_cnt[i] : 0;
    uint64_t total;
    const uint64_t ex = block_excl_scan_1024(v, wsum, total);
    if (i < ntiles) tile_base[i] = ex;
    if (threadIdx.x == 0) {
        __hip_atomic_store(&group_tot[blockIdx.x], total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t k = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        last = k + 1 == gridDim.x;
        carry = 0;
    }
    __syncthreads();
    if (!last) return;
    __threadfence();
    for (uint64_t g0 = 0; g0 < ngroups; g0 += 1024) {
        const uint64_t g = g0 + threadIdx.x;
        const uint64_t gv = g < ngroups ? __hip_atomic_load(&group_tot[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
        uint64_t gt;
        const uint64_t gx = block_excl_scan_1024(gv, wsum, gt);
        const uint64_t c = carry;
        if (g < ngroups) group_tot[g] = c + gx;       // group base
        __syncthreads();
        if (threadIdx.x == 0) carry = c + gt;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        tile_base[ntiles] = carry;
        *d_nl = carry;
    }
}

// NUL bytes are rare in FASTQ text: a sequence line holding one is appended (once per lane) to a
// short list in the workspace, and k_fq_nulfix re-measures those lines with a strlen scan.  A list
// that overflows makes k_fq_nulfix re-measure every line (exact either way).  Neither the offsets
// nor the ends need a reset: every sequence line of the chunk gets both from its two newlines,
// except a final line without '\n', which k_fq_lens recognises by its line number.
constexpr uint32_t kNulCap = 1u << 16;

struct FqOut {
    uint64_t* offsets;
    uint64_t* ends;      // aux: '\n' position closing sequence line i
    uint32_t* nul_cnt;   // sequence lines with a NUL byte (may exceed kNulCap: overflow)
    uint32_t* nul_list;  // [kNulCap] their indices
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

// 16-bit mask of the '\n' bytes of a 16-B chunk (bit b = byte b)
__device__ __forceinline__ uint32_t nib(uint32_t e) {            // 0x80 per hit byte -> 4 bits
    return (((e >> 7) * 0x00204081u) >> 21) & 0xFu;
}
__device__ __forceinline__ uint32_t nl_mask16(const uint4& x) {
    return nib(eq_bytes(x.x, 0x0A0A0A0Au)) | nib(eq_bytes(x.y, 0x0A0A0A0Au)) << 4 |
           nib(eq_bytes(x.z, 0x0A0A0A0Au)) << 8 | nib(eq_bytes(x.w, 0x0A0A0A0Au)) << 12;
}
__device__ __forceinline__ bool has_nul(const uint4& x) {
    return (eq_bytes(x.x, 0u) | eq_bytes(x.y, 0u) | eq_bytes(x.z, 0u) | eq_bytes(x.w, 0u)) != 0u;
}

// Block-wide inclusive scan of the 16-bit per-chunk newline counts, four chunk rows per u64 (each
// field's block total <= 4096): excl[k] = this lane's exclusive prefix per field, total[k] = the
// block's per-field totals.
template <int P>
__device__ __forceinline__ void scan_packed(const uint64_t (&packed)[P], uint64_t (*wtot)[P], uint64_t (&excl)[P],
                                            uint64_t (&total)[P]) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint64_t v[P];
#pragma unroll
    for (int k = 0; k < P; ++k) v[k] = packed[k];
    for (int d = 1; d < 64; d <<= 1) {
#pragma unroll
        for (int k = 0; k < P; ++k) {
            const uint64_t u = __shfl_up(v[k], d);
            if (lane >= (uint32_t)d) v[k] += u;
        }
    }
    if (lane == 63) {
#pragma unroll
        for (int k = 0; k < P; ++k) wtot[wave][k] = v[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < P; ++k) {
        uint64_t before = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < kFqT / 64; ++w) {
            if ((uint32_t)w < wave) before += wtot[w][k];
            tot += wtot[w][k];
        }
        excl[k] = before + v[k] - packed[k];
        total[k] = tot;
    }
}

// Emission of one tile given its first line index lbase: every '\n' closes a line; the lines of a
// block are ordered chunk-row j first, then lane.  Waves without a NUL byte take the 16-bit-mask
// loop (one iteration per newline of the lane's chunk); a wave with a NUL walks bytes per word and
// lists the sequence lines its NULs fall in.
template <int U>
__device__ __forceinline__ void emit_tile(const FqOut& o, const uint4 (&x)[U], uint64_t t0, uint64_t lbase,
                                          const uint64_t (&excl)[U / 4], const uint64_t (&total)[U / 4]) {
    bool nul = false;
#pragma unroll
    for (int j = 0; j < U; ++j) nul |= has_nul(x[j]);
    const bool wave_nul = __ballot(nul) != 0;
    uint64_t rows_before = 0;              // newlines in the rows j' < j (whole block)
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint64_t off = t0 + 16ull * (j * kFqT + threadIdx.x);
        uint64_t li = lbase + rows_before + ((excl[j / 4] >> (16 * (j % 4))) & 0xFFFFu);
        rows_before += (total[j / 4] >> (16 * (j % 4))) & 0xFFFFu;
        if (off >= o.nbytes) continue;
        if (!wave_nul) {
            // bytes past nbytes load as ' ': every hit is inside the chunk
            uint32_t m = nl_mask16(x[j]);
            while (m) {
                const uint32_t bit = __builtin_ctz(m);
                m &= m - 1;
                on_newline(o, off + bit, li);
                ++li;
            }
            continue;
        }
        const uint32_t xw[4] = {x[j].x, x[j].y, x[j].z, x[j].w};
        uint64_t listed = ~0ull;           // the line this lane last put on the NUL list
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
                } else if ((li & 3u) == 1u && li != listed) {
                    const uint64_t i = (li + 2) / 4 - o.sel0;
                    listed = li;
                    if (i < o.max_reads) {
                        const uint32_t k = atomicAdd(o.nul_cnt, 1u);
                        if (k < kNulCap) o.nul_list[k] = (uint32_t)i;
                    }
                }
            }
        }
    }
}

template <int U>
__device__ __forceinline__ void load_tile(const uint8_t* buf, uint64_t nbytes, uint64_t t0, uint4 (&x)[U],
                                          uint64_t (&packed)[U / 4]) {
    load_chunks<U>(buf, nbytes, t0, x);
#pragma unroll
    for (int k = 0; k < U / 4; ++k) packed[k] = 0;   // 16-bit newline count of chunk j at bits 16 (j % 4)
#pragma unroll
    for (int j = 0; j < U; ++j) packed[j / 4] |= (uint64_t)count_nl(x[j]) << (16 * (j % 4));
}

__global__ __launch_bounds__(kFqT) void k_fq_emit(const uint8_t* __restrict__ buf, FqOut o, uint64_t line0,
                                                  const uint64_t* __restrict__ tile_base,
                                                  const uint64_t* __restrict__ group_base) {
    __shared__ uint64_t wtot[kFqT / 64][kFqU / 4];
    const uint64_t t0 = (uint64_t)blockIdx.x * kFqTile;
    uint4 x[kFqU];
    uint64_t packed[kFqU / 4], excl[kFqU / 4], total[kFqU / 4];
    load_tile(buf, o.nbytes, t0, x, packed);
    scan_packed(packed, wtot, excl, total);
    emit_tile(o, x, t0, line0 + group_base[blockIdx.x >> 10] + tile_base[blockIdx.x], excl, total);
}

// One read of the file (ss_fastq_index_onepass).  A decoupled look-back over tile counts measured
// 1.25-1.47 ms for 2 GB (every waiting block polls the same status lines; the two-pass form took
// 0.82), so the line numbers are resolved after the fact instead:
//   k_fq_nlpos : 32-KiB tiles; each tile writes its newline positions in file order (u16 offsets in
//                the tile) to its own fixed run of the staging array, or, past kTileCap newlines,
//                reserves a run of its shard with one atomicAdd; plus its count, run start and
//                last newline.  The reservations go to 64 counters (tile % 64), each on its
//                own 128-B line with its own staging region: one counter word serves ~88
//                atomics per us, which capped a single shared counter at 0.75 ms per 60k tiles.
//                A region that runs full raises the overflow word (the caller retries with a larger
//                bound).  NUL bytes (rare) go to a position list.
//   k_fq_scan_last over the tile counts -> each tile's first line number (group scans, then the
//                last group block scans the group totals)
//   k_fq_place : tile-wise, the staged positions with their line numbers -> offsets / lens; the
//                sequence lines holding a NUL byte (when the chunk has any) re-measured in place
// HBM: the file once + 2 B per line written and read back (the newline's offset in its 32-KiB tile)
// + 12 B per sequence line of output.
// 16-KiB tiles (4) 0.525 ms, 64-KiB tiles (16) level with 32 KiB (tools/tune_f1.hip)
constexpr int kFqU1 = 8;                                       // 16-B chunks per thread
constexpr uint64_t kFqTile1 = (uint64_t)kFqT * kFqU1 * 16;     // 32 KiB per tile

constexpr uint32_t kStageShards = 64, kShardStride = 32;       // counters 128 B apart
constexpr uint32_t kLdsPos = (uint32_t)(kFqTile1 / 8);       // newline positions gathered in LDS (4096)
constexpr uint32_t kSubPerTile = (uint32_t)(kFqTile1 / 1024);  // 1-KiB NUL sub-blocks per tile (32)
static_assert(kSubPerTile <= 32, "a tile's NUL sub-blocks are one u32 mask");
// Every tile owns a fixed run of kTileCap staging words (after the shards' regions, 8 KiB per 32-KiB
// tile): a tile with at most that many newlines (lines of 16 B or more on average) writes its
// positions there straight from registers -- no reservation atomic, no LDS staging, no second
// barrier; a denser tile reserves a run of its shard as before.
constexpr uint32_t kTileCap = (uint32_t)(kFqTile1 / 16);      // 2048

struct FqStage {
    uint16_t* pos;        // [kStageShards * region + tiles * kTileCap] staged newline positions, as
                          // offsets inside their 32-KiB tile
    uint64_t region;      // staging words per shard
    uint32_t* used;       // [kStageShards * kShardStride] run reservations per shard
    uint32_t* ovf;        // a shard's region ran full
    uint32_t* tile_cnt;   // [t] newlines per tile
    uint32_t* tile_run;   // [t] start of the tile's run in pos
    uint32_t* tile_last;  // [t] position of the tile's last newline (kNone32: none staged)
    uint32_t* tile_nul;   // [t] the tile's 1-KiB sub-blocks holding a NUL byte (bit b: bytes 1024 b ..)
    uint32_t* nul_cnt;    // NUL bytes seen (may exceed kNulCap)
    uint32_t* nul_pos;    // [kNulCap] their positions
};

__global__ __launch_bounds__(kFqT) void k_fq_nlpos(const uint8_t* __restrict__ buf, uint64_t nbytes, FqStage st) {
    __shared__ uint64_t wtot[kFqT / 64][kFqU1 / 4];
    __shared__ uint32_t s_run, s_cnt, s_nul;
    __shared__ __attribute__((aligned(8))) uint16_t spos[kLdsPos];
    const uint64_t t0 = (uint64_t)blockIdx.x * kFqTile1;
    if (threadIdx.x == 0) s_nul = 0;
    // the chunks live only until their newline masks are taken: 16 bits per chunk, two per VGPR
    uint32_t mk[kFqU1 / 2];
    bool nul = false;
    uint32_t nsub = 0;     // the tile's 1-KiB sub-blocks with a NUL: chunk j of wave w lies in sub-block 4 j + w
    {
        uint4 x[kFqU1];
        load_chunks<kFqU1>(buf, nbytes, t0, x);
#pragma unroll
        for (int j = 0; j < kFqU1; j += 2) {
            mk[j / 2] = nl_mask16(x[j]) | nl_mask16(x[j + 1]) << 16;
            const bool n0 = has_nul(x[j]), n1 = has_nul(x[j + 1]);
            nul |= n0 | n1;
            nsub |= (n0 ? 1u << (4 * j + (threadIdx.x >> 6)) : 0u) | (n1 ? 1u << (4 * (j + 1) + (threadIdx.x >> 6)) : 0u);
        }
    }
    // the wave's NUL verdict now: left to its use at the end, the compiler keeps the chunks live
    // through the whole kernel (96 VGPRs, 5 waves per SIMD, instead of 62 and 8)
    const bool any_nul = __ballot(nul) != 0;
    uint64_t packed[kFqU1 / 4], excl[kFqU1 / 4], total[kFqU1 / 4];
#pragma unroll
    for (int k = 0; k < kFqU1 / 4; ++k) packed[k] = 0;
#pragma unroll
    for (int j = 0; j < kFqU1; ++j)
        packed[j / 4] |= (uint64_t)__popc((mk[j / 2] >> (16 * (j & 1))) & 0xFFFFu) << (16 * (j % 4));
    scan_packed(packed, wtot, excl, total);
    uint32_t cnt = 0;
#pragma unroll
    for (int k = 0; k < kFqU1 / 4; ++k)
        cnt += (uint32_t)((total[k] & 0xFFFFu) + ((total[k] >> 16) & 0xFFFFu) + ((total[k] >> 32) & 0xFFFFu) +
                          (total[k] >> 48));
    const bool fixed = cnt <= kTileCap;    // block-uniform (the scan's totals)
    if (any_nul && nsub) atomicOr(&s_nul, nsub);   // (s_nul zeroed before scan_packed's barrier)
    if (threadIdx.x == 0) {
        // the reservation's round trip overlaps the other waves' LDS staging below
        const uint32_t sh = blockIdx.x % kStageShards;
        uint64_t run = (uint64_t)sh * st.region;
        uint32_t c = cnt;
        if (fixed) {
            run = (uint64_t)kStageShards * st.region + (uint64_t)blockIdx.x * kTileCap;
        } else if (c) {
            const uint32_t r = atomicAdd(&st.used[sh * kShardStride], c);
            if (r + (uint64_t)c > st.region) {
                atomicExch(st.ovf, 1u);
                c = 0;                    // nothing staged; the call reports the overflow
            }
            run += r;
        }
        st.tile_cnt[blockIdx.x] = c;
        st.tile_run[blockIdx.x] = (uint32_t)run;
        if (cnt == 0) st.tile_last[blockIdx.x] = kNone32;
        s_run = (uint32_t)run;
        s_cnt = c;
    }
    const bool in_lds = cnt <= kLdsPos;   // typical tiles: positions gathered in LDS, stored as one run
    auto put = [&](uint32_t base) {
        uint32_t rows_before = 0;
#pragma unroll
        for (int j = 0; j < kFqU1; ++j) {
            const uint32_t off = (uint32_t)(t0 + 16ull * (j * kFqT + threadIdx.x));
            uint32_t k = base + rows_before + (uint32_t)((excl[j / 4] >> (16 * (j % 4))) & 0xFFFFu);
            rows_before += (uint32_t)((total[j / 4] >> (16 * (j % 4))) & 0xFFFFu);
            uint32_t m = (mk[j / 2] >> (16 * (j & 1))) & 0xFFFFu;   // bytes past nbytes loaded as ' '
            while (m) {
                const uint32_t bit = __builtin_ctz(m);
                m &= m - 1;
                const uint16_t rel = (uint16_t)(off + bit - (uint32_t)t0);
                if (in_lds) spos[k++] = rel;
                else st.pos[k++] = rel;
                if (k == base + cnt) st.tile_last[blockIdx.x] = off + bit;   // the tile's last newline
            }
        }
    };
    // Positions gathered in LDS and stored as one run beat each lane storing its own (scattered 2-B
    // stores: 0.435 vs 0.410 ms per 2-GB call, tools/tune_f1.hip)
    if (in_lds) put(0);
    __syncthreads();
    if (fixed && cnt) {           // the tile's own run: 8-B copies (the run is 4 KiB aligned; a copy past cnt
        const uint64_t* s8 = (const uint64_t*)spos;   // stays inside the run)
        uint64_t* d8 = (uint64_t*)(st.pos + kStageShards * st.region + (uint64_t)blockIdx.x * kTileCap);
        for (uint32_t e = threadIdx.x; 4 * e < cnt; e += kFqT) d8[e] = s8[e];
    } else if (!fixed && s_cnt) {
        if (in_lds) {
            const uint32_t run = s_run;
            for (uint32_t e = threadIdx.x; e < cnt; e += kFqT) st.pos[run + e] = spos[e];
        } else {
            put(s_run);
        }
    }
    if (threadIdx.x == 0) st.tile_nul[blockIdx.x] = s_nul;   // written after the barrier above
    if (any_nul) {                         // rare: reload the lane's chunks (keeps them out of VGPRs)
#pragma unroll 1
        for (int j = 0; j < kFqU1; ++j) {
            const uint64_t off = t0 + 16ull * (j * kFqT + threadIdx.x);
            if (off >= nbytes) break;
            const uint4 c = load_chunk(buf, off, nbytes);
            const uint32_t xw[4] = {c.x, c.y, c.z, c.w};
#pragma unroll 1
            for (int q = 0; q < 4; ++q) {
                uint32_t m = eq_bytes(xw[q], 0u);
                while (m) {
                    const uint32_t bit = __builtin_ctz(m);
                    m &= m - 1;
                    const uint64_t p = off + 4 * q + (bit >> 3);
                    if (p >= nbytes) break;
                    const uint32_t i = atomicAdd(st.nul_cnt, 1u);
                    if (i < kNulCap) st.nul_pos[i] = (uint32_t)p;
                }
            }
        }
    }
}

__device__ __forceinline__ uint64_t fq_nsel(const uint8_t* buf, const FqOut& o, uint64_t line0, int at_eof,
                                            uint64_t nl, bool& partial) {
    partial = at_eof && o.nbytes > 0 && buf[o.nbytes - 1] != '\n';
    return (line0 + nl + (partial ? 1u : 0u) + 2) / 4 - o.sel0;
}

// strlen - 1 of sequence line i from its start and its closing '\n' (or the chunk end for a final
// line without one); slen 0 -> kNone32 (the reference's size_t underflow)
__device__ __forceinline__ uint32_t fq_len(uint64_t slen) {
    return slen == 0 ? kNone32 : (uint32_t)min<uint64_t>(slen - 1, 0xFFFFFFFEull);
}

__device__ __forceinline__ bool fq_has_nl(const FqOut& o, uint64_t line0, uint64_t nl, bool partial, uint64_t i) {
    return !(partial && 4 * (o.sel0 + i) + 1 == line0 + nl);    // the unterminated last line
}

// One wave per tile (four per block): staged newline k of the tile closes line lbase + k.  The
// newline closing a sequence line (line number = 1 mod 4) gives its end; the newline before it (the
// lane below's entry by a shuffle, the previous round's last one, or the previous tile's last newline,
// tile_last) gives its start: offsets[i] and lens[i] directly, no end array and no separate length
// pass.  The wave's loads (counts, run, line base, the previous tile's last newline) are independent,
// so they go out together.  The last tile's wave also places a final sequence line without '\n' and
// writes the sequence-line count.

// start of the line that follows the last newline staged before `tile` (0: none in the chunk); a
// tile that stages none (a line longer than a tile) sends the search further back
__device__ __forceinline__ uint64_t start_before(const FqStage& st, uint64_t tile) {
    while (tile > 0) {
        --tile;
        const uint32_t l = st.tile_last[tile];
        if (l != kNone32) return (uint64_t)l + 1;
    }
    return 0;
}

// A sequence line [start, stop) (stop: its '\n', or the chunk end for an unterminated last line)
// with a NUL byte: strlen stops at the first NUL (the k_fq_nulfix rule, applied as the line is
// placed).  Only when the chunk holds NULs: a short list is searched; with more, only the line's
// 1-KiB sub-blocks that hold a NUL (k_fq_nlpos's per-tile masks) are byte-scanned, so a file with
// a thousand stray NULs re-reads a few KiB around each, not every sequence line.
constexpr uint32_t kNulListScan = 64;
__device__ __forceinline__ uint32_t nul_len(const uint8_t* __restrict__ buf, const FqStage& st, uint32_t nulc,
                                            uint64_t start, uint64_t stop, uint32_t len) {
    uint64_t first = stop;
    if (nulc <= kNulListScan) {
        for (uint32_t k = 0; k < nulc; ++k) {
            const uint64_t p = st.nul_pos[k];
            if (p >= start && p < first) first = p;
        }
    } else if (stop > start) {
        for (uint64_t sb = start >> 10; sb <= (stop - 1) >> 10 && first == stop; ++sb) {
            if (!((st.tile_nul[sb / kSubPerTile] >> (sb % kSubPerTile)) & 1u)) continue;
            const uint64_t e = min(stop, (sb + 1) << 10);
            for (uint64_t p = max(start, sb << 10); p < e; ++p)
                if (buf[p] == 0) {
                    first = p;
                    break;
                }
        }
    }
    return first < stop ? fq_len(first - start) : len;
}

__global__ __launch_bounds__(256) void k_fq_place(const uint8_t* __restrict__ buf, FqOut o, uint64_t line0,
                                                  int at_eof, FqStage st, uint64_t ntiles,
                                                  const uint64_t* __restrict__ tile_base,
                                                  const uint64_t* __restrict__ group_base,
                                                  const uint64_t* __restrict__ d_nl, uint32_t* __restrict__ lens,
                                                  uint64_t* d_nreads) {
    const uint64_t tile = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nulc = *st.nul_cnt;   // NUL bytes in the chunk (k_fq_nlpos): lines re-measured below
    if (tile < ntiles) {
        const uint32_t cnt = st.tile_cnt[tile];
        const uint32_t run = st.tile_run[tile];
        const uint64_t lbase = line0 + group_base[tile >> 10] + tile_base[tile];
        const uint32_t prev = tile ? st.tile_last[tile - 1] : kNone32;
        // start of the tile's first line: after the previous newline (0 for the chunk's first line)
        uint64_t carry = lbase == line0 ? 0 : (prev != kNone32 ? (uint64_t)prev + 1 : kNone64);
        const uint32_t tb = (uint32_t)(tile * kFqTile1);
        if (run >= kStageShards * st.region) {
            // a fixed run (16-B aligned): 8 positions per lane per load, 512 per wave round (a tile's
            // ~550 newlines in two rounds instead of nine dependent 64-wide ones)
            for (uint32_t k0 = 0; k0 < cnt; k0 += 512) {
                const uint32_t kb = k0 + 8u * lane;
                const uint32_t nv = kb < cnt ? min(8u, cnt - kb) : 0u;
                uint4 v = make_uint4(0, 0, 0, 0);
                if (nv) v = *(const uint4*)(st.pos + run + kb);
                const uint32_t vw[4] = {v.x, v.y, v.z, v.w};
                uint32_t pp[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) pp[q] = tb + ((vw[q >> 1] >> (16 * (q & 1))) & 0xFFFFu);
                uint32_t lastp = pp[7];
#pragma unroll
                for (int q = 0; q < 7; ++q)
                    if ((uint32_t)q + 1 == nv) lastp = pp[q];
                const uint32_t below = (uint32_t)__shfl_up((int)lastp, 1);
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const uint64_t li = lbase + kb + q;
                    if ((uint32_t)q < nv && (li & 3u) == 1u) {
                        const uint64_t i = (li >> 2) - o.sel0;
                        if (i < o.max_reads) {
                            uint64_t start = q ? (uint64_t)pp[q - 1] + 1 : (lane ? (uint64_t)below + 1 : carry);
                            if (start == kNone64) start = start_before(st, tile);
                            o.offsets[i] = start;
                            uint32_t len = fq_len((uint64_t)pp[q] - start + 1);
                            if (nulc) len = nul_len(buf, st, nulc, start, pp[q], len);
                            lens[i] = len;
                        }
                    }
                }
                carry = (uint64_t)(uint32_t)__shfl((int)pp[7], 63) + 1;
            }
        } else for (uint32_t k0 = 0; k0 < cnt; k0 += 64) {
            const uint32_t k = k0 + lane;
            const uint32_t p = tb + st.pos[run + min(k, cnt - 1)];
            const uint32_t below = (uint32_t)__shfl_up((int)p, 1);
            const uint64_t li = lbase + k;
            if (k < cnt && (li & 3u) == 1u) {
                const uint64_t i = (li >> 2) - o.sel0;
                if (i < o.max_reads) {
                    uint64_t start = lane ? (uint64_t)below + 1 : carry;
                    if (start == kNone64) start = start_before(st, tile);
                    o.offsets[i] = start;
                    uint32_t len = fq_len((uint64_t)p - start + 1);
                    if (nulc) len = nul_len(buf, st, nulc, start, p, len);
                    lens[i] = len;
                }
            }
            carry = (uint64_t)(uint32_t)__shfl((int)p, 63) + 1;
        }
    }
    if (tile + 1 == ntiles && lane == 0) {
        const uint64_t nl = *d_nl;
        bool partial;
        *d_nreads = fq_nsel(buf, o, line0, at_eof, nl, partial);
        d_nreads[1] = *st.ovf;                             // status word (a staging region ran full)
        const uint64_t last = line0 + nl;                  // the unterminated final line, if any
        if (partial && (last & 3u) == 1u) {
            const uint64_t i = (last >> 2) - o.sel0;
            if (i < o.max_reads) {
                const uint64_t start = nl ? start_before(st, ntiles) : 0;
                o.offsets[i] = start;
                const uint32_t len = fq_len(o.nbytes - start);
                lens[i] = nulc ? nul_len(buf, st, nulc, start, o.nbytes, len) : len;
            }
        }
    }
}

__global__ __launch_bounds__(256) void k_fq_lens(const uint8_t* __restrict__ buf, FqOut o, uint64_t line0,
                                                 int at_eof, const uint64_t* __restrict__ d_nl,
                                                 uint32_t* __restrict__ lens, uint64_t* d_nreads) {
    const uint64_t nl = *d_nl;
    bool partial;
    const uint64_t nsel = fq_nsel(buf, o, line0, at_eof, nl, partial);
    if (blockIdx.x == 0 && threadIdx.x == 0) *d_nreads = nsel;
    const uint64_t lim = min(nsel, o.max_reads);
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < lim; i += (uint64_t)gridDim.x * 256) {
        uint64_t start = o.offsets[i];
        if (i == 0 && (line0 & 3u) == 1u) {
            start = 0;                      // the chunk opens with a sequence line
            o.offsets[0] = 0;
        }
        const bool has_nl = fq_has_nl(o, line0, nl, partial, i);
        lens[i] = fq_len(has_nl ? o.ends[i] - start + 1 : o.nbytes - start);
    }
}

// Sequence lines with a NUL byte: strlen stops at the first NUL.  The lines that hold a listed NUL
// (or, after a list overflow, all lines) are re-measured byte by byte; runs after the lengths pass.
// BYLINE: the list holds sequence-line indices (two-pass emit); otherwise NUL byte positions (one
// pass), mapped to their line by a binary search over the line starts.
template <bool BYLINE>
__global__ __launch_bounds__(256) void k_fq_nulfix(const uint8_t* __restrict__ buf, FqOut o, uint64_t line0,
                                                   int at_eof, const uint64_t* __restrict__ d_nl,
                                                   uint32_t* __restrict__ lens) {
    const uint32_t cnt = *o.nul_cnt;
    if (cnt == 0) return;
    bool partial;
    const uint64_t lim = min(fq_nsel(buf, o, line0, at_eof, *d_nl, partial), o.max_reads);
    if (lim == 0) return;
    const bool all = cnt > kNulCap;
    const uint64_t n = all ? lim : cnt;
    for (uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (uint64_t)gridDim.x * 256) {
        uint64_t i = e;
        if (!all) {
            if (BYLINE) {
                i = o.nul_list[e];
            } else {
                const uint64_t p = o.nul_list[e];      // last line starting at or before p
                uint64_t lo = 0, hi = lim;
                while (hi - lo > 1) {
                    const uint64_t mid = (lo + hi) / 2;
                    if (o.offsets[mid] <= p) lo = mid; else hi = mid;
                }
                i = lo;
                if (o.offsets[i] > p) continue;
            }
        }
        const uint64_t start = o.offsets[i];    // strlen: stop at the line's '\n', a NUL or the chunk end
        uint64_t p = start;
        while (p < o.nbytes && buf[p] != 0 && buf[p] != '\n') ++p;
        if (p < o.nbytes && buf[p] == 0) lens[i] = fq_len(p - start);
    }
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

// two-pass workspace: tile_base u64 [t + 1] | group_base u64 [g + 1] | nul_cnt u32 (8-B slot) |
// nul_list u32 [kNulCap] | tile_cnt u32 [t]
uint64_t ss_fastq_scan_ws_bytes(uint64_t nbytes) {
    const uint64_t t = fq_tiles(nbytes);
    return 8 * (t + 1) + 8 * (fq_groups(t) + 1) + 8 + 4ull * kNulCap + 4 * t + 16;
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
    uint32_t* tile_cnt = (uint32_t*)(group_base + g + 1) + 2 + kNulCap;
    if (t) {
        hipLaunchKernelGGL(k_fq_count, dim3((unsigned)t), dim3(kFqT), 0, s, d_buf, nbytes, tile_cnt);
        hipLaunchKernelGGL(k_fq_scan_local, dim3((unsigned)g), dim3(1024), 0, s, (const uint32_t*)tile_cnt, t,
                           tile_base, group_base);
    }
    hipLaunchKernelGGL(k_fq_scan_groups, dim3(1), dim3(1024), 0, s, group_base, g, t, tile_base, d_nlines);
    return ss_check(hipGetLastError(), "k_fq_count/k_fq_scan");
}

static int fq_check(const uint8_t* d_buf, uint64_t nbytes, const void* d_ws, const void* d_out, uint64_t max_reads,
                    const void* d_offsets, const void* d_lens, const void* d_aux) {
    if (nbytes >= (1ull << 32)) return ss_fail(SS_EARG, "FASTQ chunk must be < 4 GiB");
    if (!d_ws || !d_out || (nbytes && !d_buf)) return ss_fail(SS_EARG, "null buffer");
    if (max_reads && (!d_offsets || !d_lens || !d_aux)) return ss_fail(SS_EARG, "null output buffer");
    if ((((uintptr_t)d_buf) & 15) || (((uintptr_t)d_ws) & 7)) return ss_fail(SS_EARG, "d_buf must be 16-B aligned, d_ws 8-B");
    return SS_OK;
}

static FqOut fq_out(uint64_t* d_offsets, uint64_t* d_aux, uint32_t* nul_cnt, uint64_t max_reads, uint64_t line0,
                    uint64_t nbytes) {
    FqOut o;
    o.offsets = d_offsets;
    o.ends = d_aux;
    o.nul_cnt = nul_cnt;
    o.nul_list = nul_cnt + 2;
    o.max_reads = max_reads;
    o.sel0 = (line0 + 2) / 4;
    o.nbytes = nbytes;
    return o;
}

// lens + NUL fix-up (grid-stride, at most 256 x 64 blocks)
static int fq_finish(hipStream_t s, const uint8_t* d_buf, const FqOut& o, uint64_t line0, int at_eof,
                     const uint64_t* d_nl, uint32_t* d_lens, uint64_t* d_nreads) {
    uint64_t g = o.max_reads ? (o.max_reads + 255) / 256 : 1;
    if (g > 256ull * 64) g = 256ull * 64;
    hipLaunchKernelGGL(k_fq_lens, dim3((unsigned)g), dim3(256), 0, s, d_buf, o, line0, at_eof, d_nl, d_lens, d_nreads);
    hipLaunchKernelGGL(k_fq_nulfix<true>, dim3(256), dim3(256), 0, s, d_buf, o, line0, at_eof, d_nl, d_lens);
    return ss_check(hipGetLastError(), "k_fq_lens/k_fq_nulfix");
}

int ss_fastq_index(const uint8_t* d_buf, uint64_t nbytes, uint64_t line0, int at_eof, void* d_ws,
                   uint64_t* d_offsets, uint32_t* d_lens, uint64_t* d_aux, uint64_t max_reads,
                   uint64_t* d_nreads, void* stream) {
    int rc = fq_check(d_buf, nbytes, d_ws, d_nreads, max_reads, d_offsets, d_lens, d_aux);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    const uint64_t t = fq_tiles(nbytes);
    const uint64_t* tile_base = (const uint64_t*)d_ws;
    const uint64_t* group_base = tile_base + t + 1;
    uint32_t* nul_cnt = (uint32_t*)(group_base + fq_groups(t) + 1);
    rc = ss_check(hipMemsetAsync(nul_cnt, 0, 4, s), "fastq NUL counter reset");
    if (rc) return rc;
    const FqOut o = fq_out(d_offsets, d_aux, nul_cnt, max_reads, line0, nbytes);
    if (t) hipLaunchKernelGGL(k_fq_emit, dim3((unsigned)t), dim3(kFqT), 0, s, d_buf, o, line0, tile_base, group_base);
    rc = ss_check(hipGetLastError(), "k_fq_emit");
    return rc ? rc : fq_finish(s, d_buf, o, line0, at_eof, tile_base + t, d_lens, d_nreads);
}

// one-pass workspace: tile_base u64 [t + 1] | group_base u64 [g + 1] | used u32 [64 x 32] | ovf u32,
// nul_cnt u32, 2 pad u32 | nul_pos u32 [kNulCap] | tile_cnt u32 [t] | tile_run u32 [t] | tile_last u32 [t] |
// tile_nul u32 [t] |
// pos u16 [64 x region + t x kTileCap] (256-B aligned)
inline uint64_t fq_tiles1(uint64_t nbytes) { return (nbytes + kFqTile1 - 1) / kFqTile1; }

// staging words per shard: the lines max_reads implies (4 per sequence line) + 25 %, spread over the
// shards, plus one whole tile of single-byte lines per shard for the uneven spread
inline uint64_t fq_region(uint64_t max_reads) {
    const uint64_t lines = 4 * max_reads + 8;
    return (((lines + lines / 4) / kStageShards + kFqTile1) + 3) & ~3ull;   // x4: the fixed runs stay 8-B aligned
}

uint64_t ss_fastq_onepass_ws_bytes(uint64_t nbytes, uint64_t max_reads) {
    const uint64_t t = fq_tiles1(nbytes);
    return 8 * (t + 1) + 8 * (fq_groups(t) + 1) + 4ull * kStageShards * kShardStride + 16 + 4ull * kNulCap + 16 * t +
           2 * kStageShards * fq_region(max_reads) + 2ull * kTileCap * t + 256;
}

int ss_fastq_index_onepass(const uint8_t* d_buf, uint64_t nbytes, uint64_t line0, int at_eof, void* d_ws,
                           uint64_t ws_bytes, uint64_t* d_offsets, uint32_t* d_lens, uint64_t* d_aux,
                           uint64_t max_reads, uint64_t* d_counts, void* stream) {
    int rc = fq_check(d_buf, nbytes, d_ws, d_counts, max_reads, d_offsets, d_lens, d_aux);
    if (rc) return rc;
    if (ws_bytes < ss_fastq_onepass_ws_bytes(nbytes, max_reads)) return ss_fail(SS_EARG, "workspace too small");
    if (kStageShards * fq_region(max_reads) + (uint64_t)kTileCap * fq_tiles1(nbytes) >= (1ull << 32))
        return ss_fail(SS_EARG, "max_reads too large");
    hipStream_t s = (hipStream_t)stream;
    const uint64_t t = fq_tiles1(nbytes), g = fq_groups(t);
    uint64_t* tile_base = (uint64_t*)d_ws;
    uint64_t* group_base = tile_base + t + 1;
    FqStage st;
    st.used = (uint32_t*)(group_base + g + 1);
    st.ovf = st.used + kStageShards * kShardStride;
    st.nul_cnt = st.ovf + 1;
    st.nul_pos = st.ovf + 4;      // ovf + 2: k_fq_scan_last's ticket, ovf + 3 pad: one 16-B-sized reset fill
    st.tile_cnt = st.nul_pos + kNulCap;
    st.tile_run = st.tile_cnt + t;
    st.tile_last = st.tile_run + t;
    st.tile_nul = st.tile_last + t;
    // 256-B aligned: the fixed runs (4 KiB apart) are then 16-B aligned for k_fq_place's wide loads
    st.pos = (uint16_t*)(((uintptr_t)(st.tile_nul + t) + 255) & ~(uintptr_t)255);
    st.region = fq_region(max_reads);
    static_assert((4 * (kStageShards * kShardStride + 4)) % 16 == 0, "one fill packet");
    rc = ss_check(hipMemsetAsync(st.used, 0, 4 * (kStageShards * kShardStride + 4), s), "fastq staging reset");
    if (rc) return rc;
    FqOut o = fq_out(d_offsets, d_aux, st.nul_cnt, max_reads, line0, nbytes);
    o.nul_list = st.nul_pos;
    if (t) {
        hipLaunchKernelGGL(k_fq_nlpos, dim3((unsigned)t), dim3(kFqT), 0, s, d_buf, nbytes, st);
        hipLaunchKernelGGL(k_fq_scan_last, dim3((unsigned)g), dim3(1024), 0, s, (const uint32_t*)st.tile_cnt, t,
                           tile_base, group_base, g, st.ovf + 2, d_counts);
        // NUL-holding sequence lines are re-measured inside k_fq_place (no k_fq_nulfix pass)
        hipLaunchKernelGGL(k_fq_place, dim3((unsigned)((t + 3) / 4)), dim3(256), 0, s, d_buf, o, line0, at_eof, st, t, tile_base,
                           group_base, (const uint64_t*)d_counts, d_lens, d_counts + 1);
    } else {
        hipLaunchKernelGGL(k_fq_scan_groups, dim3(1), dim3(1024), 0, s, group_base, g, t, tile_base, d_counts);
    }
    rc = ss_check(hipGetLastError(), "k_fq_nlpos/k_fq_scan_last/k_fq_place");
    // k_fq_place's last block wrote the read count and the status word; an empty chunk has no tiles
    if (!rc && t == 0) rc = ss_check(hipMemsetAsync(d_counts + 1, 0, 16, s), "fastq read count / status");
    return rc;
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
