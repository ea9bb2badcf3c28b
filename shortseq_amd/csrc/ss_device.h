// ss_device.h — gfx950 device primitives shared by the encode / decode / hamming / counter kernels.
//
// Everything here is integer SWAR on 32-bit lanes (4 ASCII bytes per VGPR): no MFMA, no LDS tables.
// Bit contract (README.md:101-112): code(c) = (c >> 1) & 3 for A C T G (0 1 2 3);
// nt j of a read lives in word j/32 at bits 2*(j%32).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ssd {

constexpr uint64_t kEmpty = ~0ull;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Streamed-once input: non-temporal 16-byte load (global_load_dwordx4 ... nt).
__device__ __forceinline__ uint4 ld_stream(const uint4* p) {
    const u32x4 v = __builtin_nontemporal_load((const u32x4*)p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

// util.pxd:98-99 validity rule, restated per byte without the 64-bit bloom shift:
// a byte is a base iff (c & 63) is one of {1, 3, 20, 7}, and that value is fixed by its own code
// bits p = c & 6 (A:1 C:3 T:20 G:7).  v_perm_b32 with selector p looks the expected value up from
// the constant pair {0x00070014, 0x00030001}, so 4 bytes are validated with ~2 VALU ops.
//
// Packing: p_i = x_i & 0x06060606 holds the codes of nts 4i..4i+3 at bits 1-2 of each byte.
// M = p0>>1 | p1<<1 | p2<<3 | p3<<5 puts code(nt 4i+b) at bit 8b+2i; a 4x4 transpose of 2-bit
// fields (two delta swaps) moves it to bit 2(4i+b).  ~16 VALU ops per 16 bytes, no per-byte loop.
//
// Table path (short_seq_64.pyx:96-108, util.pyx:125-140): a valid byte with bit 6 clear
// (\x01 \x03 \x07 \x14) has table_91 value 4 -> its own 2 bits are 0 and bit 2 carries into the
// next nucleotide.  Full-block PEXT path (util.pyx:100-119): no carry (Q2).  The check is
// one AND of the 4 words; the alias fix-up runs only when a lane sees such a byte.
// Valid bytes >= 0x80 index table_91 out of bounds in the reference (Q3, outside the parity
// domain); here they follow the same bit-6 rule (oracle/ss_oracle.c and host_codec.h agree).

__device__ __forceinline__ uint32_t transpose2x4(uint32_t m) {
    uint32_t t = ((m >> 12) ^ m) & 0x0000F0F0u;
    m ^= t ^ (t << 12);
    t = ((m >> 6) ^ m) & 0x00CC00CCu;
    m ^= t ^ (t << 6);
    return m;
}

struct Enc32 {     // 16 bytes -> 32 code bits
    uint32_t v;    // packed codes (| alias carries shifted in, for table chunks)
    uint32_t cout; // carry out of bit 31 (nt 15 aliased on the table path) -> bit 0 of next half
    uint32_t bad;  // nonzero iff some byte is not a base
};

// x0..x3: 16 ASCII bytes (little-endian in each u32).  table: table-path semantics for this chunk.
__device__ __forceinline__ Enc32 encode16(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3, bool table) {
    const uint32_t p0 = x0 & 0x06060606u, p1 = x1 & 0x06060606u;
    const uint32_t p2 = x2 & 0x06060606u, p3 = x3 & 0x06060606u;
    uint32_t bad = ((x0 & 0x3F3F3F3Fu) ^ __builtin_amdgcn_perm(0x00070014u, 0x00030001u, p0)) |
                   ((x1 & 0x3F3F3F3Fu) ^ __builtin_amdgcn_perm(0x00070014u, 0x00030001u, p1)) |
                   ((x2 & 0x3F3F3F3Fu) ^ __builtin_amdgcn_perm(0x00070014u, 0x00030001u, p2)) |
                   ((x3 & 0x3F3F3F3Fu) ^ __builtin_amdgcn_perm(0x00070014u, 0x00030001u, p3));
    uint32_t v = transpose2x4((p0 >> 1) | (p1 << 1) | (p2 << 3) | (p3 << 5));
    uint32_t cout = 0;
    if (table && (x0 & x1 & x2 & x3 & 0x40404040u) != 0x40404040u) {
        const uint32_t a = transpose2x4(((~x0 >> 6) & 0x01010101u) | ((~x1 >> 4) & 0x04040404u) |
                                        ((~x2 >> 2) & 0x10101010u) | (~x3 & 0x40404040u));
        v = (v & ~(a | (a << 1))) | (a << 2);
        cout = a >> 30;
    }
    Enc32 e;
    e.v = v;
    e.cout = cout;
    e.bad = bad;
    return e;
}

// 16 codes (32 bits) -> 16 ASCII bytes via charmap "ACTG" (util.pyx:52): inverse transpose, then
// one v_perm per 4 output bytes.
__device__ __forceinline__ uint4 decode16(uint32_t v) {
    const uint32_t m = transpose2x4(v);
    uint32_t o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = __builtin_amdgcn_perm(0u, 0x47544341u, (m >> (2 * i)) & 0x03030303u);
    return make_uint4(o[0], o[1], o[2], o[3]);
}

// Streamed-once output (the packed words / ASCII are not re-read by this kernel): non-temporal
// stores (global_store ... nt).  Measured +2..4% on the 32-nt encode (tools/tune_encode.hip).
__device__ __forceinline__ void st_stream(uint32_t* p, uint32_t v) { __builtin_nontemporal_store(v, p); }
__device__ __forceinline__ void st_stream(uint4* p, uint4 v) {
    const u32x4 q = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(q, (u32x4*)p);
}

// Hamming contribution of one 32- or 64-bit xor (short_seq_64.pyx:82-84): codes that xor to 3
// collapse onto the low bit, then popcount.
__device__ __forceinline__ uint32_t ham32(uint32_t x) { return __popc(((x >> 1) | x) & 0x55555555u); }
__device__ __forceinline__ uint32_t ham64(uint64_t x) {
    return __popcll(((x >> 1) | x) & 0x5555555555555555ull);
}

__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Value of the neighbouring lane (lane ^ 1): one DPP quad_perm [1,0,3,2] VALU op, no LDS traffic.
__device__ __forceinline__ uint32_t swap_pair(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
}

// 64-bit fingerprint of a multi-word key (W words, compared whole): the slot key of the multi-word
// counter tables (ss_counter.hip) and the drop-in engine's class rows (k_encode_classes emits it per
// row, so the partition passes need not re-read the rows).  ~0 is reserved for free slots.  One
// xorshift-multiply round per word (the xorshift first, so a difference in a word's top bits reaches
// the multiply's low bits and cannot cancel against the next word's), then a final xorshift-multiply
// so the top bits (slot position, sketch register) depend on every word: one 64-bit multiply per
// word where splitmix64 per word took two.  Equal keys are decided on the words (a collision only
// sends a chunk down the exact path), so the function is a speed choice, not a correctness one.
__device__ __forceinline__ uint64_t fp_seed(uint32_t W) { return 0x243F6A8885A308D3ull ^ W; }
__device__ __forceinline__ uint64_t fp_step(uint64_t h, uint64_t x) {
    h ^= x;
    h ^= h >> 29;
    return h * 0xBF58476D1CE4E5B9ull;
}
__device__ __forceinline__ uint64_t fp_final(uint64_t h) {
    h ^= h >> 32;
    h *= 0x94D049BB133111EBull;
    h ^= h >> 29;
    return h == ~0ull ? ~1ull : h;
}
__device__ __forceinline__ uint64_t words_fp(const uint64_t* w, uint32_t W) {
    uint64_t h = fp_seed(W);
    for (uint32_t j = 0; j < W; ++j) h = fp_step(h, w[j]);
    return fp_final(h);
}

// First-invalid-read report where the read index is only needed on the (rare) bad path:
// read = slot / div, computed inside the ballot branch.
__device__ __forceinline__ void report_bad_div(bool bad, uint64_t slot, uint64_t div, unsigned long long* first_bad) {
    if (__ballot(bad)) {
        if (bad) atomicMin(first_bad, (unsigned long long)(slot / div));
    }
}

// First-invalid-read report: one atomic per wave that saw a bad lane (rare path).
__device__ __forceinline__ void report_bad(bool bad, uint64_t read, unsigned long long* first_bad) {
    if (__ballot(bad)) {
        if (bad) atomicMin(first_bad, (unsigned long long)read);
    }
}

}  // namespace ssd
