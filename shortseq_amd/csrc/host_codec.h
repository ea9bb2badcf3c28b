// host_codec.h — per-object host codec (one read per call), header-only.
//
// This is product code for the drop-in per-object API (sq.pack / str() / ^ on single objects),
// where a kernel launch would cost ~10x the work.  It implements the reference
// semantics bit for bit, including the error detail the reference puts in its messages:
//   short_seq.pyx:54-74   length-class switch and the >1024 error
//   short_seq_64.pyx:96-108 / util.pyx:125-140   table path (reverse scan, Q1 carry, last bad byte)
//   util.pyx:97-119       full 32-nt blocks (chunks 3->0, 8-byte chunk named on error, no carry)
//   short_seq_64.pyx:114-121 etc.  decode;  short_seq_64.pyx:77-84 etc.  hamming
// Full blocks use BMI2 PEXT when the host compiler targets it (the GPU box hosts do).
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#if defined(__BMI2__) || defined(__AVX2__)
#include <immintrin.h>
#endif

#ifndef SHORTSEQ_AMD_H
typedef struct ss_err {
    int32_t kind;
    int32_t nbytes;
    int64_t read_index;
    int64_t byte_offset;
} ss_err;
#endif

namespace ssh {

constexpr uint64_t kBloom = 0xFFFFFFFFFFEFFF75ull;   // util.pyx:75
constexpr size_t kMaxNt = 1024;                      // short_seq_var.pyx:9

inline bool is_base(uint8_t c) { return ((kBloom >> (c & 63u)) & 1u) == 0; }   // util.pxd:98-99

// Table value for a byte that passed is_base (util.pyx:44-50): A C G T -> codes; \x01 \x03 \x07 \x14
// (bit 6 clear) -> 4.  Bytes >= 0x80 are outside the parity domain (Q3) and follow the same rule.
inline uint64_t table_code(uint8_t c) { return (c & 0x40u) == 0 ? 4u : ((c >> 1) & 3u); }

// Reverse scan like the reference; returns -1 or the offset of the LAST offending byte.
inline int64_t table_block(const uint8_t* s, size_t n, uint64_t* out) {
    uint64_t acc = 0;
    for (size_t k = n; k-- > 0;) {
        const uint8_t c = s[k];
        if (!is_base(c)) return (int64_t)k;
        acc = (acc << 2) | table_code(c);
    }
    *out = acc;
    return -1;
}

// _bloom_filter_64 (util.pxd:116-127)
inline bool chunk_ok(uint64_t x) {
    uint64_t q = 0;
    for (int b = 0; b < 8; ++b) q |= 1ull << ((x >> (8 * b)) & 63u);
    return (kBloom & q) == 0;
}

inline uint64_t pext_chunk(uint64_t x) {
#if defined(__BMI2__)
    return _pext_u64(x, 0x0606060606060606ull);      // util.pyx:39, :116
#else
    uint64_t r = 0;
    for (int b = 0; b < 8; ++b) r |= ((x >> (8 * b + 1)) & 3u) << (2 * b);
    return r;
#endif
}

// One full 32-nt block; returns -1 or the byte offset of the failing 8-byte chunk.
inline int64_t full_block(const uint8_t* s, uint64_t* out) {
    uint64_t block = 0;
    for (int j = 3; j >= 0; --j) {
        uint64_t chunk;
        memcpy(&chunk, s + 8 * j, 8);
        if (!chunk_ok(chunk)) return 8 * j;
        block = (block << 16) | pext_chunk(chunk);
    }
    *out = block;
    return -1;
}

#if defined(__AVX2__) && defined(__BMI2__)
// Fast path for the common case: if all 32 bytes at s are exactly 'A' 'C' 'G' 'T' (no aliased or
// invalid byte), the table rule and the PEXT rule agree ((c >> 1) & 3, no alias carry), so the
// block packs with four PEXTs.  Each byte is checked against the only ACGT letter with its low
// nibble ('A' 1, 'C' 3, 'T' 4, 'G' 7).  Returns false (nothing written) for any other byte.
inline bool acgt_block32(const uint8_t* s, uint64_t* out) {
    // non-ACGT slots hold i ^ 8: their low nibble differs from i, so no byte can match them
    const __m256i lut = _mm256_setr_epi8(0x08, 0x41, 0x0A, 0x43, 0x54, 0x0D, 0x0E, 0x47, 0x00, 0x01, 0x02, 0x03,
                                         0x04, 0x05, 0x06, 0x07, 0x08, 0x41, 0x0A, 0x43, 0x54, 0x0D, 0x0E, 0x47,
                                         0x00, 0x01, 0x02, 0x03, 0x04, 0x05, 0x06, 0x07);
    const __m256i x = _mm256_loadu_si256((const __m256i*)s);
    const __m256i lo = _mm256_and_si256(x, _mm256_set1_epi8(0x0F));
    const __m256i eq = _mm256_cmpeq_epi8(_mm256_shuffle_epi8(lut, lo), x);
    if ((uint32_t)_mm256_movemask_epi8(eq) != 0xFFFFFFFFu) return false;
    uint64_t c[4];
    memcpy(c, s, 32);
    *out = _pext_u64(c[0], 0x0606060606060606ull) | (_pext_u64(c[1], 0x0606060606060606ull) << 16) |
           (_pext_u64(c[2], 0x0606060606060606ull) << 32) | (_pext_u64(c[3], 0x0606060606060606ull) << 48);
    return true;
}
#define SSH_HAVE_ACGT_FAST 1
#endif

// Encode one read as shortseq._new would.  `words` receives ceil(L/32) words (the caller zeroes
// any further words).  Returns 0, 1 (unsupported base) or 2 (too long); err may be null.
inline int encode(const uint8_t* s, size_t L, uint64_t* words, ss_err* err) {
    if (err) {
        err->kind = 0;
        err->nbytes = 0;
        err->read_index = 0;
        err->byte_offset = -1;
    }
    if (L > kMaxNt) {
        if (err) err->kind = 2;
        return 2;
    }
    if (L == 0) return 0;
#ifdef SSH_HAVE_ACGT_FAST
    if (L == 32 && acgt_block32(s, &words[0])) return 0;
#endif
    if (L <= 32) {
        int64_t bad = table_block(s, L, &words[0]);
        if (bad >= 0) {
            if (err) { err->kind = 1; err->nbytes = 1; err->byte_offset = bad; }
            return 1;
        }
        return 0;
    }
    const size_t full = L / 32, rem = L % 32;
    for (size_t b = 0; b < full; ++b) {
#ifdef SSH_HAVE_ACGT_FAST
        if (acgt_block32(s + 32 * b, &words[b])) continue;
#endif
        int64_t bad = full_block(s + 32 * b, &words[b]);
        if (bad >= 0) {
            if (err) { err->kind = 1; err->nbytes = 8; err->byte_offset = (int64_t)(32 * b) + bad; }
            return 1;
        }
    }
    if (rem) {
        int64_t bad = table_block(s + 32 * full, rem, &words[full]);
        if (bad >= 0) {
            if (err) { err->kind = 1; err->nbytes = 1; err->byte_offset = (int64_t)(32 * full) + bad; }
            return 1;
        }
    }
    return 0;
}

// "ACTG"[code] (util.pyx:52) four nucleotides at a time: entry b of the table is the 4 characters
// of the 8-bit packed byte b (nt 0 in the low bits -> the first character, little-endian u32).
struct DecodeTable {
    uint32_t v[256];
    DecodeTable() {
        static const char kMap[4] = {'A', 'C', 'T', 'G'};
        for (uint32_t b = 0; b < 256; ++b) {
            uint32_t x = 0;
            for (uint32_t j = 0; j < 4; ++j) x |= (uint32_t)(uint8_t)kMap[(b >> (2 * j)) & 3u] << (8 * j);
            v[b] = x;
        }
    }
};

inline void decode(const uint64_t* words, size_t L, char* out) {
    static const DecodeTable t;
    static const char kMap[4] = {'A', 'C', 'T', 'G'};
    size_t i = 0;
    for (; i + 32 <= L; i += 32) {   // one word -> 32 characters
        uint64_t w = words[i >> 5];
        for (int q = 0; q < 8; ++q, w >>= 8) {
            const uint32_t c = t.v[w & 0xFFu];
            memcpy(out + i + 4 * q, &c, 4);
        }
    }
    for (; i < L; ++i) out[i] = kMap[(words[i >> 5] >> (2 * (i & 31))) & 3u];
}

inline uint64_t hamming(const uint64_t* a, const uint64_t* b, size_t L) {
    const size_t n = L <= 32 ? 1 : (L + 31) / 32;
    uint64_t cnt = 0;
    for (size_t i = 0; i < n; ++i) {
        uint64_t x = a[i] ^ b[i];
        x = ((x >> 1) | x) & 0x5555555555555555ull;
        cnt += (uint64_t)__builtin_popcountll(x);
    }
    return cnt;
}

}  // namespace ssh
