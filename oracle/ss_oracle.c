/*
 * oracle/ss_oracle.c — TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * A plain-C, scalar restatement of the reference's 2-bit encode / decode / hamming / counter
 * semantics (AlexTate/ShortSeq @ /root/reference).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library.  shortseq_amd/ never links or calls it.
 *
 * Pinned against: tests/golden/ fixtures (generated from the unmodified reference built by
 * oracle/build_ref.sh, script tests/golden/gen_golden.py) — see tests/test_oracle_golden.py.
 *
 * Every function cites the reference line it restates.  The restatement deliberately does NOT use
 * PEXT/BZHI: each bit is computed from the documented per-byte rule, so it is an independent check
 * of both the reference and the HIP kernels.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORA_NT_PER_BLOCK 32u                    /* util.pyx:42 */
#define ORA_MAX_NT 1024u                        /* short_seq_var.pyx:9 */
static const uint64_t ORA_BLOOM = 0xFFFFFFFFFFEFFF75ull;   /* util.pyx:75 */
static const char ORA_CHARMAP[4] = {'A', 'C', 'T', 'G'};   /* util.pyx:52 */

/* Error record: kind 0 ok, 1 unsupported base, 2 too long.  For kind 1, byte_offset/nbytes name the
 * bytes the reference would put in its message: one byte on the table path (short_seq_64.pyx:105,
 * util.pyx:137), an 8-byte chunk on the full-block path (util.pyx:115). */
typedef struct {
    int32_t kind;
    int32_t nbytes;
    int64_t read_index;
    int64_t byte_offset;
} ora_err;

/* util.pxd:98-99 — is_base(c): bloom & (1 << (c & 63)) == 0 */
static inline int ora_is_base(uint8_t c) { return ((ORA_BLOOM >> (c & 63u)) & 1u) == 0; }

/* util.pyx:44-50 — table_91.  Restated by rule: 'A'->0 'C'->1 'G'->3 'T'->2 'U'->2, every other
 * index < 91 -> 4.  Indices >= 91 are out of bounds in the reference (UB); only bloom-
 * passing bytes >= 0x80 reach that case, and they are outside the parity domain.  We define them by
 * the same rule as the low aliases (bit 6 clear -> 4, else (c >> 1) & 3), as the HIP path does. */
static inline uint32_t ora_table_code(uint8_t c) {
    if (c >= 91) return (c & 0x40u) ? ((c >> 1) & 3u) : 4u;
    switch (c) {
        case 'A': return 0; case 'C': return 1; case 'G': return 3;
        case 'T': return 2; case 'U': return 2;
        default: return 4;
    }
}

/* short_seq_64.pyx:96-108 and util.pyx:125-140 (identical loops): reverse scan, validate each byte,
 * acc = (acc << 2) | table_91[c].  A table value of 4 ORs into the NEXT nucleotide's low bit
 * (SURVEY Q1).  On failure the reported byte is the LAST offending one (reverse scan). */
static int ora_table_block(const uint8_t* s, uint32_t n, uint64_t* out, int64_t* bad_off) {
    uint64_t acc = 0;
    for (int64_t i = (int64_t)n - 1; i >= 0; --i) {
        uint8_t c = s[i];
        if (!ora_is_base(c)) { *bad_off = i; return 1; }
        acc = (acc << 2) | ora_table_code(c);
    }
    *out = acc;
    return 0;
}

/* util.pyx:100-119 — one 32-nt block: chunks j = 3..0 of 8 bytes; each chunk must pass
 * _bloom_filter_64 (util.pxd:116-127, i.e. every byte passes is_base); PEXT(chunk, 0x0606..06)
 * (util.pyx:39) == for each byte (c >> 1) & 3, packed little-endian.  No carry. */
static int ora_full_block(const uint8_t* s, uint64_t* out, int64_t* bad_off) {
    uint64_t block = 0;
    for (int j = 3; j >= 0; --j) {
        const uint8_t* chunk = s + 8 * j;
        for (int b = 0; b < 8; ++b)
            if (!ora_is_base(chunk[b])) { *bad_off = 8 * j; return 1; }
        uint64_t bits = 0;
        for (int b = 0; b < 8; ++b) bits |= (uint64_t)((chunk[b] >> 1) & 3u) << (2 * b);
        block = (block << 16) | bits;
    }
    *out = block;
    return 0;
}

/* Number of 64-bit words for L nucleotides: util.pyx:30-33 (ceil via double; exact for L <= 2^52). */
uint32_t ora_words_for(uint32_t L) { return (L + ORA_NT_PER_BLOCK - 1) / ORA_NT_PER_BLOCK; }

/* Encode ONE read exactly as shortseq._new (short_seq.pyx:54-74) would:
 *   L == 0            -> empty singleton, packed 0                       (short_seq.pyx:55-56)
 *   L <= 32           -> _marshall_bytes_64 (table path)                  (short_seq.pyx:57-62)
 *   33 <= L <= 1024   -> _marshall_bytes_array: L/32 full blocks + table tail (util.pyx:78-94)
 *   L > 1024          -> "Sequences longer than 1024 bases are not supported." (short_seq.pyx:74)
 * `dst` receives ceil(L/32) words (the caller zero-pads any further words, as tp_alloc/Calloc do). */
int ora_encode(const uint8_t* s, uint32_t L, uint64_t* dst, ora_err* err) {
    int64_t off = 0;
    if (err) { err->kind = 0; err->nbytes = 0; err->byte_offset = -1; }
    if (L > ORA_MAX_NT) { if (err) err->kind = 2; return 2; }
    if (L == 0) return 0;
    if (L <= 32) {
        if (ora_table_block(s, L, &dst[0], &off)) {
            if (err) { err->kind = 1; err->nbytes = 1; err->byte_offset = off; }
            return 1;
        }
        return 0;
    }
    uint32_t full = L / 32, rem = L % 32;
    for (uint32_t b = 0; b < full; ++b) {
        if (ora_full_block(s + 32 * b, &dst[b], &off)) {
            if (err) { err->kind = 1; err->nbytes = 8; err->byte_offset = 32 * (int64_t)b + off; }
            return 1;
        }
    }
    if (rem) {
        if (ora_table_block(s + 32 * full, rem, &dst[full], &off)) {
            if (err) { err->kind = 1; err->nbytes = 1; err->byte_offset = 32 * (int64_t)full + off; }
            return 1;
        }
    }
    return 0;
}

/* _unmarshall_bytes_64/_192/_var (short_seq_64.pyx:114-121, short_seq_192.pyx:114-127,
 * short_seq_var.pyx:98-120): nt i = charmap[(word[i/32] >> 2*(i%32)) & 3].  The var decoder's
 * one-word over-read contributes no output byte and is not replicated. */
void ora_decode(const uint64_t* words, uint32_t L, uint8_t* out) {
    for (uint32_t i = 0; i < L; ++i) out[i] = (uint8_t)ORA_CHARMAP[(words[i / 32] >> (2 * (i % 32))) & 3u];
}

/* __xor__ (short_seq_64.pyx:77-84; short_seq_192.pyx:74-91; short_seq_var.pyx:64-81):
 * per word x = a ^ b; x = ((x >> 1) | x) & 0x5555..; popcount.  ShortSeq64 always uses one word
 * (also for L == 0); the others use ceil(L/32). Operates on whole words, so Q1 tail bits count. */
uint32_t ora_hamming(const uint64_t* a, const uint64_t* b, uint32_t L) {
    uint32_t n = L <= 32 ? 1u : ora_words_for(L), cnt = 0;
    for (uint32_t i = 0; i < n; ++i) {
        uint64_t x = a[i] ^ b[i];
        x = ((x >> 1) | x) & 0x5555555555555555ull;
        cnt += (uint32_t)__builtin_popcountll(x);
    }
    return cnt;
}

/* ---------------------------------------------------------------------------------------------
 * Batch helpers (fixed length L, read i at ascii + i*stride; words at out + i*wpr).
 * err->read_index = first invalid read in input order (the read a sequential caller such as
 * ShortSeqCounter._count_py_bytes_list, counter.pyx:22-29, would raise on).
 * ------------------------------------------------------------------------------------------- */
int ora_encode_batch(const uint8_t* ascii, uint64_t n, uint32_t L, uint64_t stride,
                     uint64_t* out, uint32_t wpr, ora_err* err) {
    uint32_t W = L <= 32 ? 1u : ora_words_for(L);
    if (err) { err->kind = 0; err->read_index = -1; }
    for (uint64_t i = 0; i < n; ++i) {
        uint64_t* o = out + i * wpr;
        for (uint32_t w = 0; w < wpr; ++w) o[w] = 0;
        ora_err e;
        int rc = ora_encode(ascii + i * stride, L, o, &e);
        if (rc) { if (err) { *err = e; err->read_index = (int64_t)i; } return rc; }
        (void)W;
    }
    return 0;
}

void ora_decode_batch(const uint64_t* words, uint64_t n, uint32_t L, uint32_t wpr,
                      uint8_t* out, uint64_t stride) {
    for (uint64_t i = 0; i < n; ++i) ora_decode(words + i * wpr, L, out + i * stride);
}

void ora_hamming_ref_batch(const uint64_t* words, uint64_t n, uint32_t L, uint32_t wpr,
                           const uint64_t* ref, uint32_t* out) {
    for (uint64_t i = 0; i < n; ++i) out[i] = ora_hamming(words + i * wpr, ref, L);
}

void ora_hamming_pair_batch(const uint64_t* a, const uint64_t* b, uint64_t n, uint32_t L,
                            uint32_t wpr, uint32_t* out) {
    for (uint64_t i = 0; i < n; ++i) out[i] = ora_hamming(a + i * wpr, b + i * wpr, L);
}

/* ---------------------------------------------------------------------------------------------
 * Synthetic read generator; shared bit-for-bit with the device generator.
 * read i, word w (W = ceil(L/32)): r = splitmix64(seed + i*W + w) masked to 2*min(32, L-32w) bits;
 * ascii byte j of that word = "ACTG"[(r >> 2j) & 3].  Known answer: encode(ascii) == r.
 * ------------------------------------------------------------------------------------------- */
static inline uint64_t ora_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

uint64_t ora_gen_word(uint64_t seed, uint64_t i, uint32_t L, uint32_t w) {
    uint32_t W = ora_words_for(L);
    uint32_t nt = L - 32 * w; if (nt > 32) nt = 32;
    uint64_t r = ora_splitmix64(seed + i * W + w);
    return nt == 32 ? r : (r & ((1ull << (2 * nt)) - 1));
}

void ora_gen_reads(uint64_t seed, uint64_t i0, uint64_t n, uint32_t L, uint64_t stride, uint8_t* ascii) {
    uint32_t W = ora_words_for(L);
    for (uint64_t k = 0; k < n; ++k) {
        uint8_t* s = ascii + k * stride;
        for (uint32_t w = 0; w < W; ++w) {
            uint64_t r = ora_gen_word(seed, i0 + k, L, w);
            uint32_t nt = L - 32 * w; if (nt > 32) nt = 32;
            for (uint32_t j = 0; j < nt; ++j) s[32 * w + j] = (uint8_t)ORA_CHARMAP[(r >> (2 * j)) & 3u];
        }
    }
}

/* Pool-drawn reads for the counter workload: read i is pool item
 * p = splitmix64(pool_seed ^ (i * 0xD1B54A32D192ED03)) % U, whose bases are gen_reads(seed, p). */
uint64_t ora_pool_index(uint64_t pool_seed, uint64_t i, uint64_t U) {
    return ora_splitmix64(pool_seed ^ (i * 0xD1B54A32D192ED03ull)) % U;
}

void ora_gen_pool_reads(uint64_t seed, uint64_t pool_seed, uint64_t U, uint64_t i0, uint64_t n,
                        uint32_t L, uint64_t stride, uint8_t* ascii) {
    for (uint64_t k = 0; k < n; ++k)
        ora_gen_reads(seed, ora_pool_index(pool_seed, i0 + k, U), 1, L, stride, ascii + k * stride);
}

/* Zipf-drawn pool reads (SURVEY §8(d) C5 skew): read i is pool item rank = #{k : cdf[k] <= u63},
 * u63 = splitmix64(pool_seed ^ (i * 0xD1B54A32D192ED03)) >> 1, cdf = the Zipf CDF scaled to 2^63
 * (cdf[U-1] = 2^63; the table is an input, built once on the host). */
uint64_t ora_zipf_index(uint64_t pool_seed, uint64_t i, const uint64_t* cdf, uint64_t U) {
    const uint64_t u63 = ora_splitmix64(pool_seed ^ (i * 0xD1B54A32D192ED03ull)) >> 1;
    uint64_t lo = 0, hi = U;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        if (cdf[mid] <= u63) lo = mid + 1; else hi = mid;
    }
    return lo < U ? lo : U - 1;
}

void ora_gen_zipf_reads(uint64_t seed, uint64_t pool_seed, const uint64_t* cdf, uint64_t U, uint64_t i0,
                        uint64_t n, uint32_t L, uint64_t stride, uint8_t* ascii) {
    for (uint64_t k = 0; k < n; ++k)
        ora_gen_reads(seed, ora_zipf_index(pool_seed, i0 + k, cdf, U), 1, L, stride, ascii + k * stride);
}

/* ---------------------------------------------------------------------------------------------
 * Counter (counter.pyx:41-54): dict keyed on (length, packed words) — ShortSeq64.__eq__ compares
 * (length, packed) (short_seq_64.pyx:41-44), ShortSeq192/Var compare length + memcmp of ceil(L/32)
 * words (short_seq_192.pyx:35-41).  Count 1 on first sight, +1 after; iteration order = first
 * occurrence (dict insertion order).  Content dedup for ShortSeqVar too (documented deviation Q6).
 * Input: concatenated reads with per-read lengths/offsets.  Output: unique keys in first-occurrence
 * order: uwords[u*32 ...], ulen[u], ucount[u], ufirst[u].  Returns #unique or -1 on error.
 * ------------------------------------------------------------------------------------------- */
typedef struct { int64_t slot_uid; } ora_slot;

static uint64_t ora_hash_key(const uint64_t* w, uint32_t nw, uint32_t L) {
    uint64_t h = 0x243F6A8885A308D3ull ^ L;
    for (uint32_t i = 0; i < nw; ++i) h = ora_splitmix64(h ^ w[i]);
    return h;
}

int64_t ora_count(const uint8_t* ascii, const uint64_t* offsets, const uint32_t* lens, uint64_t n,
                  uint64_t* uwords /* n*32 capacity */, uint32_t* ulen, uint64_t* ucount,
                  uint64_t* ufirst, ora_err* err) {
    uint64_t cap = 16; while (cap < 2 * n + 16) cap <<= 1;
    int64_t* table = (int64_t*)malloc(cap * sizeof(int64_t));
    if (!table) return -1;
    for (uint64_t i = 0; i < cap; ++i) table[i] = -1;
    int64_t nu = 0;
    uint64_t w[32];
    if (err) { err->kind = 0; err->read_index = -1; }
    for (uint64_t i = 0; i < n; ++i) {
        uint32_t L = lens[i];
        memset(w, 0, sizeof w);
        ora_err e;
        if (ora_encode(ascii + offsets[i], L, w, &e)) {
            if (err) { *err = e; err->read_index = (int64_t)i; }
            free(table); return -1;
        }
        uint32_t nw = L <= 32 ? 1u : ora_words_for(L);
        uint64_t h = ora_hash_key(w, nw, L) & (cap - 1);
        for (;;) {
            int64_t u = table[h];
            if (u < 0) {
                table[h] = nu;
                memcpy(uwords + 32 * nu, w, sizeof w);
                ulen[nu] = L; ucount[nu] = 1; ufirst[nu] = i; ++nu;
                break;
            }
            if (ulen[u] == L && memcmp(uwords + 32 * u, w, nw * 8) == 0) { ucount[u]++; break; }
            h = (h + 1) & (cap - 1);
        }
    }
    free(table);
    return nu;
}

/* ------------------------------------------------------------------------------------------------
 * FASTQ sequence-line selection (test infrastructure; restates fast_read.pyx:3-20 and
 * short_seq.pyx:49-52 as a plain scalar loop).  getline() semantics: a line is everything up to and
 * including '\n', the last line may lack it.  count starts at 1; kept iff count % 2 == 0 and
 * count % 4 != 0.  len = strlen(line) - 1, strlen stopping at the first NUL of the line buffer.
 * lens[i] = 0xFFFFFFFF when strlen is 0 (size_t underflow in the reference).  Returns the number of
 * kept lines (only the first `cap` are written).
 * ---------------------------------------------------------------------------------------------- */
uint64_t ora_fastq_index(const uint8_t* buf, uint64_t nbytes, uint64_t* offsets, uint32_t* lens, uint64_t cap) {
    uint64_t pos = 0, count = 1, kept = 0;
    while (pos < nbytes) {                                  /* getline returns -1 at EOF */
        uint64_t end = pos;
        while (end < nbytes && buf[end] != '\n') ++end;
        const uint64_t line_len = (end < nbytes) ? end - pos + 1 : end - pos;   /* incl. '\n' */
        if (count % 2 == 0 && count % 4 != 0) {
            uint64_t slen = 0;
            while (slen < line_len && buf[pos + slen] != 0) ++slen;
            if (kept < cap) {
                offsets[kept] = pos;
                lens[kept] = slen == 0 ? 0xFFFFFFFFu : (uint32_t)(slen - 1 > 0xFFFFFFFEu ? 0xFFFFFFFEu : slen - 1);
            }
            ++kept;
        }
        ++count;
        pos += line_len;
    }
    return kept;
}

/* ------------------------------------------------------------------------------------------------
 * Slice (test infrastructure; restates short_seq.pyx:93-238): nts [start, start + n) of a packed
 * read `src` (wpr words), as _slice: offset = 2*start bits into block start/32; ShortSeq64 result
 * (n <= 32): (packed[0] >> offset) | (packed[1] << (64 - offset)) when the slice crosses the block,
 * _bzhi to 2n bits; longer: _shift_copy_trim (memcpy at offset 0, else per destination block
 * (src[i] >> offset) | (src[i+1] << (64 - offset)), the final block trimmed to tail bits).
 * Reads of src beyond wpr words count as 0 here (the reference reads past its array there; those
 * bits are always trimmed away).  dst gets ceil(2n/64) words (>= 1).
 * ---------------------------------------------------------------------------------------------- */
static inline uint64_t ora_bzhi(uint64_t x, uint64_t nbits) { return nbits >= 64 ? x : (x & ((1ull << nbits) - 1)); }

void ora_slice(const uint64_t* src, uint32_t wpr, uint32_t start, uint32_t n, uint64_t* dst) {
    const uint32_t blk = start / 32, off = 2 * (start % 32);
    const uint64_t bits = 2ull * n;
    const uint64_t* p = src + blk;
    const uint32_t avail = wpr - blk;                 /* words readable from p */
#define ORA_SRC(i) ((uint32_t)(i) < avail ? p[(i)] : 0ull)
    if (n <= 32) {
        uint64_t r;
        if (off + bits > 64) r = ora_bzhi((ORA_SRC(0) >> off) | (ORA_SRC(1) << (64 - off)), bits);
        else r = ora_bzhi(ORA_SRC(0) >> off, bits);
        dst[0] = r;
        return;
    }
    const uint64_t nblk = (bits + 63) / 64, tail = bits % 64;
    for (uint64_t i = 0; i < nblk; ++i)
        dst[i] = off == 0 ? ORA_SRC(i) : ((ORA_SRC(i) >> off) | (ORA_SRC(i + 1) << (64 - off)));
    if (tail) dst[nblk - 1] = ora_bzhi(dst[nblk - 1], tail);
#undef ORA_SRC
}
