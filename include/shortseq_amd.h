/*
 * shortseq_amd.h — C ABI of the MI355X (gfx950) batch 2-bit DNA engine.
 *
 * Drop-in boundary for the reference's native kernel layer (AlexTate/ShortSeq, Cython cdef functions
 * exported as PyCapsules in each module's __pyx_capi__).  The reference kernels work
 * on ONE read per call; each entry point below does the same work for a whole batch on the GPU.
 *
 * Conventions
 *   - Plain C types only.  `d_*` arguments are device pointers (hipMalloc / torch CUDA tensors);
 *     `h_*` arguments are host pointers.  `stream` is a hipStream_t passed as void* (NULL = default).
 *   - Device entry points are asynchronous on `stream`, never allocate, never synchronise, and are
 *     safe to capture in a hipGraph.  They return SS_OK or a launch/argument error immediately.
 *     Exceptions, each documented at its declaration: the counter and ingest handles (their own
 *     workspaces; the ingest calls are synchronous), and ss_hamming_all_pairs / _ex when they take
 *     the pigeonhole form (a per-device scratch buffer cached across calls; AUTO reads its candidate
 *     totals back with one stream sync).  SS_ALLPAIRS_TILES keeps the plain contract.
 *   - Validation mirrors util.pxd:98-99 (bloom filter 0xFFFFFFFFFFEFFF75, util.pyx:75).  A kernel
 *     that meets an invalid byte writes the index of the FIRST invalid read (input order) into
 *     *d_first_bad (atomicMin; the entry point resets it to UINT64_MAX first).  The caller re-scans
 *     that read with ss_host_encode() to obtain the reference's exact error (byte or 8-byte chunk).
 *   - Layouts: read i of a fixed-length batch starts at d_ascii + i*stride (bytes); its packed words
 *     are d_words[i*wpr .. i*wpr + wpr), nt j in word j/32 at bits 2*(j%32) (nt 0 = LSBs), codes
 *     A=0 C=1 T=2 G=3 (README.md:101-112).  wpr >= ceil(L/32) (>= 1); extra words are written 0.
 *
 * Error codes (ss_status): negative = API/runtime error, positive = data error.
 */
#ifndef SHORTSEQ_AMD_H
#define SHORTSEQ_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SS_ABI_VERSION 1

enum ss_status {
    SS_OK = 0,
    SS_EINVALID_BASE = 1,   /* "Unsupported base character: ..."  (short_seq_64.pyx:105, util.pyx:115/137) */
    SS_ETOO_LONG = 2,       /* "Sequences longer than 1024 bases are not supported." (short_seq.pyx:74) */
    SS_EARG = -1,           /* bad argument (NULL pointer, L out of range, wpr too small, misalignment) */
    SS_EHIP = -2,           /* HIP runtime error; see ss_last_error_string() */
    SS_ENOMEM = -3,         /* device allocation failed (counter handles, forced pigeonhole all-pairs) */
    SS_EFULL = -4           /* counter table full */
};

#define SS_MAX_NT 1024u     /* short_seq_var.pyx:9 */
#define SS_MAX_64_NT 32u    /* short_seq_64.pyx:28 */
#define SS_MAX_192_NT 96u   /* short_seq_192.pyx:22 */

/* Error detail for the host codec (ss_host_encode).  kind = ss_status; for SS_EINVALID_BASE,
 * [byte_offset, byte_offset + nbytes) are the bytes the reference names in its message: 1 byte on
 * the table path (the LAST offending byte, reverse scan), 8 bytes (the chunk) on the full-block path
 * (blocks in order, chunks 3->0 within a block). */
typedef struct ss_err {
    int32_t kind;
    int32_t nbytes;
    int64_t read_index;
    int64_t byte_offset;
} ss_err;

/* ------------------------------------------------------------------------------------------------
 * Library / runtime
 * ---------------------------------------------------------------------------------------------- */
int ss_abi_version(void);
const char* ss_last_error_string(void);          /* thread-local message of the last SS_EHIP/EARG */
int ss_device_count(int* h_count);
int ss_set_device(int device);
int ss_get_device(int* h_device);                   /* the calling thread's current device */

/* Pinned host staging buffers (hipHostMalloc / hipHostFree) for H2D batch staging. */
int ss_pinned_alloc(void** h_ptr, size_t bytes);
int ss_pinned_free(void* h_ptr);

/* ------------------------------------------------------------------------------------------------
 * Batch encode — replaces, per read:
 *   _marshall_bytes_64   (short_seq_64.pyx:96-108)   L <= 32: table path (SURVEY Q1 carry kept)
 *   _marshall_bytes_192  (short_seq_192.pyx:103-108) 33..96  -> _marshall_bytes_array
 *   _marshall_bytes_var  (short_seq_var.pyx:123-132) 97..1024 -> _marshall_bytes_array
 *   _marshall_bytes_array/_full_blocks/_partial_block (util.pyx:78-140): full 32-nt blocks by the
 *   PEXT rule (c>>1)&3, the L%32 tail by the table rule.
 * Fixed length L (1..1024) for every read.  Fast path when L % 16 == 0, stride % 16 == 0 and
 * d_ascii is 16-byte aligned; otherwise a general path (any L, stride >= L).
 * ---------------------------------------------------------------------------------------------- */
int ss_encode_fixed(const uint8_t* d_ascii, uint64_t n, uint32_t L, uint64_t stride,
                    uint64_t* d_words, uint32_t wpr, uint64_t* d_first_bad, void* stream);

/* Variable-length batch: read i = d_ascii[d_offsets[i] .. + d_lens[i]), 0 <= len <= 1024
 * (short_seq.pyx:54-74 length-class switch: 0 -> packed 0, <= 32 table path, else array path).
 * Reads longer than 1024 are reported through *d_first_bad like invalid bases.  The kernel reads the
 * blob in whole 16-B-aligned chunks around each read (device allocations are at least 256-B aligned,
 * so this never leaves the allocation). */
int ss_encode_var(const uint8_t* d_ascii, const uint64_t* d_offsets, const uint32_t* d_lens,
                  uint64_t n, uint64_t* d_words, uint32_t wpr, uint64_t* d_first_bad, void* stream);

/* ------------------------------------------------------------------------------------------------
 * Batch decode — replaces _unmarshall_bytes_64/_192/_var (short_seq_64.pyx:114-121,
 * short_seq_192.pyx:114-127, short_seq_var.pyx:98-120): nt j -> "ACTG"[code] (util.pyx:52).
 * Writes exactly L bytes per read at d_ascii + i*stride (no terminator).
 * ---------------------------------------------------------------------------------------------- */
int ss_decode_fixed(const uint64_t* d_words, uint64_t n, uint32_t L, uint32_t wpr,
                    uint8_t* d_ascii, uint64_t stride, void* stream);

int ss_decode_var(const uint64_t* d_words, const uint32_t* d_lens, uint64_t n, uint32_t wpr,
                  uint8_t* d_ascii, const uint64_t* d_offsets, void* stream);

/* ------------------------------------------------------------------------------------------------
 * Hamming — replaces ShortSeq64/192/Var.__xor__ (short_seq_64.pyx:77-84, short_seq_192.pyx:74-91,
 * short_seq_var.pyx:64-81): sum over W = (L <= 32 ? 1 : ceil(L/32)) words of
 * popcount(((x >> 1) | x) & 0x5555555555555555), x = a ^ b.  Whole-word, like the reference.
 * Dense rows (wpr == W) with 16-B aligned word arrays and an 8-B aligned d_out take the streaming
 * kernels (k_ham_dense / k_ham_dense3w); any other layout the lane-group kernel.  Same results.
 * ---------------------------------------------------------------------------------------------- */
int ss_hamming_ref(const uint64_t* d_words, uint64_t n, uint32_t L, uint32_t wpr,
                   const uint64_t* d_ref, uint32_t* d_out, void* stream);
int ss_hamming_pair(const uint64_t* d_a, const uint64_t* d_b, uint64_t n, uint32_t L, uint32_t wpr,
                    uint32_t* d_out, void* stream);

/* Fused encode + hamming vs one packed reference read (d_ref_words, wpr words, e.g. read 0 encoded
 * first): one pass over the ASCII, writes the packed words (if d_words != NULL) and the distance. */
int ss_encode_hamming_ref(const uint8_t* d_ascii, uint64_t n, uint32_t L, uint64_t stride,
                          uint64_t* d_words, uint32_t wpr, const uint64_t* d_ref_words,
                          uint32_t* d_out, uint64_t* d_first_bad, void* stream);

/* ------------------------------------------------------------------------------------------------
 * Batch slice / subscript — replaces ShortSeq64/192/Var.__getitem__ (short_seq_64.pyx:53-75,
 * short_seq_192.pyx:50-72, short_seq_var.pyx:37-59) -> _slice / _slice_to_ShortSeq64/192/Var /
 * _shift_copy_trim (short_seq.pyx:93-238) and _subscript (short_seq.pyx:78-90, a 1-nt slice):
 * out row r = nts [start, start + len) of read r, packed from bit 0, trimmed to 2*len bits, words
 * past the slice zero.  out_wpr >= max(1, ceil(len/32)).
 * fixed: one (start, len) for the batch, start + len <= L.
 * var:   per-read d_starts / d_lens; with d_read_lens (nullable) they are clamped to the read
 *        (start' = min(start, L_r), len' = min(len, L_r - start')), as Python slice bounds are.
 * ---------------------------------------------------------------------------------------------- */
int ss_slice_fixed(const uint64_t* d_words, uint64_t n, uint32_t L, uint32_t wpr, uint32_t start, uint32_t len,
                   uint64_t* d_out, uint32_t out_wpr, void* stream);
int ss_slice_var(const uint64_t* d_words, uint64_t n, uint32_t wpr, const uint32_t* d_read_lens,
                 const uint32_t* d_starts, const uint32_t* d_lens, uint64_t* d_out, uint32_t out_wpr, void* stream);

/* All-pairs thresholded hamming (UMI-style dedup; distance = __xor__ above) over
 * one batch of n < 2^32 packed reads of length L: for every unordered pair i < j with distance
 * <= max_dist, d_counts[i] and d_counts[j] += 1 (neighbours per read; if d_counts != NULL) and the
 * pair (i, j) is appended as two u32 to d_pairs (if != NULL) while fewer than max_pairs were written.
 * *d_npairs = all such pairs (may exceed max_pairs).  The entry point zeroes d_counts / *d_npairs.
 * Pair order is unspecified (each pair is written as i < j).  n <= 65535 * 1024 per call (L <= 32).
 * Same as ss_hamming_all_pairs_ex(..., SS_ALLPAIRS_AUTO, stream). */
int ss_hamming_all_pairs(const uint64_t* d_words, uint64_t n, uint32_t L, uint32_t wpr, uint32_t max_dist,
                         uint32_t* d_counts, uint32_t* d_pairs, uint64_t max_pairs, uint64_t* d_npairs,
                         void* stream);

/* Method of ss_hamming_all_pairs_ex; every method gives the same counts, total and pair set.
 * TILES: every pair checked (MFMA one-hot tiles for L <= 128, bit-plane tiles above).
 * PIGEONHOLE (L <= 128, max_dist < 16): the min(L + 1, 32 W) positions split into max_dist + 1
 *   segments (W = ceil(L/32) words; a segment may cross a word boundary); only pairs with an equal
 *   segment are checked (bucketed per segment on the device; a segment past 11 nt by a hash).
 *   Blocks the calling thread once on the stream (the candidate totals are read back) only in AUTO;
 *   forced, it queues everything.  Its scratch lives on the device that holds d_words.
 * AUTO: PIGEONHOLE when L <= 128, segments >= 3 nt, n >= 32768 and the bucket histogram shows fewer
 *   than 1/16 of all pairs as candidates; TILES otherwise.  A stream under hipGraph capture always
 *   gets TILES in AUTO (no allocation, no host read-back: the call stays capturable). */
#define SS_ALLPAIRS_AUTO 0u
#define SS_ALLPAIRS_TILES 1u
#define SS_ALLPAIRS_PIGEONHOLE 2u
int ss_hamming_all_pairs_ex(const uint64_t* d_words, uint64_t n, uint32_t L, uint32_t wpr, uint32_t max_dist,
                            uint32_t* d_counts, uint32_t* d_pairs, uint64_t max_pairs, uint64_t* d_npairs,
                            uint32_t method, void* stream);

/* ------------------------------------------------------------------------------------------------
 * Dedup counter — replaces ShortSeqCounter._count_sequence (counter.pyx:41-54): key = (length,
 * packed words) (short_seq_64.pyx:41-44; short_seq_192.pyx:35-41), count += 1, first-occurrence
 * index kept so the host can rebuild dict insertion order.  Open-addressing table in HBM, one per
 * handle; all keys of one handle share one length L <= 1024 (the length is part of the key).
 * L <= 32: the slot key is the packed word.  L > 32: W = ceil(L/32) words per key, kept beside the
 * slots; the slot holds a 64-bit fingerprint of the words and equality is decided on the words.
 * A slot is 16 B (key u64, count u32, first index u32): global read indices of one handle stay below
 * 2^32 - 1 (inserts past that return SS_EARG).  Counts are u64 (ShortSeqCounter's are Python ints,
 * counter.pyx:53): before the reads inserted since the last spill could wrap a slot's u32, every
 * count moves into a per-slot u64 array (allocated then, 8 B per slot) and ss_counter_merge /
 * _merge_words carry past 32 bits into it; extracts return the sum.  The packed exchange records
 * (ss_counter_pack_ranges) carry u32 counts and flag bit 2 for a count past that.  Packed-word
 * handles (ss_counter_set_words) keep u32 slot counts: the drop-in engine that keys them spills
 * their counts per row itself (its per-row u64 counts).
 * ---------------------------------------------------------------------------------------------- */
typedef struct ss_counter ss_counter;

int ss_counter_create(uint64_t capacity, ss_counter** out);      /* capacity rounded up to 2^k */
int ss_counter_destroy(ss_counter* c);
int ss_counter_reset(ss_counter* c, void* stream);
uint64_t ss_counter_capacity(const ss_counter* c);

/* Reserve workspace (~100 B per read + a small per-region table) so inserts of up to max_reads
 * reads take the partitioned path: reads are bucketed by table region and each region is
 * aggregated by one workgroup in LDS (no per-read global atomics).  Host call (allocates).  L 16/32
 * with 16-B aligned rows encode inside the first partition pass (a key repeated within a 4096-read
 * tile leaves it as one weighted record when its bin is heavy, so skewed inputs keep the partition
 * balanced; records finding their bucket full are counted by a direct insert afterwards); any other
 * L <= 32 / layout is packed into the workspace first.  Inserts larger than the reservation use the
 * direct atomic-insert kernels.  Requires capacity <= 2^26 (32768 regions).  max_reads < 2^31. */
int ss_counter_reserve(ss_counter* c, uint64_t max_reads);
uint64_t ss_counter_reserved(const ss_counter* c);
int ss_counter_release(ss_counter* c);       /* free the workspace (inserts take the direct path) */

/* Encode + count a fixed-length batch (L <= 1024).  Read i gets global index base_index + i.
 * Multi-word handles (L > 32) always take the partitioned path and grow the workspace to n reads
 * (plus n * W words for the packed batch) when the reservation is smaller. 
 * If the batch holds an invalid read (reported through *d_first_bad) the table's contents are
 * unspecified afterwards, like the reference counter that raises mid-list (counter.pyx:22-29). */
int ss_counter_insert_fixed(ss_counter* c, const uint8_t* d_ascii, uint64_t n, uint32_t L,
                            uint64_t stride, uint64_t base_index, uint64_t* d_first_bad, void* stream);

/* Merge already-counted entries (e.g. received from other GPUs): counts add, first index = min. */
int ss_counter_merge(ss_counter* c, const uint64_t* d_keys, const uint32_t* d_lens,
                     const uint64_t* d_counts, const uint64_t* d_first, uint64_t m, void* stream);

/* Merge already-counted multi-word entries (L > 32): d_words[m * W] the key words of entry i (row
 * i), counts add, first index = min.  The m entries must be distinct keys (e.g. the extraction of
 * another handle of the same length, ss_counter_extract_words); keys already in the table are
 * found by their words.  Used to grow a per-length table (ss_ingest).  New in this ABI version;
 * replaces no reference interface (the reference's dict grows by itself, counter.pyx:41-54). */
int ss_counter_merge_words(ss_counter* c, const uint64_t* d_words, const uint64_t* d_counts,
                           const uint64_t* d_first, uint64_t m, void* stream);

/* Test hook: spill the u32 slot counts into the u64 array once more than `reads` (1 .. 2^32 - 1,
 * default 2^32 - 1) reads were inserted since the last spill.  New in this ABI version. */
int ss_counter_set_spill_limit(ss_counter* c, uint64_t reads);

/* Fix the key length of an empty handle (also done by the first insert); -1 from ss_counter_length
 * means not fixed yet, -2 a packed-word handle (ss_counter_set_words). */
int ss_counter_set_length(ss_counter* c, uint32_t L);
int ss_counter_length(const ss_counter* c);

/* Packed-word keys: an empty handle (or one after ss_counter_reset) set to keys of W = 2..64 words,
 * compared whole; ss_counter_insert_words counts n rows d_words[n * W] already packed on the device
 * (row i gets global index base_index + i; partitioned path, workspace grown to n as for multi-word
 * ss_counter_insert_fixed).  The drop-in engine keys one handle per length class this way: the
 * ceil(L/32) words of a read of 32(W-2)+1 .. 32(W-1) nt plus its length as the last word, so one
 * table holds every length of the class (key = (length, words), short_seq_192.pyx:35-41 /
 * short_seq_var.pyx:22-28).  Extract with ss_counter_extract_words (lens = 0: the length is the
 * caller's word); grow with ss_counter_merge_words.  New in this ABI version; replaces no
 * reference interface. */
int ss_counter_set_words(ss_counter* c, uint32_t W);
int ss_counter_insert_words(ss_counter* c, const uint64_t* d_words, uint64_t n, uint64_t base_index, void* stream);

/* Copy the handle's overflow word to *d_flag (device u64): bit 0 = table full during an insert or
 * merge, bit 1 = an extract found more entries than `cap`, bit 2 = a merged count did not fit 32
 * bits, bit 3 = a read index did not fit 32 bits.  Nonzero means the result is invalid. */
int ss_counter_overflow(ss_counter* c, uint64_t* d_flag, void* stream);

/* Per-pass timing of the optimistic partitioned insert (tracing: bench.py's C5 lines attribute the
 * insert's time to its passes).  With on != 0 every such insert records HIP events on its stream
 * between its passes (a ring of 64 inserts, folded as it wraps); ss_counter_pass_times returns the
 * mean ms per insert since the last call of: [0] coarse partition (k_prep + k_pf_coarse), [1] sub-bin
 * order (k_pf_order), [2] fine scatter (k_pf_scatter), [3] aggregate (k_pc_aggregate_slice), [4]
 * spill insert (k_spill_insert), and *h_inserts; then resets the sums.  Host calls.  New in this
 * ABI version; replaces no reference interface. */
int ss_counter_set_timing(ss_counter* c, int on);
int ss_counter_pass_times(ss_counter* c, double* h_ms, uint64_t* h_inserts);

/* Number of occupied slots -> *d_size (device u64). */
int ss_counter_size(ss_counter* c, uint64_t* d_size, void* stream);

/* Compact the table into arrays of capacity `cap` (>= size).  Entries are grouped by owner
 * (hash % n_parts); d_part_counts[n_parts] receives the entries per part, in part order.
 * n_parts = 1 gives a plain compaction.  Order inside a part is unspecified (sort by first index
 * on the host to recover insertion order). */
int ss_counter_extract(ss_counter* c, uint32_t n_parts, uint64_t* d_keys, uint32_t* d_lens,
                       uint64_t* d_counts, uint64_t* d_first, uint64_t cap,
                       uint64_t* d_part_counts, void* stream);

/* Words per key of the handle: 1 for L <= 32, ceil(L/32) for multi-word keys (L 33..1024, the
 * ShortSeq192 / ShortSeqVar keys of short_seq_192.pyx:35-41 / short_seq_var.pyx:22-28; counted
 * under a 64-bit fingerprint of the words, equality always on the full words).  0 for NULL. */
int ss_counter_words(const ss_counter* c);

/* ss_counter_extract for any key length: as ss_counter_extract, plus d_words[cap * W] receives the
 * W packed words of each entry (row i = entry i).  For multi-word handles d_fps gets the entries'
 * fingerprints (the owner partition is owner_of(fingerprint)); for single-word handles d_fps and
 * d_words both get the packed word.  ss_counter_extract itself rejects multi-word handles, and
 * ss_counter_merge takes single-word keys only. */
int ss_counter_extract_words(ss_counter* c, uint32_t n_parts, uint64_t* d_fps, uint32_t* d_lens,
                             uint64_t* d_words, uint64_t* d_counts, uint64_t* d_first, uint64_t cap,
                             uint64_t* d_part_counts, void* stream);

/* ------------------------------------------------------------------------------------------------
 * FASTQ ingest on the device — replaces _read_fastq_short_seqs (fast_read.pyx:3-20) + _from_chars
 * (short_seq.pyx:49-52) as called by read_and_count_fastq (counter.pyx:57-70): lines split at '\n',
 * 0-based line j kept iff j % 4 == 1, length = strlen(line) - 1 (the '\n' dropped; a final line
 * without '\n' loses its last character; an embedded NUL ends the line).
 * A chunk is < 4 GiB, starts at a line boundary and ends right after a '\n' (or at EOF: at_eof != 0);
 * line0 = lines before the chunk.  d_buf 16-B aligned.
 *   1. ss_fastq_scan: newlines per 16-KiB tile + scan into d_ws (ss_fastq_scan_ws_bytes(nbytes)
 *      bytes); *d_nlines = newlines in the chunk.
 *   2. ss_fastq_index (same d_ws): d_offsets[i] / d_lens[i] of sequence line i (chunk-relative),
 *      *d_nreads = sequence lines in the chunk (may exceed max_reads: then only max_reads are
 *      written; size max_reads from *d_nlines: at most nlines / 4 + 1).  d_aux: max_reads u64 of
 *      scratch.  d_lens[i] = 0xFFFFFFFF where strlen is 0 (the reference's size_t underflow, i.e.
 *      the too-long error); > 1024 is the too-long error as well.
 * or, reading the chunk once:
 *   ss_fastq_index_onepass: the same outputs from one read of the chunk (each 32-KiB tile stages its
 *      newline positions, 4 B per line, and the line numbers are resolved from the tile counts);
 *      d_ws of ss_fastq_onepass_ws_bytes(nbytes, max_reads) bytes; d_counts[3] = {newlines,
 *      sequence lines, staging full}.  max_reads is the caller's bound (a sequence line takes >= 4
 *      bytes of the file: nbytes / 4 + 2 always suffices); the outputs are complete iff
 *      d_counts[2] == 0 and d_counts[1] <= max_reads, otherwise the call is repeated with a larger
 *      max_reads (>= d_counts[1]; doubled when d_counts[2] != 0).
 * The (d_offsets, d_lens) pair is the ragged layout of ss_encode_var and ss_gather_rows.
 * ---------------------------------------------------------------------------------------------- */
uint64_t ss_fastq_scan_ws_bytes(uint64_t nbytes);
int ss_fastq_scan(const uint8_t* d_buf, uint64_t nbytes, void* d_ws, uint64_t ws_bytes, uint64_t* d_nlines,
                  void* stream);
int ss_fastq_index(const uint8_t* d_buf, uint64_t nbytes, uint64_t line0, int at_eof, void* d_ws,
                   uint64_t* d_offsets, uint32_t* d_lens, uint64_t* d_aux, uint64_t max_reads,
                   uint64_t* d_nreads, void* stream);
uint64_t ss_fastq_onepass_ws_bytes(uint64_t nbytes, uint64_t max_reads);
int ss_fastq_index_onepass(const uint8_t* d_buf, uint64_t nbytes, uint64_t line0, int at_eof, void* d_ws,
                           uint64_t ws_bytes, uint64_t* d_offsets, uint32_t* d_lens, uint64_t* d_aux,
                           uint64_t max_reads, uint64_t* d_counts, void* stream);

/* Gather ragged rows into a dense batch: dst row r = d_src[d_offsets[s] .. + L) with s = d_sel[r]
 * (or r when d_sel is NULL); dst_stride % 16 == 0, >= round_up(L, 16); d_dst 16-B aligned; bytes of
 * the last 16-B chunk past L are 'A'.  Reads of d_src stay below src_bytes.  Feeds one length
 * group of a ragged batch (FASTQ, ShortSeqCounter lists) to the fixed-length encode / counter. */
int ss_gather_rows(const uint8_t* d_src, uint64_t src_bytes, const uint64_t* d_offsets, const uint64_t* d_sel,
                   uint64_t m, uint32_t L, uint8_t* d_dst, uint64_t dst_stride, void* stream);

/* Multi-GPU counter with region-range ownership: part p of n owns the table regions
 * [ceil(p R / n), ceil((p + 1) R / n)) (R = capacity / slice slots, ss_counter_geometry); the sentinel
 * key ~0 belongs to the owner of its hash region.  Every rank counts its own reads into its own
 * table, extracts the entries of the OTHER ranks' regions (ss_counter_extract_ranges: grouped by
 * part, each part sorted by region, the sentinel last), exchanges them (all-to-all), and folds what it
 * receives into its own table's owned regions (ss_counter_merge_runs).  The regions a rank does not own
 * are stale afterwards; the union of all ranks' owned regions is the exact counter.
 *   ss_counter_geometry:       host query, log2(capacity) and log2(slots per region).
 *   ss_counter_extract_ranges: as ss_counter_extract with parts = region ranges (single-word keys).
 *   ss_counter_merge_runs:     d_run_offsets = n_runs (begin, end) u64 pairs (device) into the received
 *                              arrays; every run sorted by region and all keys in `part`'s regions;
 *                              d_bounds: n_runs * (regions of part + 1) u32 of scratch. */
int ss_counter_geometry(const ss_counter* c, uint32_t* h_log2cap, uint32_t* h_slice_log);
int ss_counter_extract_ranges(ss_counter* c, uint32_t n_parts, uint64_t* d_keys, uint32_t* d_lens,
                              uint64_t* d_counts, uint64_t* d_first, uint64_t cap, uint64_t* d_part_counts,
                              void* stream);
int ss_counter_merge_runs(ss_counter* c, const uint64_t* d_keys, const uint64_t* d_counts, const uint64_t* d_first,
                          const uint64_t* d_run_offsets, uint32_t n_runs, uint64_t m, uint32_t part,
                          uint32_t n_parts, uint32_t L, uint32_t* d_bounds, void* stream);

/* Packed exchange (the multi-GPU counter's one exchange step in 16-B records instead of three u64
 * arrays): record = {key u64, count u32 | (first - first_base) u32 << 32}.
 * ss_counter_pack_ranges: the entries of every part except skip_part (-1 = none; the caller's own
 *   part stays in its table), grouped by part in part order, inside a part by table region, the
 *   sentinel key ~0 last in its owner's segment; written to d_rec (16-byte aligned, cap records);
 *   d_part_counts[n_parts] (0 for skip_part).  One pass over the table after a partitioned insert
 *   (its aggregate keeps the per-region occupancy), two otherwise.  A count or first - first_base
 *   that does not fit 32 bits, or more than cap records, raises the overflow word (bits 4 / 2).
 * ss_counter_merge_packed: as ss_counter_merge_runs for packed runs; run r's first indices are
 *   relative to d_run_first_base[r] (the source rank's first_base). */
int ss_counter_pack_ranges(ss_counter* c, uint32_t n_parts, int32_t skip_part, uint64_t first_base, void* d_rec,
                           uint64_t cap, uint64_t* d_part_counts, void* stream);
int ss_counter_merge_packed(ss_counter* c, const void* d_rec, const uint64_t* d_run_offsets,
                            const uint64_t* d_run_first_base, uint32_t n_runs, uint64_t m, uint32_t part,
                            uint32_t n_parts, uint32_t L, uint32_t* d_bounds, void* stream);

/* ------------------------------------------------------------------------------------------------
 * Ragged read streams counted on the GPU — the batch engine behind the drop-in ShortSeqCounter(list)
 * (counter.pyx:22-39: _count_py_bytes_list -> _from_py_bytes -> _count_sequence) and
 * read_and_count_fastq (counter.pyx:57-70 + fast_read.pyx:3-20).  Host calls, synchronous, one
 * engine per thread; the engine owns its stream, pinned staging and counter tables (one for lengths 1-31 --
 * the packed word with a length marker at bit 2L + 1 -- one for 32, one per length class).
 *   ss_ingest_staging:  a pinned buffer of >= nbytes the caller fills with the reads back to back
 *                       (valid until the next staging / add call).
 *   ss_ingest_add_blob: count n reads of h_blob (read i = the next h_lens[i] bytes); global indices
 *                       continue across calls.
 *   ss_ingest_add_fastq: the sequence lines of a FASTQ file (the fast_read.pyx rule; lengths as
 *                       ss_fastq_index), read in chunks of chunk_bytes (0 = 1 GiB); *h_nseqs = lines.
 *   ss_ingest_error:    the first rejected read in input order: *h_index (UINT64_MAX = none), *h_kind
 *                       (SS_EINVALID_BASE, its bytes -> h_read[0..cap), *h_len; or SS_ETOO_LONG).  The
 *                       caller raises the reference's exception for it (ss_host_encode gives the
 *                       message of an invalid base); nothing after that read is counted.
 *   ss_ingest_finish:   orders the distinct keys by first occurrence (dict insertion order);
 *                       *h_nkeys entries, *h_nwords packed words in total.
 *   ss_ingest_results:  pinned arrays valid until the next reset: lengths u32 [nkeys], counts u64
 *                       [nkeys], words u64 (entry k's max(0, ceil(L/32)) words follow entry k-1's; a
 *                       length-0 entry is the empty read and has none).
 *   ss_ingest_reset:    drop the counts (tables are pooled for the next call).
 *   ss_ingest_set_exact: 1 = size every length class's table by its rows (the 2 x rows bound).  By
 *                       default a class table (lengths 33..1024, one per ceil(L/32)) is sized by a
 *                       HyperLogLog sketch of its distinct keys over the call (1.2 x the estimate +
 *                       256, at most half full); a table that still runs full makes the add call
 *                       return SS_EFULL, and the caller counts again with exact sizing (the drop-in
 *                       front does).  2 = size them by 1/64 of the sketch (a test hook that makes
 *                       the SS_EFULL path run).  3 = test hook: the classes' fingerprint count takes
 *                       its exact fallback (as if two keys shared a 64-bit fingerprint).  4 = as 3,
 *                       but found only after the deferred fold and the speculative finish were queued.
 *                       5 = test hook: the speculative finish's result bound as if the sketch said 0,
 *                       so it is dropped and the finish runs the ordinary way.  New in this ABI
 *                       version; the reference dict has no sizing.
 * ---------------------------------------------------------------------------------------------- */
typedef struct ss_ingest ss_ingest;
int ss_ingest_create(int device, ss_ingest** h_out);
int ss_ingest_destroy(ss_ingest* g);
int ss_ingest_reset(ss_ingest* g);
int ss_ingest_set_exact(ss_ingest* g, int exact);
/* Global read indices of one engine are u64 (a call counts any number of reads); a length's or class's
 * table indexes its rows with a u32 first index, so a group about to pass 2^32 - 1 rows is re-keyed
 * (its distinct keys become its first rows).  Test hook: lower that bound to `rows` (>= 1024) so the
 * re-keying runs at small sizes.  New in this ABI version. */
int ss_ingest_set_row_limit(ss_ingest* g, uint64_t rows);
/* A slot's count is u32: before the reads counted since the last spill pass 2^32 - 2, every table's
 * counts move into its group's u64 row counts (added back at finish / export), so a key's count is
 * exact past 2^32.  Test hook: spill once `reads` (1 .. 2^32 - 2) reads have been counted since the
 * last spill.  New in this ABI version. */
int ss_ingest_set_count_limit(ss_ingest* g, uint64_t reads);
int ss_ingest_staging(ss_ingest* g, uint64_t nbytes, uint8_t** h_ptr);
int ss_ingest_add_blob(ss_ingest* g, const uint8_t* h_blob, const uint32_t* h_lens, uint64_t n);
int ss_ingest_add_fastq(ss_ingest* g, const char* path, uint64_t chunk_bytes, uint64_t* h_nseqs);
/* Multi-GPU FASTQ (counter.pyx:57-70 over one file, split across devices): ss_fastq_split cuts the
 * file into nparts byte ranges h_begin[p] .. h_begin[p + 1] (h_begin has nparts + 1 entries), each
 * starting at a line start and ending after a newline or at the end of the file, and gives the
 * lines before each range (h_line0[p]).  ss_ingest_add_fastq_range counts one range (line0 = the
 * lines before it, so the j % 4 == 1 selection of fast_read.pyx:13 stays global); the ranges'
 * results, taken in range order, are the file's counter (first-occurrence order kept: every read of
 * range p precedes every read of range p + 1).  Host calls.  A range longer than one chunk
 * (chunk_bytes; 0 = 1 GiB) is read by a reader thread into two pinned chunk slots: chunk k + 1's
 * file reads and H2D copies (their own stream) run while chunk k is indexed and counted.  The reader
 * runs on the GPU's NUMA node's CPUs within the process's affinity mask (SHORTSEQ_FQ_PIN=0: not
 * pinned), so its pinned slots and the bytes copied into them are node-local. */
int ss_fastq_split(const char* path, uint32_t nparts, uint64_t* h_begin, uint64_t* h_line0);
int ss_ingest_add_fastq_range(ss_ingest* g, const char* path, uint64_t begin, uint64_t end, uint64_t line0,
                              uint64_t chunk_bytes, uint64_t* h_nseqs);
/* A ragged batch already on this engine's device: read i = d_blob[d_offsets[i], + d_lens[i]) of an
 * nbytes-byte blob (e.g. the output of ss_fastq_index_onepass, or a device-generated batch); counted
 * as ss_ingest_add_blob counts a staged list (same length split, tables and first-occurrence order).
 * Synchronous; the caller's buffers are not kept. */
int ss_ingest_add_device(ss_ingest* g, const uint8_t* d_blob, uint64_t nbytes, const uint64_t* d_offsets,
                         const uint32_t* d_lens, uint64_t n);
int ss_ingest_error(ss_ingest* g, uint64_t* h_index, int* h_kind, uint8_t* h_read, uint64_t cap, uint64_t* h_len);
int ss_ingest_finish(ss_ingest* g, uint64_t* h_nkeys, uint64_t* h_nwords);
/* Stage split of the engine's FASTQ calls since the last call of this (new,
 * replaces nothing): h_ms[5] = host ms of the file reads (pread into pinned memory, in pieces whose
 * H2D copies overlap the next piece's read), device ms of those H2D copies (summed), host ms of the
 * device index to its sync (incl. the wait for its chunk's copies), host ms of the chunk counts,
 * host ms of ss_ingest_finish (reads and copies of a later chunk overlap the index and count of an
 * earlier one, so the stages of a multi-chunk range sum to more than its wall time); *h_h2d_bytes =
 * the bytes the H2D copies moved (their rate = the PCIe rate the call saw). */
int ss_ingest_fastq_stages(ss_ingest* g, double* h_ms, uint64_t* h_h2d_bytes);
int ss_ingest_results(ss_ingest* g, const uint32_t** h_lens, const uint64_t** h_counts, const uint64_t** h_words);
/* Compact results (new in this ABI version; replaces nothing -- the reference's dict holds Python
 * ints): with ss_ingest_set_results_format(g, 1) the finish writes lengths as u16 and counts as u32
 * (*h_count_bytes = 4) unless a count needs u64 (8); the words are as above.  About 15 % fewer bytes
 * over PCIe for ragged keys.  ss_ingest_results refuses the compact format and
 * ss_ingest_results_compact the plain one.  Format 2: compact with u64 counts always (a test hook). */
int ss_ingest_set_results_format(ss_ingest* g, int compact);
int ss_ingest_results_compact(ss_ingest* g, const uint16_t** h_lens, const void** h_counts, uint32_t* h_count_bytes,
                              const uint64_t** h_words);

/* Multi-device reduce of one call (ShortSeqCounter(list) / read_and_count_fastq sharded over several
 * engines, counter.pyx:10-70; north_star: "an RCCL reduce over xGMI only for the final histogram
 * merge").  Engines that counted contiguous shards of one input fold into the first shard's engine on
 * the devices, so every distinct key crosses PCIe once and the host builds the dict from one
 * first-occurrence-ordered row list (no per-shard dict merge).
 *   ss_ingest_export: extract every table of the engine on its own device (entries, counts, and each
 *                     entry's first read); *h_nkeys = its distinct keys.  Run it in the shard's own
 *                     thread after its adds (the shards' exports run concurrently).
 *   ss_ingest_merge:  fold an exported engine into dst: its entries cross to dst's device (peer copies
 *                     over xGMI, hipMemcpyPeerAsync; a device copy when both share a device), become
 *                     rows of dst's tables (short group, length 32, classes) appended as one block (first read =
 *                     src_base + the entry's own), counts add, first index = min.  Sources follow
 *                     dst's reads in input order (src_base = the reads before the source's shard,
 *                     increasing from call to call).  Then ss_ingest_finish(dst) orders the union.
 *                     The caller checks ss_ingest_error of every shard first (the first rejected read
 *                     in input order raises).  Synchronous.  A dst that received merges may itself be
 *                     merged into an engine before it (a reduction tree of adjacent shards: export it
 *                     again first; the merge marks dst un-exported).  Merges into distinct dst
 *                     engines may run concurrently from different host threads.  New in this ABI
 *                     version; the reference has one process-wide dict (counter.pyx:41-54). */
int ss_ingest_export(ss_ingest* g, uint64_t* h_nkeys);
int ss_ingest_merge(ss_ingest* dst, ss_ingest* src, uint64_t src_base);
/* Optional, before a destination's merges: size dst's tables and row maps once for the union of
 * the nsrc (exported) sources' entries, so the merges that follow do not grow a table -- re-inserting
 * every entry it holds -- one merge at a time.  Synchronous.  New in this ABI version. */
int ss_ingest_reserve_merge(ss_ingest* dst, ss_ingest* const* srcs, uint32_t nsrc);

/* ------------------------------------------------------------------------------------------------
 * Synthetic reads on the device (SURVEY §8(d) generator; identical to oracle/ss_oracle.c):
 * read i word w: r = splitmix64(seed + i*W + w) masked to its nts, byte j = "ACTG"[(r >> 2j) & 3].
 * Pool variant: read i is pool item splitmix64(pool_seed ^ (i * 0xD1B54A32D192ED03)) % U.
 * Zipf variant (SURVEY §8(d) C5 skew): read i is pool item rank = #{k : d_cdf[k] <= u63}, u63 =
 * splitmix64(pool_seed ^ (i * 0xD1B54A32D192ED03)) >> 1, for a device table d_cdf[U] of the Zipf
 * CDF scaled to 2^63 (d_cdf[k] = floor(2^63 * P(rank <= k)), d_cdf[U-1] = 2^63; built on the host by
 * shortseq_amd.batch.zipf_cdf).  Item 0 is the most frequent.
 * ---------------------------------------------------------------------------------------------- */
int ss_synth_reads(uint8_t* d_ascii, uint64_t seed, uint64_t i0, uint64_t n, uint32_t L,
                   uint64_t stride, void* stream);
int ss_synth_pool_reads(uint8_t* d_ascii, uint64_t seed, uint64_t pool_seed, uint64_t U,
                        uint64_t i0, uint64_t n, uint32_t L, uint64_t stride, void* stream);
int ss_synth_zipf_reads(uint8_t* d_ascii, uint64_t seed, uint64_t pool_seed, const uint64_t* d_cdf, uint64_t U,
                        uint64_t i0, uint64_t n, uint32_t L, uint64_t stride, void* stream);
/* Ragged pool reads (mixed lengths): read i draws pool item
 * p = splitmix64(pool_seed ^ i * 0xD1B54A32D192ED03) % U of length
 * Lmin + splitmix64(seed ^ 0x6A09E667F3BCC909 ^ p) % (Lmax - Lmin + 1), word w = splitmix64(seed + 32 p + w)
 * masked.  ss_synth_ragged_lens writes the n lengths; the caller lays the blob out (d_offsets, e.g.
 * an exclusive prefix sum of the lengths) and ss_synth_ragged_reads writes the ASCII there. */
int ss_synth_ragged_lens(uint32_t* d_lens, uint64_t seed, uint64_t pool_seed, uint64_t U, uint64_t i0, uint64_t n,
                         uint32_t Lmin, uint32_t Lmax, void* stream);
int ss_synth_ragged_reads(uint8_t* d_blob, const uint64_t* d_offsets, uint64_t seed, uint64_t pool_seed, uint64_t U,
                          uint64_t i0, uint64_t n, uint32_t Lmin, uint32_t Lmax, void* stream);

/* ------------------------------------------------------------------------------------------------
 * Host-resident batches (the host side stages read batches in pinned
 * memory).  Replaces, for a whole host array, the per-object marshal/unmarshal loops the Cython front
 * runs today (short_seq_64.pyx:96-121, util.pyx:78-140, short_seq_var.pyx:98-120).
 * A stager owns a ring of `nslots` (2..16) pinned + device chunk slots of `chunk_bytes` each and
 * three HIP streams (H2D, kernel, D2H); a call streams the batch through it chunk by chunk so the
 * copies and the kernel of neighbouring chunks overlap.  Host buffers may be pageable (staged by
 * `copy_threads` memcpy threads; 0 = the calling thread) or pinned (DMA'd directly, detected per
 * call).  Calls are synchronous (they return when the outputs are in host memory) and must not be
 * made concurrently on one stager.  *h_first_bad = first invalid read (input order) or UINT64_MAX;
 * the rc stays SS_OK for data errors, as for the device entry points.
 * ss_decode_host writes L bytes per read at h_ascii + i*stride; bytes L..stride of a row are
 * unspecified.  d_ref_words (encode_hamming) is a device pointer, ready before the call.
 * ---------------------------------------------------------------------------------------------- */
typedef struct ss_stager ss_stager;
int ss_stager_create(int device, uint64_t chunk_bytes, uint32_t nslots, uint32_t copy_threads,
                     ss_stager** h_out);
int ss_stager_destroy(ss_stager* st);
/* Stage split and placement of a stager (new, replaces nothing).  With timing on,
 * every call records event pairs per chunk.  ss_stager_stats returns, per call since its last call
 * (timed calls), h_ms[6] = host ms of the pageable -> pinned copies, host ms of the pinned ->
 * pageable copies, device ms of the H2D copies, the kernels and the D2H copies (sums over chunks:
 * they overlap across chunks), host ms waiting on the D2H events; and h_info[4] = copy threads, CPUs
 * in the process's affinity mask, the GPU's NUMA node (-1 unknown), CPUs the copy threads are pinned
 * to (the node's CPUs within the mask; 0 = not pinned, also with SHORTSEQ_STAGE_PIN=0). */
int ss_stager_set_timing(ss_stager* st, int on);
int ss_stager_stats(ss_stager* st, double* h_ms, int32_t* h_info);
int ss_encode_host(ss_stager* st, const uint8_t* h_ascii, uint64_t n, uint32_t L, uint64_t stride,
                   uint64_t* h_words, uint32_t wpr, uint64_t* h_first_bad);
int ss_encode_hamming_ref_host(ss_stager* st, const uint8_t* h_ascii, uint64_t n, uint32_t L, uint64_t stride,
                               uint64_t* h_words, uint32_t wpr, const uint64_t* d_ref_words, uint32_t* h_out,
                               uint64_t* h_first_bad);
int ss_decode_host(ss_stager* st, const uint64_t* h_words, uint64_t n, uint32_t L, uint32_t wpr,
                   uint8_t* h_ascii, uint64_t stride);

/* ------------------------------------------------------------------------------------------------
 * Host codec (per-object path, no GPU): the drop-in Python objects use these for single reads,
 * where a kernel launch (~µs) would cost more than the work (SURVEY §7 hard parts).
 * ---------------------------------------------------------------------------------------------- */
int ss_host_encode(const uint8_t* h_seq, uint64_t L, uint64_t* h_words, ss_err* h_err);
void ss_host_decode(const uint64_t* h_words, uint64_t L, char* h_out);
uint64_t ss_host_hamming(const uint64_t* h_a, const uint64_t* h_b, uint64_t L);

#ifdef __cplusplus
}
#endif
#endif /* SHORTSEQ_AMD_H */
