// ss_internal.h — shared host-side helpers for the C ABI implementation (not installed).
#pragma once
#include <hip/hip_runtime.h>
#include "../../include/shortseq_amd.h"

#include <vector>

// The CPUs of `device`'s NUMA node (sysfs, by PCI bus id) that this process's affinity mask allows;
// *node = that node (-1: unknown), *allowed = the mask's CPU count.  Empty when the node is unknown
// or the intersection is empty (ss_stage.hip: the stager's copy threads, the FASTQ reader ring).
std::vector<int> ss_gpu_numa_cpus(int device, int* node, int* allowed);
// Record `msg` as the thread's last error and return `code`.
int ss_fail(int code, const char* msg);
// SS_OK if e == hipSuccess, otherwise record "<what>: <hip error string>" and return SS_EHIP.
int ss_check(hipError_t e, const char* what);
// Launch-side entry shared by ss_encode_fixed / ss_encode_hamming_ref.
extern "C" int ss_encode_fixed_impl(const uint8_t* d_ascii, uint64_t n, uint32_t L, uint64_t stride,
                                    uint64_t* d_words, uint32_t wpr, uint64_t* d_first_bad,
                                    const uint64_t* d_ref_words, uint32_t* d_out, void* stream);
// All multi-word classes of a chunk in one read-order pass (k_encode_classes; every class present has
// W + 1 <= w1max <= 16 words), over k_len_count's nblk block ranges: class W's rows at d_out + h_woff[W]
// (W = 2..32; the block's first row of class W = d_blkoff[(bin0 + W) * nblk + block], k_len_binscan's
// in-bin offsets; rows in read order), each row's fingerprint (words_fp over its W + 1 words) at
// d_fps[h_fpoff[W] + row] when d_fps is given, its global read index (base + chunk read) at
// h_rmap[W][row] when h_rmap[W] is given, and the classes' HyperLogLog registers d_hll[W << kHllLog
// ...] (u32, max-updated; zeroed by the caller).
constexpr uint32_t kHllLog = 11;
// ss_counter_reset in two halves: the host state now, its three device words (p[0..2] = v[0..2])
// queued later, several tables' words in one ss_prep_words dispatch (n <= kPrepMany), before any use
// of the tables on that stream
constexpr uint32_t kPrepMany = 32;
extern "C" int ss_counter_reset_host(ss_counter* c, unsigned long long** p, unsigned long long* v);
extern "C" int ss_prep_words(unsigned long long* const* p, const unsigned long long* v, uint32_t n, void* stream);
extern "C" int ss_encode_classes_impl(const uint8_t* d_buf, const uint64_t* d_offs, const uint32_t* d_lens, uint64_t n,
                                      const uint32_t* d_blkoff, uint32_t nblk, const uint64_t* h_woff,
                                      const uint64_t* h_fpoff, uint64_t* const* h_rmap, uint64_t base, uint32_t bin0,
                                      uint32_t w1max, uint64_t* d_out, uint64_t* d_fps, uint32_t* d_hll,
                                      uint64_t* d_first_bad, void* stream);
// A chunk of class reads of at most S - 1 words (3 <= S <= 6; k_encode_rows): read r's row at
// d_out + r * S (its W words, its length, zeros), its fingerprint (words_fp over W + 1 words) at
// d_fps[r], its class's HyperLogLog registers updated; a read that is not a class read (empty) gets a
// zero row and words_fp of one zero word.  *d_first_bad (not reset) = min read with a rejected byte.
// d_gate (or null): the kernel does nothing unless *d_gate == S when it runs (an encode queued before
// the host has seen the length split).
extern "C" int ss_encode_rows_impl(const uint8_t* d_buf, const uint64_t* d_offs, const uint32_t* d_lens, uint64_t n,
                                   uint32_t S, uint64_t* d_out, uint64_t* d_fps, uint32_t* d_hll,
                                   uint64_t* d_first_bad, void* stream, const uint64_t* d_gate = nullptr);
// The drop-in engine's short reads (1..31 nt) as keys of one table: d_keys[i] = the packed word of
// read d_sel[i] (d_sel null: read i) | 1 << (2L + 1), the length marker above the word and its
// table-path carry bit (k_short_keys, ss_codec.hip); dense_L > 0: reads back to back of that length.
// *d_first_bad (not reset) = min chunk read index with a rejected byte.
extern "C" int ss_short_keys_impl(const uint8_t* d_buf, const uint64_t* d_offs, const uint32_t* d_lens,
                                  const uint64_t* d_sel, uint64_t m, uint32_t dense_L, uint64_t* d_keys,
                                  uint64_t* d_first_bad, void* stream);
// Single-word keys already computed on the device (d_keys[n], any 64-bit values): counted with the
// optimistic partitioned insert (12-B records, LDS aggregation) -- e.g. the class rows' fingerprints.
extern "C" int ss_counter_insert_keys(ss_counter* c, const uint64_t* d_keys, uint64_t n, uint64_t base_index,
                                      void* stream);
// One length class of the drop-in engine's chunk for ss_classes_verify_fold: its table (set_words(W1)),
// its m packed rows of W1 words, and the table's first row index for them.
struct ss_class_rows {
    ss_counter* table;
    const uint64_t* rows;
    uint64_t m;
    uint64_t base;
    uint32_t W1;
};
// After ss_counter_insert_keys(fpt, d_fps, sum of m, 0) over the classes' fingerprints (class after
// class, in cls order): every row compared with its fingerprint's first row (a mismatch -- two keys
// sharing a fingerprint -- sets *d_flag, zeroed by the caller) and, unless *d_flag, every fpt entry
// folded into its class's table (count, first = base + row).  With *d_flag set the class tables are
// untouched and the caller counts the classes on the exact multi-word path instead.
extern "C" int ss_classes_verify_fold(ss_counter* fpt, const uint64_t* d_fps, const ss_class_rows* cls, uint32_t ncls,
                                      uint32_t* d_flag, void* stream);
// The same for read-order rows (ss_encode_rows_impl, stride S <= 6, fingerprints d_fps[n], after
// ss_counter_insert_keys(fpt, d_fps, n, 0)): cls[W] (W = 2 .. S - 1; null table: no reads of class W)
// holds class W's table, its first free row (base) and its row map at that row (rmap).  Each new key
// of class W takes the next row (base + the new keys before it: at most the class's reads) and
// rmap[row] = base + its first read; the zero rows of reads that are no class reads are skipped.
struct ss_flat_class {
    ss_counter* table;
    uint64_t base;
    uint64_t* rmap;
};
extern "C" int ss_classes_flat_verify_fold(ss_counter* fpt, const uint64_t* d_rows, uint32_t S, uint64_t n,
                                           const uint64_t* d_fps, const ss_flat_class* cls, uint64_t base,
                                           uint32_t* d_flag, void* stream);
// The same in two steps, so the fold can be deferred: ss_classes_flat_verify (representatives +
// verify: sets *d_flag on a difference; ev_reps, when given, is recorded between the two) then ss_classes_flat_fold (into the class tables; a no-op when
// *d_flag).  The scratch (fpt and its representatives) must be left untouched in between.
extern "C" int ss_classes_flat_verify(ss_counter* fpt, const uint64_t* d_rows, uint32_t S, uint64_t n,
                                      const uint64_t* d_fps, uint32_t* d_flag, void* stream, void* ev_reps);
extern "C" int ss_classes_flat_fold(ss_counter* fpt, uint32_t S, const ss_flat_class* cls, uint64_t base,
                                    const uint32_t* d_flag, void* stream);
// Instead of a fold into class tables that hold no earlier rows (cls[W].base == 0): the scratch's
// entries as dense per-class arrays in the rows the fold would give them -- words [m][W + 1] (the
// class table's key words), counts, first = row -- with cls[W].rmap[row] written as the fold writes
// it, and the entry count into *total (u64).  The finish then orders them like extracted entries; a
// later ss_classes_flat_fold of the same scratch gives the same rows.  d_zero: a device u32 holding 0.
struct ss_flat_out {
    uint64_t* words;
    uint64_t* counts;
    uint64_t* first;
    uint64_t* total;
    uint64_t* ovf;        // set nonzero when the class has more than cap entries (those are dropped)
    uint64_t cap;
};
extern "C" int ss_classes_flat_extract(ss_counter* fpt, uint32_t S, const ss_flat_class* cls, uint64_t base,
                                       const ss_flat_out* out, const uint32_t* d_zero, void* stream);
// Every entry's count moved into d_acc[first] (u64, indexed by the entry's first index: the drop-in
// engine's rows) and the slot's count zeroed (the single-word sentinel keeps 1), so later inserts
// cannot wrap a slot's u32 count (k_spill_counts).
extern "C" int ss_counter_spill_counts(ss_counter* c, uint64_t* d_acc, void* stream);
// HyperLogLog registers (2^kHllLog u32 at d_hll) of m packed rows of W1 words, k_encode_classes' hash.
extern "C" int ss_hll_rows_impl(const uint64_t* d_rows, uint64_t m, uint32_t W1, uint32_t* d_hll, void* stream);
// Drop-in engine (ss_ingest), one multi-word length class: rows of W words + the length (k_encode_class).
// Row i = read d_sel[i] of the chunk (d_buf + d_offs[r], d_lens[r] bytes), or read i at i * dense_L
// when d_sel is null.  *d_first_bad (not reset here) = min chunk read index with a rejected byte.
extern "C" int ss_encode_class_impl(const uint8_t* d_buf, const uint64_t* d_offs, const uint32_t* d_lens,
                                    const uint64_t* d_sel, uint32_t dense_L, uint64_t m, uint32_t W,
                                    uint64_t* d_out, uint64_t* d_first_bad, void* stream);
