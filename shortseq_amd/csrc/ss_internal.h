// ss_internal.h — shared host-side helpers for the C ABI implementation (not installed).
#pragma once
#include <hip/hip_runtime.h>
#include "../../include/shortseq_amd.h"

// Record `msg` as the thread's last error and return `code`.
int ss_fail(int code, const char* msg);
// SS_OK if e == hipSuccess, otherwise record "<what>: <hip error string>" and return SS_EHIP.
int ss_check(hipError_t e, const char* what);
// Launch-side entry shared by ss_encode_fixed / ss_encode_hamming_ref.
extern "C" int ss_encode_fixed_impl(const uint8_t* d_ascii, uint64_t n, uint32_t L, uint64_t stride,
                                    uint64_t* d_words, uint32_t wpr, uint64_t* d_first_bad,
                                    const uint64_t* d_ref_words, uint32_t* d_out, void* stream);
// Drop-in engine (ss_ingest), one multi-word length class: rows of W words + the length (k_encode_class).
// Row i = read d_sel[i] of the chunk (d_buf + d_offs[r], d_lens[r] bytes), or read i at i * dense_L
// when d_sel is null.  *d_first_bad (not reset here) = min chunk read index with a rejected byte.
extern "C" int ss_encode_class_impl(const uint8_t* d_buf, const uint64_t* d_offs, const uint32_t* d_lens,
                                    const uint64_t* d_sel, uint32_t dense_L, uint64_t m, uint32_t W,
                                    uint64_t* d_out, uint64_t* d_first_bad, void* stream);
