/*
 * oracle/ref_harness.c — TEST INFRASTRUCTURE ONLY (bench.py cpu_baseline leg + oracle validation).
 *
 * Drives the reference's OWN compiled kernels (built by oracle/build_ref.sh into oracle/_ref/) over a
 * contiguous batch, the way SURVEY §6 timed them.  The kernels are the Cython cdef functions the
 * reference exports through its modules' __pyx_capi__ PyCapsules:
 *   shortseq.short_seq_64._marshall_bytes_64   "uint64_t (uint8_t *, uint8_t)"   short_seq_64.pyx:96
 *   shortseq.util._marshall_bytes_array         "void (uint64_t *, uint8_t *, size_t)" util.pyx:78
 * The caller passes the raw function pointer (PyCapsule_GetPointer).  Inputs must be valid bases:
 * the reference raises a Python exception (GIL re-acquired) on a bad byte, which this loop does not
 * check for.
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>

typedef uint64_t (*ref_m64_fn)(uint8_t*, uint8_t);
typedef void (*ref_marr_fn)(uint64_t*, uint8_t*, size_t);

/* short_seq.pyx:57-61: ShortSeq64 path, one call per read. */
void ref_encode64_batch(void* fn, const uint8_t* ascii, uint64_t n, uint32_t L, uint64_t stride,
                        uint64_t* out) {
    ref_m64_fn f = (ref_m64_fn)fn;
    for (uint64_t i = 0; i < n; ++i) out[i] = f((uint8_t*)ascii + i * stride, (uint8_t)L);
}

/* short_seq.pyx:63-72: ShortSeq192 / Var path (both call _marshall_bytes_array into zeroed words). */
void ref_encode_array_batch(void* fn, const uint8_t* ascii, uint64_t n, uint32_t L, uint64_t stride,
                            uint64_t* out, uint32_t wpr) {
    ref_marr_fn f = (ref_marr_fn)fn;
    for (uint64_t i = 0; i < n; ++i) {
        uint64_t* o = out + i * wpr;
        memset(o, 0, (size_t)wpr * 8);
        f(o, (uint8_t*)ascii + i * stride, L);
    }
}
