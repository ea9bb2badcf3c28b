// tools/tune_counter.hip — time the production partitioned counter insert (C5: 125M x 32 nt from a
// pool of 2^24, table 2^25) built with compile-time knobs, e.g.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include -DSS_PC_TILE=4096 tools/tune_counter.hip \
//         shortseq_amd/csrc/ss_codec.hip shortseq_amd/csrc/ss_runtime.hip -o tools/tune_counter_4096
// prints ms per insert (table reset excluded) and checks the total count and the unique count.

#include "../shortseq_amd/csrc/ss_counter.hip"


#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
#define CS(x) do { int r_ = (x); if (r_) { printf("ss error %d: %s @%d\n", r_, ss_last_error_string(), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 125000000ull;
    const int reps = argc > 2 ? atoi(argv[2]) : 10;
    const uint32_t L = 32;
    uint8_t* ascii;
    uint64_t *fb, *size;
    CK(hipMalloc(&ascii, n * L));
    CK(hipMalloc(&fb, 8));
    CK(hipMalloc(&size, 8));
    CS(ss_synth_pool_reads(ascii, 5, 77, 1ull << 24, 0, n, L, L, nullptr));
    ss_counter* c;
    CS(ss_counter_create(1ull << 25, &c));
    CS(ss_counter_reserve(c, n));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    double tot = 0, mn = 1e9;
    for (int r = -3; r < reps; ++r) {
        CS(ss_counter_reset(c, nullptr));
        CK(hipEventRecord(e0, 0));
        CS(ss_counter_insert_fixed(c, ascii, n, L, L, 0, fb, nullptr));
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 0) {
            tot += ms;
            mn = ms < mn ? ms : mn;
        }
    }
    CS(ss_counter_size(c, size, nullptr));
    uint64_t hs, hfb;
    CK(hipMemcpy(&hs, size, 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&hfb, fb, 8, hipMemcpyDeviceToHost));
    printf("tile %d: insert avg %.3f ms min %.3f ms  (%.1f G reads/s)  unique %llu first_bad %llx\n", (int)SS_PC_TILE,
           tot / reps, mn, n / (tot / reps) / 1e6, (unsigned long long)hs, (unsigned long long)hfb);
    return 0;
}
