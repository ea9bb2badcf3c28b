// tools/diag_alloc.hip — why the same encode kernel is ~4% slower inside bench.py than in the tuner:
// allocation size (TLB fragments) vs the per-call first_bad memset node.
#include "../shortseq_amd/csrc/ss_codec.hip"
#include "../shortseq_amd/csrc/ss_runtime.hip"
#include <stdio.h>
#include <functional>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static void timeit(const char* name, double bytes, int reps, const std::function<void()>& f) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int i = 0; i < 5; ++i) f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; ++r) f();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-60s %8.4f ms/launch  %7.1f GB/s\n", name, ms / reps, bytes / (ms / reps) / 1e6);
    fflush(stdout);
}

int main() {
    const uint64_t n = 100000000; const uint32_t L = 32;
    const double bytes = n * 40.0;
    uint64_t* fb; CK(hipMalloc(&fb, 8)); CK(hipMemset(fb, 0xFF, 8));
    uint8_t* big; CK(hipMalloc(&big, 26ull << 30));
    uint64_t* bigw; CK(hipMalloc(&bigw, 7ull << 30));
    uint8_t* ex; CK(hipMalloc(&ex, n * L));
    uint64_t* exw; CK(hipMalloc(&exw, n * 8));
    for (int round = 0; round < 2; ++round) {
        for (int which = 0; which < 2; ++which) {
            uint8_t* in = which ? ex : big;
            uint64_t* w = which ? exw : bigw;
            if (ss_synth_reads(in, 1, 0, n, L, L, nullptr)) return 1;
            const char* tag = which ? "exact-size allocs" : "26 GB / 7 GB allocs";
            char name[128];
            snprintf(name, sizeof name, "%s: kernel only", tag);
            timeit(name, bytes, 40, [&] {
                G16Args a; a.in = (const uint4*)in; a.in_stride16 = 2; a.out32 = (uint32_t*)w; a.wpr2 = 2; a.n = n;
                a.cpr = 2; a.full2 = 2; a.all_table = 1; a.logG = 1; a.ref32 = nullptr; a.ham2 = 2; a.counts = nullptr;
                a.first_bad = (unsigned long long*)fb;
                launch_g16<false, true, kPathTable, 768, 2, false, true>(a, 0);
            });
            snprintf(name, sizeof name, "%s: ss_encode_fixed (memset + kernel)", tag);
            timeit(name, bytes, 40, [&] { ss_encode_fixed(in, n, L, L, w, 1, fb, nullptr); });
        }
    }
    return 0;
}
