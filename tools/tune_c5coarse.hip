// tools/tune_c5coarse.hip — where the C5 coarse pass's time goes (VERDICT r5 item 1 follow-up):
// the production kernel k_pf_coarse<512, 8, false, true> on the C5 batch (125M x 32-nt reads drawn
// from a 2^24 pool), timed alone (fill counters reset before each launch, HIP events, median).  It is
// compiled against a copy of ss_counter.hip named by SS_COUNTER_SRC, so scripts/build_c5coarse.sh
// can make diagnostic variants of the kernel (its record stores cut out, its loads served from a
// 4-MB window, both) whose output is wrong on purpose -- nothing runs after the coarse pass here.
//   scripts/build_c5coarse.sh  ->  tools/tune_c5coarse_{prod,nost,l2ld,both}
#include SS_COUNTER_SRC

#include <algorithm>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
#define CS(x) do { int r_ = (x); if (r_) { printf("ss error %d: %s @%d\n", r_, ss_last_error_string(), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
    const uint64_t n = 125000000ull, U = 1ull << 24;
    const int reps = argc > 1 ? atoi(argv[1]) : 15;
    uint8_t* ascii;
    uint64_t* fb;
    CK(hipMalloc(&ascii, n * 32));
    CK(hipMalloc(&fb, 16));
    CS(ss_synth_pool_reads(ascii, 5, 77, U, 0, n, 32, 32, nullptr));
    ss_counter* c;
    CS(ss_counter_create(2 * U, &c));
    CS(ss_counter_reserve(c, n));
    CS(ss_counter_set_length(c, 32));
    Tbl t = tbl_of(c);
    PartWs w{};
    w.akey = c->ws_akey;
    w.acnt = c->ws_acnt;
    w.areg = c->ws_areg;
    w.spill = c->ws_spill;
    w.spill_cap = c->ws_reads;
    w.R = (uint32_t)(c->cap >> c->slice_log);
    w.rbits = c->log2cap - c->slice_log;
    w.slab = (uint32_t)c->ws_slab;
    w.spill_ctr = c->ws_fill + fill_at(kSpillCtr);
    int dev = 0, cus = 0, per = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)k_pf_coarse<kPfT, kPfRPL, false, true>, kPfT, 0));
    const int grid = cus * per;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> ts;
    for (int r = -3; r < reps; ++r) {
        CK(hipMemsetAsync(c->ws_fill, 0, kFillWords * sizeof(uint32_t), 0));
        CK(hipMemsetAsync(fb, 0xFF, 8, 0));
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL((k_pf_coarse<kPfT, kPfRPL, false, true>), dim3(grid), dim3(kPfT), 0, 0, t, w,
                           (const uint4*)ascii, (uint64_t)2, n, 2u, c->ws_cap1, c->ws_fill, (unsigned long long*)fb);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 0) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    printf("coarse %s: median %.3f ms (min %.3f), grid %d (%d per CU)\n", SS_VARIANT, ts[ts.size() / 2], ts[0], grid, per);
    return 0;
}
