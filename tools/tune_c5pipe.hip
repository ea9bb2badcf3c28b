// tools/tune_c5pipe.hip — experiment: do the C5 partition passes of two halves of the shard overlap
// when issued on two streams (coarse of half 1 beside the fine scatter of half 0)?
//
//   full : coarse + order + fine over all n reads (one workspace), one stream
//   seq  : coarse(h0) order(h0) fine(h0) coarse(h1) order(h1) fine(h1), one stream
//   pipe : s0: coarse(h0) -> order(h0) fine(h0) ; s1: [after coarse(h0)] coarse(h1) -> [after fine(h0)]
//          order(h1) fine(h1)
// The aggregate is left out (it runs once over both halves' fine records either way).
//
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include tools/tune_c5pipe.hip \
//          shortseq_amd/csrc/ss_codec.hip shortseq_amd/csrc/ss_runtime.hip -o tools/tune_c5pipe
#include "../shortseq_amd/csrc/ss_counter.hip"

#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
#define CS(x) do { int r_ = (x); if (r_) { printf("ss error %d: %s @%d\n", r_, ss_last_error_string(), __LINE__); exit(1); } } while (0)

namespace {
PartWs ws_of(ss_counter* c) {
    PartWs w{};
    w.keys = c->ws_keys; w.akey = c->ws_akey; w.aidx = c->ws_aidx; w.acnt = c->ws_acnt; w.areg = c->ws_areg;
    w.bidx = c->ws_bidx; w.bcnt = c->ws_bcnt; w.spill = c->ws_spill; w.spill_cap = c->ws_reads;
    w.hist = c->ws_hist; w.rstart = c->ws_rstart; w.tot = c->ws_tot;
    w.R = (uint32_t)(c->cap >> c->slice_log); w.rbits = c->log2cap - c->slice_log;
    w.slab = 1; w.spill_ctr = c->ws_fill + fill_at(kSpillCtr);
    w.seg_end = c->ws_segend;
    w.slabs = c->ws_order + kNFill;
    return w;
}

int g_grid = 0;
int g_mul = 1;

void coarse(ss_counter* c, const uint8_t* ascii, uint64_t n, uint64_t* fb, hipStream_t s) {
    Tbl t = tbl_of(c);
    PartWs w = ws_of(c);
    CK(hipMemsetAsync(c->ws_fill, 0, kFillWords * sizeof(uint32_t), s));
    hipLaunchKernelGGL((k_pf_coarse<kPfT, kPfRPL, false, false>), dim3(g_grid * g_mul), dim3(kPfT), 0, s, t, w, (const uint4*)ascii,
                       (uint64_t)2, n, 2u, c->ws_cap1, c->ws_fill, (unsigned long long*)fb);
}

void fine(ss_counter* c, hipStream_t s) {
    Tbl t = tbl_of(c);
    PartWs w = ws_of(c);
    hipLaunchKernelGGL(k_pf_order, dim3(1), dim3(512), 0, s, (const uint32_t*)c->ws_fill, c->ws_cap1, c->ws_order,
                       1u << (w.rbits - kCoarseBits), c->ws_order + kNFill);
    hipLaunchKernelGGL((k_pf_scatter<kFsT, kFsTile>), dim3(kNFill), dim3(kFsT), 0, s, t, w, c->ws_cap1,
                       (const uint32_t*)c->ws_fill, (const uint32_t*)c->ws_order);
}
}  // namespace

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 125000000ull;
    const int reps = argc > 2 ? atoi(argv[2]) : 10;
    const uint64_t U = 1ull << 24, h = n / 2;
    uint8_t* ascii;
    uint64_t* fb;
    CK(hipMalloc(&ascii, n * 32));
    CK(hipMalloc(&fb, 16));
    CS(ss_synth_pool_reads(ascii, 5, 77, U, 0, n, 32, 32, nullptr));
    ss_counter *cf, *c0, *c1;
    CS(ss_counter_create(2 * U, &cf));
    CS(ss_counter_create(2 * U, &c0));
    CS(ss_counter_create(2 * U, &c1));
    CS(ss_counter_reserve(cf, n));
    CS(ss_counter_reserve(c0, h));
    CS(ss_counter_reserve(c1, n - h));
    int dev = 0, cus = 0, per = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)k_pf_coarse<kPfT, kPfRPL, false, false>, kPfT, 0));
    g_grid = cus * per;
    hipStream_t s0, s1;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    hipEvent_t t0, t1, ec0, ef0, ee1;
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    CK(hipEventCreateWithFlags(&ec0, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&ef0, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&ee1, hipEventDisableTiming));
    const char* names[6] = {"full", "seq", "pipe", "pipe2", "fullx2", "fullx3"};
    for (int mode = 0; mode < 6; ++mode) {
        g_mul = mode == 4 ? 2 : mode == 5 ? 3 : 1;
        double tot = 0;
        for (int r = -3; r < reps; ++r) {
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(t0, s0));
            if (mode == 0 || mode >= 4) {
                coarse(cf, ascii, n, fb, s0);
                fine(cf, s0);
            } else if (mode == 1) {
                coarse(c0, ascii, h, fb, s0);
                fine(c0, s0);
                coarse(c1, ascii + h * 32, n - h, fb + 1, s0);
                fine(c1, s0);
            } else if (mode == 2) {
                coarse(c0, ascii, h, fb, s0);
                CK(hipEventRecord(ec0, s0));
                fine(c0, s0);
                CK(hipEventRecord(ef0, s0));
                CK(hipStreamWaitEvent(s1, ec0, 0));
                coarse(c1, ascii + h * 32, n - h, fb + 1, s1);
                CK(hipStreamWaitEvent(s1, ef0, 0));
                fine(c1, s1);
                CK(hipEventRecord(ee1, s1));
                CK(hipStreamWaitEvent(s0, ee1, 0));
            } else {   // both coarse passes at once, then both fine passes at once
                CK(hipEventRecord(ec0, s0));
                CK(hipStreamWaitEvent(s1, ec0, 0));
                coarse(c0, ascii, h, fb, s0);
                coarse(c1, ascii + h * 32, n - h, fb + 1, s1);
                fine(c0, s0);
                fine(c1, s1);
                CK(hipEventRecord(ee1, s1));
                CK(hipStreamWaitEvent(s0, ee1, 0));
            }
            CK(hipEventRecord(t1, s0));
            CK(hipEventSynchronize(t1));
            float ms;
            CK(hipEventElapsedTime(&ms, t0, t1));
            if (r >= 0) tot += ms;
        }
        printf("%-5s coarse+order+fine over %llu reads: %.3f ms\n", names[mode], (unsigned long long)n, tot / reps);
        fflush(stdout);
    }
    return 0;
}
