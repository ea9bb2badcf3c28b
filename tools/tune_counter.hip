// tools/tune_counter.hip — time the production partitioned counter insert (C5: 125M x 32 nt from a
// pool of 2^24, table 2^25) built with compile-time knobs, e.g.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include tools/tune_counter.hip \
//         shortseq_amd/csrc/ss_codec.hip shortseq_amd/csrc/ss_runtime.hip -o tools/tune_counter_4096
// prints ms per insert (table reset excluded) and checks the total count and the unique count.

#include "../shortseq_amd/csrc/ss_counter.hip"


#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <vector>
#include <unordered_map>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
#define CS(x) do { int r_ = (x); if (r_) { printf("ss error %d: %s @%d\n", r_, ss_last_error_string(), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
    // tune_counter [n=125M] [reps=10] [U_log2=24] [zipf_s=0 (uniform)]
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 125000000ull;
    const int reps = argc > 2 ? atoi(argv[2]) : 10;
    const int ulog = argc > 3 ? atoi(argv[3]) : 24;
    const double zs = argc > 4 ? atof(argv[4]) : 0.0;
    const uint64_t U = 1ull << ulog;
    const uint32_t L = 32;
    uint8_t* ascii;
    uint64_t *fb, *size;
    CK(hipMalloc(&ascii, n * L));
    CK(hipMalloc(&fb, 8));
    CK(hipMalloc(&size, 8));
    if (zs > 0) {   // the table of shortseq_amd.batch.zipf_cdf
        uint64_t* h = (uint64_t*)malloc(U * 8);
        double* c = (double*)malloc(U * 8);
        double acc = 0;
        for (uint64_t k = 0; k < U; ++k) c[k] = (acc += pow((double)(k + 1), -zs));
        for (uint64_t k = 0; k < U; ++k) h[k] = (uint64_t)floor(c[k] / acc * 9223372036854775808.0);
        h[U - 1] = 1ull << 63;
        uint64_t* d;
        CK(hipMalloc(&d, U * 8));
        CK(hipMemcpy(d, h, U * 8, hipMemcpyHostToDevice));
        CS(ss_synth_zipf_reads(ascii, 5, 77, d, U, 0, n, L, L, nullptr));
        CK(hipDeviceSynchronize());
        CK(hipFree(d));
        free(h);
        free(c);
    } else {
        CS(ss_synth_pool_reads(ascii, 5, 77, U, 0, n, L, L, nullptr));
    }
    ss_counter* c;
    CS(ss_counter_create(2 * U, &c));
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
    uint32_t hspill = 0;
    CK(hipMemcpy(&hspill, c->ws_fill + fill_at(kSpillCtr), 4, hipMemcpyDeviceToHost));
    if (getenv("SS_DIAG") && c->ws_slab && hspill) {   // where do the spills come from
        const uint32_t nb = (uint32_t)((c->cap >> c->slice_log) >> kCoarseBits);
        std::vector<uint32_t> sl(2 * kNFill), hist((size_t)kNFill * nb), se((size_t)kNFill * nb), fl(kFillWords);
        CK(hipMemcpy(sl.data(), c->ws_order + kNFill, sl.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hist.data(), c->ws_hist, hist.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(se.data(), c->ws_segend, se.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(fl.data(), c->ws_fill, fl.size() * 4, hipMemcpyDeviceToHost));
        uint64_t full = 0, fullfb = 0;
        for (uint32_t f = 0; f < kNFill; ++f) {
            uint32_t nf = 0;
            for (uint32_t i = 0; i < nb; ++i) nf += se[(size_t)f * nb + i] - hist[(size_t)f * nb + i] >= sl[kNFill + f];
            full += nf;
            fullfb += nf > 0;
            if (nf && fullfb <= 6) printf("  fb %u fill %u slab %u full regions %u\n", f, fl[fill_at(f)], sl[kNFill + f], nf);
        }
        std::vector<uint4> sp(std::min<uint64_t>(hspill, c->ws_reads));
        CK(hipMemcpy(sp.data(), c->ws_spill, sp.size() * 16, hipMemcpyDeviceToHost));
        std::unordered_map<uint64_t, uint64_t> kc;
        uint64_t weighted = 0;
        for (auto& r : sp) { kc[((uint64_t)r.y << 32) | r.x] += 1; weighted += r.z > 1; }
        uint64_t mx = 0;
        for (auto& e : kc) mx = std::max(mx, e.second);
        printf("  full slabs %llu in %llu sub-bins; spill records %zu distinct keys %zu weighted %llu max per key %llu\n",
               (unsigned long long)full, (unsigned long long)fullfb, sp.size(), kc.size(), (unsigned long long)weighted,
               (unsigned long long)mx);
    }
    printf("U=2^%d zipf=%.2f: insert avg %.3f ms min %.3f ms  (%.1f G reads/s)  unique %llu first_bad %llx  spill %u\n", ulog, zs,
           tot / reps, mn, n / (tot / reps) / 1e6, (unsigned long long)hs, (unsigned long long)hfb, hspill);
    return 0;
}
