// tools/tune_allpairs.hip — MFMA all-pairs variants (row blocks per wave RB, table vs arithmetic
// one-hot build) on the production kernel template; checks hits/counts against the production
// launch.  hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include tools/tune_allpairs.hip \
//   shortseq_amd/csrc/ss_codec.hip shortseq_amd/csrc/ss_runtime.hip -o tools/tune_allpairs
#include "../shortseq_amd/csrc/ss_allpairs.hip"
#include <stdio.h>
#include <stdlib.h>
#include <functional>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int KS, int RB, bool TAB>
double run(AllPairsArgs a, uint32_t P, int reps, unsigned long long* hits) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 2; ++i) {
        CK(hipMemset(a.npairs, 0, 8));
        launch_allpairs_mfma<KS, RB, TAB>(a, P, 0);
    }
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) launch_allpairs_mfma<KS, RB, TAB>(a, P, 0);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipMemset(a.npairs, 0, 8));
    launch_allpairs_mfma<KS, RB, TAB>(a, P, 0);
    CK(hipMemcpy(hits, a.npairs, 8, hipMemcpyDeviceToHost));
    return ms / reps;
}

int main() {
    for (int cfg = 0; cfg < 2; ++cfg) {
        const uint64_t n = cfg == 0 ? 200000 : 50000;
        const uint32_t L = cfg == 0 ? 12 : 32, k = cfg == 0 ? 1 : 6;
        uint64_t* w;
        CK(hipMalloc(&w, n * 8));
        uint64_t* hw = (uint64_t*)malloc(n * 8);
        uint64_t x = 12345;
        for (uint64_t i = 0; i < n; ++i) {
            x = x * 6364136223846793005ull + 1442695040888963407ull;
            uint64_t v = x ^ (x >> 29);
            if (i % 3 == 1) v = hw[i - 1] ^ (1ull << (2 * (i % L)));   // near neighbours
            hw[i] = L < 32 ? v & ((1ull << (2 * L)) - 1) : v;
        }
        CK(hipMemcpy(w, hw, n * 8, hipMemcpyHostToDevice));
        AllPairsArgs a;
        a.words = w; a.n = n; a.wpr = 1; a.W = 1; a.k = k; a.ntiles = 0; a.counts = nullptr; a.pairs = nullptr;
        a.max_pairs = 0;
        CK(hipMalloc(&a.npairs, 8));
        const uint32_t P = L + 1 < 32 ? L + 1 : 32;
        const double pairs = (double)n * (n - 1) / 2;
        unsigned long long hits;
        double ms;
#define V(KS, RB, TAB) ms = run<KS, RB, TAB>(a, P, 10, &hits); \
        printf("L %2u n %6llu KS %d RB %d TAB %d: %.3f ms  %.2f T pairs/s  hits %llu\n", L, (unsigned long long)n, KS, RB, (int)TAB, ms, pairs / ms / 1e9, hits);
        if (cfg == 0) { V(2, 4, false) V(2, 4, true) V(2, 2, true) V(2, 8, true) V(2, 2, false) V(2, 4, true) }
        else { V(4, 4, false) V(4, 4, true) V(4, 2, true) V(4, 2, false) V(4, 8, true) V(4, 4, true) }
        CK(hipFree(w));
        free(hw);
    }
    return 0;
}
