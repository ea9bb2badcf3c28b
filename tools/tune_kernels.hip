// tools/tune_kernels.hip — block-shape sweep of the PRODUCTION streaming kernels on the BASELINE
// configs (C2 32-nt encode, C3 96-nt fused encode+hamming, C4 512-nt encode/decode).
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include tools/tune_kernels.hip -o tools/tune_kernels
//   tools/tune_kernels [reps=20]
//
// The production translation units are included directly so the sweep times exactly the kernels
// the library launches (same templates, different <T, U, XCD, NT> instantiations).  GB/s are
// algorithmic bytes per launch / hipEvent time (SURVEY §8(d) byte model).
#include "../shortseq_amd/csrc/ss_codec.hip"
#include "../shortseq_amd/csrc/ss_runtime.hip"

#include <stdio.h>
#include <stdlib.h>
#include <functional>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static int g_reps = 20;

static void timeit(const char* name, double bytes, const std::function<void()>& f) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i) f();
    CK(hipDeviceSynchronize());
    double s = 0, mn = 1e9;
    for (int r = 0; r < g_reps; ++r) {
        float ms;
        CK(hipEventRecord(e0, 0));
        f();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        s += ms;
        mn = std::min<double>(mn, ms);
    }
    CK(hipGetLastError());
    const double avg = s / g_reps;
    printf("%-52s avg %8.4f ms  min %8.4f ms  %7.1f GB/s avg  %7.1f GB/s best\n", name, avg, mn, bytes / avg / 1e6,
           bytes / mn / 1e6);
    fflush(stdout);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

static G16Args make_args(const uint8_t* in, uint64_t n, uint32_t L, uint64_t* words, const uint64_t* ref,
                         uint32_t* counts, unsigned long long* fb) {
    G16Args a;
    a.in = (const uint4*)in;
    a.in_stride16 = L / 16;
    a.out32 = (uint32_t*)words;
    a.wpr2 = 2 * ((L + 31) / 32);
    a.n = n;
    a.cpr = L / 16;
    a.full2 = 2 * (L / 32);
    a.all_table = L <= 32;
    a.logG = log2_ceil(a.wpr2);
    a.ref32 = (const uint32_t*)ref;
    a.ham2 = 2 * ham_words(L);
    a.counts = counts;
    a.first_bad = fb;
    return a;
}

#define ENC(PATH, T, U, XCD, NT, tag) \
    timeit("enc " tag " T" #T " U" #U " xcd=" #XCD " ntst=" #NT, bytes, \
           [&] { launch_g16<false, true, PATH, T, U, XCD, NT>(a, 0); })
#define HAMD(PATH, T, U, tag) \
    timeit("ham-dense " tag " T" #T " U" #U, bytes, [&] { launch_ham_dense<PATH, T, U, true>(a, 0); })
#define DEC(T, U, NTLD, NTST, tag) \
    timeit("dec " tag " T" #T " U" #U " ntld=" #NTLD " ntst=" #NTST, bytes, \
           [&] { launch_decode_g16<T, U, NTLD, NTST>((const uint32_t*)words, a.wpr2, n, a.cpr, log2_ceil(a.cpr), \
                                                     (uint4*)out, L / 16, 0); })

int main(int argc, char** argv) {
    g_reps = argc > 1 ? atoi(argv[1]) : 20;
    const uint64_t max_bytes = 50000000ull * 512;
    uint8_t *in, *out;
    uint64_t *words, *ref;
    uint32_t* counts;
    unsigned long long* fb;
    CK(hipMalloc(&in, max_bytes));
    CK(hipMalloc(&out, max_bytes));
    CK(hipMalloc(&words, max_bytes / 4));
    CK(hipMalloc(&counts, 400000000ull));
    CK(hipMalloc(&ref, 256));
    CK(hipMalloc(&fb, 8));
    CK(hipMemset(fb, 0xFF, 8));
    {   // ---- C2: 100M x 32 nt
        const uint64_t n = 100000000;
        const uint32_t L = 32;
        CK((hipError_t)(ss_synth_reads(in, 1, 0, n, L, L, nullptr) == 0 ? hipSuccess : hipErrorUnknown));
        G16Args a = make_args(in, n, L, words, ref, counts, fb);
        const double bytes = n * 40.0;
        printf("== C2 encode 100M x 32 nt\n");
        ENC(kPathTable, 384, 2, false, true, "32 (warm-up)");
        for (int round = 0; round < 3; ++round) {
            ENC(kPathTable, 384, 2, false, true, "32 (production)");
            ENC(kPathTable, 384, 2, true, true, "32");
            ENC(kPathTable, 320, 2, false, true, "32");
            ENC(kPathTable, 448, 2, false, true, "32");
        }
        printf("== decode 100M x 32 nt\n");
        for (int round = 0; round < 2; ++round) {
            DEC(256, 2, false, false, "32 (production)");
            DEC(256, 2, false, true, "32 nt-store");
        }
    }
    {   // ---- C4: 50M x 512 nt
        const uint64_t n = 50000000;
        const uint32_t L = 512;
        CK((hipError_t)(ss_synth_reads(in, 3, 0, n, L, L, nullptr) == 0 ? hipSuccess : hipErrorUnknown));
        G16Args a = make_args(in, n, L, words, ref, counts, fb);
        double bytes = n * 640.0;
        printf("== C4 encode 50M x 512 nt\n");
        for (int round = 0; round < 3; ++round) {
            ENC(kPathPext, 128, 2, false, true, "512 (production)");
            ENC(kPathPext, 128, 2, true, true, "512");
            ENC(kPathPext, 96, 2, false, true, "512");
            ENC(kPathPext, 160, 2, false, true, "512");
        }
        printf("== C4 decode 50M x 512 nt\n");
        for (int round = 0; round < 3; ++round) {
            DEC(256, 2, false, false, "512 (production)");
            DEC(256, 2, false, true, "512 nt-store");
            DEC(256, 2, true, true, "512 nt-load nt-store");
            DEC(256, 4, false, true, "512 nt-store");
            DEC(512, 2, false, true, "512 nt-store");
            DEC(256, 1, false, true, "512 nt-store");
        }
    }
    return 0;
}
