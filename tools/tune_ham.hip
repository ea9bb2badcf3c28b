// tools/tune_ham.hip — C3' hamming vs one read on dense packed rows (k_ham_dense, power-of-two W):
// block shapes of the production kernel for 32 nt (W = 1, 100M rows) and 512 nt (W = 16, 50M rows);
// every shape's distances are checked against the production launch before timing.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include tools/tune_ham.hip -o tools/tune_ham
#include "../shortseq_amd/csrc/ss_codec.hip"
#include "../shortseq_amd/csrc/ss_runtime.hip"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void k_fill_words(uint64_t* w, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        w[i] = splitmix64(i * 0x9E3779B97F4A7C15ull + 777);
}

typedef void (*Fn)(const uint64_t*, const uint64_t*, uint64_t, uint32_t, uint32_t*);

static void bytes_before(const uint64_t* a, const uint64_t* ref, uint64_t n, uint32_t W, uint32_t* out) {
    const uint32_t rpb = ((2u * 256 * 4) / W) & ~1u;
    hipLaunchKernelGGL((k_ham_dense<false, false, 256, 4, false>), dim3((unsigned)((n + rpb - 1) / rpb)), dim3(256), 0, 0,
                       (const uint4*)a, (const uint4*)a, ref, n, W, rpb, 1.0f / (float)W, out);
}

template <int T, int U>
static void shape(const uint64_t* a, const uint64_t* ref, uint64_t n, uint32_t W, uint32_t* out) {
    launch_ham_dense_k<T, U>(a, ref, n, W, out, false, 0);
}

static void prod(const uint64_t* a, const uint64_t* ref, uint64_t n, uint32_t W, uint32_t* out) {
    if (ss_hamming_ref(a, n, W == 1 ? 32 : 32 * W, W, ref, out, 0)) { printf("prod failed\n"); exit(1); }
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 30;
    uint64_t *w, *ref;
    uint32_t *d0, *d1;
    const uint64_t maxw = 800000000ull;
    CK(hipMalloc(&w, maxw * 8));
    CK(hipMalloc(&ref, 16 * 8));
    CK(hipMalloc(&d0, 100000000ull * 4));
    CK(hipMalloc(&d1, 100000000ull * 4));
    hipLaunchKernelGGL(k_fill_words, dim3(8192), dim3(256), 0, 0, w, maxw);
    CK(hipMemcpy(ref, w + 16 * 4321, 16 * 8, hipMemcpyDeviceToDevice));
    const struct { const char* name; Fn f; } vs[] = {
        {"prod", prod}, {"byte loop (before)", bytes_before}, {"T256 U4 (before)", shape<256, 4>}, {"T512 U2", shape<512, 2>}, {"T128 U4", shape<128, 4>},
        {"T128 U2", shape<128, 2>}, {"T64 U8", shape<64, 8>}, {"T64 U4", shape<64, 4>}, {"T128 U8", shape<128, 8>},
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    bool all = true;
    for (uint32_t W : {5u, 6u, 7u}) {
        const uint64_t n = 50000000ull;
        std::vector<uint32_t> h0(n), h1(n);
        prod(w, ref, n, W, d0);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h0.data(), d0, n * 4, hipMemcpyDeviceToHost));
        const double bytes = (double)n * (8.0 * W + 4.0);
        for (int pass = 0; pass < 2; ++pass)
            for (const auto& v : vs) {
                CK(hipMemset(d1, 0xAB, n * 4));
                v.f(w, ref, n, W, d1);
                CK(hipDeviceSynchronize());
                CK(hipMemcpy(h1.data(), d1, n * 4, hipMemcpyDeviceToHost));
                const bool ok = h0 == h1;
                all &= ok;
                for (int i = 0; i < 5; ++i) v.f(w, ref, n, W, d1);
                CK(hipEventRecord(e0, 0));
                for (int i = 0; i < reps; ++i) v.f(w, ref, n, W, d1);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                ms /= reps;
                printf("W=%-2u %-16s %s %.4f ms  %.3f of 8 TB/s\n", W, v.name, ok ? "OK " : "BAD", ms, bytes / (ms * 1e-3) / 8e12);
            }
    }
    printf(all ? "ALL OK\n" : "SOME BAD\n");
    return all ? 0 : 2;
}
