// tools/tune_ham3.hip — C3' 96-nt hamming vs one read (k_ham_dense3w) block shapes on 100M dense
// rows (or argv[2] rows, e.g. an odd count for the tails); each variant's distances are checked
// against the production launch before timing.  Same-box history of the kernel: 63-lane chunks with
// two 4-B stores per triple 0.718 of 8 TB/s, one 8-B store 0.750, whole 1-KiB chunks in 3-chunk
// groups 0.779.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include tools/tune_ham3.hip -o tools/tune_ham3
#include "../shortseq_amd/csrc/ss_codec.hip"
#include "../shortseq_amd/csrc/ss_runtime.hip"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void k_fill_words(uint64_t* w, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = i * 0x9E3779B97F4A7C15ull + 12345;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        w[i] = z ^ (z >> 31);
    }
}

template <int T, int G>
static void launch_w(const uint64_t* a, const uint64_t* ref, uint64_t n, uint32_t* out) {
    const uint64_t per = (uint64_t)128 * (T / 64) * G;
    hipLaunchKernelGGL((k_ham_dense3w<false, T, G>), dim3((unsigned)((n + per - 1) / per)), dim3(T), 0, 0,
                       (const uint4*)a, (const uint4*)a, ref, n, out);
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 30;
    const uint64_t n = argc > 2 ? strtoull(argv[2], 0, 10) : 100000000ull;
    uint64_t *w, *ref;
    uint32_t *d0, *d1;
    CK(hipMalloc(&w, n * 24));
    CK(hipMalloc(&ref, 24));
    CK(hipMalloc(&d0, n * 4));
    CK(hipMalloc(&d1, n * 4));
    hipLaunchKernelGGL(k_fill_words, dim3(8192), dim3(256), 0, 0, w, n * 3);
    CK(hipMemcpy(ref, w + 3 * 12345, 24, hipMemcpyDeviceToDevice));
    launch_w<256, 1>(w, ref, n, d0);
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> h0(n), h1(n);
    CK(hipMemcpy(h0.data(), d0, n * 4, hipMemcpyDeviceToHost));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, void (*f)(const uint64_t*, const uint64_t*, uint64_t, uint32_t*)) {
        CK(hipMemset(d1, 0xAB, n * 4));
        f(w, ref, n, d1);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h1.data(), d1, n * 4, hipMemcpyDeviceToHost));
        const bool ok = memcmp(h0.data(), h1.data(), n * 4) == 0;
        for (int i = 0; i < 20; ++i) f(w, ref, n, d1);
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < reps; ++i) f(w, ref, n, d1);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("%-28s %s  %.4f ms  %.3f of 8 TB/s\n", name, ok ? "OK " : "BAD", ms, n * 28.0 / (ms * 1e-3) / 8e12);
    };
    for (int pass = 0; pass < 2; ++pass) {
        run("prod T256 G1", launch_w<256, 1>);
        run("T256 G2", launch_w<256, 2>);
        run("T512 G1", launch_w<512, 1>);
        run("T128 G2", launch_w<128, 2>);
        run("T1024 G1", launch_w<1024, 1>);
    }
    return 0;
}
