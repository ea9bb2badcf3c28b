// tools/tune_encvar.hip — ss_encode_var on the F2 bench batch (50M reads of 50-150 nt from a 2^20
// pool, wpr 5): the production kernel (one word per lane) against forms where a lane takes K words
// of its wave's 64 K-word span and issues every offset / length load, then every chunk load, before
// packing any (more bytes in flight per lane).  Output compared with the production launch.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include tools/tune_encvar.hip \
//     shortseq_amd/csrc/ss_runtime.hip -o tools/tune_encvar
#include "../shortseq_amd/csrc/ss_codec.hip"

#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
#define CS(x) do { int r_ = (x); if (r_) { printf("ss error %d: %s @%d\n", r_, ss_last_error_string(), __LINE__); exit(1); } } while (0)

namespace {
template <int K>
__global__ __launch_bounds__(kThreads) void k_encvar_k(const uint8_t* in, const uint64_t* __restrict__ offs,
                                                       const uint32_t* __restrict__ lens, uint64_t n,
                                                       uint64_t* __restrict__ out, uint32_t wpr, double inv_wpr,
                                                       unsigned long long* first_bad) {
    const uint64_t total = n * wpr;
    const uint64_t base = ((uint64_t)blockIdx.x * kThreads + (threadIdx.x & ~63u)) * K + (threadIdx.x & 63u);
    uint64_t r[K];
    uint32_t w[K], L[K];
    uint64_t off[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t g = base + 64u * k;
        uint64_t rr = (uint64_t)((double)g * inv_wpr);
        if (rr * wpr > g) --rr;
        else if ((rr + 1) * wpr <= g) ++rr;
        r[k] = g < total ? rr : 0;
        w[k] = (uint32_t)(g - rr * wpr);
        L[k] = g < total ? lens[r[k]] : 0u;
        off[k] = g < total ? offs[r[k]] : 0u;
    }
    Chunks3 c[K];
    uint32_t nb[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        nb[k] = (L[k] <= SS_MAX_NT && 32u * w[k] < L[k]) ? min(32u, L[k] - 32u * w[k]) : 0u;
        if (nb[k]) c[k] = load_word_q(in + off[k] + 32u * w[k], nb[k]);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t g = base + 64u * k;
        if (g >= total) continue;
        uint32_t bad = 0;
        uint64_t word = 0;
        if (L[k] > SS_MAX_NT) bad = (w[k] == 0);
        else if (nb[k]) word = pack_word_q(c[k], nb[k], (L[k] <= 32u) || (nb[k] < 32u), bad);
        out[g] = word;
        report_bad(bad != 0u, r[k], first_bad);
    }
}
}  // namespace

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 50000000ull;
    const int reps = argc > 2 ? atoi(argv[2]) : 10;
    const uint32_t Lmin = 50, Lmax = 150, wpr = 5;
    uint32_t* lens;
    uint64_t *offs, *out0, *out1, *fb;
    CK(hipMalloc(&lens, n * 4));
    CK(hipMalloc(&offs, n * 8));
    CK(hipMalloc(&fb, 8));
    CS(ss_synth_ragged_lens(lens, 41, 42, 1u << 20, 0, n, Lmin, Lmax, nullptr));
    std::vector<uint32_t> hl(n);
    std::vector<uint64_t> ho(n);
    CK(hipMemcpy(hl.data(), lens, n * 4, hipMemcpyDeviceToHost));
    uint64_t tot = 0;
    for (uint64_t i = 0; i < n; ++i) {
        ho[i] = tot;
        tot += hl[i];
    }
    CK(hipMemcpy(offs, ho.data(), n * 8, hipMemcpyHostToDevice));
    uint8_t* blob;
    CK(hipMalloc(&blob, tot + 64));
    CS(ss_synth_ragged_reads(blob, offs, 41, 42, 1u << 20, 0, n, Lmin, Lmax, nullptr));
    CK(hipMalloc(&out0, n * wpr * 8));
    CK(hipMalloc(&out1, n * wpr * 8));
    const double bytes = (double)tot + n * 12.0 + n * wpr * 8.0;
    printf("%llu reads, %.3f GB of bases, %.3f GB algorithmic\n", (unsigned long long)n, tot / 1e9, bytes / 1e9);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<uint64_t> h0(n * wpr), h1(n * wpr);
    for (int mode = 0; mode < 4; ++mode) {
        const int K = mode == 0 ? 1 : mode == 1 ? 2 : mode == 2 ? 4 : 8;
        auto launch = [&](uint64_t* out) {
            if (mode == 0) {
                CS(ss_encode_var(blob, offs, lens, n, out, wpr, fb, nullptr));
                return;
            }
            const uint64_t lanes = (n * wpr + K - 1) / K;
            const unsigned grid = (unsigned)((lanes + kThreads - 1) / kThreads);
            if (K == 2) hipLaunchKernelGGL(k_encvar_k<2>, dim3(grid), dim3(kThreads), 0, 0, blob, offs, lens, n, out, wpr, 1.0 / wpr, (unsigned long long*)fb);
            if (K == 4) hipLaunchKernelGGL(k_encvar_k<4>, dim3(grid), dim3(kThreads), 0, 0, blob, offs, lens, n, out, wpr, 1.0 / wpr, (unsigned long long*)fb);
            if (K == 8) hipLaunchKernelGGL(k_encvar_k<8>, dim3(grid), dim3(kThreads), 0, 0, blob, offs, lens, n, out, wpr, 1.0 / wpr, (unsigned long long*)fb);
        };
        uint64_t* out = mode == 0 ? out0 : out1;
        launch(out);
        CK(hipDeviceSynchronize());
        bool ok = true;
        if (mode) {
            CK(hipMemcpy(h0.data(), out0, n * wpr * 8, hipMemcpyDeviceToHost));
            CK(hipMemcpy(h1.data(), out1, n * wpr * 8, hipMemcpyDeviceToHost));
            ok = h0 == h1;
        }
        for (int i = 0; i < 2; ++i) launch(out);
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < reps; ++i) launch(out);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("K=%d %s  %.4f ms  %.3f of 8 TB/s\n", K, ok ? "OK" : "MISMATCH", ms, bytes / ms / 1e6 / 8000.0);
        fflush(stdout);
    }
    return 0;
}
