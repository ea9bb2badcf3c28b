// tools/tune_encvar.hip — ss_encode_var on the F2 bench batch (50M reads of 50-150 nt from a 2^20
// pool, wpr 5): the production kernel (one word per lane) against forms where a lane takes K words
// of its wave's 64 K-word span and issues every offset / length load, then every chunk load, before
// packing any (more bytes in flight per lane), and block-of-reads forms that stage a dense span of
// the blob in LDS with coalesced loads (profiles/r3/tune_encvar_span.log: 0.33-0.45 of 8 TB/s against
// 0.59 for the production kernel, not kept).  Output compared with the production launch.
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

__device__ __forceinline__ uint64_t shx64(uint64_t v, int m) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m), hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m);
    return ((uint64_t)hi << 32) | lo;
}
// Block of R reads: when their bytes form one dense span (<= CAP bytes, <= 2x the reads' bytes),
// the span is staged in LDS with coalesced 16-B loads and every word is packed from LDS chunks;
// otherwise each word loads its chunks from global memory (k_encode_var_dense's path).
template <uint32_t R, int T, int K, uint32_t CAP>
__global__ __launch_bounds__(T) void k_encvar_span(const uint8_t* in, const uint64_t* __restrict__ offs,
                                                   const uint32_t* __restrict__ lens, uint64_t n,
                                                   uint64_t* __restrict__ out, uint32_t wpr, float inv_wpr,
                                                   unsigned long long* first_bad) {
    __shared__ uint4 sbuf[CAP / 16];
    __shared__ uint64_t soff[R];
    __shared__ uint32_t slen[R];
    __shared__ uint64_t red[3][T / 64];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint64_t r0 = (uint64_t)blockIdx.x * R;
    const uint32_t nr = (uint32_t)min((uint64_t)R, n - r0);
    uint64_t lo = ~0ull, hi = 0, sum = 0;
    for (uint32_t i = threadIdx.x; i < R; i += T) {
        const uint64_t o = offs[r0 + min(i, nr - 1)];
        const uint32_t L = lens[r0 + min(i, nr - 1)];
        soff[i] = o;
        slen[i] = L;
        if (i < nr && L && L <= SS_MAX_NT) {
            lo = min(lo, o);
            hi = max(hi, o + L);
            sum += L;
        }
    }
    for (int m = 32; m; m >>= 1) {
        lo = min(lo, shx64(lo, m));
        hi = max(hi, shx64(hi, m));
        sum += shx64(sum, m);
    }
    if (lane == 0) {
        red[0][wave] = lo;
        red[1][wave] = hi;
        red[2][wave] = sum;
    }
    __syncthreads();
    lo = red[0][0];
    hi = red[1][0];
    sum = red[2][0];
#pragma unroll
    for (int v = 1; v < T / 64; ++v) {
        lo = min(lo, red[0][v]);
        hi = max(hi, red[1][v]);
        sum += red[2][v];
    }
    const uint64_t base = lo & ~15ull;
    const bool staged = hi > lo && hi - base <= CAP && hi - base <= 2 * sum + 256;
    if (staged) {
        const uint32_t nch = (uint32_t)((hi - base + 15) >> 4);
        const uint4* src = (const uint4*)(in + base);
        for (uint32_t c = threadIdx.x; c < nch; c += T) sbuf[c] = ld_stream(&src[c]);
        __syncthreads();
    }
    const uint32_t words = nr * wpr;
    for (uint32_t g0 = 0; g0 < words; g0 += T * K) {
        uint32_t w[K], nb[K], L[K], rl[K];
        uint64_t off[K];
        Chunks3 c[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t g = min(g0 + (uint32_t)k * T + threadIdx.x, words - 1u);
            uint32_t r = (uint32_t)((float)g * inv_wpr);
            if (r * wpr > g) --r;
            else if ((r + 1) * wpr <= g) ++r;
            rl[k] = r;
            w[k] = g - r * wpr;
            L[k] = slen[r];
            off[k] = soff[r];
            nb[k] = (L[k] <= SS_MAX_NT && 32u * w[k] < L[k]) ? min(32u, L[k] - 32u * w[k]) : 0u;
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (!nb[k]) continue;
            if (staged) {
                const uint32_t p = (uint32_t)(off[k] + 32u * w[k] - base), q = p >> 4;
                c[k].sh = p & 15u;
                const uint32_t last = (c[k].sh + nb[k] - 1u) >> 4;
                c[k].c0 = sbuf[q];
                c[k].c1 = sbuf[q + min(1u, last)];
                c[k].c2 = sbuf[q + min(2u, last)];
            } else {
                c[k] = load_word_q(in + off[k] + 32u * w[k], nb[k]);
            }
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t g = g0 + (uint32_t)k * T + threadIdx.x;
            if (g >= words) continue;
            uint32_t bad = 0;
            uint64_t word = 0;
            if (L[k] > SS_MAX_NT) bad = (w[k] == 0);
            else if (nb[k]) word = pack_word_q(c[k], nb[k], (L[k] <= 32u) || (nb[k] < 32u), bad);
            out[r0 * wpr + g] = word;
            report_bad(bad != 0u, r0 + rl[k], first_bad);
        }
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
    const char* names[6] = {"prod", "span R128 T256 K3", "span R64 T128 K3", "span R256 T256 K5", "span R128 T128 K5", "span R256 T512 K3"};
    for (int mode = 0; mode < 6; ++mode) {
        const int K = mode;
        auto launch = [&](uint64_t* out) {
            const float inv = 1.0f / (float)wpr;
            switch (mode) {
            case 0: CS(ss_encode_var(blob, offs, lens, n, out, wpr, fb, nullptr)); return;
            case 1: hipLaunchKernelGGL((k_encvar_span<128, 256, 3, 24576>), dim3((unsigned)((n + 127) / 128)), dim3(256), 0, 0, blob, offs, lens, n, out, wpr, inv, (unsigned long long*)fb); return;
            case 2: hipLaunchKernelGGL((k_encvar_span<64, 128, 3, 12288>), dim3((unsigned)((n + 63) / 64)), dim3(128), 0, 0, blob, offs, lens, n, out, wpr, inv, (unsigned long long*)fb); return;
            case 3: hipLaunchKernelGGL((k_encvar_span<256, 256, 5, 49152>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, blob, offs, lens, n, out, wpr, inv, (unsigned long long*)fb); return;
            case 4: hipLaunchKernelGGL((k_encvar_span<128, 128, 5, 24576>), dim3((unsigned)((n + 127) / 128)), dim3(128), 0, 0, blob, offs, lens, n, out, wpr, inv, (unsigned long long*)fb); return;
            case 5: hipLaunchKernelGGL((k_encvar_span<256, 512, 3, 49152>), dim3((unsigned)((n + 255) / 256)), dim3(512), 0, 0, blob, offs, lens, n, out, wpr, inv, (unsigned long long*)fb); return;
            }
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
        (void)K;
        printf("%-20s %s  %.4f ms  %.3f of 8 TB/s\n", names[mode], ok ? "OK" : "MISMATCH", ms, bytes / ms / 1e6 / 8000.0);
        fflush(stdout);
    }
    return 0;
}
