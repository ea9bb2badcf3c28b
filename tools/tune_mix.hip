// tools/tune_mix.hip — is C3's fused encode + hamming (96 B in, 24 B words + 4 B distance out per
// read) capped by its byte mix?  VERDICT r5 item 6: same-box stream kernels with the same bytes
// and trivial compute, beside the production kernels:
//   mix_lds<T>   C3's shape: one lane per 16-B chunk (dwordx4 nt load), a 4-B "word" per lane stored
//                dense (the encode's output shape), the chunk's byte into LDS, a barrier, then one
//                thread per read sums its 6 bytes and stores the u32 distance
//   mix_plain<T> the same loads and word stores; the distance stored by the read's first lane from
//                its own chunk (no LDS, no barrier): the byte mix alone
//   c2_plain<T>  C2's mix for reference: 32 B in, 4 B per chunk out (8 B per read), nothing else
//   prod C3      ss_encode_hamming_ref (k_encode_ham_dense) on the same 100M x 96-nt reads
//   prod C2      ss_encode_fixed (k_encode_g16) on 100M x 32-nt reads
// Prints ms and the fraction of 8 TB/s over each kernel's bytes (min over reps).
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include tools/tune_mix.hip -o tools/tune_mix
//   tools/tune_mix [reps=20]
#include "../shortseq_amd/csrc/ss_codec.hip"
#include "../shortseq_amd/csrc/ss_runtime.hip"

#include <stdio.h>
#include <stdlib.h>

namespace {

constexpr uint32_t kCpr = 6;      // 16-B chunks per 96-nt read

// T threads, U chunks per lane per block (a block = T * U chunks = T * U / 6 reads; T * U % 6 == 0)
template <int T, int U>
__global__ __launch_bounds__(T) void k_mix_lds(const uint4* __restrict__ in, uint32_t* __restrict__ words,
                                               uint32_t* __restrict__ dist, uint64_t nchunks) {
    constexpr uint32_t CB = T * U, RB = CB / kCpr;
    static_assert(CB % kCpr == 0, "whole reads per block");
    __shared__ uint8_t part[CB];
    const uint64_t c0 = (uint64_t)blockIdx.x * CB;
    uint4 x[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint64_t c = c0 + (uint64_t)j * T + threadIdx.x;
        x[j] = ld_stream(&in[min(c, nchunks - 1)]);
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint64_t c = c0 + (uint64_t)j * T + threadIdx.x;
        const uint32_t v = x[j].x ^ x[j].y ^ x[j].z ^ x[j].w;
        if (c < nchunks) st_stream(&words[c], v);
        part[j * T + threadIdx.x] = (uint8_t)__popc(v);
    }
    __syncthreads();
    for (uint32_t r = threadIdx.x; r < RB; r += T) {
        const uint64_t g = c0 / kCpr + r;
        uint32_t s = 0;
#pragma unroll
        for (uint32_t k = 0; k < kCpr; ++k) s += part[r * kCpr + k];
        if (g * kCpr < nchunks) st_stream(&dist[g], s);
    }
}

template <int T, int U>
__global__ __launch_bounds__(T) void k_mix_plain(const uint4* __restrict__ in, uint32_t* __restrict__ words,
                                                 uint32_t* __restrict__ dist, uint64_t nchunks) {
    constexpr uint32_t CB = T * U;
    const uint64_t c0 = (uint64_t)blockIdx.x * CB;
    uint4 x[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint64_t c = c0 + (uint64_t)j * T + threadIdx.x;
        x[j] = ld_stream(&in[min(c, nchunks - 1)]);
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint64_t c = c0 + (uint64_t)j * T + threadIdx.x;
        const uint32_t v = x[j].x ^ x[j].y ^ x[j].z ^ x[j].w;
        if (c < nchunks) {
            st_stream(&words[c], v);
            if (c % kCpr == 0) st_stream(&dist[c / kCpr], v);
        }
    }
}

template <int T, int U>
__global__ __launch_bounds__(T) void k_c2_plain(const uint4* __restrict__ in, uint32_t* __restrict__ words,
                                                uint64_t nchunks) {
    constexpr uint32_t CB = T * U;
    const uint64_t c0 = (uint64_t)blockIdx.x * CB;
    uint4 x[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint64_t c = c0 + (uint64_t)j * T + threadIdx.x;
        x[j] = ld_stream(&in[min(c, nchunks - 1)]);
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint64_t c = c0 + (uint64_t)j * T + threadIdx.x;
        if (c < nchunks) st_stream(&words[c], x[j].x ^ x[j].y ^ x[j].z ^ x[j].w);
    }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
#define CS(x) do { int r_ = (x); if (r_) { printf("ss error %d: %s @%d\n", r_, ss_last_error_string(), __LINE__); exit(1); } } while (0)

int g_reps = 20;

template <typename F>
void timeit(const char* name, double bytes, F f) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 5; ++i) f();
    CK(hipDeviceSynchronize());
    float best = 1e9f, sum = 0;
    for (int i = 0; i < g_reps; ++i) {
        CK(hipEventRecord(a, 0));
        f();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        best = ms < best ? ms : best;
        sum += ms;
    }
    printf("%-28s min %.4f ms  mean %.4f ms  %.0f GB/s  frac %.3f (mean %.3f)\n", name, best, sum / g_reps,
           bytes / best * 1e-6, bytes / best * 1e-6 / 8000.0, bytes / (sum / g_reps) * 1e-6 / 8000.0);
    fflush(stdout);
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
}

}  // namespace

int main(int argc, char** argv) {
    g_reps = argc > 1 ? atoi(argv[1]) : 20;
    const uint64_t n = 100000000ull;
    uint8_t *a96, *a32;
    uint64_t *w, *fb;
    uint32_t *d, *w32;
    CK(hipMalloc(&a96, n * 96));
    CK(hipMalloc(&w, n * 24));
    CK(hipMalloc(&d, n * 4));
    CK(hipMalloc(&fb, 8));
    CS(ss_synth_reads(a96, 1, 0, n, 96, 96, nullptr));
    CK(hipDeviceSynchronize());
    const uint64_t nch = n * kCpr;
    w32 = (uint32_t*)w;
    const double b3 = (double)n * (96 + 24 + 4);
    // production C3 (the reference read packed first, as in bench.py)
    CS(ss_encode_fixed(a96, 1, 96, 96, w, 3, fb, nullptr));
    uint64_t* ref;
    CK(hipMalloc(&ref, 24));
    CK(hipMemcpy(ref, w, 24, hipMemcpyDeviceToDevice));
    timeit("prod C3 k_encode_ham_dense", b3, [&] { CS(ss_encode_hamming_ref(a96, n, 96, 96, w, 3, ref, d, fb, nullptr)); });
    timeit("mix_lds<256,6>", b3, [&] {
        hipLaunchKernelGGL((k_mix_lds<256, 6>), dim3((unsigned)((nch + 1535) / 1536)), dim3(256), 0, 0,
                           (const uint4*)a96, w32, d, nch);
    });
    timeit("mix_lds<512,6>", b3, [&] {
        hipLaunchKernelGGL((k_mix_lds<512, 6>), dim3((unsigned)((nch + 3071) / 3072)), dim3(512), 0, 0,
                           (const uint4*)a96, w32, d, nch);
    });
    timeit("mix_plain<256,6>", b3, [&] {
        hipLaunchKernelGGL((k_mix_plain<256, 6>), dim3((unsigned)((nch + 1535) / 1536)), dim3(256), 0, 0,
                           (const uint4*)a96, w32, d, nch);
    });
    timeit("mix_plain<256,4>", b3, [&] {
        hipLaunchKernelGGL((k_mix_plain<256, 4>), dim3((unsigned)((nch + 1023) / 1024)), dim3(256), 0, 0,
                           (const uint4*)a96, w32, d, nch);
    });
    timeit("mix_plain<512,8>", b3, [&] {
        hipLaunchKernelGGL((k_mix_plain<512, 8>), dim3((unsigned)((nch + 4095) / 4096)), dim3(512), 0, 0,
                           (const uint4*)a96, w32, d, nch);
    });
    timeit("prod C3 k_encode_ham_dense", b3, [&] { CS(ss_encode_hamming_ref(a96, n, 96, 96, w, 3, ref, d, fb, nullptr)); });
    CK(hipFree(a96));
    CK(hipFree(d));
    // C2's mix on the same box: 32 B in + 8 B out per read
    CK(hipMalloc(&a32, n * 32));
    CS(ss_synth_reads(a32, 1, 0, n, 32, 32, nullptr));
    CK(hipDeviceSynchronize());
    const double b2 = (double)n * 40;
    const uint64_t nc2 = n * 2;
    timeit("prod C2 k_encode_g16", b2, [&] { CS(ss_encode_fixed(a32, n, 32, 32, w, 1, fb, nullptr)); });
    timeit("c2_plain<256,4>", b2, [&] {
        hipLaunchKernelGGL((k_c2_plain<256, 4>), dim3((unsigned)((nc2 + 1023) / 1024)), dim3(256), 0, 0,
                           (const uint4*)a32, w32, nc2);
    });
    timeit("c2_plain<256,8>", b2, [&] {
        hipLaunchKernelGGL((k_c2_plain<256, 8>), dim3((unsigned)((nc2 + 2047) / 2048)), dim3(256), 0, 0,
                           (const uint4*)a32, w32, nc2);
    });
    CK(hipFree(a32));
    CK(hipFree(w));
    return 0;
}
