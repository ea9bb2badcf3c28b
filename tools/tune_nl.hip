// tools/tune_nl.hip — read-ceiling probe for k_fq_nlpos: how fast can a kernel read 2 GB and count
// its newlines with the production tile shape (256 threads x 8 chunks of 16 B = 32 KiB per block)?
//   once   : one tile per block, the block exits (k_fq_nlpos's launch shape)
//   gs     : grid-stride over tiles, resident blocks only, no prefetch
//   gspf   : grid-stride with the next tile's loads issued before this tile's counting
//   once16 : one tile per block, 512 threads (64 KiB per block)
// Each block writes one u32 (its newline count) per tile so nothing is dead code.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/tune_nl.hip -o tools/tune_nl
#include "../shortseq_amd/csrc/ss_device.h"
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int kU = 8;

__device__ __forceinline__ uint32_t nl16(uint4 c) {
    auto eq = [](uint32_t w) {
        const uint32_t x = w ^ 0x0A0A0A0Au;
        return ((x - 0x01010101u) & ~x & 0x80808080u);
    };
    return __popc(eq(c.x)) + __popc(eq(c.y)) + __popc(eq(c.z)) + __popc(eq(c.w));
}

__device__ __forceinline__ uint4 ld(const uint4* p) { return ssd::ld_stream(p); }

template <int T>
__device__ __forceinline__ uint32_t block_sum(uint32_t v, uint32_t* red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    uint32_t s = 0;
    if (threadIdx.x == 0)
        for (int w = 0; w < T / 64; ++w) s += red[w];
    __syncthreads();
    return s;
}

template <int T>
__global__ __launch_bounds__(T) void k_once(const uint4* in, uint64_t nchunks, uint32_t* out) {
    __shared__ uint32_t red[T / 64];
    const uint64_t c0 = (uint64_t)blockIdx.x * T * kU;
    uint4 x[kU];
#pragma unroll
    for (int j = 0; j < kU; ++j) {
        const uint64_t c = c0 + j * T + threadIdx.x;
        x[j] = c < nchunks ? ld(in + c) : make_uint4(0, 0, 0, 0);
    }
    uint32_t v = 0;
#pragma unroll
    for (int j = 0; j < kU; ++j) v += nl16(x[j]);
    const uint32_t s = block_sum<T>(v, red);
    if (threadIdx.x == 0) out[blockIdx.x] = s;
}

template <bool PF>
__global__ __launch_bounds__(256) void k_gs(const uint4* in, uint64_t nchunks, uint64_t ntiles, uint32_t* out) {
    constexpr int T = 256;
    __shared__ uint32_t red[T / 64];
    uint4 x[kU];
    uint64_t t = blockIdx.x;
    auto load = [&](uint64_t tile) {
        const uint64_t c0 = tile * T * kU;
#pragma unroll
        for (int j = 0; j < kU; ++j) {
            const uint64_t c = c0 + j * T + threadIdx.x;
            x[j] = c < nchunks ? ld(in + c) : make_uint4(0, 0, 0, 0);
        }
    };
    if (PF && t < ntiles) load(t);
    for (; t < ntiles; t += gridDim.x) {
        if (!PF) load(t);
        uint32_t v = 0;
#pragma unroll
        for (int j = 0; j < kU; ++j) v += nl16(x[j]);
        if (PF && t + gridDim.x < ntiles) load(t + gridDim.x);
        const uint32_t s = block_sum<T>(v, red);
        if (threadIdx.x == 0) out[t] = s;
    }
}

__global__ void k_fill(uint8_t* b, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        b[i] = (i % 61 == 16) ? '\n' : 'A';
}

int main(int argc, char** argv) {
    const uint64_t nbytes = argc > 1 ? strtoull(argv[1], 0, 10) : 1979711488ull;
    const int reps = argc > 2 ? atoi(argv[2]) : 30;
    const uint64_t nchunks = nbytes / 16;
    uint8_t* buf;
    uint32_t* out;
    CK(hipMalloc(&buf, nbytes));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, buf, nbytes);
    const uint64_t tiles = (nchunks + 256 * kU - 1) / (256 * kU);
    CK(hipMalloc(&out, tiles * 8));
    int dev = 0, cus = 0, per = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int mode = 0; mode < 6; ++mode) {
        const char* name = "";
        auto launch = [&]() {
            if (mode == 0) {
                name = "once T256";
                hipLaunchKernelGGL(k_once<256>, dim3((unsigned)tiles), dim3(256), 0, 0, (const uint4*)buf, nchunks, out);
            } else if (mode == 1) {
                name = "once T512";
                hipLaunchKernelGGL(k_once<512>, dim3((unsigned)((nchunks + 512 * kU - 1) / (512 * kU))), dim3(512), 0, 0,
                                   (const uint4*)buf, nchunks, out);
            } else {
                const int mul = mode == 2 || mode == 4 ? 8 : 16;
                const bool pf = mode >= 4;
                name = pf ? (mul == 8 ? "gspf x8" : "gspf x16") : (mul == 8 ? "gs x8" : "gs x16");
                if (pf)
                    hipLaunchKernelGGL(k_gs<true>, dim3(cus * mul), dim3(256), 0, 0, (const uint4*)buf, nchunks, tiles, out);
                else
                    hipLaunchKernelGGL(k_gs<false>, dim3(cus * mul), dim3(256), 0, 0, (const uint4*)buf, nchunks, tiles, out);
            }
        };
        for (int i = 0; i < 5; ++i) launch();
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < reps; ++i) launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("%-10s %.4f ms  %.0f GB/s\n", name, ms, nbytes / ms / 1e6);
        fflush(stdout);
    }
    (void)per;
    return 0;
}
