// tools/probe_streams.hip — does the number of concurrent sequential streams matter on MI355X HBM?
// Read-only sum over 4 GB: (a) grid-order tiles (active blocks read one compact window),
// (b) B persistent blocks, each streaming its own contiguous 1/B of the buffer, for B = 256..8192,
// (c) B blocks, tiles interleaved (block b takes tiles b, b+B, ...).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/probe_streams.hip -o tools/probe_streams
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int T = 512, U = 4;   // 32 KiB per block-tile
template <int MODE>  // 0 grid order, 1 contiguous ranges, 2 interleaved tiles
__global__ __launch_bounds__(T) void k_read(const u32x4* __restrict__ in, uint64_t n16, uint32_t* out) {
    const uint64_t tiles = n16 / (T * U);
    uint32_t acc = 0;
    auto tile = [&](uint64_t t) {
        u32x4 x[U];
#pragma unroll
        for (int j = 0; j < U; ++j) x[j] = __builtin_nontemporal_load(&in[t * T * U + j * T + threadIdx.x]);
#pragma unroll
        for (int j = 0; j < U; ++j) acc ^= x[j].x ^ x[j].y ^ x[j].z ^ x[j].w;
    };
    if (MODE == 0) {
        tile(blockIdx.x);
    } else if (MODE == 1) {
        const uint64_t per = tiles / gridDim.x;
        for (uint64_t t = blockIdx.x * per; t < (blockIdx.x + 1) * per; ++t) tile(t);
    } else {
        for (uint64_t t = blockIdx.x; t < tiles; t += gridDim.x) tile(t);
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

template <int MODE>
void run(const char* name, const u32x4* in, uint64_t n16, uint32_t* out, unsigned grid) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k_read<MODE>), dim3(grid), dim3(T), 0, 0, in, n16, out);
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL((k_read<MODE>), dim3(grid), dim3(T), 0, 0, in, n16, out);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= 10;
    printf("%-40s grid %6u  %.3f ms  %.0f GB/s\n", name, grid, ms, n16 * 16 / ms / 1e6);
}

int main() {
    const uint64_t bytes = 4ull << 30, n16 = bytes / 16;
    u32x4* in;
    uint32_t* out;
    CK(hipMalloc(&in, bytes));
    CK(hipMalloc(&out, 1 << 20));
    CK(hipMemset(in, 1, bytes));
    const uint64_t tiles = n16 / (T * U);
    run<0>("grid order", in, n16, out, (unsigned)tiles);
    for (unsigned B : {256u, 512u, 1024u, 2048u, 4096u, 8192u}) {
        char nm[64];
        snprintf(nm, sizeof nm, "contiguous ranges B=%u", B);
        run<1>(nm, in, n16, out, B);
        snprintf(nm, sizeof nm, "interleaved tiles B=%u", B);
        run<2>(nm, in, n16, out, B);
    }
    run<0>("grid order (repeat)", in, n16, out, (unsigned)tiles);
    return 0;
}
