// tools/probe_zerocopy.hip — device -> pinned host bandwidth for the ingest engine's results (~42 MB
// on the f2 batch): hipMemcpyAsync (blit) vs a kernel storing straight into the mapped pinned buffer
// with 16-B and 8-B coalesced stores.
//   hipcc -O3 --offload-arch=gfx950 tools/probe_zerocopy.hip -o tools/probe_zerocopy
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void k_copy16(const uint4* __restrict__ src, uint4* dst, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) dst[i] = src[i];
}
__global__ void k_copy8(const uint64_t* __restrict__ src, uint64_t* dst, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) dst[i] = src[i];
}

int main() {
    const uint64_t bytes = 42ull << 20;
    void *d, *h;
    CK(hipMalloc(&d, bytes));
    CK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
    CK(hipMemset(d, 1, bytes));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int mode = 0; mode < 3; ++mode) {
        for (int rep = 0; rep < 6; ++rep) {
            CK(hipEventRecord(a, 0));
            if (mode == 0) CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, 0));
            else if (mode == 1) hipLaunchKernelGGL(k_copy16, dim3(1024), dim3(256), 0, 0, (const uint4*)d, (uint4*)h, bytes / 16);
            else hipLaunchKernelGGL(k_copy8, dim3(1024), dim3(256), 0, 0, (const uint64_t*)d, (uint64_t*)h, bytes / 8);
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            if (rep >= 3) printf("%s: %.3f ms, %.1f GB/s\n", mode == 0 ? "hipMemcpyAsync D2H" : mode == 1 ? "kernel 16-B stores" : "kernel 8-B stores", ms, bytes / ms / 1e6);
        }
    }
    return 0;
}
