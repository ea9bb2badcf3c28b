// tools/tune_ham3.hip — C3' 96-nt hamming vs one read (k_ham_dense3w) block shapes on 100M dense
// rows (or argv[2] rows, e.g. an odd count for the tails); each variant's distances are checked
// against the production launch before timing.  Same-box history of the kernel: 63-lane chunks with
// two 4-B stores per triple 0.718 of 8 TB/s, one 8-B store 0.750, whole 1-KiB chunks in 3-chunk
// groups 0.779.
// The lane-pair dwordx3 form (k_ham_dense3x) is the production kernel since round 3.
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

template <int T, int U>
static void launch_w(const uint64_t* a, const uint64_t* ref, uint64_t n, uint32_t* out) {   // production
    const uint64_t per = (uint64_t)32 * (T / 64) * U;
    hipLaunchKernelGGL((k_ham_dense3x<false, T, U>), dim3((unsigned)((n + per - 1) / per)), dim3(T), 0, 0,
                       (const uint32_t*)a, (const uint32_t*)a, ref, n, out);
}

// LDS-sum form with each read's per-word distances padded to 8 bytes (byte 8 rl + k), summed with one
// 8-B LDS read and one v_sad_u8 (the C3 fused kernel's tail): block = rpb whole reads as dwordx4
template <int T, int U>
__global__ __launch_bounds__(T) void k_ham3_pad8(const uint4* __restrict__ a, const uint64_t* __restrict__ ref,
                                                 uint64_t n, uint32_t rpb, uint32_t* __restrict__ out) {
    __shared__ uint64_t part8[2 * T * U / 3 + 2];
    uint8_t* part = (uint8_t*)part8;
    const uint64_t r0 = (uint64_t)blockIdx.x * rpb;
    const uint32_t nr = (uint32_t)min((uint64_t)rpb, n - r0);
    const uint32_t nw = nr * 3, nfull = nw / 2;
    const uint64_t q0 = r0 * 3 / 2;
    const uint64_t rf0 = ref[0], rf1 = ref[1], rf2 = ref[2];
    uint4 x[U];
    if (nr == rpb) {   // whole block (rpb even: whole dwordx4): clamped unconditional loads
#pragma unroll
        for (int j = 0; j < U; ++j) x[j] = ld_stream(&a[q0 + min((uint32_t)(j * T + threadIdx.x), nfull - 1)]);
    } else {
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint32_t ql = j * T + threadIdx.x;
            if (ql < nfull) x[j] = ld_stream(&a[q0 + ql]);
            else if (2 * ql < nw) { const uint64_t v = ((const uint64_t*)a)[2 * (q0 + ql)]; x[j] = make_uint4((uint32_t)v, (uint32_t)(v >> 32), 0u, 0u); }
            else x[j] = make_uint4(0u, 0u, 0u, 0u);
        }
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint32_t ql = j * T + threadIdx.x;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t w = 2 * ql + h;
            const uint32_t rl = (uint32_t)__fmul_rn(__fadd_rn((float)w, 0.5f), 1.0f / 3.0f);
            const uint32_t k = w - 3 * rl;
            const uint64_t v = h ? (((uint64_t)x[j].w << 32) | x[j].z) : (((uint64_t)x[j].y << 32) | x[j].x);
            const uint64_t rv = k == 0 ? rf0 : (k == 1 ? rf1 : rf2);
            if (w < nw) part[8 * rl + k] = (uint8_t)ham64(v ^ rv);
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nr; i += T)
        __builtin_nontemporal_store(__builtin_amdgcn_sad_u8((uint32_t)part8[i] & 0xFFFFFFu, 0u, 0u), &out[r0 + i]);
}

template <int T, int U>
static void launch_p8(const uint64_t* a, const uint64_t* ref, uint64_t n, uint32_t* out) {
    const uint32_t rpb = ((2u * T * U) / 3u) & ~1u;
    hipLaunchKernelGGL((k_ham3_pad8<T, U>), dim3((unsigned)((n + rpb - 1) / rpb)), dim3(T), 0, 0, (const uint4*)a, ref, n,
                       rpb, out);
}

// glds form: each wave DMAs G whole 3-KiB groups (128 reads) straight into its own LDS region
// (global_load_lds_dwordx4: coalesced 1-KiB wave-instructions, no VGPRs), waits for its own DMAs
// (no block barrier: the region is wave-private), then lane l reads reads 2l, 2l+1 of a group as three
// conflict-free ds_read_b128 (48-B lane stride) and stores both distances with one 8-B store.
typedef __attribute__((address_space(3))) void* lds_void_ptr;
template <int T, int G>
__global__ __launch_bounds__(T) void k_ham3_glds(const uint4* __restrict__ a, const uint64_t* __restrict__ ref,
                                                 uint64_t n, uint32_t* __restrict__ out) {
    constexpr uint32_t NWV = T / 64;
    __shared__ uint4 sbuf[NWV][G][192];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const uint64_t q = (((uint64_t)blockIdx.x * G + g) * NWV + wv) * 192 + j * 64 + lane;
            __builtin_amdgcn_global_load_lds((const void*)&a[q], (lds_void_ptr)&sbuf[wv][g][j * 64], 16, 0, 0);
        }
    const uint64_t rf0 = ref[0], rf1 = ref[1], rf2 = ref[2];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const uint4 u0 = sbuf[wv][g][3 * lane], u1 = sbuf[wv][g][3 * lane + 1], u2 = sbuf[wv][g][3 * lane + 2];
        const uint64_t w0 = ((uint64_t)u0.y << 32) | u0.x, w1 = ((uint64_t)u0.w << 32) | u0.z;
        const uint64_t w2 = ((uint64_t)u1.y << 32) | u1.x, w3 = ((uint64_t)u1.w << 32) | u1.z;
        const uint64_t w4 = ((uint64_t)u2.y << 32) | u2.x, w5 = ((uint64_t)u2.w << 32) | u2.z;
        const uint32_t d0 = ham64(w0 ^ rf0) + ham64(w1 ^ rf1) + ham64(w2 ^ rf2);
        const uint32_t d1 = ham64(w3 ^ rf0) + ham64(w4 ^ rf1) + ham64(w5 ^ rf2);
        const uint64_t r = (((uint64_t)blockIdx.x * G + g) * NWV + wv) * 128 + 2 * lane;
        if (r + 1 < n) ham_store2(&out[r], d0, d1);
        else if (r < n) ham_store(&out[r], d0);
    }
}

// x4-store form: the production lane-triple sums, then the 64 triples' two distances (packed in one
// u32) are gathered so that lanes 0..31 each store four reads' distances as one dwordx4 (one store
// instruction per 128-read group instead of three partial ones)
template <int T, int G>
__global__ __launch_bounds__(T) void k_ham3_x4(const uint4* __restrict__ a, const uint64_t* __restrict__ ref,
                                               uint64_t n, uint32_t* __restrict__ out) {
    constexpr uint32_t NWV = T / 64;
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    uint4 x[G][3];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const uint64_t q = (((uint64_t)blockIdx.x * G + g) * NWV + wv) * 192 + j * 64 + lane;
            x[g][j] = ld_stream(&a[q]);
        }
    const uint64_t rw[3] = {ref[0], ref[1], ref[2]};
#pragma unroll
    for (int g = 0; g < G; ++g) {
        uint32_t dl[3], dh[3], pk[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const uint64_t wlo = ((uint64_t)x[g][j].y << 32) | x[g][j].x, whi = ((uint64_t)x[g][j].w << 32) | x[g][j].z;
            const uint32_t pos = (2u * ((uint32_t)j + lane)) % 3u;
            const uint64_t clo = pos == 0 ? rw[0] : (pos == 1 ? rw[1] : rw[2]);
            const uint64_t chi = pos == 0 ? rw[1] : (pos == 1 ? rw[2] : rw[0]);
            dl[j] = ham64(wlo ^ clo);
            dh[j] = ham64(whi ^ chi);
        }
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const uint32_t sm = dl[j] + dh[j];
            uint32_t n1l = __shfl(dl[j], (int)min(lane + 1u, 63u)), n1h = __shfl(dh[j], (int)min(lane + 1u, 63u));
            uint32_t n2 = __shfl(sm, (int)min(lane + 2u, 63u));
            if (j < 2) {
                const uint32_t l0 = __builtin_amdgcn_readlane(dl[j + 1], 0), h0 = __builtin_amdgcn_readlane(dh[j + 1], 0);
                const uint32_t s1 = __builtin_amdgcn_readlane(dl[j + 1] + dh[j + 1], 1);
                if (lane == 62) n2 = l0 + h0;
                if (lane == 63) {
                    n1l = l0;
                    n1h = h0;
                    n2 = s1;
                }
            }
            pk[j] = (sm + n1l) | ((n1h + n2) << 16);    // reads 2m, 2m + 1 of triple lane 3m (valid there)
        }
        // output lane q < 32: triples 2q (global lane 6q) and 2q + 1 (6q + 3)
        const uint32_t L0 = 6u * (lane & 31u), L1 = L0 + 3u;
        uint32_t v0 = 0, v1 = 0;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const uint32_t a0 = __shfl(pk[j], (int)(L0 & 63u)), a1 = __shfl(pk[j], (int)(L1 & 63u));
            if (L0 / 64u == (uint32_t)j) v0 = a0;
            if (L1 / 64u == (uint32_t)j) v1 = a1;
        }
        const uint64_t grp = ((uint64_t)blockIdx.x * G + g) * NWV + wv;
        const uint64_t r = grp * 128 + 4 * lane;
        if (lane < 32 && r + 3 < n) {
            const u32x4 o = {v0 & 0xFFFFu, v0 >> 16, v1 & 0xFFFFu, v1 >> 16};
            __builtin_nontemporal_store(o, (u32x4*)&out[r]);
        }
    }
}

template <int T, int G>
static void launch_x4(const uint64_t* a, const uint64_t* ref, uint64_t n, uint32_t* out) {
    const uint64_t per = (uint64_t)128 * (T / 64) * G;   // whole groups only (n a multiple of per)
    hipLaunchKernelGGL((k_ham3_x4<T, G>), dim3((unsigned)(n / per)), dim3(T), 0, 0, (const uint4*)a, ref, n, out);
}

template <int T, int U>
static void launch_x3(const uint64_t* a, const uint64_t* ref, uint64_t n, uint32_t* out) { launch_w<T, U>(a, ref, n, out); }

template <int T, int G>
static void launch_glds(const uint64_t* a, const uint64_t* ref, uint64_t n, uint32_t* out) {
    const uint64_t per = (uint64_t)128 * (T / 64) * G;   // whole groups only (n a multiple of per)
    hipLaunchKernelGGL((k_ham3_glds<T, G>), dim3((unsigned)(n / per)), dim3(T), 0, 0, (const uint4*)a, ref, n, out);
}


// x3 with the wave's U x 32 distances gathered through LDS into dwordx4 stores (U * 8 lanes, one
// store instruction) instead of U stores of 4 B from 32 even lanes
template <int T, int U>
__global__ __launch_bounds__(T) void k_ham3_x3s(const uint32_t* __restrict__ a, const uint64_t* __restrict__ ref,
                                                uint64_t n, uint32_t* __restrict__ out) {
    constexpr uint32_t NWV = T / 64;
    __shared__ __attribute__((aligned(16))) uint32_t sd[NWV][U * 32];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6, h = lane & 1u;
    const uint64_t g0 = ((uint64_t)blockIdx.x * NWV + wv) * U;
    u32x3 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t rc = min((g0 + u) * 32 + (lane >> 1), n - 1);
        x[u] = __builtin_nontemporal_load((const u32x3*)(a + rc * 6 + 3 * h));
    }
    const uint64_t r0 = ref[0], r1 = ref[1], r2 = ref[2];
    const uint32_t c0 = h ? (uint32_t)(r1 >> 32) : (uint32_t)r0;
    const uint32_t c1 = h ? (uint32_t)r2 : (uint32_t)(r0 >> 32);
    const uint32_t c2 = h ? (uint32_t)(r2 >> 32) : (uint32_t)r1;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        uint32_t d = ham32(x[u].x ^ c0) + ham32(x[u].y ^ c1) + ham32(x[u].z ^ c2);
        d += swap_pair(d);
        if (!h) sd[wv][u * 32 + (lane >> 1)] = d;
    }
    __syncthreads();
    const uint64_t rb = g0 * 32;
    if (rb + U * 32 <= n) {
        if (lane < U * 8) {
            const uint4 v = *(const uint4*)&sd[wv][4 * lane];
            const u32x4 q = {v.x, v.y, v.z, v.w};
            __builtin_nontemporal_store(q, (u32x4*)(out + rb + 4 * lane));
        }
    } else {
        for (uint32_t k = lane; k < U * 32; k += 64)
            if (rb + k < n) out[rb + k] = sd[wv][k];
    }
}

template <int T, int U>
static void launch_x3s(const uint64_t* a, const uint64_t* ref, uint64_t n, uint32_t* out) {
    const uint64_t per = (uint64_t)32 * (T / 64) * U;
    hipLaunchKernelGGL((k_ham3_x3s<T, U>), dim3((unsigned)((n + per - 1) / per)), dim3(T), 0, 0, (const uint32_t*)a, ref, n, out);
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
    launch_w<128, 2>(w, ref, n, d0);
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
    for (int pass = 0; pass < 3; ++pass) {
        run("prod (x3 T128 U2, LDS-gathered stores)", launch_w<128, 2>);
        run("x3s T256 U2", launch_x3s<256, 2>);
        run("x3s T128 U2", launch_x3s<128, 2>);
        run("x3s T512 U2", launch_x3s<512, 2>);
        run("x3s T256 U1", launch_x3s<256, 1>);
        run("x3s T512 U1", launch_x3s<512, 1>);
        run("x3s T1024 U1", launch_x3s<1024, 1>);
        run("x3s T256 U3", launch_x3s<256, 3>);
    }
    return 0;
}
