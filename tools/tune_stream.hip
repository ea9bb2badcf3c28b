// tools/tune_stream.hip — structural variants of the streaming kernels (not just block shapes):
//
//   C2 32-nt encode : production k_encode_g16 vs
//       r1   : one lane per read (2 x dwordx4 at stride 32 B), one 8-B store per lane
//       r2   : one lane per 2 reads (4 x dwordx4 at stride 64 B), one 16-B store per lane
//       pers : persistent grid, register double-buffered tiles (next tile's loads in flight while
//              the current one is encoded and stored)
//   C3 96-nt fused encode+hamming : production k_encode_ham_dense (LDS byte partials + barrier) vs
//       wave : a wave owns 64 whole reads = 64*cpr chunks loaded as cpr coalesced dwordx4 rows;
//              per-chunk distances packed 5 bits each, gathered per read with cpr ds_bpermute —
//              no LDS allocation, no barrier.
// Every variant's words (and distances) are compared with the production kernel's before timing.
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include tools/tune_stream.hip -o tools/tune_stream
//   tools/tune_stream [reps=20]
#include "../shortseq_amd/csrc/ss_codec.hip"
#include "../shortseq_amd/csrc/ss_runtime.hip"

namespace {
// (measured slower than k_encode_ham_dense: 2.32-2.45 vs 1.87-1.94 ms, gpurun_out/tune_c3.log)
// Dense fused encode + hamming for 96-nt reads (3 PEXT words, no alias carries) without LDS or a
// barrier: a lane owns one 32-nt word (its two dwordx4 chunks), a wave streams 63 consecutive words =
// 21 whole reads (lane 63 idles, 1.6 % of the lanes), and the three lanes of a read add their
// distances with two shuffles; the read's first lane stores the sum.  Word chunk c of the block =
// j * (T / 64) + wave, so at each j the block's waves read one contiguous span.
template <int T, int U, bool NTST>
__global__ __launch_bounds__(T) void k_encode_ham_w3(G16Args a) {
    constexpr uint32_t NWV = T / 64, RPC = 21, QPC = 63, RPB = RPC * NWV * U;
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t m = lane / 3u, p = lane - 3u * m;
    const uint64_t r0 = (uint64_t)blockIdx.x * RPB;
    const uint32_t nr = (uint32_t)min((uint64_t)RPB, a.n - r0);
    const uint32_t nw = 3u * nr;
    const uint64_t q0 = r0 * 3u;
    uint4 x[U][2];
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint32_t ql = (j * NWV + wv) * QPC + lane;
        const bool live = lane < QPC && ql < nw;
        x[j][0] = live ? ld_stream(&a.in[2 * (q0 + ql)]) : make_uint4(0x41414141u, 0x41414141u, 0x41414141u, 0x41414141u);
        x[j][1] = live ? ld_stream(&a.in[2 * (q0 + ql) + 1])
                       : make_uint4(0x41414141u, 0x41414141u, 0x41414141u, 0x41414141u);
    }
    const uint64_t ref = ((uint64_t)a.ref32[2 * p + 1] << 32) | a.ref32[2 * p];
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint32_t ql = (j * NWV + wv) * QPC + lane;
        const uint32_t rb = (j * NWV + wv) * RPC + m;                      // block-local read
        const bool live = lane < QPC && ql < nw;
        const Enc32 lo = encode16(x[j][0].x, x[j][0].y, x[j][0].z, x[j][0].w, false);
        const Enc32 hi = encode16(x[j][1].x, x[j][1].y, x[j][1].z, x[j][1].w, false);
        report_bad(live && (lo.bad | hi.bad) != 0u, r0 + rb, a.first_bad);
        const uint64_t v = ((uint64_t)hi.v << 32) | lo.v;
        if (live && a.out32) {
            uint64_t* dst = (uint64_t*)a.out32 + q0 + ql;
            if constexpr (NTST) __builtin_nontemporal_store(v, dst);
            else *dst = v;
        }
        const uint32_t d = live ? ham64(v ^ ref) : 0u;
        const uint32_t d1 = __shfl(d, (int)min(lane + 1u, 63u)), d2 = __shfl(d, (int)min(lane + 2u, 63u));
        if (live && p == 0) {
            if constexpr (NTST) __builtin_nontemporal_store(d + d1 + d2, &a.counts[r0 + rb]);
            else a.counts[r0 + rb] = d + d1 + d2;
        }
    }
}

template <int T, int U, bool NTST>
void launch_ham_w3(const G16Args& a, hipStream_t s) {
    const uint64_t rpb = 21ull * (T / 64) * U;
    hipLaunchKernelGGL((k_encode_ham_w3<T, U, NTST>), dim3(grid_for(a.n, rpb)), dim3(T), 0, s, a);
}
}  // namespace

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <functional>
#include <vector>
#include <unistd.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static int g_reps = 20;

static void timeit(const char* name, double bytes, const std::function<void()>& f) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 5; ++i) f();
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

// ---------------------------------------------------------------------------------------------
// C2 variants (L = 32, table path: the low chunk's alias carry goes into the high half)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t enc_read32(const uint4& lo, const uint4& hi, uint32_t& bad) {
    const Enc32 a = encode16(lo.x, lo.y, lo.z, lo.w, true);
    const Enc32 b = encode16(hi.x, hi.y, hi.z, hi.w, true);
    bad = a.bad | b.bad;
    return (uint64_t)a.v | ((uint64_t)(b.v | a.cout) << 32);
}

template <int T, int U>
__global__ __launch_bounds__(T) void k_enc_r1(const uint4* __restrict__ in, uint64_t* __restrict__ out, uint64_t n,
                                              unsigned long long* fb) {
    const uint64_t base = (uint64_t)blockIdx.x * T * U + threadIdx.x;
    uint4 x[U][2];
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint64_t r = base + (uint64_t)j * T;
        const bool ok = r < n;
        x[j][0] = ok ? ld_stream(&in[2 * r]) : make_uint4(0x41414141u, 0x41414141u, 0x41414141u, 0x41414141u);
        x[j][1] = ok ? ld_stream(&in[2 * r + 1]) : make_uint4(0x41414141u, 0x41414141u, 0x41414141u, 0x41414141u);
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint64_t r = base + (uint64_t)j * T;
        uint32_t bad;
        const uint64_t w = enc_read32(x[j][0], x[j][1], bad);
        report_bad(r < n && bad, r, fb);
        if (r < n) __builtin_nontemporal_store(w, &out[r]);
    }
}

template <int T, int U>
__global__ __launch_bounds__(T) void k_enc_r2(const uint4* __restrict__ in, uint64_t* __restrict__ out, uint64_t n,
                                              unsigned long long* fb) {
    const uint64_t np = n / 2;   // n even in this tuner
    const uint64_t base = (uint64_t)blockIdx.x * T * U + threadIdx.x;
    uint4 x[U][4];
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint64_t p = base + (uint64_t)j * T;
        const bool ok = p < np;
#pragma unroll
        for (int q = 0; q < 4; ++q)
            x[j][q] = ok ? ld_stream(&in[4 * p + q]) : make_uint4(0x41414141u, 0x41414141u, 0x41414141u, 0x41414141u);
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint64_t p = base + (uint64_t)j * T;
        uint32_t b0, b1;
        const uint64_t w0 = enc_read32(x[j][0], x[j][1], b0);
        const uint64_t w1 = enc_read32(x[j][2], x[j][3], b1);
        report_bad(p < np && (b0 | b1), 2 * p, fb);
        if (p < np) {
            const u32x4 q = {(uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32)};
            __builtin_nontemporal_store(q, (u32x4*)&out[2 * p]);
        }
    }
}

// persistent: tile = T*U chunks (production lane mapping: lane slot g = chunk, 2 lanes per read)
template <int T, int U>
__global__ __launch_bounds__(T) void k_enc_pers(const uint4* __restrict__ in, uint32_t* __restrict__ out,
                                                uint64_t nchunks, unsigned long long* fb) {
    const uint64_t tiles = (nchunks + (uint64_t)T * U - 1) / ((uint64_t)T * U);
    uint64_t t = blockIdx.x;
    uint4 x[U];
    auto load = [&](uint64_t tile) {
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint64_t g = tile * T * U + (uint64_t)j * T + threadIdx.x;
            x[j] = g < nchunks ? ld_stream(&in[g]) : make_uint4(0x41414141u, 0x41414141u, 0x41414141u, 0x41414141u);
        }
    };
    if (t < tiles) load(t);
    for (; t < tiles; t += gridDim.x) {
        uint4 cur[U];
#pragma unroll
        for (int j = 0; j < U; ++j) cur[j] = x[j];
        if (t + gridDim.x < tiles) load(t + gridDim.x);
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint64_t g = t * T * U + (uint64_t)j * T + threadIdx.x;
            const Enc32 e = encode16(cur[j].x, cur[j].y, cur[j].z, cur[j].w, true);
            const uint32_t v = e.v | ((threadIdx.x & 1u) ? swap_pair(e.cout) : 0u);
            report_bad_div(g < nchunks && e.bad != 0u, g, 2, fb);
            if (g < nchunks) st_stream(&out[g], v);
        }
    }
}

// wave-staged 16-B stores: a wave owns 64*U consecutive chunks (coalesced dwordx4 loads, lane l
// takes chunk wbase + 64 j + l), writes its U u32 results to a per-wave LDS strip, and each lane
// stores 4 consecutive results as one dwordx4 (1 KB per wave store instruction).
template <int WPB, int U, bool NTST>
__global__ __launch_bounds__(64 * WPB) void k_enc_wst(const uint4* __restrict__ in, uint32_t* __restrict__ out,
                                                     uint64_t nchunks, unsigned long long* fb) {
    __shared__ uint32_t strip[WPB][64 * U];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint64_t wbase = ((uint64_t)blockIdx.x * WPB + wave) * (64 * U);
    uint4 x[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint64_t g = wbase + j * 64 + lane;
        x[j] = g < nchunks ? ld_stream(&in[g]) : make_uint4(0x41414141u, 0x41414141u, 0x41414141u, 0x41414141u);
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint64_t g = wbase + j * 64 + lane;
        const Enc32 e = encode16(x[j].x, x[j].y, x[j].z, x[j].w, true);
        const uint32_t v = e.v | ((lane & 1u) ? swap_pair(e.cout) : 0u);
        report_bad_div(g < nchunks && e.bad != 0u, g, 2, fb);
        strip[wave][j * 64 + lane] = v;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
    for (int q = 0; q < U / 4; ++q) {
        const uint32_t c = (q * 64 + lane) * 4;          // first of 4 consecutive chunks
        const uint64_t g = wbase + c;
        if (g + 3 < nchunks) {
            const u32x4 v = {strip[wave][c], strip[wave][c + 1], strip[wave][c + 2], strip[wave][c + 3]};
            if (NTST) __builtin_nontemporal_store(v, (u32x4*)&out[g]);
            else *(u32x4*)&out[g] = v;
        } else {
            for (uint32_t k = 0; k < 4; ++k)
                if (g + k < nchunks) out[g + k] = strip[wave][c + k];
        }
    }
}

// ---------------------------------------------------------------------------------------------
// C3 variant: wave-owned reads, ds_bpermute gather of packed 5-bit chunk distances.
// CPR chunks per read (even, PEXT path, L % 32 == 0, L >= 64), CPR <= 12 (two packed words).
// ---------------------------------------------------------------------------------------------
template <int CPR, int WPB>
__global__ __launch_bounds__(64 * WPB) void k_ham_wave(const uint4* __restrict__ in, uint32_t* __restrict__ out32,
                                                      const uint32_t* __restrict__ ref32, uint32_t* __restrict__ counts,
                                                      uint64_t n, unsigned long long* fb) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t r0 = ((uint64_t)blockIdx.x * WPB + (threadIdx.x >> 6)) * 64u;   // first read of this wave
    if (r0 >= n) return;
    const uint32_t nr = (uint32_t)min((uint64_t)64, n - r0);
    const uint32_t nloc = nr * CPR;
    const uint64_t c0 = r0 * CPR;
    uint4 x[CPR];
#pragma unroll
    for (int j = 0; j < CPR; ++j) {
        const uint32_t cl = j * 64 + lane;
        x[j] = cl < nloc ? ld_stream(&in[c0 + cl]) : make_uint4(0x41414141u, 0x41414141u, 0x41414141u, 0x41414141u);
    }
    constexpr int NP = (CPR + 5) / 6;
    uint32_t H[NP];
#pragma unroll
    for (int q = 0; q < NP; ++q) H[q] = 0;
    uint32_t badacc = 0;
#pragma unroll
    for (int j = 0; j < CPR; ++j) {
        const uint32_t cl = j * 64 + lane;
        const uint32_t k = cl % CPR;
        const Enc32 e = encode16(x[j].x, x[j].y, x[j].z, x[j].w, false);
        const bool live = cl < nloc;
        badacc |= live ? e.bad : 0u;
        if (live) st_stream(&out32[c0 + cl], e.v);
        const uint32_t h = ham32(e.v ^ ref32[k]);
        H[j / 6] |= h << (5 * (j % 6));
    }
    if (__ballot(badacc != 0)) {
        // rare path: find the first bad read of this wave exactly (recompute per chunk)
#pragma unroll
        for (int j = 0; j < CPR; ++j) {
            const uint32_t cl = j * 64 + lane;
            const Enc32 e = encode16(x[j].x, x[j].y, x[j].z, x[j].w, false);
            if (cl < nloc && e.bad) atomicMin(fb, (unsigned long long)(r0 + cl / CPR));
        }
    }
    // read `lane` = chunks lane*CPR + i, i < CPR; chunk c sits in register c / 64 of lane c % 64
    uint32_t sum = 0;
#pragma unroll
    for (int i = 0; i < CPR; ++i) {
        const uint32_t c = lane * CPR + i;
        const uint32_t src = c & 63u, reg = c >> 6;     // reg < CPR
        uint32_t got[NP];
#pragma unroll
        for (int q = 0; q < NP; ++q) got[q] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)H[q]);
        uint32_t word = got[0];
#pragma unroll
        for (int q = 1; q < NP; ++q) word = (reg / 6 == (uint32_t)q) ? got[q] : word;
        sum += (word >> (5 * (reg % 6))) & 31u;
    }
    if (lane < nr) counts[r0 + lane] = sum;
}

__global__ void k_fill(uint8_t* p, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 16; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t r = splitmix64(i);
        ((uint4*)p)[i] = decode16((uint32_t)r);
    }
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

static bool same(const void* d_a, const void* d_b, size_t bytes, const char* what) {
    std::vector<uint8_t> a(bytes), b(bytes);
    CK(hipMemcpy(a.data(), d_a, bytes, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), d_b, bytes, hipMemcpyDeviceToHost));
    const bool ok = memcmp(a.data(), b.data(), bytes) == 0;
    printf("  check %-40s %s\n", what, ok ? "OK" : "MISMATCH");
    return ok;
}

int main(int argc, char** argv) {
    g_reps = argc > 1 ? atoi(argv[1]) : 20;
    const bool only_c3 = argc > 2 && strcmp(argv[2], "c3") == 0;
    const uint64_t n2 = 100000000ull;              // C2 reads
    const uint64_t n3 = 100000000ull;              // C3 reads
    uint8_t* in;
    uint64_t *w_ref, *w_var, *ref;
    uint32_t *c_ref, *c_var;
    unsigned long long* fb;
    CK(hipMalloc(&in, n3 * 96));
    CK(hipMalloc(&w_ref, n3 * 24));
    CK(hipMalloc(&w_var, n3 * 24));
    CK(hipMalloc(&c_ref, n3 * 4));
    CK(hipMalloc(&c_var, n3 * 4));
    CK(hipMalloc(&ref, 64));
    CK(hipMalloc(&fb, 8));
    CK(hipMemset(fb, 0xFF, 8));
    hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, in, n3 * 96);
    CK(hipDeviceSynchronize());

    // ---------------- clock ramp: per-launch times of the production C2 kernel from idle ----------
    {
        G16Args a = make_args(in, n2, 32, w_ref, nullptr, nullptr, fb);
        hipEvent_t ev[201];
        for (int i = 0; i <= 200; ++i) CK(hipEventCreate(&ev[i]));
        CK(hipDeviceSynchronize());
        usleep(1000000);
        CK(hipEventRecord(ev[0], 0));
        for (int i = 0; i < 200; ++i) {
            launch_g16<false, true, kPathTable, 768, 2, false, true>(a, 0);
            CK(hipEventRecord(ev[i + 1], 0));
        }
        CK(hipDeviceSynchronize());
        printf("ramp from idle (ms per launch, back-to-back):");
        for (int i = 0; i < 200; ++i) {
            float ms;
            CK(hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
            if (i % 10 == 0) printf("\n  %3d:", i);
            printf(" %.4f", ms);
        }
        printf("\n");
    }
    for (int pass = 0; pass < 2; ++pass) {
    // ---------------- C2 ----------------
    if (!only_c3) {
        const uint32_t L = 32;
        const double bytes = (double)n2 * 40;
        G16Args a = make_args(in, n2, L, w_ref, nullptr, nullptr, fb);
        printf("C2 32-nt encode, %llu reads (pass %d)\n", (unsigned long long)n2, pass);
        launch_g16<false, true, kPathTable, 768, 2, false, true>(a, 0);
        timeit("C2 production k_encode_g16 T768 U2", bytes, [&] { launch_g16<false, true, kPathTable, 768, 2, false, true>(a, 0); });
        if (pass == 0) {
            CK(hipMemset(w_var, 0, n2 * 8));
            hipLaunchKernelGGL((k_enc_wst<4, 4, true>), dim3((unsigned)((2 * n2 + 1023) / 1024)), dim3(256), 0, 0,
                               (const uint4*)in, (uint32_t*)w_var, 2 * n2, fb);
            same(w_ref, w_var, n2 * 8, "wst WPB4 U4 vs production");
        }
        timeit("C2 wst WPB4 U4 nt", bytes, [&] { hipLaunchKernelGGL((k_enc_wst<4, 4, true>), dim3((unsigned)((2 * n2 + 1023) / 1024)), dim3(256), 0, 0, (const uint4*)in, (uint32_t*)w_var, 2 * n2, fb); });
        timeit("C2 wst WPB8 U4 nt", bytes, [&] { hipLaunchKernelGGL((k_enc_wst<8, 4, true>), dim3((unsigned)((2 * n2 + 2047) / 2048)), dim3(512), 0, 0, (const uint4*)in, (uint32_t*)w_var, 2 * n2, fb); });
        timeit("C2 wst WPB12 U4 nt", bytes, [&] { hipLaunchKernelGGL((k_enc_wst<12, 4, true>), dim3((unsigned)((2 * n2 + 3071) / 3072)), dim3(768), 0, 0, (const uint4*)in, (uint32_t*)w_var, 2 * n2, fb); });
        timeit("C2 wst WPB4 U8 nt", bytes, [&] { hipLaunchKernelGGL((k_enc_wst<4, 8, true>), dim3((unsigned)((2 * n2 + 2047) / 2048)), dim3(256), 0, 0, (const uint4*)in, (uint32_t*)w_var, 2 * n2, fb); });
        timeit("C2 wst WPB8 U4", bytes, [&] { hipLaunchKernelGGL((k_enc_wst<8, 4, false>), dim3((unsigned)((2 * n2 + 2047) / 2048)), dim3(512), 0, 0, (const uint4*)in, (uint32_t*)w_var, 2 * n2, fb); });
        timeit("C2 k_encode_g16 T512 U2", bytes, [&] { launch_g16<false, true, kPathTable, 512, 2, false, true>(a, 0); });
        timeit("C2 k_encode_g16 T1024 U2", bytes, [&] { launch_g16<false, true, kPathTable, 1024, 2, false, true>(a, 0); });
        timeit("C2 k_encode_g16 T768 U1", bytes, [&] { launch_g16<false, true, kPathTable, 768, 1, false, true>(a, 0); });
        timeit("C2 k_encode_g16 T1024 U1", bytes, [&] { launch_g16<false, true, kPathTable, 1024, 1, false, true>(a, 0); });
        timeit("C2 k_encode_g16 T512 U3", bytes, [&] { launch_g16<false, true, kPathTable, 512, 3, false, true>(a, 0); });
        timeit("C2 r1 T512 U1", bytes, [&] { hipLaunchKernelGGL((k_enc_r1<512, 1>), dim3(grid_for(n2, 512)), dim3(512), 0, 0, (const uint4*)in, w_var, n2, fb); });
        timeit("C2 r1 T1024 U1", bytes, [&] { hipLaunchKernelGGL((k_enc_r1<1024, 1>), dim3(grid_for(n2, 1024)), dim3(1024), 0, 0, (const uint4*)in, w_var, n2, fb); });
        timeit("C2 pers T512 U2 x2/CU", bytes, [&] { hipLaunchKernelGGL((k_enc_pers<512, 2>), dim3(512), dim3(512), 0, 0, (const uint4*)in, (uint32_t*)w_var, 2 * n2, fb); });
        timeit("C2 pers T768 U2 x2/CU", bytes, [&] { hipLaunchKernelGGL((k_enc_pers<768, 2>), dim3(512), dim3(768), 0, 0, (const uint4*)in, (uint32_t*)w_var, 2 * n2, fb); });
        timeit("C2 pers T512 U2 x3/CU", bytes, [&] { hipLaunchKernelGGL((k_enc_pers<512, 2>), dim3(768), dim3(512), 0, 0, (const uint4*)in, (uint32_t*)w_var, 2 * n2, fb); });
    }
    // ---------------- C3 ----------------
    {
        const uint32_t L = 96;
        const double bytes = (double)n3 * 124;
        hipLaunchKernelGGL((k_encode_gen<false, false>), dim3(1), dim3(256), 0, 0, in, (uint64_t)96,
                           (const uint64_t*)nullptr, (const uint32_t*)nullptr, 96u, (uint64_t)1, ref, 3u, 2u,
                           (const uint64_t*)nullptr, 0u, (uint32_t*)nullptr, fb);
        G16Args a = make_args(in, n3, L, w_ref, ref, c_ref, fb);
        if (pass == 0) {
            launch_ham_dense<kPathPext, 768, 2, true>(a, 0);
            G16Args b = make_args(in, n3, L, w_var, ref, c_var, fb);
            CK(hipMemset(w_var, 0, n3 * 24));
            CK(hipMemset(c_var, 0, n3 * 4));
            launch_ham_dense<kPathPext, 128, 6, true>(b, 0);
            same(w_ref, w_var, n3 * 24, "ham_dense T128 U6 words");
            same(c_ref, c_var, n3 * 4, "ham_dense T128 U6 distances");
            CK(hipMemset(c_var, 0, n3 * 4));
            launch_ham_dense<kPathPext, 256, 4, true>(b, 0);
            same(c_ref, c_var, n3 * 4, "ham_dense T256 U4 distances");
        }
        if (pass == 0) {
            G16Args b = make_args(in, n3, L, w_var, ref, c_var, fb);
            CK(hipMemset(w_var, 0, n3 * 24));
            CK(hipMemset(c_var, 0, n3 * 4));
            launch_ham_w3<256, 4, true>(b, 0);
            same(w_ref, w_var, n3 * 24, "ham_w3 T256 U4 words");
            same(c_ref, c_var, n3 * 4, "ham_w3 T256 U4 distances");
            CK(hipMemset(w_var, 0, n3 * 24));
            CK(hipMemset(c_var, 0, n3 * 4));
            hipLaunchKernelGGL((k_ham_wave<6, 8>), dim3((unsigned)((n3 + 511) / 512)), dim3(512), 0, 0, (const uint4*)in,
                               (uint32_t*)w_var, (const uint32_t*)ref, c_var, n3, fb);
            same(w_ref, w_var, n3 * 24, "wave WPB8 words");
            same(c_ref, c_var, n3 * 4, "wave WPB8 distances");
        }
        printf("C3 96-nt fused encode + hamming, %llu reads (pass %d)\n", (unsigned long long)n3, pass);
        timeit("C3 ham_w3 T256 U2", bytes, [&] { launch_ham_w3<256, 2, true>(a, 0); });
        timeit("C3 wave WPB4", bytes, [&] {
            hipLaunchKernelGGL((k_ham_wave<6, 4>), dim3((unsigned)((n3 + 255) / 256)), dim3(256), 0, 0, (const uint4*)in,
                               (uint32_t*)w_var, (const uint32_t*)ref, c_var, n3, fb); });
        timeit("C3 wave WPB2", bytes, [&] {
            hipLaunchKernelGGL((k_ham_wave<6, 2>), dim3((unsigned)((n3 + 127) / 128)), dim3(128), 0, 0, (const uint4*)in,
                               (uint32_t*)w_var, (const uint32_t*)ref, c_var, n3, fb); });
        timeit("C3 wave WPB16", bytes, [&] {
            hipLaunchKernelGGL((k_ham_wave<6, 16>), dim3((unsigned)((n3 + 1023) / 1024)), dim3(1024), 0, 0, (const uint4*)in,
                               (uint32_t*)w_var, (const uint32_t*)ref, c_var, n3, fb); });
        timeit("C3 ham_dense T768 U2 (r1 production)", bytes, [&] { launch_ham_dense<kPathPext, 768, 2, true>(a, 0); });
        timeit("C3 ham_dense T256 U3", bytes, [&] { launch_ham_dense<kPathPext, 256, 3, true>(a, 0); });
        timeit("C3 ham_dense T128 U6", bytes, [&] { launch_ham_dense<kPathPext, 128, 6, true>(a, 0); });
        timeit("C3 ham_dense T384 U2", bytes, [&] { launch_ham_dense<kPathPext, 384, 2, true>(a, 0); });
        timeit("C3 ham_dense T512 U3", bytes, [&] { launch_ham_dense<kPathPext, 512, 3, true>(a, 0); });
        timeit("C3 ham_dense T192 U4", bytes, [&] { launch_ham_dense<kPathPext, 192, 4, true>(a, 0); });
        timeit("C3 ham_dense T128 U3", bytes, [&] { launch_ham_dense<kPathPext, 128, 3, true>(a, 0); });
        timeit("C3 wave WPB8", bytes, [&] {
            hipLaunchKernelGGL((k_ham_wave<6, 8>), dim3((unsigned)((n3 + 511) / 512)), dim3(512), 0, 0, (const uint4*)in,
                               (uint32_t*)w_var, (const uint32_t*)ref, c_var, n3, fb); });
    }
    }
    printf("TUNE_STREAM_DONE\n");
    return 0;
}
