// tools/tune_c3.hip — C3 fused encode + hamming (96 nt, dense): the production kernel k_encode_ham_dense
// (production) in block shapes (T192 U4 stays best of 17; profiles/r4/tune_c3_shapes_r4.log) and a
// no-LDS lane-row form k_encode_ham6w (measured slower:
// 0.772 vs 0.784 of 8 TB/s for the best shape, T256 G1, same box, gpurun_out/tune_c3_6w.log).  Every
// variant's packed words, distances and first-bad read are checked against the production launch
// (ss_encode_hamming_ref) on a tail-heavy small batch with an invalid byte and on the timed batch.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include tools/tune_c3.hip -o tools/tune_c3
#include "../shortseq_amd/csrc/ss_codec.hip"
#include "../shortseq_amd/csrc/ss_runtime.hip"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

namespace {
// Dense fused encode + hamming for 96-nt reads (6 chunks = 3 words) with no LDS and no barrier, in
// k_ham_dense3w's layout: a wave streams groups of 3 whole 1-KiB rows of chunks (192 dwordx4 =
// 32 reads, line-aligned, every lane busy).  Group lane Lg = 64 j + lane holds chunk Lg (chunk
// k = Lg % 6 of read Lg / 6; 64 = 4 mod 6).  Per-chunk distances are summed over lane pairs by one
// DPP op, lane 6m adds the pairs at 6m + 2 and 6m + 4 by shuffle (the two reads that straddle a
// row boundary, Lg = 60..65 and 126..131, take the next row's lanes 0 / 2 by readlane) and stores
// read m's distance.  Loads are unconditional from a clamped chunk index (no per-load branch).
template <int T, int G>
__global__ __launch_bounds__(T) void k_encode_ham6w(G16Args a) {
    constexpr uint32_t NWV = T / 64;
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint64_t nq = a.n * 6, qmax = nq - 1;
    uint4 x[G][3];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const uint64_t q = (((uint64_t)blockIdx.x * G + g) * NWV + wv) * 192 + j * 64 + lane;
            x[g][j] = ld_stream(&a.in[min(q, qmax)]);
        }
    uint32_t rf[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) rf[k] = a.ref32[k];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const uint64_t grp = ((uint64_t)blockIdx.x * G + g) * NWV + wv;
        uint32_t p[3], kk[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const uint64_t q = grp * 192 + j * 64 + lane;
            const bool live = q < nq;
            kk[j] = (lane + 4u * j) % 6u;
            uint32_t bad;
            const uint32_t v = encode_chunk<kPathPext>(x[g][j], kk[j], a, bad);
            report_bad_div(live && bad != 0u, q, 6, a.first_bad);
            if (live && a.out32) st_stream(&a.out32[q], v);
            const uint32_t r = kk[j] == 0 ? rf[0] : kk[j] == 1 ? rf[1] : kk[j] == 2 ? rf[2]
                             : kk[j] == 3 ? rf[3] : kk[j] == 4 ? rf[4] : rf[5];
            const uint32_t d = live ? ham32(v ^ r) : 0u;
            p[j] = d + swap_pair(d);                   // even lanes: chunks Lg, Lg + 1
        }
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            uint32_t p2 = __shfl(p[j], (int)min(lane + 2u, 63u));
            uint32_t p4 = __shfl(p[j], (int)min(lane + 4u, 63u));
            if (j == 0) {           // Lg = 60: chunks 64, 65 are row 1's lanes 0, 1
                const uint32_t n0 = __builtin_amdgcn_readlane(p[1], 0);
                if (lane == 60) p4 = n0;
            } else if (j == 1) {    // Lg = 126: chunks 128..131 are row 2's lanes 0..3
                const uint32_t n0 = __builtin_amdgcn_readlane(p[2], 0), n2 = __builtin_amdgcn_readlane(p[2], 2);
                if (lane == 62) {
                    p2 = n0;
                    p4 = n2;
                }
            }
            if (kk[j] == 0) {
                const uint64_t r = grp * 32 + (64u * j + lane) / 6u;
                if (r < a.n) st_stream(&a.counts[r], p[j] + p2 + p4);
            }
        }
    }
}

// LDS-sum kernel with each read's per-chunk distances padded to 8 bytes: the tail sums a read with
// one 8-B LDS read and two v_sad_u8 instead of cpr byte reads (cpr <= 8)
template <int T, int U>
__global__ __launch_bounds__(T) void k_encode_ham_dense8(G16Args a, uint32_t rpb, float inv_cpr) {
    __shared__ uint64_t part8[T * U / 4];              // >= rpb reads (rpb = T U / cpr, cpr >= 4)
    uint8_t* part = (uint8_t*)part8;
    const uint64_t r0 = (uint64_t)blockIdx.x * rpb;
    const uint32_t nr = (uint32_t)min((uint64_t)rpb, a.n - r0);
    const uint32_t nloc = nr * a.cpr;
    const uint64_t c0 = r0 * a.cpr;
    for (uint32_t i = threadIdx.x; i < rpb; i += T) part8[i] = 0;
    uint4 x[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint32_t cl = j * T + threadIdx.x;
        x[j] = cl < nloc ? ld_stream(&a.in[c0 + cl]) : make_uint4(0x41414141u, 0x41414141u, 0x41414141u, 0x41414141u);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint32_t cl = j * T + threadIdx.x;
        const uint32_t rl = (uint32_t)__fmul_rn(__fadd_rn((float)cl, 0.5f), inv_cpr);
        const uint32_t k = cl - rl * a.cpr;
        uint32_t bad;
        const uint32_t v = encode_chunk<kPathPext>(x[j], k, a, bad);
        const bool live = cl < nloc;
        report_bad(live && bad != 0u, r0 + rl, a.first_bad);
        if (live && a.out32) st_stream(&a.out32[c0 + cl], v);
        if (live && k < a.ham2) part[8 * rl + k] = (uint8_t)ham32(v ^ a.ref32[k]);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nr; i += T) {
        const uint64_t p = part8[i];
        const uint32_t s = __builtin_amdgcn_sad_u8((uint32_t)p, 0u, 0u) + __builtin_amdgcn_sad_u8((uint32_t)(p >> 32), 0u, 0u);
        st_stream(&a.counts[r0 + i], s);
    }
}

// Per-wave LDS form (no block barrier): a wave owns 64 whole reads = 384 consecutive chunks, 6
// coalesced dwordx4 loads per lane; per-chunk distances go to the wave's own 512-B PAD8 LDS slice,
// ordered by a wave barrier only, then lane i sums read i and stores its distance (256-B store).
template <int T>
__global__ __launch_bounds__(T) void k_encode_ham_wave(G16Args a) {
    constexpr uint32_t NWV = T / 64;
    __shared__ uint64_t part8[NWV * 64];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    uint8_t* part = (uint8_t*)(part8 + wv * 64);
    const uint64_t r0 = ((uint64_t)blockIdx.x * NWV + wv) * 64;
    const uint64_t nq = a.n * 6, qmax = nq - 1, c0 = r0 * 6;
    uint4 x[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) x[j] = ld_stream(&a.in[min(c0 + j * 64 + lane, qmax)]);
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        const uint32_t cl = j * 64 + lane, rl = cl / 6u, k = cl - 6u * rl;
        uint32_t bad;
        const uint32_t v = encode_chunk<kPathPext>(x[j], k, a, bad);
        const bool live = c0 + cl < nq;
        report_bad(live && bad != 0u, r0 + rl, a.first_bad);
        if (live && a.out32) st_stream(&a.out32[c0 + cl], v);
        part[8 * rl + k] = (uint8_t)((live && k < a.ham2) ? ham32(v ^ a.ref32[k]) : 0u);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint64_t p = part8[wv * 64 + lane] & 0xFFFFFFFFFFFFull;
    const uint32_t s = __builtin_amdgcn_sad_u8((uint32_t)p, 0u, 0u) + __builtin_amdgcn_sad_u8((uint32_t)(p >> 32), 0u, 0u);
    if (r0 + lane < a.n) st_stream(&a.counts[r0 + lane], s);
}

// Persistent, software-pipelined form of the production kernel (round 5): the grid is the resident
// blocks; each block walks tiles of rpb reads with the NEXT tile's U chunk loads issued before this
// tile's encode / LDS sum / barrier, so the block's epilogue overlaps the next tile's fetch.
template <int T, int U>
__global__ __launch_bounds__(T) void k_encode_ham_pipe(G16Args a, uint32_t rpb, float inv_cpr, uint64_t ntiles) {
    __shared__ uint64_t part8[T * U / 2];
    uint8_t* part = (uint8_t*)part8;
    uint4 xn[U];
    auto load = [&](uint64_t tile, uint4 (&x)[U]) {
        const uint64_t r0 = tile * rpb;
        const uint32_t nr = (uint32_t)min((uint64_t)rpb, a.n - r0);
        const uint32_t nloc = nr * a.cpr;
        const uint64_t c0 = r0 * a.cpr;
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint32_t cl = j * T + threadIdx.x;
            x[j] = cl < nloc ? ld_stream(&a.in[c0 + cl]) : make_uint4(0x41414141u, 0x41414141u, 0x41414141u, 0x41414141u);
        }
    };
    uint64_t tile = blockIdx.x;
    if (tile < ntiles) load(tile, xn);
    for (; tile < ntiles; tile += gridDim.x) {
        uint4 x[U];
#pragma unroll
        for (int j = 0; j < U; ++j) x[j] = xn[j];
        if (tile + gridDim.x < ntiles) load(tile + gridDim.x, xn);
        const uint64_t r0 = tile * rpb;
        const uint32_t nr = (uint32_t)min((uint64_t)rpb, a.n - r0);
        const uint32_t nloc = nr * a.cpr;
        const uint64_t c0 = r0 * a.cpr;
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint32_t cl = j * T + threadIdx.x;
            const uint32_t rl = (uint32_t)__fmul_rn(__fadd_rn((float)cl, 0.5f), inv_cpr);
            const uint32_t k = cl - rl * a.cpr;
            uint32_t bad;
            const uint32_t v = encode_chunk<kPathPext>(x[j], k, a, bad);
            const bool live = cl < nloc;
            report_bad(live && bad != 0u, r0 + rl, a.first_bad);
            if (live && a.out32) st_stream(&a.out32[c0 + cl], v);
            const uint8_t d = (uint8_t)((live && k < a.ham2) ? ham32(v ^ a.ref32[k]) : 0u);
            if (live) part[8 * rl + k] = d;
        }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < nr; i += T) {
            const uint64_t p = part8[i] & (~0ull >> (64 - 8 * a.cpr));
            const uint32_t sum = __builtin_amdgcn_sad_u8((uint32_t)p, 0u, 0u) + __builtin_amdgcn_sad_u8((uint32_t)(p >> 32), 0u, 0u);
            st_stream(&a.counts[r0 + i], sum);
        }
        __syncthreads();
    }
}

// Production kernel with XCD-contiguous block order (block b -> XCD b % 8 gets one contiguous eighth
// of the stream) and/or plain (temporal) loads
template <int T, int U, bool XCDO, bool NTLD>
__global__ __launch_bounds__(T) void k_encode_ham_x(G16Args a, uint32_t rpb, float inv_cpr) {
    __shared__ uint64_t part8[T * U / 2];
    uint8_t* part = (uint8_t*)part8;
    const uint64_t bo = XCDO ? (uint64_t)(blockIdx.x % 8u) * ((gridDim.x + 7u) / 8u) + blockIdx.x / 8u : blockIdx.x;
    const uint64_t r0 = bo * rpb;
    if (r0 >= a.n) return;
    const uint32_t nr = (uint32_t)min((uint64_t)rpb, a.n - r0);
    const uint32_t nloc = nr * a.cpr;
    const uint64_t c0 = r0 * a.cpr;
    uint4 x[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint32_t cl = j * T + threadIdx.x;
        x[j] = cl < nloc ? (NTLD ? ld_stream(&a.in[c0 + cl]) : a.in[c0 + cl])
                         : make_uint4(0x41414141u, 0x41414141u, 0x41414141u, 0x41414141u);
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint32_t cl = j * T + threadIdx.x;
        const uint32_t rl = (uint32_t)__fmul_rn(__fadd_rn((float)cl, 0.5f), inv_cpr);
        const uint32_t k = cl - rl * a.cpr;
        uint32_t bad;
        const uint32_t v = encode_chunk<kPathPext>(x[j], k, a, bad);
        const bool live = cl < nloc;
        report_bad(live && bad != 0u, r0 + rl, a.first_bad);
        if (live && a.out32) st_stream(&a.out32[c0 + cl], v);
        const uint8_t d = (uint8_t)((live && k < a.ham2) ? ham32(v ^ a.ref32[k]) : 0u);
        if (live) part[8 * rl + k] = d;
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nr; i += T) {
        const uint64_t p = part8[i] & (~0ull >> (64 - 8 * a.cpr));
        const uint32_t sum = __builtin_amdgcn_sad_u8((uint32_t)p, 0u, 0u) + __builtin_amdgcn_sad_u8((uint32_t)(p >> 32), 0u, 0u);
        st_stream(&a.counts[r0 + i], sum);
    }
}
}  // namespace

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static G16Args args(const uint8_t* in, uint64_t n, uint64_t* words, const uint64_t* ref, uint32_t* out, uint64_t* fb) {
    G16Args a;
    a.in = (const uint4*)in;
    a.in_stride16 = 6;
    a.out32 = (uint32_t*)words;
    a.wpr2 = 6;
    a.n = n;
    a.cpr = 6;
    a.full2 = 6;
    a.all_table = 0;
    a.logG = 3;
    a.ref32 = (const uint32_t*)ref;
    a.ham2 = 6;
    a.counts = out;
    a.first_bad = (unsigned long long*)fb;
    return a;
}

template <int T, int U>
static void v8(const uint8_t* in, uint64_t n, uint64_t* words, const uint64_t* ref, uint32_t* out, uint64_t* fb) {
    reset_first_bad(fb, 0);
    const uint32_t rpb = (U * T) / 6;
    hipLaunchKernelGGL((k_encode_ham_dense8<T, U>), dim3((unsigned)((n + rpb - 1) / rpb)), dim3(T), 0, 0,
                       args(in, n, words, ref, out, fb), rpb, 1.0f / 6.0f);
}

template <int T, int U>
static void vp(const uint8_t* in, uint64_t n, uint64_t* words, const uint64_t* ref, uint32_t* out, uint64_t* fb) {
    reset_first_bad(fb, 0);
    launch_ham_dense<kPathPext, T, U, true>(args(in, n, words, ref, out, fb), 0);
}

template <int T, int G>
static void v6w(const uint8_t* in, uint64_t n, uint64_t* words, const uint64_t* ref, uint32_t* out, uint64_t* fb) {
    reset_first_bad(fb, 0);
    const uint64_t per = (uint64_t)32 * (T / 64) * G;
    hipLaunchKernelGGL((k_encode_ham6w<T, G>), dim3((unsigned)((n + per - 1) / per)), dim3(T), 0, 0,
                       args(in, n, words, ref, out, fb));
}

static void prod(const uint8_t* in, uint64_t n, uint64_t* words, const uint64_t* ref, uint32_t* out, uint64_t* fb) {
    if (ss_encode_hamming_ref(in, n, 96, 96, words, 3, ref, out, fb, 0)) { printf("prod failed\n"); exit(1); }
}

template <int T>
static void vw(const uint8_t* in, uint64_t n, uint64_t* words, const uint64_t* ref, uint32_t* out, uint64_t* fb) {
    reset_first_bad(fb, 0);
    const uint64_t per = (uint64_t)64 * (T / 64);
    hipLaunchKernelGGL((k_encode_ham_wave<T>), dim3((unsigned)((n + per - 1) / per)), dim3(T), 0, 0,
                       args(in, n, words, ref, out, fb));
}

template <int T, int U, int BPC>
static void vpipe(const uint8_t* in, uint64_t n, uint64_t* words, const uint64_t* ref, uint32_t* out, uint64_t* fb) {
    reset_first_bad(fb, 0);
    const uint32_t rpb = (U * T) / 6;
    const uint64_t ntiles = (n + rpb - 1) / rpb;
    hipLaunchKernelGGL((k_encode_ham_pipe<T, U>), dim3(256 * BPC), dim3(T), 0, 0, args(in, n, words, ref, out, fb), rpb,
                       1.0f / 6.0f, ntiles);
}

template <int T, int U, bool XCDO, bool NTLD>
static void vx(const uint8_t* in, uint64_t n, uint64_t* words, const uint64_t* ref, uint32_t* out, uint64_t* fb) {
    reset_first_bad(fb, 0);
    const uint32_t rpb = (U * T) / 6;
    unsigned grid = (unsigned)((n + rpb - 1) / rpb);
    if (XCDO) grid = (grid + 7u) / 8u * 8u;
    hipLaunchKernelGGL((k_encode_ham_x<T, U, XCDO, NTLD>), dim3(grid), dim3(T), 0, 0, args(in, n, words, ref, out, fb), rpb,
                       1.0f / 6.0f);
}

typedef void (*Fn)(const uint8_t*, uint64_t, uint64_t*, const uint64_t*, uint32_t*, uint64_t*);

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 30;
    const uint64_t n = argc > 2 ? strtoull(argv[2], 0, 10) : 100000000ull;
    const uint64_t ns = 1000003;   // small check batch: tails, an invalid byte
    uint8_t* in;
    uint64_t *w0, *w1, *ref, *fb;
    uint32_t *d0, *d1;
    CK(hipMalloc(&in, n * 96));
    CK(hipMalloc(&w0, n * 24));
    CK(hipMalloc(&w1, n * 24));
    CK(hipMalloc(&ref, 24));
    CK(hipMalloc(&fb, 8));
    CK(hipMalloc(&d0, n * 4));
    CK(hipMalloc(&d1, n * 4));
    if (ss_synth_reads(in, 7, 0, n, 96, 96, 0)) { printf("synth failed\n"); exit(1); }
    prod(in, n, w0, w0, d0, fb);           // words of read 12345 as the reference
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(ref, w0 + 3 * 12345, 24, hipMemcpyDeviceToDevice));
    const struct { const char* name; Fn f; } vs[] = {
        {"prod k_encode_ham_dense<192,4>", prod},
        {"x T192 U4 xcd", vx<192, 4, true, true>}, {"x T192 U4 temporal-ld", vx<192, 4, false, false>},
        {"x T192 U4 xcd temporal-ld", vx<192, 4, true, false>}, {"x T192 U4 (same as prod)", vx<192, 4, false, true>},
        {"x T256 U3 xcd", vx<256, 3, true, true>},
        {"prod T128 U3", vp<128, 3>}, {"prod T96 U4", vp<96, 4>}, {"prod T192 U2", vp<192, 2>},
        {"prod T64 U6", vp<64, 6>}, {"prod T128 U6", vp<128, 6>}, {"prod T256 U3", vp<256, 3>},
        {"prod T64 U3", vp<64, 3>},
        {"prod T256 U6", vp<256, 6>}, {"prod T384 U2", vp<384, 2>}, {"prod T384 U4", vp<384, 4>},
        {"prod T512 U3", vp<512, 3>}, {"prod T768 U2", vp<768, 2>}, {"prod T1024 U3", vp<1024, 3>},
        {"prod T192 U8", vp<192, 8>}, {"prod T96 U8", vp<96, 8>},
    };
    const int nv = sizeof(vs) / sizeof(vs[0]);
    // correctness: small batch with an invalid byte in read 777777 (chunk 4), then the full batch
    std::vector<uint8_t> hb(1);
    bool all_ok = true;
    for (int pass = 0; pass < 2; ++pass) {
        const uint64_t m = pass == 0 ? ns : n;
        if (pass == 0) { uint8_t nb = 'N'; CK(hipMemcpy(in + 777777ull * 96 + 70, &nb, 1, hipMemcpyHostToDevice)); }
        std::vector<uint32_t> hd0(m), hd1(m);
        std::vector<uint64_t> hw0(m * 3), hw1(m * 3);
        uint64_t f0, f1;
        prod(in, m, w0, ref, d0, fb);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(hd0.data(), d0, m * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hw0.data(), w0, m * 24, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&f0, fb, 8, hipMemcpyDeviceToHost));
        for (int v = 1; v < nv; ++v) {
            CK(hipMemset(d1, 0xAB, m * 4));
            CK(hipMemset(w1, 0xAB, m * 24));
            vs[v].f(in, m, w1, ref, d1, fb);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(hd1.data(), d1, m * 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(hw1.data(), w1, m * 24, hipMemcpyDeviceToHost));
            CK(hipMemcpy(&f1, fb, 8, hipMemcpyDeviceToHost));
            const bool ok = hd0 == hd1 && hw0 == hw1 && f0 == f1;
            all_ok &= ok;
            printf("check n=%llu %-32s %s (first_bad %llu vs %llu)\n", (unsigned long long)m, vs[v].name,
                   ok ? "OK" : "MISMATCH", (unsigned long long)f1, (unsigned long long)f0);
        }
        if (pass == 0) { uint8_t ab = 'A'; CK(hipMemcpy(in + 777777ull * 96 + 70, &ab, 1, hipMemcpyHostToDevice)); }
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = 124.0 * (double)n;
    for (int round = 0; round < 3; ++round) {
        for (int v = 0; v < nv; ++v) {
            for (int i = 0; i < 5; ++i) vs[v].f(in, n, w1, ref, d1, fb);
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < reps; ++i) vs[v].f(in, n, w1, ref, d1, fb);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ms /= reps;
            printf("round %d %-32s %.4f ms  %.0f GB/s  frac %.3f\n", round, vs[v].name, ms, bytes / ms / 1e6,
                   bytes / ms / 1e6 / 8000.0);
        }
    }
    printf(all_ok ? "ALL OK\n" : "SOME MISMATCH\n");
    return all_ok ? 0 : 2;
}
