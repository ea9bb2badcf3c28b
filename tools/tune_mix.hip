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
// and for ss_encode_var (flat at 0.67, bound unnamed), on the F2 batch (50M
// ragged reads of 50-150 nt, wpr 5):
//   var_pattern  k_encode_var_dense's exact access pattern (a lane per output word, its read's offset
//                and length, the three 16-B chunks holding the word) with the encode replaced by a
//                XOR fold: if it runs at the production kernel's rate, the pattern bounds it
//   var_dense    the same bytes as one dense stream (blob + offsets + lengths in, wpr words out)
// Prints ms and the fraction of 8 TB/s over each kernel's bytes (min over reps).
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include tools/tune_mix.hip -o tools/tune_mix
//   tools/tune_mix [reps=20]
#include "../shortseq_amd/csrc/ss_codec.hip"
#include "../shortseq_amd/csrc/ss_runtime.hip"

#include <stdio.h>
#include <stdlib.h>

#include <vector>

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

// k_encode_var_dense with the encode math removed (see the header): kVarK = 2 words per lane
__global__ __launch_bounds__(256) void k_var_pattern(const uint8_t* in, const uint64_t* __restrict__ offs,
                                                     const uint32_t* __restrict__ lens, uint64_t n,
                                                     uint64_t* __restrict__ out, uint32_t wpr, double inv_wpr) {
    constexpr int K = 2;
    const uint64_t total = n * wpr;
    const uint64_t base = ((uint64_t)blockIdx.x * 256 + (threadIdx.x & ~63u)) * K + (threadIdx.x & 63u);
    uint64_t r[K], off[K];
    uint32_t w[K], L[K], nb[K];
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
    uint4 c0[K], c1[K], c2[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        nb[k] = 32u * w[k] < L[k] ? min(32u, L[k] - 32u * w[k]) : 0u;
        c0[k] = c1[k] = c2[k] = make_uint4(0u, 0u, 0u, 0u);
        if (nb[k]) {
            const uintptr_t addr = (uintptr_t)(in + off[k] + 32u * w[k]);
            const uint4* q = (const uint4*)(addr & ~(uintptr_t)15);
            const uint32_t last = ((uint32_t)(addr & 15) + nb[k] - 1u) >> 4;
            c0[k] = q[0];
            c1[k] = q[min(1u, last)];
            c2[k] = q[min(2u, last)];
        }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t g = base + 64u * k;
        if (g >= total) continue;
        const uint32_t lo = c0[k].x ^ c1[k].y ^ c2[k].z ^ c0[k].w, hi = c1[k].x ^ c2[k].y ^ c0[k].z ^ c2[k].w;
        out[g] = nb[k] ? ((uint64_t)hi << 32 | lo) : 0ull;
    }
}

// a dense stream of the same bytes: nch 16-B chunks read, nout 8-B words written (4 words per lane)
__global__ __launch_bounds__(256) void k_var_dense(const uint4* __restrict__ in, uint64_t nch, uint64_t* __restrict__ out,
                                                   uint64_t nout) {
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x, nt = (uint64_t)gridDim.x * 256;
    uint32_t acc = 0;
    for (uint64_t c = t; c < nch; c += nt) {
        const uint4 v = ld_stream(&in[c]);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    for (uint64_t o = t; o < nout; o += nt) out[o] = acc + o;
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
    {   // ss_encode_var on the F2 batch (bench.py bench_ragged: seed 41, pool 42, 2^20 items, 50-150 nt)
        const uint64_t nv = 50000000ull;
        const uint32_t wpr = 5;
        uint32_t* lens;
        uint64_t *offs, *out;
        CK(hipMalloc(&lens, nv * 4));
        CK(hipMalloc(&offs, nv * 8));
        CS(ss_synth_ragged_lens(lens, 41, 42, 1u << 20, 0, nv, 50, 150, nullptr));
        std::vector<uint32_t> hl(nv);
        std::vector<uint64_t> ho(nv);
        CK(hipMemcpy(hl.data(), lens, nv * 4, hipMemcpyDeviceToHost));
        uint64_t tot = 0;
        for (uint64_t i = 0; i < nv; ++i) {
            ho[i] = tot;
            tot += hl[i];
        }
        CK(hipMemcpy(offs, ho.data(), nv * 8, hipMemcpyHostToDevice));
        uint8_t* blob;
        CK(hipMalloc(&blob, tot + 12 * nv + 64));     // (var_dense streams blob-sized + metadata-sized bytes)
        CS(ss_synth_ragged_reads(blob, offs, 41, 42, 1u << 20, 0, nv, 50, 150, nullptr));
        CK(hipMalloc(&out, nv * wpr * 8));
        CK(hipDeviceSynchronize());
        const double bv = (double)tot + 12.0 * nv + 8.0 * wpr * nv;
        printf("F2 batch: %llu reads, %.3f GB blob, algorithmic %.3f GB per call\n", (unsigned long long)nv, tot * 1e-9, bv * 1e-9);
        const double inv = 1.0 / wpr;
        const uint64_t words = nv * wpr;
        const unsigned grid = (unsigned)((words + 511) / 512);
        timeit("prod ss_encode_var", bv, [&] { CS(ss_encode_var(blob, offs, lens, nv, out, wpr, fb, nullptr)); });
        timeit("var_pattern (no encode)", bv, [&] {
            hipLaunchKernelGGL(k_var_pattern, dim3(grid), dim3(256), 0, 0, (const uint8_t*)blob, (const uint64_t*)offs,
                               (const uint32_t*)lens, nv, out, wpr, inv);
        });
        const uint64_t nch = ((uint64_t)tot + 12ull * nv + 15) / 16;
        timeit("var_dense (same bytes)", bv, [&] {
            hipLaunchKernelGGL(k_var_dense, dim3(8192), dim3(256), 0, 0, (const uint4*)blob, nch,
                               out, words);
        });
        timeit("prod ss_encode_var", bv, [&] { CS(ss_encode_var(blob, offs, lens, nv, out, wpr, fb, nullptr)); });
        CK(hipFree(blob));
        CK(hipFree(lens));
        CK(hipFree(offs));
        CK(hipFree(out));
    }
    return 0;
}
