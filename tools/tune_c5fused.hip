// tools/tune_c5fused.hip — experiment: cut the C5 fine scatter (a pass over 12 B read + 12 B written
// per read) by partitioning the coarse pass into 1024 bins (10 of the 14 region bits) and letting
// the aggregate read a bin's records directly.  A bin's table slice (16 regions of 2048 slots) does
// not fit one workgroup's LDS, so G regions per workgroup and 16 / G workgroups per bin each read
// the whole bin and keep their regions (the other reads of a bin should hit L2 / MALL: the bin's
// workgroups are placed on one XCD and dispatched back to back).
//   prod : ss_counter_insert_fixed (coarse + order + fine scatter + aggregate), same box
//   xG   : k_x_coarse (1024 bins x 8 per-XCD sub-bins, one 64-bit atomic per (tile, bin pair))
//          + k_x_agg<G> (fresh slices); uniform pool, no dedup / spill (measurement only)
// The tables are compared by an order-independent signature of their (key, count, first) slots.
//
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include tools/tune_c5fused.hip \
//          shortseq_amd/csrc/ss_codec.hip shortseq_amd/csrc/ss_runtime.hip -o tools/tune_c5fused
#include "../shortseq_amd/csrc/ss_counter.hip"

namespace {
// the whole linear probe of the production aggregate's rule (ss_counter.hip now probes per round)
template <int G>
__device__ __forceinline__ uint32_t lds_probe(unsigned long long* skey, uint32_t mask, uint32_t off, uint64_t key) {
    uint32_t done = 0, at;
    while (!lds_probe_round<G>(skey, mask, kEmpty, key, off, done, at)) {
    }
    return at;
}
}  // namespace

#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
#define CS(x) do { int r_ = (x); if (r_) { printf("ss error %d: %s @%d\n", r_, ss_last_error_string(), __LINE__); exit(1); } } while (0)

namespace {
constexpr uint32_t kXB = 10, kXNB = 1u << kXB, kXSub = 8, kXPairs = kXNB / 2;

template <int T, int RPL>
__global__ __launch_bounds__(T) __attribute__((amdgpu_waves_per_eu(4))) void k_x_coarse(
        Tbl t, uint32_t rbits, Rec12* __restrict__ out, uint64_t cap, unsigned long long* __restrict__ fill,
        const uint4* __restrict__ in, uint64_t n, unsigned long long* ovf, unsigned long long* first_bad) {
    constexpr uint32_t TILE = T * RPL;
    static_assert(T * 2 == kXNB, "thread t scans bins 2t, 2t + 1");
    __shared__ uint32_t lcount[kXNB], lstart[kXNB], gbase[kXNB];
    __shared__ uint32_t wsum[T / 64];
    __shared__ uint64_t skey[TILE];
    __shared__ uint32_t sidx[TILE];
    __shared__ uint16_t sbin[TILE];
    const uint32_t shift = rbits - kXB;
    const uint64_t tiles = (n + TILE - 1) / TILE;
    const uint32_t sub = blockIdx.x % kXSub;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    for (uint32_t i = threadIdx.x; i < kXNB; i += T) lcount[i] = 0;
    __syncthreads();
    uint4 nx[RPL][2];
    for (uint64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
        const uint64_t t0 = tile * TILE;
#pragma unroll
        for (int j = 0; j < RPL; ++j) {
            const uint64_t r = min(t0 + j * T + threadIdx.x, n - 1);
            nx[j][0] = ld_stream(&in[r * 2]);
            nx[j][1] = ld_stream(&in[r * 2 + 1]);
        }
        const uint32_t cnt = (uint32_t)min((uint64_t)TILE, n - t0);
        uint64_t key[RPL];
        uint32_t bin[RPL], rank[RPL];
#pragma unroll
        for (int j = 0; j < RPL; ++j) {
            const uint64_t r = t0 + j * T + threadIdx.x;
            const Enc32 a = encode16(nx[j][0].x, nx[j][0].y, nx[j][0].z, nx[j][0].w, true);
            const Enc32 b = encode16(nx[j][1].x, nx[j][1].y, nx[j][1].z, nx[j][1].w, true);
            const bool live = r < n;
            report_bad(live && (a.bad | b.bad) != 0u, r, first_bad);
            key[j] = (uint64_t)a.v | ((uint64_t)(b.v | a.cout) << 32);
            bin[j] = region_of(t, key[j]) >> shift;
            if (live) rank[j] = atomicAdd(&lcount[bin[j]], 1u);
        }
        __syncthreads();                                                  // (A)
        {
            const uint32_t b0 = 2 * threadIdx.x;
            const uint32_t c0 = lcount[b0], c1 = lcount[b0 + 1];
            uint32_t incl = c0 + c1;
            for (uint32_t off = 1; off < 64; off <<= 1) {
                const uint32_t y = __shfl_up(incl, off);
                if (lane >= off) incl += y;
            }
            if (lane == 63) wsum[wave] = incl;
            const uint32_t excl = incl - c0 - c1;
            lstart[b0] = excl;
            lstart[b0 + 1] = excl + c0;
            const uint64_t add = (uint64_t)c0 | ((uint64_t)c1 << 32);
            const uint64_t g2 = add ? atomicAdd(&fill[sub * kXPairs + threadIdx.x], (unsigned long long)add) : 0ull;
            gbase[b0] = (uint32_t)g2;
            gbase[b0 + 1] = (uint32_t)(g2 >> 32);
            lcount[b0] = 0;
            lcount[b0 + 1] = 0;
        }
        __syncthreads();                                                  // (B)
        uint32_t wp[T / 64];
        {
            uint32_t run = 0;
#pragma unroll
            for (int w = 0; w < T / 64; ++w) {
                wp[w] = run;
                run += wsum[w];
            }
        }
        auto wpre = [&](uint32_t b) {   // exclusive prefix of the waves before bin b's scanning wave
            uint32_t v = 0;
#pragma unroll
            for (int w = 0; w < T / 64; ++w)
                if ((uint32_t)w == (b >> 7)) v = wp[w];
            return v;
        };
#pragma unroll
        for (int j = 0; j < RPL; ++j) {
            const uint32_t e = j * T + threadIdx.x;
            if (e < cnt) {
                const uint32_t sp = lstart[bin[j]] + wpre(bin[j]) + rank[j];
                skey[sp] = key[j];
                sidx[sp] = (uint32_t)(t0 + e);
                sbin[sp] = (uint16_t)bin[j];
            }
        }
        __syncthreads();                                                  // (C)
        for (uint32_t i = threadIdx.x; i < cnt; i += T) {
            const uint32_t b = sbin[i];
            const uint32_t local = i - (lstart[b] + wpre(b));
            const uint64_t pos = (uint64_t)gbase[b] + local;
            const uint64_t k = skey[i];
            if (pos < cap) {
                Rec12 r;
                r.klo = (uint32_t)k;
                r.khi = (uint32_t)(k >> 32);
                r.idx = sidx[i];
                out[(uint64_t)(b * kXSub + sub) * cap + pos] = r;
            } else {
                atomicOr(ovf, 1ull);
            }
        }
    }
}

// workgroup -> (bin, group q of G regions): the 16 / G workgroups of a bin sit on one XCD
// (blockIdx % 8) and are dispatched back to back
template <int T, int G>
__global__ __launch_bounds__(T) void k_x_agg(Tbl t, uint32_t rbits, const Rec12* __restrict__ rec, uint64_t cap,
                                             const unsigned long long* __restrict__ fill) {
    constexpr uint32_t S = 2048, Q = (1u << 4) / G;   // 16 regions per bin
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned long long* skey = (unsigned long long*)smem;   // [G S]
    uint32_t* bcnt = (uint32_t*)(skey + G * S);
    uint32_t* bfst = bcnt + G * S;
    const uint32_t xcd = blockIdx.x % 8, j = blockIdx.x / 8;
    const uint32_t bin = xcd + 8 * (j / Q), q = j % Q;
    const uint32_t region0 = bin * 16 + q * G;
    const uint32_t rshift = 64 - rbits;   // region of a key = top rbits of the slot hash
    for (uint32_t i = threadIdx.x; i < G * S; i += T) {
        skey[i] = kEmpty;
        bcnt[i] = 0;
        bfst[i] = 0xFFFFFFFFu;
    }
    uint32_t seg0[kXSub], pre[kXSub + 1];
    pre[0] = 0;
#pragma unroll
    for (uint32_t s = 0; s < kXSub; ++s) {
        const unsigned long long w = fill[s * kXPairs + bin / 2];
        const uint32_t f = (uint32_t)(bin & 1u ? (w >> 32) : w);
        seg0[s] = (bin * kXSub + s) * (uint32_t)cap;
        pre[s + 1] = pre[s] + (uint32_t)min((uint64_t)f, cap);
    }
    __syncthreads();
    const uint32_t total = pre[kXSub];
    auto flat_at = [&](uint32_t f) -> uint32_t {
        uint32_t e = seg0[0] + f;
#pragma unroll
        for (uint32_t s = 1; s < kXSub; ++s)
            if (f >= pre[s]) e = seg0[s] + (f - pre[s]);
        return e;
    };
    constexpr int kP = 4;
    uint64_t nkey[kP];
    uint32_t nidx[kP];
    auto load_step = [&](uint32_t e0) {
#pragma unroll
        for (int p = 0; p < kP; ++p) {
            const uint32_t f = min(e0 + p * T + threadIdx.x, total - 1u);
            const Rec12 r = rec[flat_at(f)];
            nkey[p] = ((uint64_t)r.khi << 32) | r.klo;
            nidx[p] = r.idx;
        }
    };
    if (total) load_step(0);
    for (uint32_t e0 = 0; e0 < total; e0 += kP * T) {
        uint64_t key[kP];
        uint32_t idx[kP];
#pragma unroll
        for (int p = 0; p < kP; ++p) {
            key[p] = nkey[p];
            idx[p] = nidx[p];
        }
        load_step(e0 + kP * T);
#pragma unroll
        for (int p = 0; p < kP; ++p) {
            const bool valid = e0 + p * T + threadIdx.x < total;
            const uint64_t h = slot_top(t, key[p]);
            const uint32_t lr = (uint32_t)(h >> t.slice_log) - region0;
            if (!valid || lr >= G || key[p] == kEmpty) continue;
            unsigned long long* sk = skey + lr * S;
            const uint32_t off = lds_probe<kAggProbe>(sk, S - 1, (uint32_t)(h & (S - 1)), key[p]);
            if (off == S) {
                atomicOr(t.overflow, kOvfTable);
                continue;
            }
            atomicAdd(&bcnt[lr * S + off], 1u);
            atomicMin(&bfst[lr * S + off], idx[p]);
        }
    }
    (void)rshift;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < G * S; i += T) {
        const unsigned long long k = skey[i];
        const uint32_t bc = bcnt[i];
        uint4* sl = (uint4*)&t.slots[((uint64_t)region0 << t.slice_log) + i];
        *sl = make_uint4((uint32_t)k, (uint32_t)(k >> 32), ~bc, bc ? bfst[i] : kNoFirst);
    }
}

__global__ void k_sig(Tbl t, unsigned long long* out) {
    unsigned long long s = 0, u = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= t.mask; i += (uint64_t)gridDim.x * blockDim.x) {
        const Slot sl = t.slots[i];
        if (sl.key == kEmpty) continue;
        s += splitmix64(sl.key ^ splitmix64(((uint64_t)~sl.ncount << 32) | sl.first));
        u += 1;
    }
    atomicAdd(&out[0], s);
    atomicAdd(&out[1], u);
}
}  // namespace

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 125000000ull;
    const int reps = argc > 2 ? atoi(argv[2]) : 10;
    const int modes = argc > 3 ? atoi(argv[3]) : 15;   // bit m: run mode m
    const uint64_t U = 1ull << 24;
    uint8_t* ascii;
    uint64_t* fb;
    CK(hipMalloc(&ascii, n * 32));
    CK(hipMalloc(&fb, 16));
    CS(ss_synth_pool_reads(ascii, 5, 77, U, 0, n, 32, 32, nullptr));
    ss_counter *cp, *cx;
    CS(ss_counter_create(2 * U, &cp));
    CS(ss_counter_create(2 * U, &cx));
    CS(ss_counter_reserve(cp, n));
    const Tbl tx = tbl_of(cx);
    const uint32_t rbits = cx->log2cap - cx->slice_log;
    if (rbits != 14 || cx->slice_log != 11) {
        printf("unexpected geometry rbits %u slice_log %u\n", rbits, cx->slice_log);
        return 1;
    }
    const uint64_t capx = ((5 * n / 2 + kXNB * kXSub - 1) / (kXNB * kXSub) + 256 + 15) & ~15ull;
    Rec12* xrec;
    unsigned long long *xfill, *xovf, *sig;
    CK(hipMalloc(&xrec, (size_t)kXNB * kXSub * capx * sizeof(Rec12)));
    CK(hipMalloc(&xfill, (size_t)kXSub * kXPairs * 8));
    CK(hipMalloc(&xovf, 8));
    CK(hipMalloc(&sig, 16));
    CK(hipMemset(xovf, 0, 8));
    int dev = 0, cus = 0, per = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)k_x_coarse<512, 8>, 512, 0));
    const int cgrid = cus * per;
    printf("coarse: %d CUs x %d blocks, capx %llu records per sub-bin\n", cus, per, (unsigned long long)capx);
    CK(hipFuncSetAttribute((const void*)k_x_agg<512, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, 4 * 2048 * 16));
    CK(hipFuncSetAttribute((const void*)k_x_agg<512, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * 2048 * 16));
    CK(hipFuncSetAttribute((const void*)k_x_agg<1024, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, 4 * 2048 * 16));
    hipEvent_t e0, e1, e2;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreate(&e2));
    auto signature = [&](const Tbl& t, unsigned long long (&h)[2]) {
        CK(hipMemset(sig, 0, 16));
        hipLaunchKernelGGL(k_sig, dim3(2048), dim3(256), 0, 0, t, sig);
        CK(hipMemcpy(h, sig, 16, hipMemcpyDeviceToHost));
    };
    unsigned long long hp[2] = {0, 0};
    const char* names[4] = {"prod", "x4 T512", "x2 T512", "x4 T1024"};
    for (int mode = 0; mode < 4; ++mode) {
        if (!((modes >> mode) & 1)) continue;
        double tc = 0, ta = 0;
        for (int r = -2; r < reps; ++r) {
            CK(hipDeviceSynchronize());
            if (mode == 0) {
                CS(ss_counter_reset(cp, nullptr));
                CK(hipEventRecord(e0, 0));
                CS(ss_counter_insert_fixed(cp, ascii, n, 32, 32, 0, fb, nullptr));
                CK(hipEventRecord(e1, 0));
                CK(hipEventRecord(e2, 0));
            } else {
                CK(hipEventRecord(e0, 0));
                CK(hipMemsetAsync(xfill, 0, (size_t)kXSub * kXPairs * 8, 0));
                hipLaunchKernelGGL((k_x_coarse<512, 8>), dim3(cgrid), dim3(512), 0, 0, tx, rbits, xrec, capx, xfill,
                                   (const uint4*)ascii, n, xovf, (unsigned long long*)fb);
                CK(hipEventRecord(e1, 0));
                if (mode == 1)
                    hipLaunchKernelGGL((k_x_agg<512, 4>), dim3(kXNB * 4), dim3(512), 4 * 2048 * 16, 0, tx, rbits, xrec,
                                       capx, (const unsigned long long*)xfill);
                else if (mode == 2)
                    hipLaunchKernelGGL((k_x_agg<512, 2>), dim3(kXNB * 8), dim3(512), 2 * 2048 * 16, 0, tx, rbits, xrec,
                                       capx, (const unsigned long long*)xfill);
                else
                    hipLaunchKernelGGL((k_x_agg<1024, 4>), dim3(kXNB * 4), dim3(1024), 4 * 2048 * 16, 0, tx, rbits,
                                       xrec, capx, (const unsigned long long*)xfill);
                CK(hipEventRecord(e2, 0));
            }
            CK(hipEventSynchronize(e2));
            CK(hipGetLastError());
            float m1, m2;
            CK(hipEventElapsedTime(&m1, e0, e1));
            CK(hipEventElapsedTime(&m2, e1, e2));
            if (r >= 0) {
                tc += m1;
                ta += m2;
            }
        }
        unsigned long long h[2];
        signature(mode == 0 ? tbl_of(cp) : tx, h);
        if (mode == 0) {
            hp[0] = h[0];
            hp[1] = h[1];
        }
        unsigned long long ov = 0;
        CK(hipMemcpy(&ov, xovf, 8, hipMemcpyDeviceToHost));
        printf("%-9s %s  part1 %.3f ms  part2 %.3f ms  total %.3f ms  (used %llu, sig %016llx, ovf %llu)\n", names[mode],
               (h[0] == hp[0] && h[1] == hp[1]) ? "OK " : "BAD", tc / reps, ta / reps, (tc + ta) / reps, h[1], h[0], ov);
        fflush(stdout);
    }
    return 0;
}
