// tools/tune_c5u.hip — experiment: C5 partition passes WITHOUT the LDS tile staging.
//
// The production k_pf_coarse / k_pf_scatter stage every tile bin-sorted in LDS so that the record
// stores are coalesced; that costs an LDS write + read of each record and a block barrier per
// phase.  Here each lane stores its own 12-B record at gbase[bin] + rank (the rank from the LDS
// histogram atomic): a run of one bin in one tile is still written whole (by several lanes / waves),
// so the XCD's L2 merges the partial lines before they leave; LDS holds only the histograms and a
// small dedup table, so occupancy is set by VGPRs alone.
//
// Build:  hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include tools/tune_c5u.hip \
//           shortseq_amd/csrc/ss_codec.hip shortseq_amd/csrc/ss_runtime.hip -o tools/tune_c5u
// Run:    tools/tune_c5u [n=125M] [reps=10] [U_log2=24] [zipf_s=0]
#include "../shortseq_amd/csrc/ss_counter.hip"

#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <vector>
#include <algorithm>

#ifndef CU_T
#define CU_T 512
#endif
#ifndef CU_RPL
#define CU_RPL 8
#endif
#ifndef CU_HT
#define CU_HT 512
#endif
#ifndef FU_T
#define FU_T 512
#endif
#ifndef FU_RPL
#define FU_RPL 8
#endif
#ifndef FU_HT
#define FU_HT 512
#endif
#ifndef CU_WPE
#define CU_WPE 1
#endif
#ifndef FU_WPE
#define FU_WPE 1
#endif

namespace {

constexpr uint32_t ilog2c(uint32_t v) { return v <= 1 ? 0 : 1 + ilog2c(v >> 1); }

// LDS dedup table insert: the entry holding `key` (claimed with a CAS when new); -1 when the probe
// limit is reached (the element then leaves as its own record)
template <uint32_t HT>
__device__ __forceinline__ int ht_insert(unsigned long long* hkey, uint32_t* hc, uint32_t* hi, uint64_t key,
                                         uint32_t c, uint32_t idx) {
    constexpr uint32_t kLog = ilog2c(HT);
    uint32_t h = dedup_home(key, kLog);
#pragma unroll 1
    for (uint32_t p = 0; p < 32; ++p) {
        unsigned long long cur = hkey[h];
        if (cur == kEmpty) cur = atomicCAS(&hkey[h], (unsigned long long)kEmpty, (unsigned long long)key);
        if (cur == kEmpty || cur == key) {
            atomicAdd(&hc[h], c);
            atomicMin(&hi[h], idx);
            return (int)h;
        }
        h = (h + 1) & (HT - 1);
    }
    return -1;
}

template <int T, int RPL, uint32_t HT>
__global__ __launch_bounds__(T) __attribute__((amdgpu_waves_per_eu(CU_WPE))) void k_cu(
        Tbl t, PartWs w, const uint4* __restrict__ in, uint64_t stride16, uint64_t n, uint32_t cpr,
        uint64_t cap1, uint32_t* fill, unsigned long long* first_bad) {
    constexpr uint32_t TILE = T * RPL;
    __shared__ uint32_t lcount[kCB], gbase[kCB], sbase[kCB], hcnt[kCB];
    __shared__ uint8_t hflag[kCB];
    __shared__ uint32_t any_heavy;
    __shared__ unsigned long long hkey[HT];
    __shared__ uint32_t hc[HT], hix[HT];
    uint32_t* spill_ctr = fill + fill_at(kSpillCtr);
    const uint32_t shift = w.rbits - kCoarseBits;
    const uint64_t tiles = (n + TILE - 1) / TILE;
    const uint32_t sub = blockIdx.x % kFinePerBin;
    const uint32_t hi16 = cpr > 1 ? 1u : 0u;
    Rec12* const arec = (Rec12*)w.akey;
    for (uint32_t i = threadIdx.x; i < kCB; i += T) {
        lcount[i] = 0;
        hcnt[i] = 0;
    }
    for (uint32_t i = threadIdx.x; i < HT; i += T) {
        hkey[i] = kEmpty;
        hc[i] = 0;
        hix[i] = 0xFFFFFFFFu;
    }
    __syncthreads();
    auto reserve = [&](uint32_t b0, uint32_t c0, uint32_t c1, uint32_t mask) {
        const uint64_t add = ((mask & 1u) ? (uint64_t)c0 : 0ull) | ((mask & 2u) ? (uint64_t)c1 << 32 : 0ull);
        const uint64_t g2 = add ? atomicAdd((unsigned long long*)&fill[fill_at(b0 * kFinePerBin + sub)],
                                            (unsigned long long)add) : 0ull;
#pragma unroll
        for (uint32_t k = 0; k < 2; ++k) {
            if (!(mask & (1u << k))) continue;
            const uint32_t g = (uint32_t)(g2 >> (32 * k)), c = k ? c1 : c0;
            gbase[b0 + k] = g;
            const uint64_t end = (uint64_t)g + c, from = max((uint64_t)g, cap1);
            sbase[b0 + k] = end > from ? atomicAdd(spill_ctr, (uint32_t)(end - from)) : 0u;
        }
    };
    auto emit = [&](uint32_t b, uint32_t pos, uint64_t k, uint32_t idx, uint32_t c) {
        if (pos < cap1) {
            const uint64_t at = (uint64_t)(b * kFinePerBin + sub) * cap1 + pos;
            Rec12 r;
            r.klo = (uint32_t)k;
            r.khi = (uint32_t)(k >> 32);
            r.idx = c > 1 ? (idx | kWeighted) : idx;
            arec[at] = r;
            if (c > 1) w.acnt[at] = c;
        } else {
            const uint64_t sp = (uint64_t)sbase[b] + (pos - max((uint64_t)gbase[b], cap1));
            if (sp < w.spill_cap) w.spill[sp] = make_uint4((uint32_t)k, (uint32_t)(k >> 32), c, idx);
            else atomicOr(t.overflow, kOvfTable);
        }
    };
    for (uint64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
        uint4 nx[RPL][2];
#pragma unroll
        for (int j = 0; j < RPL; ++j) {
            const uint64_t r = min(tile * TILE + j * T + threadIdx.x, n - 1);
            nx[j][0] = ld_stream(&in[r * stride16]);
            nx[j][1] = ld_stream(&in[r * stride16 + hi16]);
        }
        uint64_t key[RPL];
        uint32_t bin[RPL], rank[RPL];
        const uint64_t t0 = tile * TILE;
#pragma unroll
        for (int j = 0; j < RPL; ++j) {
            const uint64_t r = t0 + j * T + threadIdx.x;
            const Enc32 a = encode16(nx[j][0].x, nx[j][0].y, nx[j][0].z, nx[j][0].w, true);
            const uint4 h = hi16 ? nx[j][1] : make_uint4(0x41414141u, 0x41414141u, 0x41414141u, 0x41414141u);
            const Enc32 b = encode16(h.x, h.y, h.z, h.w, true);
            const bool live = r < n;
            report_bad(live && (a.bad | b.bad) != 0u, r, first_bad);
            key[j] = (uint64_t)a.v | ((uint64_t)(b.v | a.cout) << 32);
            bin[j] = region_of(t, key[j]) >> shift;
            rank[j] = live ? atomicAdd(&lcount[bin[j]], 1u) : 0u;
        }
        __syncthreads();                                                  // (A) ranks counted
        if (threadIdx.x < 64) {
            const uint32_t lane = threadIdx.x, b0 = 2 * lane;
            const uint32_t c0 = lcount[b0], c1 = lcount[b0 + 1];
            const bool h0 = c0 > kHeavy, h1 = c1 > kHeavy;
            hflag[b0] = h0;
            hflag[b0 + 1] = h1;
            reserve(b0, c0, c1, (h0 ? 0u : 1u) | (h1 ? 0u : 2u));
            const uint64_t hv = __ballot(h0 || h1);
            if (lane == 0) any_heavy = hv != 0;
            lcount[b0] = 0;
            lcount[b0 + 1] = 0;
        }
        __syncthreads();                                                  // (B) runs reserved
        if (!any_heavy) {
#pragma unroll
            for (int j = 0; j < RPL; ++j) {
                const uint64_t r = t0 + j * T + threadIdx.x;
                if (r < n) emit(bin[j], gbase[bin[j]] + rank[j], key[j], (uint32_t)r, 1u);
            }
            continue;
        }
        // heavy tile: elements of heavy bins are deduplicated in the LDS table (wave fold first);
        // the rest (and a table that runs full) leave as their own records
        uint32_t cc[RPL], mi[RPL], orank[RPL];
        bool ov[RPL];
#pragma unroll
        for (int j = 0; j < RPL; ++j) {
            const uint64_t r = t0 + j * T + threadIdx.x;
            const bool live = r < n;
            const bool hv = live && hflag[bin[j]];
            ov[j] = false;
            cc[j] = 1;
            mi[j] = (uint32_t)r;
            if (live && !hv) emit(bin[j], gbase[bin[j]] + rank[j], key[j], (uint32_t)r, 1u);
            bool act = hv && key[j] != kEmpty;
            wave_fold<SS_COARSE_FOLD>(act, key[j], cc[j], mi[j]);
            if (act && ht_insert<HT>(hkey, hc, hix, key[j], cc[j], mi[j]) < 0) ov[j] = true;
            if (hv && key[j] == kEmpty) ov[j] = true;
            if (ov[j]) orank[j] = atomicAdd(&hcnt[bin[j]], 1u);
        }
        __syncthreads();                                                  // (D) deduplicated
        constexpr int kE = (HT + T - 1) / T;
        uint32_t erank[kE];
#pragma unroll
        for (int q = 0; q < kE; ++q) {
            const uint32_t e = q * T + threadIdx.x;
            if (e < HT && hkey[e] != kEmpty) erank[q] = atomicAdd(&hcnt[region_of(t, hkey[e]) >> shift], 1u);
        }
        __syncthreads();                                                  // (E) survivors counted
        if (threadIdx.x < 64) {
            const uint32_t b0 = 2 * threadIdx.x;
            reserve(b0, hcnt[b0], hcnt[b0 + 1], (hflag[b0] ? 1u : 0u) | (hflag[b0 + 1] ? 2u : 0u));
            hcnt[b0] = 0;
            hcnt[b0 + 1] = 0;
        }
        __syncthreads();                                                  // (F) heavy runs reserved
#pragma unroll
        for (int j = 0; j < RPL; ++j)
            if (ov[j]) emit(bin[j], gbase[bin[j]] + orank[j], key[j], mi[j], cc[j]);
#pragma unroll
        for (int q = 0; q < kE; ++q) {
            const uint32_t e = q * T + threadIdx.x;
            if (e < HT && hkey[e] != kEmpty) {
                const uint64_t k = hkey[e];
                emit(region_of(t, k) >> shift, gbase[region_of(t, k) >> shift] + erank[q], k, hix[e], hc[e]);
                hkey[e] = kEmpty;
                hc[e] = 0;
                hix[e] = 0xFFFFFFFFu;
            }
        }
    }
}

// fine pass, unstaged: block per sub-bin (largest first), per-region cursors in LDS; one barrier
// per tile (histograms and cursors rotate through 3 / 2 buffers)
template <int T, int RPL, uint32_t HT>
__global__ __launch_bounds__(T) __attribute__((amdgpu_waves_per_eu(FU_WPE))) void k_fu(Tbl t, PartWs w, uint64_t cap1, const uint32_t* fill,
                                          const uint32_t* __restrict__ order) {
    constexpr uint32_t TILE = T * RPL;
    constexpr uint32_t kNB = 256;
    __shared__ uint32_t cur[2][kNB], lc[3][kNB], hcnt[kNB];
    __shared__ uint32_t heavyf[3];
    __shared__ unsigned long long hkey[HT];
    __shared__ uint32_t hc[HT], hix[HT];
    const uint32_t nb = 1u << (w.rbits - kCoarseBits);
    const uint32_t heavy_at = max(64u, SS_HEAVY_FINE * (TILE / nb));
    const uint32_t fb = order[blockIdx.x];
    const uint32_t bin = fb / kFinePerBin;
    const uint32_t hi_ = (uint32_t)min((uint64_t)fill[fill_at(fb)], cap1);
    const uint32_t r0 = bin * nb;
    const Rec12* srec = (const Rec12*)w.akey + (uint64_t)fb * cap1;
    const uint32_t* src_cnt = w.acnt + (uint64_t)fb * cap1;
    const uint32_t sbase = w.slabs[fb], ssize = w.slabs[kNFill + fb];
    Rec12* const brec = (Rec12*)w.keys;
    for (uint32_t i = threadIdx.x; i < nb; i += T) {
        cur[0][i] = sbase + i * ssize;
        w.hist[(uint64_t)fb * nb + i] = sbase + i * ssize;   // the aggregate's segment starts
        lc[0][i] = lc[1][i] = lc[2][i] = 0;
        hcnt[i] = 0;
    }
    for (uint32_t i = threadIdx.x; i < HT; i += T) {
        hkey[i] = kEmpty;
        hc[i] = 0;
        hix[i] = 0xFFFFFFFFu;
    }
    if (threadIdx.x < 3) heavyf[threadIdx.x] = 0;
    __syncthreads();
    auto emit = [&](uint32_t lb, uint32_t gpos, uint64_t k, uint32_t xi, uint32_t c) {
        if (gpos >= sbase + (lb + 1) * ssize) {
            const uint64_t sp = atomicAdd(w.spill_ctr, 1u);
            if (sp < w.spill_cap) w.spill[sp] = make_uint4((uint32_t)k, (uint32_t)(k >> 32), c, xi & ~kWeighted);
            else atomicOr(t.overflow, kOvfTable);
            return;
        }
        Rec12 r;
        r.klo = (uint32_t)k;
        r.khi = (uint32_t)(k >> 32);
        r.idx = c > 1 ? (xi | kWeighted) : (xi & ~kWeighted);
        brec[gpos] = r;
        if (c > 1) w.bcnt[gpos] = c;
    };
    const uint32_t ntiles = (hi_ + TILE - 1) / TILE;
    uint64_t nk[RPL];
    uint32_t ni[RPL];
    auto load_tile = [&](uint32_t t0) {
#pragma unroll
        for (int j = 0; j < RPL; ++j) {
            const uint32_t at = min(t0 + j * T + threadIdx.x, hi_ - 1);
            const Rec12 r = srec[at];
            nk[j] = ((uint64_t)r.khi << 32) | r.klo;
            ni[j] = r.idx;
        }
    };
    if (hi_) load_tile(0);
    for (uint32_t it = 0; it < ntiles; ++it) {
        const uint32_t p3 = it % 3, p2 = it & 1, z3 = (it + 2) % 3;
        const uint32_t t0 = it * TILE;
        uint64_t key[RPL];
        uint32_t idx[RPL], lb[RPL], rank[RPL];
#pragma unroll
        for (int j = 0; j < RPL; ++j) {
            key[j] = nk[j];
            idx[j] = ni[j];
        }
        if (it + 1 < ntiles) load_tile(t0 + TILE);
#pragma unroll
        for (int j = 0; j < RPL; ++j) {
            const bool live = t0 + j * T + threadIdx.x < hi_;
            lb[j] = region_of(t, key[j]) - r0;
            rank[j] = live ? atomicAdd(&lc[p3][lb[j]], 1u) : 0u;
            if (live && rank[j] == heavy_at) heavyf[p3] = 1;
        }
        __syncthreads();                                                  // (A)
        if (!heavyf[p3]) {
#pragma unroll
            for (int j = 0; j < RPL; ++j) {
                const uint32_t e = t0 + j * T + threadIdx.x;
                if (e >= hi_) continue;
                uint32_t c = 1;
                if (idx[j] & kWeighted) c = src_cnt[e];
                emit(lb[j], cur[p2][lb[j]] + rank[j], key[j], idx[j], c);
            }
            for (uint32_t i = threadIdx.x; i < nb; i += T) {
                cur[p2 ^ 1][i] = cur[p2][i] + lc[p3][i];
                lc[z3][i] = 0;
            }
            if (threadIdx.x == 0) heavyf[z3] = 0;
            continue;
        }
        uint32_t cc[RPL], mi[RPL], orank[RPL];
        bool ov[RPL];
#pragma unroll
        for (int j = 0; j < RPL; ++j) {
            const uint32_t e = t0 + j * T + threadIdx.x;
            const bool live = e < hi_;
            const bool hv = live && lc[p3][lb[j]] > heavy_at;
            const bool wt = live && (idx[j] & kWeighted);
            cc[j] = wt ? src_cnt[e] : 1u;
            mi[j] = idx[j] & ~kWeighted;
            ov[j] = false;
            if (live && !hv) emit(lb[j], cur[p2][lb[j]] + rank[j], key[j], idx[j], cc[j]);
            bool act = hv && !wt && key[j] != kEmpty;
            wave_fold<SS_FINE_FOLD>(act, key[j], cc[j], mi[j]);
            if (act && ht_insert<HT>(hkey, hc, hix, key[j], cc[j], mi[j]) < 0) ov[j] = true;
            if (hv && (wt || key[j] == kEmpty)) ov[j] = true;
            if (ov[j]) orank[j] = atomicAdd(&hcnt[lb[j]], 1u);
        }
        __syncthreads();                                                  // (D)
        constexpr int kE = (HT + T - 1) / T;
        uint32_t erank[kE];
#pragma unroll
        for (int q = 0; q < kE; ++q) {
            const uint32_t e = q * T + threadIdx.x;
            if (e < HT && hkey[e] != kEmpty) erank[q] = atomicAdd(&hcnt[region_of(t, hkey[e]) - r0], 1u);
        }
        __syncthreads();                                                  // (E)
#pragma unroll
        for (int j = 0; j < RPL; ++j)
            if (ov[j]) emit(lb[j], cur[p2][lb[j]] + orank[j], key[j], mi[j], cc[j]);
#pragma unroll
        for (int q = 0; q < kE; ++q) {
            const uint32_t e = q * T + threadIdx.x;
            if (e < HT && hkey[e] != kEmpty) {
                const uint64_t k = hkey[e];
                const uint32_t b = region_of(t, k) - r0;
                emit(b, cur[p2][b] + erank[q], k, hix[e], hc[e]);
                hkey[e] = kEmpty;
                hc[e] = 0;
                hix[e] = 0xFFFFFFFFu;
            }
        }
        for (uint32_t i = threadIdx.x; i < nb; i += T) {
            cur[p2 ^ 1][i] = cur[p2][i] + (lc[p3][i] > heavy_at ? hcnt[i] : lc[p3][i]);
            hcnt[i] = 0;
            lc[z3][i] = 0;
        }
        if (threadIdx.x == 0) heavyf[z3] = 0;
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nb; i += T)
        w.seg_end[(uint64_t)fb * nb + i] = min(cur[ntiles & 1][i], sbase + (i + 1) * ssize);
}

}  // namespace

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
#define CS(x) do { int r_ = (x); if (r_) { printf("ss error %d: %s @%d\n", r_, ss_last_error_string(), __LINE__); exit(1); } } while (0)

// order-independent checksum of the table: sum over used slots of splitmix(key ^ splitmix(count, first))
static unsigned long long table_sum(ss_counter* c, uint64_t* used) {
    std::vector<Slot> h(c->cap + 1);
    CK(hipMemcpy(h.data(), c->slots, (c->cap + 1) * sizeof(Slot), hipMemcpyDeviceToHost));
    unsigned long long s = 0;
    uint64_t u = 0;
    for (uint64_t i = 0; i <= c->cap; ++i) {
        const bool used_ = i < c->cap ? h[i].key != kEmpty : h[i].ncount != 0xFFFFFFFFu;
        if (!used_) continue;
        ++u;
        s += splitmix64(h[i].key ^ splitmix64(((uint64_t)~h[i].ncount << 32) | h[i].first));
    }
    *used = u;
    return s;
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 125000000ull;
    const int reps = argc > 2 ? atoi(argv[2]) : 10;
    const int ulog = argc > 3 ? atoi(argv[3]) : 24;
    const double zs = argc > 4 ? atof(argv[4]) : 0.0;
    const uint64_t U = 1ull << ulog;
    const uint32_t L = 32;
    uint8_t* ascii;
    uint64_t* fb;
    CK(hipMalloc(&ascii, n * L));
    CK(hipMalloc(&fb, 8));
    if (zs > 0) {
        uint64_t* h = (uint64_t*)malloc(U * 8);
        double* cd = (double*)malloc(U * 8);
        double acc = 0;
        for (uint64_t k = 0; k < U; ++k) cd[k] = (acc += pow((double)(k + 1), -zs));
        for (uint64_t k = 0; k < U; ++k) h[k] = (uint64_t)floor(cd[k] / acc * 9223372036854775808.0);
        h[U - 1] = 1ull << 63;
        uint64_t* d;
        CK(hipMalloc(&d, U * 8));
        CK(hipMemcpy(d, h, U * 8, hipMemcpyHostToDevice));
        CS(ss_synth_zipf_reads(ascii, 5, 77, d, U, 0, n, L, L, nullptr));
        CK(hipDeviceSynchronize());
        CK(hipFree(d));
        free(h);
        free(cd);
    } else {
        CS(ss_synth_pool_reads(ascii, 5, 77, U, 0, n, L, L, nullptr));
    }
    ss_counter* c;
    CS(ss_counter_create(2 * U, &c));
    CS(ss_counter_reserve(c, n));
    if (!c->ws_slab) { printf("no slabs\n"); return 1; }
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    int per_p = 0, per_u = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_p, (const void*)k_pf_coarse<kPfT, kPfRPL>, kPfT, 0));
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_u, (const void*)k_cu<CU_T, CU_RPL, CU_HT>, CU_T, 0));
    printf("coarse blocks/CU: prod %d, unstaged %d (T %d RPL %d HT %d); fine T %d RPL %d HT %d\n", per_p, per_u,
           CU_T, CU_RPL, CU_HT, FU_T, FU_RPL, FU_HT);
    hipEvent_t ev[8];
    for (auto& e : ev) CK(hipEventCreate(&e));
    const char* names[2] = {"prod", "unstaged"};
    const char* modes[4] = {"P/P", "U/P", "P/U", "U/U"};
    for (int mode = 0; mode < 4; ++mode) {
        const bool cu = mode & 1, fu = mode & 2;
        double tc = 0, tf = 0, ta = 0, tt = 0, tmin = 1e9;
        for (int r = -3; r < reps; ++r) {
            CS(ss_counter_reset(c, nullptr));
            Tbl t = tbl_of(c);
            PartWs w{};
            w.keys = c->ws_keys; w.akey = c->ws_akey; w.aidx = c->ws_aidx; w.acnt = c->ws_acnt; w.areg = c->ws_areg;
            w.bidx = c->ws_bidx; w.bcnt = c->ws_bcnt; w.spill = c->ws_spill; w.spill_cap = c->ws_reads;
            w.hist = c->ws_hist; w.rstart = c->ws_rstart; w.tot = c->ws_tot;
            w.R = (uint32_t)(c->cap >> c->slice_log); w.rbits = c->log2cap - c->slice_log;
            w.slab = 1; w.spill_ctr = c->ws_fill + fill_at(kSpillCtr);
            const bool fresh = c->reset_pending;
            c->reset_pending = false;
            const uint64_t cap1 = c->ws_cap1;
            CK(hipMemsetAsync(fb, 0xFF, 8, nullptr));
            CK(hipMemsetAsync(c->ws_fill, 0, kFillWords * sizeof(uint32_t), nullptr));
            CK(hipEventRecord(ev[0], 0));
            if (cu)
                hipLaunchKernelGGL((k_cu<CU_T, CU_RPL, CU_HT>), dim3(cus * per_u), dim3(CU_T), 0, 0, t, w,
                                   (const uint4*)ascii, (uint64_t)2, n, 2u, cap1, c->ws_fill, (unsigned long long*)fb);
            else
                hipLaunchKernelGGL((k_pf_coarse<kPfT, kPfRPL>), dim3(cus * per_p), dim3(kPfT), 0, 0, t, w,
                                   (const uint4*)ascii, (uint64_t)2, n, 2u, cap1, c->ws_fill, (unsigned long long*)fb);
            CK(hipEventRecord(ev[1], 0));
            w.seg_end = c->ws_segend;
            w.slabs = c->ws_order + kNFill;
            hipLaunchKernelGGL(k_pf_order, dim3(1), dim3(512), 0, 0, (const uint32_t*)c->ws_fill, cap1, c->ws_order,
                               1u << (w.rbits - kCoarseBits), c->ws_order + kNFill);
            if (fu)
                hipLaunchKernelGGL((k_fu<FU_T, FU_RPL, FU_HT>), dim3(kNFill), dim3(FU_T), 0, 0, t, w, cap1,
                                   (const uint32_t*)c->ws_fill, (const uint32_t*)c->ws_order);
            else
                hipLaunchKernelGGL((k_pf_scatter<SS_FS_T, SS_FS_TILE>), dim3(kNFill), dim3(SS_FS_T), 0, 0, t, w, cap1,
                                   (const uint32_t*)c->ws_fill, (const uint32_t*)c->ws_order);
            CK(hipEventRecord(ev[2], 0));
            w.brec = (const Rec12*)w.keys;
            hipLaunchKernelGGL((k_pc_aggregate_slice<kAggSliceT, true>), dim3(w.R), dim3(kAggSliceT),
                               ((size_t)1 << c->slice_log) * 16, 0, t, w, (uint64_t)0, fresh);
            hipLaunchKernelGGL(k_spill_insert, dim3(1024), dim3(256), 0, 0, t, w, (const uint32_t*)c->ws_fill,
                               (uint64_t)0);
            CK(hipEventRecord(ev[3], 0));
            CK(hipGetLastError());
            CK(hipEventSynchronize(ev[3]));
            float a, b, d;
            CK(hipEventElapsedTime(&a, ev[0], ev[1]));
            CK(hipEventElapsedTime(&b, ev[1], ev[2]));
            CK(hipEventElapsedTime(&d, ev[2], ev[3]));
            if (r >= 0) {
                tc += a; tf += b; ta += d; tt += a + b + d;
                tmin = std::min(tmin, (double)(a + b + d));
            }
        }
        uint64_t used, hfb;
        const unsigned long long sum = table_sum(c, &used);
        uint32_t hspill = 0;
        unsigned long long ovf = 0;
        CK(hipMemcpy(&hspill, c->ws_fill + fill_at(kSpillCtr), 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&ovf, c->work, 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&hfb, fb, 8, hipMemcpyDeviceToHost));
        printf("%s coarse %s fine %s: coarse %.3f  fine(+order) %.3f  agg(+spill) %.3f  total %.3f ms (min %.3f)"
               "  used %llu sum %016llx spill %u ovf %llx fb %llx\n",
               modes[mode], names[cu], names[fu], tc / reps, tf / reps, ta / reps, tt / reps, tmin,
               (unsigned long long)used, sum, hspill, ovf, (unsigned long long)hfb);
        fflush(stdout);
    }
    return 0;
}
