// tools/tune_nlpos.hip — k_fq_nlpos (one tile per block) vs a persistent form (resident blocks loop
// over tiles, optionally loading the next tile's chunks before this tile's scan / staging), on the
// F1 bench's synthetic FASTQ (1.98 GB).  Outputs (tile counts / runs / last newline, staged
// positions) compared with the production kernel's.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include tools/tune_nlpos.hip -o tools/tune_nlpos
#include "../shortseq_amd/csrc/ss_fastq.hip"
#include "../shortseq_amd/csrc/ss_runtime.hip"

#include <stdio.h>
#include <stdlib.h>
#include <random>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

namespace {
template <bool PF>
__global__ __launch_bounds__(kFqT) void k_nlpos_p(const uint8_t* __restrict__ buf, uint64_t nbytes, FqStage st,
                                                 uint64_t ntiles) {
    __shared__ uint64_t wtot[kFqT / 64][kFqU1 / 4];
    __shared__ uint32_t s_run, s_cnt;
    __shared__ __attribute__((aligned(8))) uint16_t spos[kLdsPos];
    uint4 x[kFqU1];
    if (blockIdx.x < ntiles) load_chunks<kFqU1>(buf, nbytes, (uint64_t)blockIdx.x * kFqTile1, x);
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const uint64_t t0 = tile * kFqTile1;
    uint32_t mk[kFqU1 / 2];
    bool nul = false;
    {
#pragma unroll
        for (int j = 0; j < kFqU1; j += 2) {
            mk[j / 2] = nl_mask16(x[j]) | nl_mask16(x[j + 1]) << 16;
            nul |= has_nul(x[j]) | has_nul(x[j + 1]);
        }
        if (!PF && tile + gridDim.x < ntiles) {}   // no prefetch
        if (PF && tile + gridDim.x < ntiles) load_chunks<kFqU1>(buf, nbytes, (tile + gridDim.x) * kFqTile1, x);
    }
    // the wave's NUL verdict now: left to its use at the end, the compiler keeps the chunks live
    // through the whole kernel (96 VGPRs, 5 waves per SIMD, instead of 62 and 8)
    const bool any_nul = __ballot(nul) != 0;
    uint64_t packed[kFqU1 / 4], excl[kFqU1 / 4], total[kFqU1 / 4];
#pragma unroll
    for (int k = 0; k < kFqU1 / 4; ++k) packed[k] = 0;
#pragma unroll
    for (int j = 0; j < kFqU1; ++j)
        packed[j / 4] |= (uint64_t)__popc((mk[j / 2] >> (16 * (j & 1))) & 0xFFFFu) << (16 * (j % 4));
    scan_packed(packed, wtot, excl, total);
    uint32_t cnt = 0;
#pragma unroll
    for (int k = 0; k < kFqU1 / 4; ++k)
        cnt += (uint32_t)((total[k] & 0xFFFFu) + ((total[k] >> 16) & 0xFFFFu) + ((total[k] >> 32) & 0xFFFFu) +
                          (total[k] >> 48));
    const bool fixed = cnt <= kTileCap;    // block-uniform (the scan's totals)
    if (threadIdx.x == 0) {
        // the reservation's round trip overlaps the other waves' LDS staging below
        const uint32_t sh = tile % kStageShards;
        uint64_t run = (uint64_t)sh * st.region;
        uint32_t c = cnt;
        if (fixed) {
            run = (uint64_t)kStageShards * st.region + (uint64_t)tile * kTileCap;
        } else if (c) {
            const uint32_t r = atomicAdd(&st.used[sh * kShardStride], c);
            if (r + (uint64_t)c > st.region) {
                atomicExch(st.ovf, 1u);
                c = 0;                    // nothing staged; the call reports the overflow
            }
            run += r;
        }
        st.tile_cnt[tile] = c;
        st.tile_run[tile] = (uint32_t)run;
        if (cnt == 0) st.tile_last[tile] = kNone32;
        s_run = (uint32_t)run;
        s_cnt = c;
    }
    const bool in_lds = cnt <= kLdsPos;   // typical tiles: positions gathered in LDS, stored as one run
    auto put = [&](uint32_t base) {
        uint32_t rows_before = 0;
#pragma unroll
        for (int j = 0; j < kFqU1; ++j) {
            const uint32_t off = (uint32_t)(t0 + 16ull * (j * kFqT + threadIdx.x));
            uint32_t k = base + rows_before + (uint32_t)((excl[j / 4] >> (16 * (j % 4))) & 0xFFFFu);
            rows_before += (uint32_t)((total[j / 4] >> (16 * (j % 4))) & 0xFFFFu);
            uint32_t m = (mk[j / 2] >> (16 * (j & 1))) & 0xFFFFu;   // bytes past nbytes loaded as ' '
            while (m) {
                const uint32_t bit = __builtin_ctz(m);
                m &= m - 1;
                const uint16_t rel = (uint16_t)(off + bit - (uint32_t)t0);
                if (in_lds) spos[k++] = rel;
                else st.pos[k++] = rel;
                if (k == base + cnt) st.tile_last[tile] = off + bit;   // the tile's last newline
            }
        }
    };
    // Positions gathered in LDS and stored as one run beat each lane storing its own (scattered 2-B
    // stores: 0.435 vs 0.410 ms per 2-GB call, tools/tune_f1.hip)
    if (in_lds) put(0);
    __syncthreads();
    if (fixed && cnt) {           // the tile's own run: 8-B copies (the run is 4 KiB aligned; a copy past cnt
        const uint64_t* s8 = (const uint64_t*)spos;   // stays inside the run)
        uint64_t* d8 = (uint64_t*)(st.pos + kStageShards * st.region + (uint64_t)tile * kTileCap);
        for (uint32_t e = threadIdx.x; 4 * e < cnt; e += kFqT) d8[e] = s8[e];
    } else if (!fixed && s_cnt) {
        if (in_lds) {
            const uint32_t run = s_run;
            for (uint32_t e = threadIdx.x; e < cnt; e += kFqT) st.pos[run + e] = spos[e];
        } else {
            put(s_run);
        }
    }
    if (any_nul) {                         // rare: reload the lane's chunks (keeps them out of VGPRs)
#pragma unroll 1
        for (int j = 0; j < kFqU1; ++j) {
            const uint64_t off = t0 + 16ull * (j * kFqT + threadIdx.x);
            if (off >= nbytes) break;
            const uint4 c = load_chunk(buf, off, nbytes);
            const uint32_t xw[4] = {c.x, c.y, c.z, c.w};
#pragma unroll 1
            for (int q = 0; q < 4; ++q) {
                uint32_t m = eq_bytes(xw[q], 0u);
                while (m) {
                    const uint32_t bit = __builtin_ctz(m);
                    m &= m - 1;
                    const uint64_t p = off + 4 * q + (bit >> 3);
                    if (p >= nbytes) break;
                    const uint32_t i = atomicAdd(st.nul_cnt, 1u);
                    if (i < kNulCap) st.nul_pos[i] = (uint32_t)p;
                }
            }
        }
    }
    __syncthreads();   // spos / s_run reused by the next tile
    if (!PF && tile + gridDim.x < ntiles) load_chunks<kFqU1>(buf, nbytes, (tile + gridDim.x) * kFqTile1, x);
  }
}

template <int MODE>
__global__ __launch_bounds__(kFqT) void k_nlpos_v(const uint8_t* __restrict__ buf, uint64_t nbytes, FqStage st) {
    __shared__ uint64_t wtot[kFqT / 64][kFqU1 / 4];
    __shared__ uint32_t s_run, s_cnt;
    __shared__ __attribute__((aligned(8))) uint16_t spos[kLdsPos];
    const uint64_t t0 = (uint64_t)blockIdx.x * kFqTile1;
    // the chunks live only until their newline masks are taken: 16 bits per chunk, two per VGPR
    uint32_t mk[kFqU1 / 2];
    bool nul = false;
    {
        uint4 x[kFqU1];
        load_chunks<kFqU1>(buf, nbytes, t0, x);
#pragma unroll
        for (int j = 0; j < kFqU1; j += 2) {
            mk[j / 2] = nl_mask16(x[j]) | nl_mask16(x[j + 1]) << 16;
            nul |= has_nul(x[j]) | has_nul(x[j + 1]);
        }
    }
    // the wave's NUL verdict now: left to its use at the end, the compiler keeps the chunks live
    // through the whole kernel (96 VGPRs, 5 waves per SIMD, instead of 62 and 8)
    const bool any_nul = __ballot(nul) != 0;
    uint64_t packed[kFqU1 / 4], excl[kFqU1 / 4], total[kFqU1 / 4];
#pragma unroll
    for (int k = 0; k < kFqU1 / 4; ++k) packed[k] = 0;
#pragma unroll
    for (int j = 0; j < kFqU1; ++j)
        packed[j / 4] |= (uint64_t)__popc((mk[j / 2] >> (16 * (j & 1))) & 0xFFFFu) << (16 * (j % 4));
    scan_packed(packed, wtot, excl, total);
    uint32_t cnt = 0;
#pragma unroll
    for (int k = 0; k < kFqU1 / 4; ++k)
        cnt += (uint32_t)((total[k] & 0xFFFFu) + ((total[k] >> 16) & 0xFFFFu) + ((total[k] >> 32) & 0xFFFFu) +
                          (total[k] >> 48));
    const bool fixed = cnt <= kTileCap;    // block-uniform (the scan's totals)
    if (threadIdx.x == 0) {
        // the reservation's round trip overlaps the other waves' LDS staging below
        const uint32_t sh = blockIdx.x % kStageShards;
        uint64_t run = (uint64_t)sh * st.region;
        uint32_t c = cnt;
        if (fixed) {
            run = (uint64_t)kStageShards * st.region + (uint64_t)blockIdx.x * kTileCap;
        } else if (c) {
            const uint32_t r = atomicAdd(&st.used[sh * kShardStride], c);
            if (r + (uint64_t)c > st.region) {
                atomicExch(st.ovf, 1u);
                c = 0;                    // nothing staged; the call reports the overflow
            }
            run += r;
        }
        st.tile_cnt[blockIdx.x] = c;
        st.tile_run[blockIdx.x] = (uint32_t)run;
        if (cnt == 0) st.tile_last[blockIdx.x] = kNone32;
        s_run = (uint32_t)run;
        s_cnt = c;
    }
    const bool in_lds = cnt <= kLdsPos;   // typical tiles: positions gathered in LDS, stored as one run
    auto put = [&](uint32_t base) {
        uint32_t rows_before = 0;
#pragma unroll
        for (int j = 0; j < kFqU1; ++j) {
            const uint32_t off = (uint32_t)(t0 + 16ull * (j * kFqT + threadIdx.x));
            uint32_t k = base + rows_before + (uint32_t)((excl[j / 4] >> (16 * (j % 4))) & 0xFFFFu);
            rows_before += (uint32_t)((total[j / 4] >> (16 * (j % 4))) & 0xFFFFu);
            uint32_t m = (mk[j / 2] >> (16 * (j & 1))) & 0xFFFFu;   // bytes past nbytes loaded as ' '
            while (m) {
                const uint32_t bit = __builtin_ctz(m);
                m &= m - 1;
                const uint16_t rel = (uint16_t)(off + bit - (uint32_t)t0);
                if (in_lds) spos[k++] = rel;
                else st.pos[k++] = rel;
                if (k == base + cnt) st.tile_last[blockIdx.x] = off + bit;   // the tile's last newline
            }
        }
    };
    // Positions gathered in LDS and stored as one run beat each lane storing its own (scattered 2-B
    // stores: 0.435 vs 0.410 ms per 2-GB call, tools/tune_f1.hip)
    if (MODE == 1) return;
    if (in_lds && MODE != 3) put(0);
    __syncthreads();
    if (MODE == 2) return;
    if (fixed && cnt) {           // the tile's own run: 8-B copies (the run is 4 KiB aligned; a copy past cnt
        const uint64_t* s8 = (const uint64_t*)spos;   // stays inside the run)
        uint64_t* d8 = (uint64_t*)(st.pos + kStageShards * st.region + (uint64_t)blockIdx.x * kTileCap);
        if (MODE == 11) d8 = (uint64_t*)(st.pos + kStageShards * st.region + (uint64_t)(blockIdx.x & 7) * kTileCap);
        if (MODE == 8) {
            for (uint32_t e = threadIdx.x; 4 * e < cnt; e += kFqT) __builtin_nontemporal_store(s8[e], d8 + e);
        } else if (MODE == 9 || MODE == 10) {
            const uint4* s16 = (const uint4*)spos;
            uint4* d16 = (uint4*)d8;
            for (uint32_t e = threadIdx.x; 8 * e < cnt; e += kFqT) {
                if (MODE == 9) d16[e] = s16[e];
                else ssd::st_stream(d16 + e, s16[e]);
            }
        } else {
            for (uint32_t e = threadIdx.x; 4 * e < cnt; e += kFqT) d8[e] = s8[e];
        }
    } else if (!fixed && s_cnt) {
        if (in_lds) {
            const uint32_t run = s_run;
            for (uint32_t e = threadIdx.x; e < cnt; e += kFqT) st.pos[run + e] = spos[e];
        } else {
            put(s_run);
        }
    }
    if (any_nul) {                         // rare: reload the lane's chunks (keeps them out of VGPRs)
#pragma unroll 1
        for (int j = 0; j < kFqU1; ++j) {
            const uint64_t off = t0 + 16ull * (j * kFqT + threadIdx.x);
            if (off >= nbytes) break;
            const uint4 c = load_chunk(buf, off, nbytes);
            const uint32_t xw[4] = {c.x, c.y, c.z, c.w};
#pragma unroll 1
            for (int q = 0; q < 4; ++q) {
                uint32_t m = eq_bytes(xw[q], 0u);
                while (m) {
                    const uint32_t bit = __builtin_ctz(m);
                    m &= m - 1;
                    const uint64_t p = off + 4 * q + (bit >> 3);
                    if (p >= nbytes) break;
                    const uint32_t i = atomicAdd(st.nul_cnt, 1u);
                    if (i < kNulCap) st.nul_pos[i] = (uint32_t)p;
                }
            }
        }
    }
}
}  // namespace

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 30;
    const int L = 100;
    std::mt19937_64 rng(1);
    const int m = 1 << 16;
    std::string block;
    for (int i = 0; i < m; ++i) {
        char h[64];
        snprintf(h, sizeof h, "@SYN:%08d:", i);
        block += h;
        block += std::string(8 + rng() % 20, 'x');
        block += '\n';
        for (int j = 0; j < L; ++j) block += "ACGT"[rng() & 3];
        block += "\n+\n";
        block += std::string(L, 'I');
        block += '\n';
    }
    const uint64_t reps_blk = 128, nrec = (uint64_t)m * reps_blk, nbytes = block.size() * reps_blk;
    uint8_t* buf;
    CK(hipMalloc(&buf, nbytes + 16));
    for (uint64_t r = 0; r < reps_blk; ++r) CK(hipMemcpy(buf + r * block.size(), block.data(), block.size(), hipMemcpyHostToDevice));
    const uint64_t t = fq_tiles1(nbytes);
    const uint64_t region = fq_region(nrec + 2);
    const uint64_t npos = kStageShards * region + (uint64_t)kTileCap * t;
    FqStage st[2];
    for (int v = 0; v < 2; ++v) {
        CK(hipMalloc(&st[v].used, 4 * (kStageShards * kShardStride + 4)));
        st[v].ovf = st[v].used + kStageShards * kShardStride;
        st[v].nul_cnt = st[v].ovf + 1;
        CK(hipMalloc(&st[v].nul_pos, 4ull * kNulCap));
        CK(hipMalloc(&st[v].tile_cnt, 4 * t));
        CK(hipMalloc(&st[v].tile_run, 4 * t));
        CK(hipMalloc(&st[v].tile_last, 4 * t));
        CK(hipMalloc(&st[v].pos, 2 * npos));
        CK(hipMemset(st[v].pos, 0, 2 * npos));
        st[v].region = region;
    }
    int dev = 0, cus = 0, per5 = 0, perp = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&perp, (const void*)k_nlpos_p<true>, kFqT, 0));
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per5, (const void*)k_nlpos_p<false>, kFqT, 0));
    printf("file %.3f GB, %llu tiles; resident blocks per CU: pf %d, no-pf %d\n", nbytes / 1e9, (unsigned long long)t, perp, per5);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](int mode, int v, int mul) {
        CK(hipMemsetAsync(st[v].used, 0, 4 * (kStageShards * kShardStride + 4), 0));
        if (mode == 0) hipLaunchKernelGGL(k_fq_nlpos, dim3((unsigned)t), dim3(kFqT), 0, 0, buf, nbytes, st[v]);
        else if (mode == 1) hipLaunchKernelGGL(k_nlpos_p<true>, dim3(cus * perp * mul), dim3(kFqT), 0, 0, buf, nbytes, st[v], t);
        else if (mode == 2) hipLaunchKernelGGL(k_nlpos_p<false>, dim3(cus * per5 * mul), dim3(kFqT), 0, 0, buf, nbytes, st[v], t);
        else if (mode == 5) hipLaunchKernelGGL(k_nlpos_v<1>, dim3((unsigned)t), dim3(kFqT), 0, 0, buf, nbytes, st[v]);
        else if (mode == 6) hipLaunchKernelGGL(k_nlpos_v<2>, dim3((unsigned)t), dim3(kFqT), 0, 0, buf, nbytes, st[v]);
        else if (mode == 7) hipLaunchKernelGGL(k_nlpos_v<3>, dim3((unsigned)t), dim3(kFqT), 0, 0, buf, nbytes, st[v]);
        else if (mode == 8) hipLaunchKernelGGL(k_nlpos_v<8>, dim3((unsigned)t), dim3(kFqT), 0, 0, buf, nbytes, st[v]);
        else if (mode == 9) hipLaunchKernelGGL(k_nlpos_v<9>, dim3((unsigned)t), dim3(kFqT), 0, 0, buf, nbytes, st[v]);
        else if (mode == 10) hipLaunchKernelGGL(k_nlpos_v<10>, dim3((unsigned)t), dim3(kFqT), 0, 0, buf, nbytes, st[v]);
        else hipLaunchKernelGGL(k_nlpos_v<11>, dim3((unsigned)t), dim3(kFqT), 0, 0, buf, nbytes, st[v]);
    };
    run(0, 0, 1);
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> c0(t), r0(t), l0(t), c1(t), r1(t), l1(t);
    std::vector<uint16_t> p0(npos), p1(npos);
    CK(hipMemcpy(c0.data(), st[0].tile_cnt, 4 * t, hipMemcpyDeviceToHost));
    CK(hipMemcpy(r0.data(), st[0].tile_run, 4 * t, hipMemcpyDeviceToHost));
    CK(hipMemcpy(l0.data(), st[0].tile_last, 4 * t, hipMemcpyDeviceToHost));
    CK(hipMemcpy(p0.data(), st[0].pos, 2 * npos, hipMemcpyDeviceToHost));
    const char* names[12] = {"one tile per block", "persistent + prefetch", "persistent", "persistent + prefetch x2", "persistent x2", "no staging (scan + metadata only)", "LDS put, no copy-out", "no put, copy-out", "copy-out 8-B NT", "copy-out 16-B", "copy-out 16-B NT", "copy-out to 8 runs only (L2-resident)"};
    for (int mode = 0; mode < 12; ++mode) {
        const int md = mode >= 5 ? mode : mode >= 3 ? mode - 2 : mode, mul = mode >= 3 && mode < 5 ? 2 : 1;
        run(md, 1, mul);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(c1.data(), st[1].tile_cnt, 4 * t, hipMemcpyDeviceToHost));
        CK(hipMemcpy(r1.data(), st[1].tile_run, 4 * t, hipMemcpyDeviceToHost));
        CK(hipMemcpy(l1.data(), st[1].tile_last, 4 * t, hipMemcpyDeviceToHost));
        CK(hipMemcpy(p1.data(), st[1].pos, 2 * npos, hipMemcpyDeviceToHost));
        bool ok = (md >= 5 && md <= 7) || md == 11 ? true : (c0 == c1 && l0 == l1 && r0 == r1);
        for (uint64_t i = 0; ok && i < t; ++i)
            for (uint32_t k = 0; k < c0[i]; ++k) ok = ok && p0[r0[i] + k] == p1[r1[i] + k];
        for (int i = 0; i < 3; ++i) run(md, 1, mul);
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < reps; ++i) run(md, 1, mul);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("%-26s %s  %.4f ms (incl. 8-KB reset)  %.0f GB/s of file\n", names[mode], ok ? "OK" : "MISMATCH", ms, nbytes / ms / 1e6);
        fflush(stdout);
    }
    return 0;
}
