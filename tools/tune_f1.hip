// tools/tune_f1.hip — F1 one-pass FASTQ index (ss_fastq_index_onepass) on the bench's synthetic file
// (8.4M records of 100 nt, 20-40-byte headers, 1.98 GB device-resident), built with compile-time knobs:
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include [-D(int)kTileCap=1024] tools/tune_f1.hip -o tools/tune_f1_<v>
// Checks offsets / lengths / read count against the two-pass index (ss_fastq_scan + ss_fastq_index)
// and prints the mean time per call over hipEvents.
#include "../shortseq_amd/csrc/ss_fastq.hip"
#include "../shortseq_amd/csrc/ss_runtime.hip"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <random>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
#define CS(x) do { int r_ = (x); if (r_) { printf("ss error %d: %s @%d\n", r_, ss_last_error_string(), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 30;
    const int L = argc > 2 ? atoi(argv[2]) : 100;
    const uint64_t nrec_target = argc > 3 ? strtoull(argv[3], 0, 10) : (8ull << 20);
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
    const uint64_t reps_blk = nrec_target / m, nrec = (uint64_t)m * reps_blk, nbytes = block.size() * reps_blk;
    uint8_t* buf;
    CK(hipMalloc(&buf, nbytes + 16));
    for (uint64_t r = 0; r < reps_blk; ++r) CK(hipMemcpy(buf + r * block.size(), block.data(), block.size(), hipMemcpyHostToDevice));
    printf("file %.3f GB, %llu records of %d nt\n", nbytes / 1e9, (unsigned long long)nrec, L);
    const uint64_t maxr = nrec + 2;
    const uint64_t ws_b = ss_fastq_onepass_ws_bytes(nbytes, maxr), ws2_b = ss_fastq_scan_ws_bytes(nbytes);
    void *ws, *ws2;
    uint64_t *offs, *offs2, *aux, *cnt, *cnt2;
    uint32_t *lens, *lens2;
    CK(hipMalloc(&ws, ws_b));
    CK(hipMalloc(&ws2, ws2_b));
    CK(hipMalloc(&offs, maxr * 8));
    CK(hipMalloc(&offs2, maxr * 8));
    CK(hipMalloc(&aux, maxr * 8));
    CK(hipMalloc(&lens, maxr * 4));
    CK(hipMalloc(&lens2, maxr * 4));
    CK(hipMalloc(&cnt, 24));
    CK(hipMalloc(&cnt2, 24));
    CS(ss_fastq_scan(buf, nbytes, ws2, ws2_b, cnt2, 0));
    CS(ss_fastq_index(buf, nbytes, 0, 1, ws2, offs2, lens2, aux, maxr, cnt2 + 1, 0));
    CS(ss_fastq_index_onepass(buf, nbytes, 0, 1, ws, ws_b, offs, lens, aux, maxr, cnt, 0));
    CK(hipDeviceSynchronize());
    uint64_t hc[3], hc2[3];
    CK(hipMemcpy(hc, cnt, 24, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hc2, cnt2, 16, hipMemcpyDeviceToHost));
    std::vector<uint64_t> o1(nrec), o2(nrec);
    std::vector<uint32_t> l1(nrec), l2(nrec);
    CK(hipMemcpy(o1.data(), offs, nrec * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(o2.data(), offs2, nrec * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(l1.data(), lens, nrec * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(l2.data(), lens2, nrec * 4, hipMemcpyDeviceToHost));
    const bool ok = hc[1] == nrec && hc2[1] == nrec && hc[2] == 0 && o1 == o2 && l1 == l2 && l1[0] == (uint32_t)L;
    printf("one-pass vs two-pass: reads %llu / %llu, status %llu, offsets+lens %s\n", (unsigned long long)hc[1],
           (unsigned long long)hc2[1], (unsigned long long)hc[2], ok ? "OK" : "MISMATCH");
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int round = 0; round < 3; ++round) {
        for (int i = 0; i < 5; ++i) CS(ss_fastq_index_onepass(buf, nbytes, 0, 1, ws, ws_b, offs, lens, aux, maxr, cnt, 0));
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < reps; ++i) CS(ss_fastq_index_onepass(buf, nbytes, 0, 1, ws, ws_b, offs, lens, aux, maxr, cnt, 0));
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("round %d tile_cap %u: onepass %.4f ms  %.0f GB/s of file\n", round, (unsigned)(int)kTileCap, ms,
               nbytes / ms / 1e6);
    }
    return ok ? 0 : 2;
}
