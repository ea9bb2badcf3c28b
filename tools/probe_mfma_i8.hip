// tools/probe_mfma_i8.hip — empirical A/B/D lane maps of v_mfma_i32_32x32x32_i8 on gfx950.
// Fills lane fragments from A[32][32], B[32][32] (small ints) under candidate k maps and checks
// D against the host product; prints which map holds.
//   hipcc -O3 --offload-arch=gfx950 tools/probe_mfma_i8.hip -o tools/probe_mfma_i8
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__global__ void k(const v4i* a, const v4i* b, v16i* d) {
    v16i c = {};
    d[threadIdx.x] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[threadIdx.x], b[threadIdx.x], c, 0, 0, 0);
}

static int kmap(int m, int h, int j) {
    if (m == 0) return 16 * h + j;                                  // contiguous 16 per half
    return (j < 8) ? 8 * h + j : 16 + 8 * h + (j - 8);             // two K=16 halves
}

int main() {
    signed char A[32][32], B[32][32];
    srand(3);
    for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
            A[i][j] = (signed char)(rand() % 7 - 3);
            B[i][j] = (signed char)(rand() % 7 - 3);
        }
    int ref[32][32];
    for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
            int s = 0;
            for (int q = 0; q < 32; ++q) s += A[i][q] * B[q][j];
            ref[i][j] = s;
        }
    v4i *da, *db;
    v16i* dd;
    hipMalloc(&da, 64 * sizeof(v4i));
    hipMalloc(&db, 64 * sizeof(v4i));
    hipMalloc(&dd, 64 * sizeof(v16i));
    for (int m = 0; m < 2; ++m) {
        signed char ha[64][16], hb[64][16];
        for (int l = 0; l < 64; ++l)
            for (int j = 0; j < 16; ++j) {
                const int r = l & 31, h = l >> 5, kk = kmap(m, h, j);
                ha[l][j] = A[r][kk];
                hb[l][j] = B[kk][r];
            }
        hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
        hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, db, dd);
        int hd[64][16];
        hipMemcpy(hd, dd, sizeof hd, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int l = 0; l < 64; ++l)
            for (int i = 0; i < 16; ++i) {
                const int row = (i & 3) + 8 * (i >> 2) + 4 * (l >> 5), col = l & 31;
                if (hd[l][i] != ref[row][col]) ++bad;
            }
        printf("k map %d: %d mismatches of 1024\n", m, bad);
    }
    return 0;
}
