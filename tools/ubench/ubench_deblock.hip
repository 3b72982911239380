// Micro-benchmark: cycles of one deblock_dir() pass (k_rows' per-MB filter)
// for one wave, on an LDS region filled with pseudo-random samples and a
// P-frame-like deblocking record.  Diagnostics only.
#include "../../broadway_amd/csrc/hip/recon_kernels.hip"
#include <stdio.h>

__global__ __launch_bounds__(64) void k_ub(unsigned long long *out, int iters, int bsmode)
{
    __shared__ RowLds L;
    const int lane = threadIdx.x;
    for (int i = lane; i < (int)sizeof(RowLds); i += 64) ((uint8_t *)&L)[i] = (uint8_t)(100 + ((i * 37) & 15));
    __syncthreads();
    if (lane < 16) {
        // bS: mode 0 = MB edges 2, internal 0; mode 1 = all 2; mode 2 = MB edge 4, internal 3
        uint16_t w = bsmode == 0 ? 0x0002 : bsmode == 1 ? 0x2222 : 0x3334;
        ((uint16_t *)L.db)[lane] = w;
    }
    if (lane < 6) {
        uint8_t *o = L.db + 16 + lane * 8;
        o[0] = 40; o[1] = 10; o[2] = 1; o[3] = 2; o[4] = 3; o[5] = 30; o[6] = o[7] = 0;
    }
    __syncthreads();
    unsigned long long t0 = clock64();
    for (int it = 0; it < iters; it++) {
        deblock_dir(0, L.db, L.ry, L.ru, L.rv, lane, true);
        wave_sync();
    }
    unsigned long long t1 = clock64();
    for (int it = 0; it < iters; it++) {
        deblock_dir(1, L.db, L.ry, L.ru, L.rv, lane, true);
        wave_sync();
    }
    unsigned long long t2 = clock64();
    if (lane == 0) { out[0] = (t1 - t0) / iters; out[1] = (t2 - t1) / iters; out[2] = L.ry[100]; }
}

int main()
{
    unsigned long long *d, h[3];
    hipMalloc(&d, 64);
    for (int mode = 0; mode < 3; mode++) {
        hipLaunchKernelGGL(k_ub, dim3(1), dim3(64), 0, 0, d, 200, mode);
        hipMemcpy(h, d, 24, hipMemcpyDeviceToHost);
        printf("bsmode %d: V %llu cycles, H %llu cycles\n", mode, h[0], h[1]);
    }
    return 0;
}
