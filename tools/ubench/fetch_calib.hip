// FETCH_SIZE calibration for the access widths k_wg uses (MI355X_MICROARCH.md:
// "other access widths are uncalibrated").  Each kernel reads a known number
// of bytes once; rocprofv3 --pmc FETCH_SIZE per dispatch / bytes = the factor.
//   k_dword   : 4 B per lane, a wave reads 256 contiguous bytes
//   k_window  : 3 dwords per lane from rows of a 1920-wide plane (MC window
//               pattern: 4 lanes per block row, blocks at pseudo-random spots)
//   k_x4      : 16 B per lane streaming (the guide's calibrated case)
//   k_x2      : 8 B per lane streaming (global_load_dwordx2: the mailbox
//               granules {dword, epoch} and chroma MC rows)
//   k_x3      : 12 B per lane streaming (global_load_dwordx3: luma MC rows)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k_dword(const uint32_t *__restrict__ src, uint32_t *out, size_t n)
{
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc += src[i];
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_x4(const uint4 *__restrict__ src, uint32_t *out, size_t n)
{
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = src[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_x2(const uint2 *__restrict__ src, uint32_t *out, size_t n)
{
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint2 v = src[i];
        acc += v.x + v.y;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// 12 B per lane: lane i of the grid reads bytes [12 i, 12 i + 12)
__global__ void k_x3(const uint32_t *__restrict__ src, uint32_t *out, size_t n)
{
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint3 v = *(const uint3 *)(src + 3 * i);
        acc += v.x + v.y + v.z;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// every 16-row x 16-col tile of a W x H plane read exactly once as 16 rows of
// 4 dwords by 64 lanes (lane = row*4 + dword), tiles visited in a scrambled order
__global__ void k_window(const uint8_t *__restrict__ plane, uint32_t *out, int W, int H, int ntiles)
{
    const int lane = threadIdx.x & 63;
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int nw = (gridDim.x * blockDim.x) >> 6;
    const int tw = W / 16;
    uint32_t acc = 0;
    for (int t = wave; t < ntiles; t += nw) {
        const int tt = (int)(((unsigned)t * 2654435761u) % (unsigned)ntiles);   // permutation (ntiles odd-free check below)
        const int tx = tt % tw, ty = tt / tw;
        const int row = lane >> 2, dw = lane & 3;
        acc += *(const uint32_t *)(plane + (size_t)(ty * 16 + row) * W + tx * 16 + dw * 4);
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main()
{
    const size_t bytes = 512ull << 20;
    uint8_t *buf; uint32_t *out;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
    if (hipMemset(buf, 1, bytes) != hipSuccess) return 1;
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    hipLaunchKernelGGL(k_dword, dim3(8192), dim3(256), 0, 0, (const uint32_t *)buf, out, bytes / 4);
    hipLaunchKernelGGL(k_x4, dim3(8192), dim3(256), 0, 0, (const uint4 *)buf, out, bytes / 16);
    hipLaunchKernelGGL(k_x2, dim3(8192), dim3(256), 0, 0, (const uint2 *)buf, out, bytes / 8);
    const size_t n3 = bytes / 12;
    hipLaunchKernelGGL(k_x3, dim3(8192), dim3(256), 0, 0, (const uint32_t *)buf, out, n3);
    // window: plane 1920 x (bytes / 1920) rows, multiple of 16
    const int W = 1920, H = (int)((bytes / W) / 16 * 16);
    const int ntiles = (W / 16) * (H / 16);   // 2654435761 is odd and ntiles = 120 * k: not a permutation in
                                              // general -> count distinct tiles on the host below
    hipLaunchKernelGGL(k_window, dim3(8192), dim3(256), 0, 0, (const uint8_t *)buf, out, W, H, ntiles);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    // distinct tiles touched by k_window
    uint8_t *seen = (uint8_t *)calloc(ntiles, 1);
    size_t distinct = 0;
    for (int t = 0; t < ntiles; t++) {
        const int tt = (int)(((unsigned)t * 2654435761u) % (unsigned)ntiles);
        if (!seen[tt]) { seen[tt] = 1; distinct++; }
    }
    printf("k_x2 bytes %zu\nk_x3 bytes %zu\n", bytes, n3 * 12);
    printf("k_dword bytes %zu\nk_x4 bytes %zu\nk_window bytes %zu (distinct tiles %zu of %d)\n", bytes, bytes,
           distinct * 256, distinct, ntiles);
    return 0;
}
