// k_conceal -- neighbour-based error concealment of a picture's missing MBs
// on the device (ConcealMb's intra branch, h264bsd_conceal.c:337-579, in the
// order of h264bsdConceal, :192-241): the host path (csrc/host/conceal.c) is
// the same arithmetic on a copy of the picture brought back to the host.
//
// One wave walks the MBs in the given order, in place on the frame slot,
// which holds the picture's decoded MBs reconstructed with the loop filter
// off (the caller's first pass).  Each concealed MB becomes a neighbour of
// the next, so the walk is sequential; within an MB the 64 lanes gather the
// neighbour rows / columns, sum them in groups, and write the 16x16 + 2 x
// 8x8 samples.  Neighbour loads are sc1 (L2, past this CU's L1) and every
// MB's stores drain before the next MB reads: a wave's own earlier stores
// are what it reads.
#include <hip/hip_runtime.h>
#include <stdint.h>

__device__ __forceinline__ uint32_t cc_ld_byte(const uint8_t *p)
{
    const uint32_t *d = (const uint32_t *)((uintptr_t)p & ~(uintptr_t)3);
    const uint32_t v = __hip_atomic_load(d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (v >> (((uintptr_t)p & 3) * 8)) & 255u;
}

__device__ __forceinline__ int cc_clip1(int v) { return v < 0 ? 0 : v > 255 ? 255 : v; }

// the reduced 4x4 transform (:592-629): only d[0], d[1], d[4] can be non-zero
__device__ __forceinline__ void cc_low_transform(int32_t *d)
{
    if (!d[1] && !d[4]) {
        for (int i = 1; i < 16; i++) d[i] = d[0];
        return;
    }
    const int32_t t0 = d[0], t1 = d[1];
    d[0] = t0 + t1;
    d[1] = t0 + (t1 >> 1);
    d[2] = t0 - (t1 >> 1);
    d[3] = t0 - t1;
    d[5] = d[6] = d[7] = d[4];
    for (int c = 0; c < 4; c++) {
        const int32_t a = d[c], b = d[4 + c];
        d[c] = a + b;
        d[4 + c] = a + (b >> 1);
        d[8 + c] = a - (b >> 1);
        d[12 + c] = a - b;
    }
}

// the 16 prediction values of one plane from its group sums S[side][4]
// (side 0 above, 1 below, 2 left, 3 right) and availability; c = 0 luma, 1
// chroma (:337-457 / :459-572)
__device__ __forceinline__ void cc_plane_fp(const int32_t (*S)[4], int A, int B, int L, int R, int c, int32_t *fp)
{
    for (int i = 0; i < 16; i++) fp[i] = 0;
    int j = 0, hor = 0, ver = 0;
    const int32_t *a = S[0], *b = S[1], *l = S[2], *r = S[3];
    if (A) { j++; hor++; fp[0] += a[0] + a[1] + a[2] + a[3]; fp[1] += a[0] + a[1] - a[2] - a[3]; }
    if (B) { j++; hor++; fp[0] += b[0] + b[1] + b[2] + b[3]; fp[1] += b[0] + b[1] - b[2] - b[3]; }
    if (L) { j++; ver++; fp[0] += l[0] + l[1] + l[2] + l[3]; fp[4] += l[0] + l[1] - l[2] - l[3]; }
    if (R) { j++; ver++; fp[0] += r[0] + r[1] + r[2] + r[3]; fp[4] += r[0] + r[1] - r[2] - r[3]; }
    if (!hor && L && R) fp[1] = (l[0] + l[1] + l[2] + l[3] - r[0] - r[1] - r[2] - r[3]) >> (5 - c);
    else if (hor) fp[1] >>= (3 - c + hor);
    if (!ver && A && B) fp[4] = (a[0] + a[1] + a[2] + a[3] - b[0] - b[1] - b[2] - b[3]) >> (5 - c);
    else if (ver) fp[4] >>= (3 - c + ver);
    switch (j) {
    case 1: fp[0] >>= 4 - c; break;
    case 2: fp[0] >>= 5 - c; break;
    case 3: fp[0] = (21 * fp[0]) >> (10 - c); break;
    default: fp[0] >>= 6 - c; break;
    }
    cc_low_transform(fp);
}

// frame: the slot (I420, w*16 x h*16); order[0..n): MB addresses in
// concealment order; dec0: nmbs flags, 1 = decoded (dynamic LDS copy, grows)
// dynamic LDS bound of k_conceal (one byte per MB): the CU's 160 KB less
// the static sums and headroom
#define CONCEAL_LDS_MAX (159 * 1024)
__global__ __launch_bounds__(64) void k_conceal(uint8_t *frame, int w, int h, int cp, const int *order, int n,
                                               const uint8_t *dec0)
{
    extern __shared__ uint8_t cc_dec[];
    __shared__ int32_t sums[3][4][4];          // plane, side, group
    const int lane = threadIdx.x;
    const int nmbs = w * h;
    for (int i = lane; i < nmbs; i += 64) cc_dec[i] = dec0[i];
    __syncthreads();
    const int W = w * 16, H = h * 16, CW = cp;     // chroma row pitch (H264MI_CPITCH)
    uint8_t *const Y = frame;
    uint8_t *const U = frame + (size_t)W * H;
    uint8_t *const V = U + (size_t)CW * (H / 2);
    for (int k = 0; k < n; k++) {
        const int mb = order[k];
        const int row = mb / w, col = mb % w;
        const int A = row && cc_dec[mb - w], B = row != h - 1 && cc_dec[mb + w];
        const int L = col && cc_dec[mb - 1], R = col != w - 1 && cc_dec[mb + 1];
        // luma: lane = side * 16 + i; chroma: lane = plane * 32 + side * 8 + i
        {
            const int side = lane >> 4, i = lane & 15;
            const int ok = side == 0 ? A : side == 1 ? B : side == 2 ? L : R;
            const int x0 = col * 16, y0 = row * 16;
            uint32_t v = 0;
            if (ok) {
                const size_t o = side == 0 ? (size_t)(y0 - 1) * W + x0 + i
                               : side == 1 ? (size_t)(y0 + 16) * W + x0 + i
                               : side == 2 ? (size_t)(y0 + i) * W + x0 - 1
                                           : (size_t)(y0 + i) * W + x0 + 16;
                v = cc_ld_byte(Y + o);
            }
            // groups of 4 consecutive samples: lanes 4g..4g+3 of the side
            v += __shfl_xor(v, 1);
            v += __shfl_xor(v, 2);
            if ((i & 3) == 0) sums[0][side][i >> 2] = (int32_t)v;
        }
        {
            const int plane = lane >> 5, side = (lane >> 3) & 3, i = lane & 7;
            const int ok = side == 0 ? A : side == 1 ? B : side == 2 ? L : R;
            const int x0 = col * 8, y0 = row * 8;
            const uint8_t *P = plane ? V : U;
            uint32_t v = 0;
            if (ok) {
                const size_t o = side == 0 ? (size_t)(y0 - 1) * CW + x0 + i
                               : side == 1 ? (size_t)(y0 + 8) * CW + x0 + i
                               : side == 2 ? (size_t)(y0 + i) * CW + x0 - 1
                                           : (size_t)(y0 + i) * CW + x0 + 8;
                v = cc_ld_byte(P + o);
            }
            v += __shfl_xor(v, 1);                // groups of 2
            if ((i & 1) == 0) sums[1 + plane][side][i >> 1] = (int32_t)v;
        }
        __syncthreads();
        int32_t fp[16];
        {   // luma: lane -> row y = lane >> 2, columns 4 * (lane & 3) .. +3
            cc_plane_fp(sums[0], A, B, L, R, 0, fp);
            const int y = lane >> 2, g = lane & 3;
            const uint32_t v = (uint32_t)cc_clip1(fp[(y >> 2) * 4 + g]) * 0x01010101u;
            *(uint32_t *)(Y + (size_t)(row * 16 + y) * W + col * 16 + g * 4) = v;
        }
        {   // chroma: lane -> plane, row y = (lane & 31) >> 2, columns 2 * (lane & 3) .. +1
            const int plane = lane >> 5, rest = lane & 31, y = rest >> 2, g = rest & 3;
            cc_plane_fp(sums[1 + plane], A, B, L, R, 1, fp);
            const uint16_t v = (uint16_t)((uint32_t)cc_clip1(fp[(y >> 1) * 4 + g]) * 0x0101u);
            *(uint16_t *)((plane ? V : U) + (size_t)(row * 8 + y) * CW + col * 8 + g * 2) = v;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this MB's samples in L2 before the next MB reads
        if (lane == 0) cc_dec[mb] = 1;
        __syncthreads();
    }
}
