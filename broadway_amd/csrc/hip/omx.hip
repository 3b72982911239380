// OpenMAX DL omxVCM4P10_* primitives (include/h264mi_omx.h) on the GPU.
//
// Each call packs its inputs -- neighbour samples, the reference window, the
// edge region, unpacked coefficients -- into one job, has the calling thread's
// resident job server (k_omx_server) run it and unpacks the result into the
// caller's strided buffers.  The arithmetic restates the reference
// implementations under Decoder/omxdl/reference/vc/m4p10/src (file cited per
// primitive); their argument checks are mirrored on the host, before any
// output is written.  tests/test_omx.py compares every primitive with the
// reference C built from those sources (oracle/Makefile.omx).
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#include "../../../include/h264mi_omx.h"

namespace {

enum { OP_I4 = 1, OP_I16, OP_ICH, OP_LUMA, OP_CHROMA, OP_DBL_V, OP_DBL_H, OP_DBC_V, OP_DBC_H, OP_LUMADC, OP_CHROMADC,
       OP_RESID };

#define WIN 21                     // luma window stride (16 + 5)

struct OmxJob {
    int op, mode, avail, w, h, dx, dy, qp, ac, has_dc;
    uint8_t alpha[2], beta[2], thr[16], bs[16];
    int16_t coef[16];
    int16_t dc;
    uint8_t in[WIN * WIN + 3];     // neighbours / window / edge region (deblocking: in place)
    uint8_t out[256];
    int16_t sout[16];
};

__device__ __forceinline__ int clip255(int v) { return v < 0 ? 0 : v > 255 ? 255 : v; }
__device__ __forceinline__ int clip3(int lo, int hi, int v) { return v < lo ? lo : v > hi ? hi : v; }
__device__ __forceinline__ int iabs(int v) { return v < 0 ? -v : v; }

// ---- intra (omxVCM4P10_PredictIntra_4x4.c, _16x16.c, PredictIntraChroma_8x8.c,
//      armVCM4P10_PredictIntraDC4x4.c).  in: [0] above-left, [1..16] above
//      (4x4: 8 entries, the last four replaced by above[3] without
//      UPPER_RIGHT), [17..32] left
__device__ int i4_pixel(const OmxJob &j, int x, int y)
{
    const uint8_t *U = j.in + 1, *L = j.in + 17;
    const int UL = j.in[0];
    auto P = [&](int px, int py) -> int {          // p[px, py], px or py == -1
        if (py < 0) return px < 0 ? UL : U[px];
        return L[py];
    };
    const int zvr = 2 * x - y, zhd = 2 * y - x, zhu = x + 2 * y;
    switch (j.mode) {
    case 0: return U[x];
    case 1: return L[y];
    case 2: {
        int s = 0, n = 0;
        if (j.avail & H264MI_OMX_VC_LEFT) { s += L[0] + L[1] + L[2] + L[3]; n++; }
        if (j.avail & H264MI_OMX_VC_UPPER) { s += U[0] + U[1] + U[2] + U[3]; n++; }
        return n == 0 ? 128 : n == 1 ? (s + 2) >> 2 : (s + 4) >> 3;
    }
    case 3:
        if (x == 3 && y == 3) return (U[6] + 3 * U[7] + 2) >> 2;
        return (U[x + y] + 2 * U[x + y + 1] + U[x + y + 2] + 2) >> 2;
    case 4: {
        const int z = x - y;
        if (z > 0) return (P(z - 2, -1) + 2 * P(z - 1, -1) + P(z, -1) + 2) >> 2;
        if (z < 0) return (P(-1, -z - 2) + 2 * P(-1, -z - 1) + P(-1, -z) + 2) >> 2;
        return (U[0] + 2 * UL + L[0] + 2) >> 2;
    }
    case 5:
        if (zvr >= 0 && !(zvr & 1)) return (P(x - (y >> 1) - 1, -1) + P(x - (y >> 1), -1) + 1) >> 1;
        if (zvr > 0) return (P(x - (y >> 1) - 2, -1) + 2 * P(x - (y >> 1) - 1, -1) + P(x - (y >> 1), -1) + 2) >> 2;
        if (zvr == -1) return (L[0] + 2 * UL + U[0] + 2) >> 2;
        return (P(-1, y - 1) + 2 * P(-1, y - 2) + P(-1, y - 3) + 2) >> 2;
    case 6:
        if (zhd >= 0 && !(zhd & 1)) return (P(-1, y - (x >> 1) - 1) + P(-1, y - (x >> 1)) + 1) >> 1;
        if (zhd > 0) return (P(-1, y - (x >> 1) - 2) + 2 * P(-1, y - (x >> 1) - 1) + P(-1, y - (x >> 1)) + 2) >> 2;
        if (zhd == -1) return (L[0] + 2 * UL + U[0] + 2) >> 2;
        return (P(x - 1, -1) + 2 * P(x - 2, -1) + P(x - 3, -1) + 2) >> 2;
    case 7:
        if (!(y & 1)) return (U[x + (y >> 1)] + U[x + (y >> 1) + 1] + 1) >> 1;
        return (U[x + (y >> 1)] + 2 * U[x + (y >> 1) + 1] + U[x + (y >> 1) + 2] + 2) >> 2;
    default:
        if (zhu > 5) return L[3];
        if (zhu == 5) return (L[2] + 3 * L[3] + 2) >> 2;
        if (!(zhu & 1)) return (L[y + (x >> 1)] + L[y + (x >> 1) + 1] + 1) >> 1;
        return (L[y + (x >> 1)] + 2 * L[y + (x >> 1) + 1] + L[y + (x >> 1) + 2] + 2) >> 2;
    }
}

// DC of one 4x4 quadrant of chroma: both (DC4x4), above first (DCUp4x4), left first (DCLeft4x4)
__device__ int dc4(const uint8_t *U, const uint8_t *L, int avail, int kind)
{
    const bool hl = avail & H264MI_OMX_VC_LEFT, hu = avail & H264MI_OMX_VC_UPPER;
    const int su = U[0] + U[1] + U[2] + U[3], sl = L[0] + L[1] + L[2] + L[3];
    if (kind == 0) {
        const int n = hl + hu, s = (hl ? sl : 0) + (hu ? su : 0);
        return n == 0 ? 128 : n == 1 ? (s + 2) >> 2 : (s + 4) >> 3;
    }
    if (kind == 1) return hu ? (su + 2) >> 2 : hl ? (sl + 2) >> 2 : 128;
    return hl ? (sl + 2) >> 2 : hu ? (su + 2) >> 2 : 128;
}

__device__ int i16_pixel(const OmxJob &j, int x, int y)
{
    const uint8_t *U = j.in + 1, *L = j.in + 17;
    const int UL = j.in[0];
    switch (j.mode) {
    case 0: return U[x];
    case 1: return L[y];
    case 2: {
        int s = 0, n = 0;
        if (j.avail & H264MI_OMX_VC_LEFT) { for (int i = 0; i < 16; i++) s += L[i]; n++; }
        if (j.avail & H264MI_OMX_VC_UPPER) { for (int i = 0; i < 16; i++) s += U[i]; n++; }
        return n == 0 ? 128 : n == 1 ? (s + 8) >> 4 : (s + 16) >> 5;
    }
    default: {
        int H = 8 * (U[15] - UL), V = 8 * (L[15] - UL);
        for (int i = 0; i < 7; i++) { H += (i + 1) * (U[8 + i] - U[6 - i]); V += (i + 1) * (L[8 + i] - L[6 - i]); }
        const int a = 16 * (U[15] + L[15]), b = (5 * H + 32) >> 6, c = (5 * V + 32) >> 6;
        return clip255((a + b * (x - 7) + c * (y - 7) + 16) >> 5);
    }
    }
}

__device__ int ich_pixel(const OmxJob &j, int x, int y)
{
    const uint8_t *U = j.in + 1, *L = j.in + 17;
    const int UL = j.in[0];
    switch (j.mode) {
    case 0: {
        const int qx = x >> 2, qy = y >> 2;
        // quadrants: (0,0) DC4x4, (1,0) DCUp4x4, (0,1) DCLeft4x4, (1,1) DC4x4
        const int kind = (qx == qy) ? 0 : qx ? 1 : 2;
        return dc4(U + 4 * qx, L + 4 * qy, j.avail, kind);
    }
    case 1: return L[y];
    case 2: return U[x];
    default: {
        int H = 4 * (U[7] - UL), V = 4 * (L[7] - UL);
        for (int i = 0; i < 3; i++) { H += (i + 1) * (U[4 + i] - U[2 - i]); V += (i + 1) * (L[4 + i] - L[2 - i]); }
        const int a = 16 * (U[7] + L[7]), b = (17 * H + 16) >> 5, c = (17 * V + 16) >> 5;
        return clip255((a + b * (x - 3) + c * (y - 3) + 16) >> 5);
    }
    }
}

// ---- interpolation (armVCM4P10_Interpolate_Luma.c, _HalfHor / _HalfVer /
//      _HalfDiag_Luma.c, armVCM4P10_Interpolate_Chroma.c).  in: the window
//      rows -2..h+2, columns -2..w+2 of the integer position, stride WIN
__device__ __forceinline__ int G(const OmxJob &j, int x, int y) { return j.in[(y + 2) * WIN + x + 2]; }
__device__ __forceinline__ int hraw(const OmxJob &j, int x, int y)   // half between (x, y) and (x + 1, y), unscaled
{
    return G(j, x - 2, y) - 5 * G(j, x - 1, y) + 20 * G(j, x, y) + 20 * G(j, x + 1, y) - 5 * G(j, x + 2, y) + G(j, x + 3, y);
}
__device__ __forceinline__ int vraw(const OmxJob &j, int x, int y)   // half between (x, y) and (x, y + 1)
{
    return G(j, x, y - 2) - 5 * G(j, x, y - 1) + 20 * G(j, x, y) + 20 * G(j, x, y + 1) - 5 * G(j, x, y + 2) + G(j, x, y + 3);
}
__device__ int luma_pixel(const OmxJob &j, int x, int y)
{
    const int dx = j.dx, dy = j.dy;
    auto b = [&](int xx, int yy) { return clip255((hraw(j, xx, yy) + 16) >> 5); };
    auto h = [&](int xx, int yy) { return clip255((vraw(j, xx, yy) + 16) >> 5); };
    auto jj = [&]() {
        const int v = hraw(j, x, y - 2) - 5 * hraw(j, x, y - 1) + 20 * hraw(j, x, y) + 20 * hraw(j, x, y + 1) -
                      5 * hraw(j, x, y + 2) + hraw(j, x, y + 3);
        return clip255((v + 512) >> 10);
    };
    auto avg = [](int a, int c) { return (a + c + 1) >> 1; };
    if (dx == 0 && dy == 0) return G(j, x, y);
    if (dy == 0) return dx == 2 ? b(x, y) : avg(b(x, y), G(j, x + (dx == 3), y));
    if (dx == 0) return dy == 2 ? h(x, y) : avg(h(x, y), G(j, x, y + (dy == 3)));
    if (dx == 2 || dy == 2) {
        int v = jj();
        if (dx != 2) v = avg(v, h(x + (dx == 3), y));
        if (dy != 2) v = avg(v, b(x, y + (dy == 3)));
        return v;
    }
    return avg(b(x, y + (dy == 3)), h(x + (dx == 3), y));
}

__device__ int chroma_pixel(const OmxJob &j, int x, int y)
{
    const int dx = j.dx, dy = j.dy;
    const uint8_t *s = j.in;           // rows 0..h, columns 0..w, stride 9
    const int A = s[y * 9 + x], B = s[y * 9 + x + 1], C = s[(y + 1) * 9 + x], D = s[(y + 1) * 9 + x + 1];
    if (dx == 0 && dy == 0) return A;
    return ((8 - dx) * (8 - dy) * A + dx * (8 - dy) * B + (8 - dx) * dy * C + dx * dy * D + 32) >> 6;
}

// ---- deblocking (armVCM4P10_DeBlockPixel.c): one line across one edge,
//      q0 at p, step between samples
__device__ void deblock_pixel(uint8_t *q, int step, int tc0, int alpha, int beta, int bs, bool chroma)
{
    if (bs == 0) return;
    const int p3 = q[-4 * step], p2 = q[-3 * step], p1 = q[-2 * step], p0 = q[-step];
    const int q0 = q[0], q1 = q[step], q2 = q[2 * step], q3 = q[3 * step];
    if (iabs(p0 - q0) >= alpha || iabs(p1 - p0) >= beta || iabs(q1 - q0) >= beta) return;
    const int ap = iabs(p2 - p0), aq = iabs(q2 - q0);
    if (bs < 4) {
        const int tc = chroma ? tc0 + 1 : tc0 + (ap < beta) + (aq < beta);
        const int d = clip3(-tc, tc, (((q0 - p0) << 2) + (p1 - q1) + 4) >> 3);
        q[-step] = (uint8_t)clip255(p0 + d);
        q[0] = (uint8_t)clip255(q0 - d);
        if (!chroma && ap < beta) q[-2 * step] = (uint8_t)(p1 + clip3(-tc0, tc0, (p2 + ((p0 + q0 + 1) >> 1) - (p1 << 1)) >> 1));
        if (!chroma && aq < beta) q[step] = (uint8_t)(q1 + clip3(-tc0, tc0, (q2 + ((p0 + q0 + 1) >> 1) - (q1 << 1)) >> 1));
        return;
    }
    const bool strong = iabs(p0 - q0) < ((alpha >> 2) + 2);
    if (!chroma && ap < beta && strong) {
        q[-step] = (uint8_t)((p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3);
        q[-2 * step] = (uint8_t)((p2 + p1 + p0 + q0 + 2) >> 2);
        q[-3 * step] = (uint8_t)((2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3);
    } else {
        q[-step] = (uint8_t)((2 * p1 + p0 + q1 + 2) >> 2);
    }
    if (!chroma && aq < beta && strong) {
        q[0] = (uint8_t)((q2 + 2 * q1 + 2 * q0 + 2 * p0 + p1 + 4) >> 3);
        q[step] = (uint8_t)((q2 + q1 + p0 + q0 + 2) >> 2);
        q[2 * step] = (uint8_t)((2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3);
    } else {
        q[0] = (uint8_t)((2 * q1 + q0 + p1 + 2) >> 2);
    }
}

// ---- residual (omxVCM4P10_DequantTransformResidualFromPairAndAdd.c,
//      TransformDequantLumaDCFromPair.c, TransformDequantChromaDCFromPair.c,
//      armVCM4P10_TransformResidual4x4.c, armVCM4P10_DequantTables.c)
__constant__ uint8_t cV[6][3] = {{10, 16, 13}, {11, 18, 14}, {13, 20, 16}, {14, 23, 18}, {16, 25, 20}, {18, 29, 23}};
__constant__ uint8_t cPosToVCol[16] = {0, 2, 0, 2, 2, 1, 2, 1, 0, 2, 0, 2, 2, 1, 2, 1};

__device__ void itrans4(int16_t *d)
{
    for (int i = 0; i < 16; i += 4) {
        const int e0 = d[i] + d[i + 2], e1 = d[i] - d[i + 2], e2 = (d[i + 1] >> 1) - d[i + 3], e3 = d[i + 1] + (d[i + 3] >> 1);
        d[i] = (int16_t)(e0 + e3); d[i + 1] = (int16_t)(e1 + e2); d[i + 2] = (int16_t)(e1 - e2); d[i + 3] = (int16_t)(e0 - e3);
    }
    for (int i = 0; i < 4; i++) {
        const int f0 = d[i], f1 = d[i + 4], f2 = d[i + 8], f3 = d[i + 12];
        const int g0 = f0 + f2, g1 = f0 - f2, g2 = (f1 >> 1) - f3, g3 = f1 + (f3 >> 1);
        d[i] = (int16_t)((g0 + g3 + 32) >> 6); d[i + 4] = (int16_t)((g1 + g2 + 32) >> 6);
        d[i + 8] = (int16_t)((g1 - g2 + 32) >> 6); d[i + 12] = (int16_t)((g0 - g3 + 32) >> 6);
    }
}

// the job lives in pinned host memory mapped into the device: one coalesced
// read into LDS, the primitive on the LDS copy, one coalesced write back --
// no H2D / D2H copies around the launch
__device__ void k_omx_body(OmxJob &j, int t);
__global__ __launch_bounds__(256) void k_omx(OmxJob *jp)
{
    __shared__ OmxJob js;
    static_assert(sizeof(OmxJob) % 4 == 0, "OmxJob copied in dwords");
    const int t = threadIdx.x;
    const uint32_t *src = (const uint32_t *)jp;
    uint32_t *dst = (uint32_t *)&js;
    for (int i = t; i < (int)(sizeof(OmxJob) / 4); i += 256) dst[i] = src[i];
    __syncthreads();
    k_omx_body(js, t);
    __syncthreads();
    for (int i = t; i < (int)(sizeof(OmxJob) / 4); i += 256) ((uint32_t *)jp)[i] = dst[i];
}
__device__ void k_omx_body(OmxJob &j, int t)
{
    switch (j.op) {
    case OP_I4:
        if (t < 16) j.out[t] = (uint8_t)i4_pixel(j, t & 3, t >> 2);
        break;
    case OP_I16:
        j.out[t] = (uint8_t)i16_pixel(j, t & 15, t >> 4);
        break;
    case OP_ICH:
        if (t < 64) j.out[t] = (uint8_t)ich_pixel(j, t & 7, t >> 3);
        break;
    case OP_LUMA:
        if (t < j.w * j.h) j.out[t] = (uint8_t)luma_pixel(j, t % j.w, t / j.w);
        break;
    case OP_CHROMA:
        if (t < j.w * j.h) j.out[t] = (uint8_t)chroma_pixel(j, t % j.w, t / j.w);
        break;
    case OP_DBL_V:          // region 16 rows x 20 columns (-4..15); one lane per row
        if (t < 16)
            for (int X = 0; X < 16; X += 4) {
                const int I = (t >> 2) + 4 * (X >> 2), in = X > 0;
                deblock_pixel(j.in + t * 20 + 4 + X, 1, j.thr[I], j.alpha[in], j.beta[in], j.bs[I], false);
            }
        break;
    case OP_DBL_H:          // region 20 rows (-4..15) x 16 columns; one lane per column
        if (t < 16)
            for (int Y = 0; Y < 16; Y += 4) {
                const int I = (t >> 2) + 4 * (Y >> 2), in = Y > 0;
                deblock_pixel(j.in + (4 + Y) * 16 + t, 16, j.thr[I], j.alpha[in], j.beta[in], j.bs[I], false);
            }
        break;
    case OP_DBC_V:          // 8 rows x 12 columns (-4..7)
        if (t < 8)
            for (int X = 0; X < 8; X += 4) {
                const int in = X > 0;
                deblock_pixel(j.in + t * 12 + 4 + X, 1, j.thr[(t >> 1) + 4 * (X >> 2)], j.alpha[in], j.beta[in],
                              j.bs[(t >> 1) + 4 * (X >> 1)], true);
            }
        break;
    case OP_DBC_H:          // 12 rows (-4..7) x 8 columns
        if (t < 8)
            for (int Y = 0; Y < 8; Y += 4) {
                const int in = Y > 0;
                deblock_pixel(j.in + (4 + Y) * 8 + t, 8, j.thr[(t >> 1) + 4 * (Y >> 2)], j.alpha[in], j.beta[in],
                              j.bs[(t >> 1) + 4 * (Y >> 1)], true);
            }
        break;
    case OP_LUMADC:
        if (t == 0) {
            int16_t d[16];
            for (int i = 0; i < 16; i++) d[i] = j.coef[i];
            for (int i = 0; i < 16; i += 4) {
                const int c0 = d[i], c1 = d[i + 1], c2 = d[i + 2], c3 = d[i + 3];
                d[i] = (int16_t)(c0 + c1 + c2 + c3); d[i + 1] = (int16_t)(c0 + c1 - c2 - c3);
                d[i + 2] = (int16_t)(c0 - c1 - c2 + c3); d[i + 3] = (int16_t)(c0 - c1 + c2 - c3);
            }
            for (int i = 0; i < 4; i++) {
                const int c0 = d[i], c1 = d[i + 4], c2 = d[i + 8], c3 = d[i + 12];
                d[i] = (int16_t)(c0 + c1 + c2 + c3); d[i + 4] = (int16_t)(c0 + c1 - c2 - c3);
                d[i + 8] = (int16_t)(c0 - c1 - c2 + c3); d[i + 12] = (int16_t)(c0 - c1 + c2 - c3);
            }
            const int sh = j.qp / 6 - 2, sc = cV[j.qp % 6][0];
            for (int i = 0; i < 16; i++)
                j.sout[i] = (int16_t)(sh >= 0 ? (d[i] * sc) << sh : (d[i] * sc + (1 << (-sh - 1))) >> -sh);
        }
        break;
    case OP_CHROMADC:
        if (t == 0) {
            const int c00 = j.coef[0], c01 = j.coef[1], c10 = j.coef[2], c11 = j.coef[3];
            int16_t d[4] = {(int16_t)(c00 + c01 + c10 + c11), (int16_t)(c00 - c01 + c10 - c11),
                            (int16_t)(c00 + c01 - c10 - c11), (int16_t)(c00 - c01 - c10 + c11)};
            const int sh = j.qp / 6 - 1, sc = cV[j.qp % 6][0];
            for (int i = 0; i < 4; i++) j.sout[i] = (int16_t)(sh >= 0 ? (d[i] * sc) << sh : (d[i] * sc) >> 1);
        }
        break;
    case OP_RESID:          // in: prediction 4x4
        if (t == 0) {
            int16_t d[16];
            for (int i = 0; i < 16; i++) d[i] = 0;
            if (j.ac)
                for (int i = 0; i < 16; i++) d[i] = (int16_t)((j.coef[i] * cV[j.qp % 6][cPosToVCol[i]]) << (j.qp / 6));
            if (j.has_dc) d[0] = j.dc;
            itrans4(d);
            for (int i = 0; i < 16; i++) j.out[i] = (uint8_t)clip255(j.in[i] + d[i]);
        }
        break;
    }
}

// ---- the per-thread job server.  A launch per call costs 16-17 us of launch
// and stream-synchronisation latency against ~1 us of work, so each calling
// thread keeps one workgroup resident that serves its jobs: the host writes the
// job and a request number into pinned coherent memory, the server (polling
// that number over PCIe) runs the primitive and writes the job and an
// acknowledgement back; no launch, no stream wait.  The server leaves after
// `idle` wall-clock ticks without a request or when asked to stop (the STOP
// bit of req), and says so in `gone` before a last look at req; a host that
// sees `gone` waits for the server's stream, and relaunches it from the last
// request it saw if its own request was not served, so a request racing the
// exit is never lost.
struct OmxCtl {
    uint32_t req, pad0[15];                 // host -> server (own 64-byte line): request number | STOP
    uint32_t ack, gone, pad1[14];           // server -> host: last request done; GONE | last request seen
};
#define OMX_GONE 0x80000000u
#define OMX_STOP 0x80000000u

__device__ __forceinline__ uint32_t ld_sys(const uint32_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(uint32_t *p, uint32_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(256) void k_omx_server(OmxJob *jp, OmxCtl *ctl, uint32_t last, uint64_t idle)
{
    __shared__ OmxJob js;
    __shared__ uint32_t s_req, s_quit;
    const int t = threadIdx.x;
    const int nw = (int)(sizeof(OmxJob) / 4);
    uint64_t t0 = wall_clock64();
    for (;;) {
        if (t == 0) {
            uint32_t r, quit = 0;
            for (;;) {
                r = ld_sys(&ctl->req);
                if (r & OMX_STOP) { quit = 1; r &= ~OMX_STOP; break; }
                if (r != last) break;
                if (wall_clock64() - t0 > idle) { quit = 1; break; }
            }
            if (quit) {                     // announce, then one last look at req
                st_sys(&ctl->gone, OMX_GONE | last);
                r = ld_sys(&ctl->req) & ~OMX_STOP;
            }
            s_req = r;
            s_quit = quit;
        }
        __syncthreads();
        const uint32_t r = s_req, quit = s_quit;
        if (r == last) break;               // quitting with nothing pending: every wave leaves here
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        const uint32_t *src = (const uint32_t *)jp;
        uint32_t *dst = (uint32_t *)&js;
        for (int i = t; i < nw; i += 256) dst[i] = src[i];
        __syncthreads();
        k_omx_body(js, t);
        __syncthreads();
        for (int i = t; i < nw; i += 256) ((uint32_t *)jp)[i] = dst[i];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __syncthreads();
        last = r;
        if (t == 0) {
            st_sys(&ctl->ack, r);
            if (quit) st_sys(&ctl->gone, OMX_GONE | r);
        }
        if (quit) break;
        t0 = wall_clock64();
    }
}

// ---- host side: one job server per calling thread, on its own stream
struct OmxCtx {
    hipStream_t st = nullptr;
    OmxJob *h = nullptr, *d = nullptr;      // pinned host job, its device address
    OmxCtl *hc = nullptr, *dc = nullptr;    // pinned control words
    uint32_t seq = 0;                       // last request posted (below the STOP bit)
    uint64_t idle = 0;                      // server idle limit in wall-clock ticks
    int ok = 0, server = 1, running = 0;
    ~OmxCtx()
    {
        if (running) {
            __atomic_store_n(&hc->req, seq | OMX_STOP, __ATOMIC_RELEASE);
            (void)hipStreamSynchronize(st);
        }
        if (st) (void)hipStreamDestroy(st);
        if (h) (void)hipHostFree(h);
        if (hc) (void)hipHostFree(hc);
    }
};
thread_local OmxCtx g_ctx;

OmxJob *job_begin(int op)
{
    OmxCtx &c = g_ctx;
    if (!c.ok) {
        int dev = 0, khz = 0;
        if (hipStreamCreateWithFlags(&c.st, hipStreamNonBlocking) != hipSuccess ||
            hipHostMalloc(&c.h, sizeof(OmxJob), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
            hipHostGetDevicePointer((void **)&c.d, c.h, 0) != hipSuccess ||
            hipHostMalloc(&c.hc, sizeof(OmxCtl), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
            hipHostGetDevicePointer((void **)&c.dc, c.hc, 0) != hipSuccess || hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0)
            return nullptr;
        memset(c.hc, 0, sizeof(OmxCtl));
        const char *e = getenv("H264MI_OMX_SERVER");    // 0: one k_omx launch per call
        c.server = !(e && e[0] == '0');
        c.idle = (uint64_t)khz * 20;                    // 20 ms without a request
        c.ok = 1;
    }
    memset(c.h, 0, offsetof(OmxJob, in));
    c.h->op = op;
    return c.h;
}

int server_launch(OmxCtx &c, uint32_t last)
{
    __atomic_store_n(&c.hc->gone, 0u, __ATOMIC_RELEASE);
    hipLaunchKernelGGL(k_omx_server, dim3(1), dim3(256), 0, c.st, c.d, c.dc, last, c.idle);
    if (hipGetLastError() != hipSuccess) return -1;
    c.running = 1;
    return 0;
}

// the job on the mapped page, run and waited for; 0 or a failure independent
// of the arguments (-1)
int job_run()
{
    OmxCtx &c = g_ctx;
    if (!c.server) {
        hipLaunchKernelGGL(k_omx, dim3(1), dim3(256), 0, c.st, c.d);
        if (hipGetLastError() != hipSuccess) return -1;
        return hipStreamSynchronize(c.st) == hipSuccess ? 0 : -1;
    }
    c.seq = (c.seq + 1) & ~OMX_STOP;
    if (!c.seq) c.seq = 1;
    const uint32_t want = c.seq;
    __atomic_store_n(&c.hc->req, want, __ATOMIC_RELEASE);
    if (!c.running && server_launch(c, want - 1)) return -1;
    for (uint64_t spin = 0;; spin++) {
        if (__atomic_load_n(&c.hc->ack, __ATOMIC_ACQUIRE) == want) return 0;
        const uint32_t g = __atomic_load_n(&c.hc->gone, __ATOMIC_ACQUIRE);
        if (g & OMX_GONE) {                 // the server left; if it left before seeing this request, relaunch
            if (hipStreamSynchronize(c.st) != hipSuccess) { c.running = 0; return -1; }
            c.running = 0;
            if (__atomic_load_n(&c.hc->ack, __ATOMIC_ACQUIRE) == want) return 0;
            if (server_launch(c, g & ~OMX_GONE)) return -1;
            spin = 0;
        }
        if ((spin & 0xFFFF) == 0xFFFF) {    // a faulted server shows on its stream
            const hipError_t q = hipStreamQuery(c.st);
            if (q != hipSuccess && q != hipErrorNotReady) { c.running = 0; return -1; }
        }
        __builtin_ia32_pause();
    }
}

inline bool misaligned(const void *p, uintptr_t a) { return ((uintptr_t)p & (a - 1)) != 0; }

// neighbours of the intra predictions into in[0 .. 32]
void pack_neighbours(OmxJob *j, const OMX_U8 *L, const OMX_U8 *U, const OMX_U8 *UL, int leftStep, int n, int nu, int avail)
{
    if ((avail & H264MI_OMX_VC_UPPER_LEFT) && UL) j->in[0] = UL[0];
    if (avail & H264MI_OMX_VC_UPPER)
        for (int i = 0; i < nu; i++) j->in[1 + i] = U[i];
    if (avail & H264MI_OMX_VC_LEFT)
        for (int i = 0; i < n; i++) j->in[17 + i] = L[i * leftStep];
}

// the pair-buffer block of armVCM4P10_UnpackBlock4x4.c / 2x2.c: per
// coefficient a flag byte (bits 0-3 position, bit 4 16-bit value, bit 5 last)
// and an 8- or 16-bit value
const OMX_U8 *unpack_pairs(const OMX_U8 *p, int16_t *dst, int n)
{
    for (int i = 0; i < n; i++) dst[i] = 0;
    int flag;
    do {
        flag = *p++;
        int v;
        if (flag & 0x10) { v = p[0] | (p[1] << 8); p += 2; if (v & 0x8000) v -= 0x10000; }
        else { v = *p++; if (v & 0x80) v -= 0x100; }
        dst[flag & 15] = (int16_t)v;
    } while (!(flag & 0x20));
    return p;
}

} // namespace

#define BADARG(c) do { if (c) return H264MI_OMX_Sts_BadArgErr; } while (0)

extern "C" OMXResult omxVCM4P10_PredictIntra_4x4(const OMX_U8 *pSrcLeft, const OMX_U8 *pSrcAbove,
                                                 const OMX_U8 *pSrcAboveLeft, OMX_U8 *pDst, OMX_INT leftStep,
                                                 OMX_INT dstStep, int predMode, OMX_S32 availability)
{
    const int a = availability, U = a & H264MI_OMX_VC_UPPER, L = a & H264MI_OMX_VC_LEFT, UL = a & H264MI_OMX_VC_UPPER_LEFT;
    BADARG(pDst == NULL || leftStep % 4 || dstStep % 4 || dstStep < 4 || misaligned(pSrcAbove, 4) || misaligned(pDst, 4));
    BADARG((U && !pSrcAbove) || (L && !pSrcLeft) || (UL && !pSrcAboveLeft));
    BADARG((predMode == 0 || predMode == 3 || predMode == 7) && !U);
    BADARG((predMode == 1 || predMode == 8) && !L);
    BADARG(predMode >= 4 && predMode <= 6 && !(U && UL && L));
    BADARG((unsigned)predMode > 8);
    OmxJob *j = job_begin(OP_I4);
    if (!j) return -1;
    j->mode = predMode; j->avail = a;
    pack_neighbours(j, pSrcLeft, pSrcAbove, pSrcAboveLeft, leftStep, 4,
                    (a & H264MI_OMX_VC_UPPER_RIGHT) ? 8 : 4, a);
    if (U && !(a & H264MI_OMX_VC_UPPER_RIGHT))         // p[4..7, -1] = p[3, -1]
        for (int i = 4; i < 8; i++) j->in[1 + i] = j->in[4];
    if (job_run()) return -1;
    for (int y = 0; y < 4; y++) memcpy(pDst + y * dstStep, j->out + y * 4, 4);
    return H264MI_OMX_Sts_NoErr;
}

extern "C" OMXResult omxVCM4P10_PredictIntra_16x16(const OMX_U8 *pSrcLeft, const OMX_U8 *pSrcAbove,
                                                   const OMX_U8 *pSrcAboveLeft, OMX_U8 *pDst, OMX_INT leftStep,
                                                   OMX_INT dstStep, int predMode, OMX_S32 availability)
{
    const int a = availability, U = a & H264MI_OMX_VC_UPPER, L = a & H264MI_OMX_VC_LEFT, UL = a & H264MI_OMX_VC_UPPER_LEFT;
    BADARG(pDst == NULL || dstStep < 16 || dstStep % 16 || leftStep % 16 || misaligned(pSrcAbove, 16) ||
           misaligned(pDst, 16));
    BADARG((U && !pSrcAbove) || (L && !pSrcLeft) || (UL && !pSrcAboveLeft));
    BADARG((predMode == 0 && !U) || (predMode == 1 && !L) || (predMode == 3 && !(U && UL && L)));
    BADARG((unsigned)predMode > 3);
    OmxJob *j = job_begin(OP_I16);
    if (!j) return -1;
    j->mode = predMode; j->avail = a;
    pack_neighbours(j, pSrcLeft, pSrcAbove, pSrcAboveLeft, leftStep, 16, 16, a);
    if (job_run()) return -1;
    for (int y = 0; y < 16; y++) memcpy(pDst + y * dstStep, j->out + y * 16, 16);
    return H264MI_OMX_Sts_NoErr;
}

extern "C" OMXResult omxVCM4P10_PredictIntraChroma_8x8(const OMX_U8 *pSrcLeft, const OMX_U8 *pSrcAbove,
                                                       const OMX_U8 *pSrcAboveLeft, OMX_U8 *pDst, OMX_INT leftStep,
                                                       OMX_INT dstStep, int predMode, OMX_S32 availability)
{
    const int a = availability, U = a & H264MI_OMX_VC_UPPER, L = a & H264MI_OMX_VC_LEFT, UL = a & H264MI_OMX_VC_UPPER_LEFT;
    BADARG(pDst == NULL || dstStep < 8 || dstStep % 8 || leftStep % 8 || misaligned(pSrcAbove, 8) || misaligned(pDst, 8));
    BADARG((U && !pSrcAbove) || (L && !pSrcLeft) || (UL && !pSrcAboveLeft));
    BADARG((predMode == 2 && !U) || (predMode == 1 && !L) || (predMode == 3 && !(U && UL && L)));
    BADARG((unsigned)predMode > 3);
    OmxJob *j = job_begin(OP_ICH);
    if (!j) return -1;
    j->mode = predMode; j->avail = a;
    pack_neighbours(j, pSrcLeft, pSrcAbove, pSrcAboveLeft, leftStep, 8, 8, a);
    if (job_run()) return -1;
    for (int y = 0; y < 8; y++) memcpy(pDst + y * dstStep, j->out + y * 8, 8);
    return H264MI_OMX_Sts_NoErr;
}

extern "C" OMXResult omxVCM4P10_InterpolateLuma(const OMX_U8 *pSrc, OMX_S32 srcStep, OMX_U8 *pDst, OMX_S32 dstStep,
                                                OMX_S32 dx, OMX_S32 dy, OMXSize roi)
{
    const int w = roi.width, h = roi.height;
    BADARG(pSrc == NULL || pDst == NULL || srcStep < w || dstStep < w || dx < 0 || dx > 3 || dy < 0 || dy > 3);
    BADARG((w != 4 && w != 8 && w != 16) || (h != 4 && h != 8 && h != 16));
    BADARG((w == 4 && misaligned(pDst, 4)) || (w == 8 && misaligned(pDst, 8)) || (w == 16 && misaligned(pDst, 16)));
    BADARG((srcStep & 7) || (dstStep & 7));
    OmxJob *j = job_begin(OP_LUMA);
    if (!j) return -1;
    j->w = w; j->h = h; j->dx = dx; j->dy = dy;
    // the samples the reference reads: columns -2..w+2 with a horizontal
    // fraction (else 0..w-1, and w for dx = 3), rows likewise
    const int x0 = dx ? -2 : 0, x1 = dx ? w + 3 : w, y0 = dy ? -2 : 0, y1 = dy ? h + 3 : h;
    for (int y = y0; y < y1; y++) memcpy(j->in + (y + 2) * WIN + x0 + 2, pSrc + y * srcStep + x0, (size_t)(x1 - x0));
    if (job_run()) return -1;
    for (int y = 0; y < h; y++) memcpy(pDst + y * dstStep, j->out + y * w, (size_t)w);
    return H264MI_OMX_Sts_NoErr;
}

extern "C" OMXResult omxVCM4P10_InterpolateChroma(const OMX_U8 *pSrc, OMX_S32 srcStep, OMX_U8 *pDst, OMX_S32 dstStep,
                                                  OMX_S32 dx, OMX_S32 dy, OMXSize roi)
{
    const int w = roi.width, h = roi.height;
    BADARG(pSrc == NULL || pDst == NULL || srcStep < 8 || dstStep < 8 || dx < 0 || dx > 7 || dy < 0 || dy > 7);
    BADARG((w != 2 && w != 4 && w != 8) || (h != 2 && h != 4 && h != 8));
    BADARG((w == 2 && misaligned(pDst, 2)) || (w == 4 && misaligned(pDst, 4)) || (w == 8 && misaligned(pDst, 8)));
    BADARG((srcStep & 7) || (dstStep & 7));
    OmxJob *j = job_begin(OP_CHROMA);
    if (!j) return -1;
    j->w = w; j->h = h; j->dx = dx; j->dy = dy;
    // rows 0..h and columns 0..w; the reference reads row h / column w only
    // with a fractional offset
    const int rw = (dx || dy) ? w + 1 : w, rh = (dx || dy) ? h + 1 : h;
    for (int y = 0; y < rh; y++) memcpy(j->in + y * 9, pSrc + y * srcStep, (size_t)rw);
    if (job_run()) return -1;
    for (int y = 0; y < h; y++) memcpy(pDst + y * dstStep, j->out + y * w, (size_t)w);
    return H264MI_OMX_Sts_NoErr;
}

namespace {
int deblock_common(OmxJob *j, const OMX_U8 *pAlpha, const OMX_U8 *pBeta, const OMX_U8 *pThresholds, const OMX_U8 *pBS)
{
    j->alpha[0] = pAlpha[0]; j->alpha[1] = pAlpha[1];
    j->beta[0] = pBeta[0]; j->beta[1] = pBeta[1];
    memcpy(j->thr, pThresholds, 16);
    memcpy(j->bs, pBS, 16);
    return 0;
}
} // namespace

#define DBARGS(al)                                                                                            \
    BADARG(pSrcDst == NULL || misaligned(pSrcDst, al) || (srcdstStep & (al - 1)) || pAlpha == NULL ||           \
           pBeta == NULL || pThresholds == NULL || misaligned(pThresholds, 4) || pBS == NULL ||              \
           misaligned(pBS, 4) || pBeta[0] > 18 || pBeta[1] > 18)

extern "C" OMXResult omxVCM4P10_FilterDeblockingLuma_VerEdge_I(OMX_U8 *pSrcDst, OMX_S32 srcdstStep,
                                                               const OMX_U8 *pAlpha, const OMX_U8 *pBeta,
                                                               const OMX_U8 *pThresholds, const OMX_U8 *pBS)
{
    DBARGS(16);
    for (int Y = 0; Y < 16; Y++)      // FilterDeblockingLuma_VerEdge_I.c: checks index pBS / pThresholds by line
        BADARG(pBS[Y] > 4 || (pBS[Y] == 4 && Y > 3) || (pBS[Y] == 4 && pBS[Y ^ 3] != 4) || pThresholds[Y] > 25);
    OmxJob *j = job_begin(OP_DBL_V);
    if (!j) return -1;
    deblock_common(j, pAlpha, pBeta, pThresholds, pBS);
    for (int y = 0; y < 16; y++) memcpy(j->in + y * 20, pSrcDst + y * srcdstStep - 4, 20);
    if (job_run()) return -1;
    for (int y = 0; y < 16; y++) memcpy(pSrcDst + y * srcdstStep - 4, j->in + y * 20, 20);
    return H264MI_OMX_Sts_NoErr;
}

extern "C" OMXResult omxVCM4P10_FilterDeblockingLuma_HorEdge_I(OMX_U8 *pSrcDst, OMX_S32 srcdstStep,
                                                               const OMX_U8 *pAlpha, const OMX_U8 *pBeta,
                                                               const OMX_U8 *pThresholds, const OMX_U8 *pBS)
{
    BADARG(pSrcDst == NULL || misaligned(pSrcDst, 8) || (srcdstStep & 7) || pAlpha == NULL || pBeta == NULL ||
           pThresholds == NULL || misaligned(pThresholds, 4) || pBS == NULL || misaligned(pBS, 4));
    for (int I = 0; I < 16; I++)
        BADARG(pBS[I] > 4 || (I > 3 && pBS[I] == 4) || (I < 4 && pBS[I] == 4 && pBS[I ^ 1] != 4));
    OmxJob *j = job_begin(OP_DBL_H);
    if (!j) return -1;
    deblock_common(j, pAlpha, pBeta, pThresholds, pBS);
    for (int y = -4; y < 16; y++) memcpy(j->in + (y + 4) * 16, pSrcDst + y * srcdstStep, 16);
    if (job_run()) return -1;
    for (int y = -4; y < 16; y++) memcpy(pSrcDst + y * srcdstStep, j->in + (y + 4) * 16, 16);
    return H264MI_OMX_Sts_NoErr;
}

extern "C" OMXResult omxVCM4P10_FilterDeblockingChroma_VerEdge_I(OMX_U8 *pSrcDst, OMX_S32 srcdstStep,
                                                                 const OMX_U8 *pAlpha, const OMX_U8 *pBeta,
                                                                 const OMX_U8 *pThresholds, const OMX_U8 *pBS)
{
    DBARGS(8);
    for (int X = 0; X < 8; X += 4)
        for (int Y = 0; Y < 8; Y++) {
            const int I = (Y >> 1) + 4 * (X >> 1);
            BADARG(pBS[I] > 4 || (I > 3 && pBS[I] == 4) || (pBS[I] == 4 && pBS[I ^ 3] != 4) || pThresholds[Y] > 25);
        }
    OmxJob *j = job_begin(OP_DBC_V);
    if (!j) return -1;
    deblock_common(j, pAlpha, pBeta, pThresholds, pBS);
    for (int y = 0; y < 8; y++) memcpy(j->in + y * 12, pSrcDst + y * srcdstStep - 4, 12);
    if (job_run()) return -1;
    for (int y = 0; y < 8; y++) memcpy(pSrcDst + y * srcdstStep - 4, j->in + y * 12, 12);
    return H264MI_OMX_Sts_NoErr;
}

extern "C" OMXResult omxVCM4P10_FilterDeblockingChroma_HorEdge_I(OMX_U8 *pSrcDst, OMX_S32 srcdstStep,
                                                                 const OMX_U8 *pAlpha, const OMX_U8 *pBeta,
                                                                 const OMX_U8 *pThresholds, const OMX_U8 *pBS)
{
    BADARG(pSrcDst == NULL || misaligned(pSrcDst, 8) || (srcdstStep & 7) || pAlpha == NULL || pBeta == NULL ||
           pThresholds == NULL || misaligned(pThresholds, 4) || pBS == NULL || misaligned(pBS, 4));
    for (int Y = 0; Y < 8; Y += 4)
        for (int X = 0; X < 8; X++) {
            const int I = (X >> 1) + 4 * (Y >> 1);
            BADARG(pBS[I] > 4 || (I > 3 && pBS[I] == 4) || (I < 4 && pBS[I] == 4 && pBS[I ^ 1] != 4));
        }
    OmxJob *j = job_begin(OP_DBC_H);
    if (!j) return -1;
    deblock_common(j, pAlpha, pBeta, pThresholds, pBS);
    for (int y = -4; y < 8; y++) memcpy(j->in + (y + 4) * 8, pSrcDst + y * srcdstStep, 8);
    if (job_run()) return -1;
    for (int y = -4; y < 8; y++) memcpy(pSrcDst + y * srcdstStep, j->in + (y + 4) * 8, 8);
    return H264MI_OMX_Sts_NoErr;
}

extern "C" OMXResult omxVCM4P10_TransformDequantLumaDCFromPair(const OMX_U8 **ppSrc, OMX_S16 *pDst, OMX_INT QP)
{
    BADARG(ppSrc == NULL || *ppSrc == NULL || pDst == NULL || misaligned(pDst, 8) || QP < 0 || QP > 51);
    OmxJob *j = job_begin(OP_LUMADC);
    if (!j) return -1;
    *ppSrc = unpack_pairs(*ppSrc, j->coef, 16);
    j->qp = QP;
    if (job_run()) return -1;
    memcpy(pDst, j->sout, 32);
    return H264MI_OMX_Sts_NoErr;
}

extern "C" OMXResult omxVCM4P10_TransformDequantChromaDCFromPair(const OMX_U8 **ppSrc, OMX_S16 *pDst, OMX_INT QP)
{
    BADARG(ppSrc == NULL || *ppSrc == NULL || pDst == NULL || misaligned(pDst, 4) || QP < 0 || QP > 51);
    OmxJob *j = job_begin(OP_CHROMADC);
    if (!j) return -1;
    *ppSrc = unpack_pairs(*ppSrc, j->coef, 4);
    j->qp = QP;
    if (job_run()) return -1;
    memcpy(pDst, j->sout, 8);
    return H264MI_OMX_Sts_NoErr;
}

extern "C" OMXResult omxVCM4P10_DequantTransformResidualFromPairAndAdd(const OMX_U8 **ppSrc, const OMX_U8 *pPred,
                                                                       const OMX_S16 *pDC, OMX_U8 *pDst,
                                                                       OMX_INT predStep, OMX_INT dstStep, OMX_INT QP,
                                                                       OMX_INT AC)
{
    BADARG(pPred == NULL || misaligned(pPred, 4) || pDst == NULL || misaligned(pDst, 4) || (predStep & 3) ||
           (dstStep & 3));
    BADARG(AC != 0 && (QP < 0 || QP > 51 || ppSrc == NULL || *ppSrc == NULL));
    BADARG(AC == 0 && pDC == NULL);
    OmxJob *j = job_begin(OP_RESID);
    if (!j) return -1;
    if (AC) *ppSrc = unpack_pairs(*ppSrc, j->coef, 16);
    j->ac = AC != 0; j->qp = QP;
    j->has_dc = pDC != NULL;
    if (pDC) j->dc = pDC[0];
    for (int y = 0; y < 4; y++) memcpy(j->in + y * 4, pPred + y * predStep, 4);
    if (job_run()) return -1;
    for (int y = 0; y < 4; y++) memcpy(pDst + y * dstStep, j->out + y * 4, 4);
    return H264MI_OMX_Sts_NoErr;
}
