// H.264 Baseline macroblock reconstruction + in-loop deblocking for gfx950.
//
// Two kernels per picture batch (one picture from each of S streams):
//   k_inter  -- every inter MB (P_L0_*, P_8x8, P_Skip) of every picture in the
//               batch, fully parallel: residual (dequant + 4x4 IDCT), 6-tap
//               luma / bilinear chroma motion compensation from HBM-resident
//               reference slots staged through LDS, clip-add, write-out, and a
//               copy of the MB's unfiltered bottom row / right column into the
//               edge buffer (intra neighbours read those after deblocking has
//               started).  Reference: h264bsdInterPrediction
//               (inter_prediction.c:364-487), h264bsdPredictSamples
//               (reconstruct.c:1819-1941), h264bsdWriteOutputBlocks
//               (image.c:171-343).
//   k_wave   -- one launch per MB anti-diagonal t = c + 2r (dependencies
//               (r,c-1), (r-1,c), (r-1,c+1)); for each MB on it: intra
//               reconstruction (I4x4 10-step sub-wavefront, I16x16, chroma,
//               I_PCM) from the edge buffers, then the MB's deblocking
//               (bS per 4x4 edge segment, thresholds, luma/chroma filters) in
//               the reference's raster-equivalent order.  Reference:
//               h264bsdIntraPrediction (intra_prediction.c:475-988),
//               h264bsdFilterPicture (deblocking.c:574-1736).
// One 64-lane wave per macroblock in both kernels.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../../include/h264mi_records.h"

#define WAVE 64

struct ReconArgs {
    uint8_t *frames;          // frame pool (I420 per slot)
    unsigned long long frame_bytes;
    const MbRec *rec;         // batch records (pictures back to back)
    const int16_t *coef;      // batch coefficient blocks
    uint8_t *edges;           // 64 B per MB of the batch
    const PicDesc *pics;
    int npics;
    int w, h;                 // picture size in MBs
    int diag;                 // k_wave: anti-diagonal index
    int diag_len;             // k_wave: max MBs on a diagonal
    unsigned int *err;        // residual range errors (per picture)
};

__constant__ uint8_t cZigzag[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
__constant__ uint8_t cLevelScale[6][3] = {
    {10, 16, 13}, {11, 18, 14}, {13, 20, 16}, {14, 23, 18}, {16, 25, 20}, {18, 29, 23}};
__constant__ uint8_t cAlpha[52] = {
    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 4, 4, 5, 6, 7, 8, 9, 10,
    12, 13, 15, 17, 20, 22, 25, 28, 32, 36, 40, 45, 50, 56, 63, 71, 80, 90,
    101, 113, 127, 144, 162, 182, 203, 226, 255, 255};
__constant__ uint8_t cBeta[52] = {
    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 2, 2, 3, 3, 3, 3, 4,
    4, 4, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13, 14, 14,
    15, 15, 16, 16, 17, 17, 18, 18};
__constant__ uint8_t cTc0[52][3] = {
    {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0},
    {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0},
    {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 1}, {0, 0, 1}, {0, 0, 1}, {0, 0, 1},
    {0, 1, 1}, {0, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 1, 2},
    {1, 1, 2}, {1, 1, 2}, {1, 1, 2}, {1, 2, 3}, {1, 2, 3}, {2, 2, 3}, {2, 2, 4},
    {2, 3, 4}, {2, 3, 4}, {3, 3, 5}, {3, 4, 6}, {3, 4, 6}, {4, 5, 7}, {4, 5, 8},
    {4, 6, 9}, {5, 7, 10}, {6, 8, 11}, {6, 8, 13}, {7, 10, 14}, {8, 11, 16},
    {9, 12, 18}, {10, 13, 20}, {11, 15, 23}, {13, 17, 25}};

__device__ __forceinline__ int clip255(int v) { return min(max(v, 0), 255); }
__device__ __forceinline__ int clip3(int lo, int hi, int v) { return min(max(v, lo), hi); }
__device__ __forceinline__ int blk_x(int b) { return ((b >> 2) & 1) * 2 + (b & 1); }
__device__ __forceinline__ int blk_y(int b) { return ((b >> 3) & 1) * 2 + ((b >> 1) & 1); }
__device__ __forceinline__ int blk_of(int x4, int y4) { return ((y4 >> 1) * 2 + (x4 >> 1)) * 4 + (y4 & 1) * 2 + (x4 & 1); }

// ---------------------------------------------------------------------------
// residual: dequant + inverse transforms (transform.c:94-398) for one MB.
// res: LDS int16[384] (luma 16x16 raster, Cb 8x8, Cr 8x8). dc: LDS int32[24].
// Returns (through *err) a nonzero flag if a sample leaves [-512,511].
// ---------------------------------------------------------------------------
__device__ void mb_residual(const MbRec &r, const int16_t *__restrict__ coef, int16_t *res,
                            int32_t *dc, int lane, int *range_err)
{
    const uint32_t cb = r.cbits;
    const int16_t *base = coef + (size_t)r.coef * 16;
    const bool i16 = r.type == MBT_I16;
    if (lane < 16) {
        int32_t v = 0;
        if (i16 && (cb & (1u << 24))) {
            const int16_t *d = base + __popc(cb & 0xFFFFFFu) * 16;
            const int i = lane >> 2, j = lane & 3;
            // f = A c A with A = [[1,1,1,1],[1,1,-1,-1],[1,-1,-1,1],[1,-1,1,-1]]:
            // A[i][k] = (-1)^popcount(k & m(i)), m = {0, 2, 3, 1}
            const int mi = i == 1 ? 2 : i == 2 ? 3 : i == 3 ? 1 : 0;
            const int mj = j == 1 ? 2 : j == 2 ? 3 : j == 3 ? 1 : 0;
            int32_t s = 0;
#pragma unroll
            for (int sp = 0; sp < 16; sp++) {
                const int rr = sp == 0 ? 0 : sp == 1 ? 1 : sp == 2 ? 4 : sp == 3 ? 8 : sp == 4 ? 5 : sp == 5 ? 2 :
                               sp == 6 ? 3 : sp == 7 ? 6 : sp == 8 ? 9 : sp == 9 ? 12 : sp == 10 ? 13 :
                               sp == 11 ? 10 : sp == 12 ? 7 : sp == 13 ? 11 : sp == 14 ? 14 : 15;
                const int neg = (__popc((rr >> 2) & mi) + __popc((rr & 3) & mj)) & 1;
                s += neg ? -(int32_t)d[sp] : (int32_t)d[sp];
            }
            const int q6 = r.qp / 6;
            const int32_t x = s * (int32_t)cLevelScale[r.qp % 6][0];
            v = q6 >= 2 ? x << (q6 - 2) : ((x << q6) + 2) >> 2;
        }
        dc[lane] = v;
    } else if (lane < 24) {
        const int comp = (lane - 16) >> 2, b = (lane - 16) & 3;
        int32_t f = 0;
        const uint32_t bit = 1u << (25 + comp);
        if (cb & bit) {
            const int16_t *d = base + __popc(cb & (bit - 1)) * 16;
            const int32_t c0 = d[0], c1 = d[1], c2 = d[2], c3 = d[3];
            f = b == 0 ? c0 + c1 + c2 + c3 : b == 1 ? c0 - c1 + c2 - c3 : b == 2 ? c0 + c1 - c2 - c3 : c0 - c1 - c2 + c3;
            f = ((f * (int32_t)cLevelScale[r.qpc % 6][0]) << (r.qpc / 6)) >> 1;
        }
        dc[lane] = f;
    }
    __syncthreads();
    if (lane < 24) {
        const bool luma = lane < 16;
        const int qp = luma ? r.qp : r.qpc;
        const int q6 = qp / 6, qm = qp % 6;
        int32_t d[16];
#pragma unroll
        for (int i = 0; i < 16; i++) d[i] = 0;
        bool nz = false;
        const uint32_t bit = 1u << lane;
        if (cb & bit) {
            const int16_t *c = base + __popc(cb & (bit - 1)) * 16;
            const bool skip0 = !luma || i16;
#pragma unroll
            for (int s = 0; s < 16; s++) {
                // raster position of scan position s (compile-time)
                const int rr = s == 0 ? 0 : s == 1 ? 1 : s == 2 ? 4 : s == 3 ? 8 : s == 4 ? 5 : s == 5 ? 2 :
                               s == 6 ? 3 : s == 7 ? 6 : s == 8 ? 9 : s == 9 ? 12 : s == 10 ? 13 :
                               s == 11 ? 10 : s == 12 ? 7 : s == 13 ? 11 : s == 14 ? 14 : 15;
                const int cls = (!(rr & 1) && !((rr >> 2) & 1)) ? 0 : (((rr & 1) && ((rr >> 2) & 1)) ? 1 : 2);
                if (s == 0 && skip0) continue;
                d[rr] = (int32_t)c[s] * ((int32_t)cLevelScale[qm][cls] << q6);
            }
            nz = true;
        }
        if (luma) {
            if (i16) { d[0] = dc[blk_y(lane) * 4 + blk_x(lane)]; nz |= d[0] != 0; }
        } else {
            d[0] = dc[lane];
            nz |= d[0] != 0;
        }
        int32_t o[16];
        if (nz) {
            int32_t t[16];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int32_t a = d[4 * i] + d[4 * i + 2], b = d[4 * i] - d[4 * i + 2];
                const int32_t c = (d[4 * i + 1] >> 1) - d[4 * i + 3], e = d[4 * i + 1] + (d[4 * i + 3] >> 1);
                t[4 * i] = a + e; t[4 * i + 1] = b + c; t[4 * i + 2] = b - c; t[4 * i + 3] = a - e;
            }
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int32_t a = t[j] + t[8 + j], b = t[j] - t[8 + j];
                const int32_t c = (t[4 + j] >> 1) - t[12 + j], e = t[4 + j] + (t[12 + j] >> 1);
                o[j] = (a + e + 32) >> 6; o[4 + j] = (b + c + 32) >> 6;
                o[8 + j] = (b - c + 32) >> 6; o[12 + j] = (a - e + 32) >> 6;
            }
            bool bad = false;
#pragma unroll
            for (int i = 0; i < 16; i++) bad |= (o[i] < -512) | (o[i] > 511);
            if (bad) *range_err = 1;
        } else {
#pragma unroll
            for (int i = 0; i < 16; i++) o[i] = 0;
        }
        if (luma) {
            const int bx = blk_x(lane) * 4, by = blk_y(lane) * 4;
#pragma unroll
            for (int i = 0; i < 16; i++) res[(by + (i >> 2)) * 16 + bx + (i & 3)] = (int16_t)o[i];
        } else {
            const int comp = (lane - 16) >> 2, b = (lane - 16) & 3;
            const int bx = (b & 1) * 4, by = (b >> 1) * 4;
#pragma unroll
            for (int i = 0; i < 16; i++) res[256 + comp * 64 + (by + (i >> 2)) * 8 + bx + (i & 3)] = (int16_t)o[i];
        }
    }
    __syncthreads();
}

// ---------------------------------------------------------------------------
// inter prediction (reconstruct.c:1819-1941): luma 6-tap from a 9x9 window
// per 4x4 block, chroma bilinear from a 3x3 window per 2x2 block.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int tap6(int a, int b, int c, int d, int e, int f)
{
    return a - 5 * b + 20 * c + 20 * d - 5 * e + f;
}

// win: 9x9 window whose (2,2) element is the integer sample G of output x=0.
// Computes 4 outputs (x = 0..3) of window row offset `yy` (0..3).
__device__ __forceinline__ void luma_row4(const uint8_t *win, int yy, int fx, int fy, int out[4])
{
#define W(x, y) ((int)win[((y) + 2 + yy) * 9 + (x) + 2])
#define B1(x, y) tap6(W((x)-2, y), W((x)-1, y), W(x, y), W((x)+1, y), W((x)+2, y), W((x)+3, y))
#define H1(x, y) tap6(W(x, (y)-2), W(x, (y)-1), W(x, y), W(x, (y)+1), W(x, (y)+2), W(x, (y)+3))
    const int pos = fy * 4 + fx;
#pragma unroll
    for (int x = 0; x < 4; x++) {
        int v;
        const int G = W(x, 0);
        if (pos == 0) { v = G; }
        else if (fy == 0) {
            const int b = clip255((B1(x, 0) + 16) >> 5);
            v = fx == 2 ? b : (fx == 1 ? (G + b + 1) >> 1 : (W(x + 1, 0) + b + 1) >> 1);
        } else if (fx == 0) {
            const int hh = clip255((H1(x, 0) + 16) >> 5);
            v = fy == 2 ? hh : (fy == 1 ? (G + hh + 1) >> 1 : (W(x, 1) + hh + 1) >> 1);
        } else if (fx == 2 || fy == 2) {
            const int j1 = tap6(B1(x, -2), B1(x, -1), B1(x, 0), B1(x, 1), B1(x, 2), B1(x, 3));
            const int j = clip255((j1 + 512) >> 10);
            if (pos == 10) v = j;
            else if (fy == 2) {           // i (fx=1) or k (fx=3)
                const int hv = clip255((H1(x + (fx == 3 ? 1 : 0), 0) + 16) >> 5);
                v = (hv + j + 1) >> 1;
            } else {                       // f (fy=1) or q (fy=3)
                const int bv = clip255((B1(x, fy == 3 ? 1 : 0) + 16) >> 5);
                v = (bv + j + 1) >> 1;
            }
        } else {                           // e, g, p, r: diagonal quarter positions
            const int bv = clip255((B1(x, fy == 3 ? 1 : 0) + 16) >> 5);
            const int hv = clip255((H1(x + (fx == 3 ? 1 : 0), 0) + 16) >> 5);
            v = (bv + hv + 1) >> 1;
        }
        out[x] = v;
    }
#undef W
#undef B1
#undef H1
}

__device__ __forceinline__ void write_edges(uint8_t *e, const uint8_t *ty, int ystride, const uint8_t *tu,
                                            const uint8_t *tv, int cstride, int lane)
{
    // e[0..15] Y bottom row, [16..23] Cb bottom, [24..31] Cr bottom,
    // [32..47] Y right col, [48..55] Cb right col, [56..63] Cr right col
    uint8_t v;
    if (lane < 16) v = ty[15 * ystride + lane];
    else if (lane < 24) v = tu[7 * cstride + lane - 16];
    else if (lane < 32) v = tv[7 * cstride + lane - 24];
    else if (lane < 48) v = ty[(lane - 32) * ystride + 15];
    else if (lane < 56) v = tu[(lane - 48) * cstride + 7];
    else v = tv[(lane - 56) * cstride + 7];
    e[lane] = v;
}

__global__ __launch_bounds__(64) void k_inter(ReconArgs a)
{
    const int nmbs = a.w * a.h;
    const int gmb = blockIdx.x;                  // MB index within the batch
    const int p = gmb / nmbs;
    const int mb = gmb - p * nmbs;
    if (p >= a.npics) return;
    const PicDesc pd = a.pics[p];
    const MbRec &r = a.rec[pd.rec_base + mb];
    if (r.type > MBT_SKIP) return;               // intra: done by k_wave
    const int lane = threadIdx.x;

    __shared__ int16_t s_res[384];
    __shared__ int32_t s_dc[24];
    __shared__ uint8_t s_win[16 * 81];
    __shared__ uint8_t s_cwin[2][16][9];
    __shared__ uint8_t s_out[384];
    __shared__ int s_err;
    if (lane == 0) s_err = 0;

    const int W16 = a.w * 16, H16 = a.h * 16, CW = W16 / 2, CH = H16 / 2;
    const int mbx = mb % a.w, mby = mb / a.w;
    const uint8_t *frames = a.frames;

    if (r.cbits) {
        int e = 0;
        mb_residual(r, a.coef + (size_t)pd.coef_base * 16, s_res, s_dc, lane, &e);
        if (e) s_err = 1;
    } else {
        for (int i = lane; i < 384; i += WAVE) s_res[i] = 0;
    }

    // stage luma windows: 16 blocks x 9x9
    for (int idx = lane; idx < 16 * 81; idx += WAVE) {
        const int b = idx / 81, rem = idx - b * 81;
        const int wy = rem / 9, wx = rem - wy * 9;
        const uint8_t *ref = frames + (unsigned long long)(pd.frame_base + r.ref[b >> 2]) * a.frame_bytes;
        const int mvx = r.mv[b][0], mvy = r.mv[b][1];
        const int x = clip3(0, W16 - 1, mbx * 16 + blk_x(b) * 4 + (mvx >> 2) - 2 + wx);
        const int y = clip3(0, H16 - 1, mby * 16 + blk_y(b) * 4 + (mvy >> 2) - 2 + wy);
        s_win[idx] = ref[y * W16 + x];
    }
    // chroma windows: 16 blocks x 2 comps x 3x3
    for (int idx = lane; idx < 16 * 2 * 9; idx += WAVE) {
        const int b = idx / 18, rem = idx - b * 18;
        const int comp = rem / 9, k = rem - comp * 9;
        const int wy = k / 3, wx = k - wy * 3;
        const uint8_t *ref = frames + (unsigned long long)(pd.frame_base + r.ref[b >> 2]) * a.frame_bytes +
                             (unsigned long long)W16 * H16 + (unsigned long long)comp * CW * CH;
        const int mvx = r.mv[b][0], mvy = r.mv[b][1];
        const int x = clip3(0, CW - 1, mbx * 8 + blk_x(b) * 2 + (mvx >> 3) + wx);
        const int y = clip3(0, CH - 1, mby * 8 + blk_y(b) * 2 + (mvy >> 3) + wy);
        s_cwin[comp][b][k] = ref[y * CW + x];
    }
    __syncthreads();

    {   // luma: lane -> (block, row)
        const int b = lane >> 2, yy = lane & 3;
        const int mvx = r.mv[b][0], mvy = r.mv[b][1];
        int o[4];
        luma_row4(s_win + b * 81, yy, mvx & 3, mvy & 3, o);
        const int bx = blk_x(b) * 4, by = blk_y(b) * 4 + yy;
#pragma unroll
        for (int x = 0; x < 4; x++) s_out[by * 16 + bx + x] = (uint8_t)clip255(o[x] + s_res[by * 16 + bx + x]);
    }
    {   // chroma: lane -> (block, comp, row), 2 samples
        const int b = lane >> 2, comp = (lane >> 1) & 1, yy = lane & 1;
        const int mvx = r.mv[b][0], mvy = r.mv[b][1];
        const int fx = mvx & 7, fy = mvy & 7;
        const uint8_t *w = s_cwin[comp][b];
        const int cx = blk_x(b) * 2, cy = blk_y(b) * 2 + yy;
#pragma unroll
        for (int x = 0; x < 2; x++) {
            const int A = w[yy * 3 + x], B = w[yy * 3 + x + 1], C = w[(yy + 1) * 3 + x], D = w[(yy + 1) * 3 + x + 1];
            const int v = ((8 - fx) * (8 - fy) * A + fx * (8 - fy) * B + (8 - fx) * fy * C + fx * fy * D + 32) >> 6;
            s_out[256 + comp * 64 + cy * 8 + cx + x] = (uint8_t)clip255(v + s_res[256 + comp * 64 + cy * 8 + cx + x]);
        }
    }
    __syncthreads();

    // write-out: luma 16 rows x 4 dwords, chroma 2 x 8 rows x 2 dwords
    uint8_t *cur = a.frames + (unsigned long long)(pd.frame_base + pd.cur_slot) * a.frame_bytes;
    {
        const int row = lane >> 2, q = lane & 3;
        *(uint32_t *)(cur + (size_t)(mby * 16 + row) * W16 + mbx * 16 + q * 4) = *(const uint32_t *)(s_out + row * 16 + q * 4);
    }
    if (lane < 32) {
        const int comp = lane >> 4, row = (lane >> 1) & 7, q = lane & 1;
        uint8_t *cp = cur + (size_t)W16 * H16 + (size_t)comp * CW * CH;
        *(uint32_t *)(cp + (size_t)(mby * 8 + row) * CW + mbx * 8 + q * 4) =
            *(const uint32_t *)(s_out + 256 + comp * 64 + row * 8 + q * 4);
    }
    write_edges(a.edges + (size_t)(pd.rec_base + mb) * 64, s_out, 16, s_out + 256, s_out + 320, 8, lane);
    if (lane == 0 && s_err) atomicOr(a.err + p, 1u);
}

// ---------------------------------------------------------------------------
// intra prediction (intra_prediction.c) into an LDS tile with a 1-sample halo
// ---------------------------------------------------------------------------
// luma tile: 17 rows x 24 cols; (row 0) = y=-1, (col 0) = x=-1; cols 17..20 = top-right
#define TY_STRIDE 24
#define TC_STRIDE 12

__device__ __forceinline__ int i4_pred(const uint8_t *T /* tile at block (0,0) i.e. &tile[(by+1)*S + bx+1] */,
                                       int S, int mode, int x, int y, bool avT, bool avL, bool avTR)
{
    // S-array of the 4x4 block: Sx[4]=p[-1,-1], Sx[5+k]=p[k,-1], Sx[3-k]=p[-1,k]
#define PT(k) ((int)T[-S + (((k) > 3 && !avTR) ? 3 : (k))])
#define PL(k) ((int)T[(k)*S - 1])
#define PTL ((int)T[-S - 1])
    int v;
    switch (mode) {
    case 0: v = PT(x); break;
    case 1: v = PL(y); break;
    case 2: {
        const int st = PT(0) + PT(1) + PT(2) + PT(3), sl = PL(0) + PL(1) + PL(2) + PL(3);
        if (avT && avL) v = (st + sl + 4) >> 3;
        else if (avL) v = (sl + 2) >> 2;
        else if (avT) v = (st + 2) >> 2;
        else v = 128;
        break;
    }
    case 3:
        if (x == 3 && y == 3) v = (PT(6) + 3 * PT(7) + 2) >> 2;
        else v = (PT(x + y) + 2 * PT(x + y + 1) + PT(x + y + 2) + 2) >> 2;
        break;
    default: {
        // modes 4..8 read a mix of left / top / corner samples: build S[13]
        int Sx[13];
        Sx[4] = PTL;
#pragma unroll
        for (int k = 0; k < 8; k++) Sx[5 + k] = PT(k);
#pragma unroll
        for (int k = 0; k < 4; k++) Sx[3 - k] = PL(k);
        if (mode == 4) {
            const int d = x - y;
            v = (Sx[3 + d] + 2 * Sx[4 + d] + Sx[5 + d] + 2) >> 2;
        } else if (mode == 5) {
            const int z = 2 * x - y, i = x - (y >> 1);
            if (z >= 0 && !(z & 1)) v = (Sx[4 + i] + Sx[5 + i] + 1) >> 1;
            else if (z > 0) v = (Sx[3 + i] + 2 * Sx[4 + i] + Sx[5 + i] + 2) >> 2;
            else if (z == -1) v = (Sx[3] + 2 * Sx[4] + Sx[5] + 2) >> 2;
            else v = (Sx[4 - y] + 2 * Sx[5 - y] + Sx[6 - y] + 2) >> 2;
        } else if (mode == 6) {
            const int z = 2 * y - x, i = y - (x >> 1);
            if (z >= 0 && !(z & 1)) v = (Sx[4 - i] + Sx[3 - i] + 1) >> 1;
            else if (z > 0) v = (Sx[5 - i] + 2 * Sx[4 - i] + Sx[3 - i] + 2) >> 2;
            else if (z == -1) v = (Sx[3] + 2 * Sx[4] + Sx[5] + 2) >> 2;
            else v = (Sx[4 + x] + 2 * Sx[3 + x] + Sx[2 + x] + 2) >> 2;
        } else if (mode == 7) {
            const int i = x + (y >> 1);
            if (!(y & 1)) v = (Sx[5 + i] + Sx[6 + i] + 1) >> 1;
            else v = (Sx[5 + i] + 2 * Sx[6 + i] + Sx[7 + i] + 2) >> 2;
        } else {
            const int z = x + 2 * y, i = y + (x >> 1);
            if (z > 5) v = Sx[0];
            else if (z == 5) v = (Sx[1] + 3 * Sx[0] + 2) >> 2;
            else if (!(z & 1)) v = (Sx[3 - i] + Sx[2 - i] + 1) >> 1;
            else v = (Sx[3 - i] + 2 * Sx[2 - i] + Sx[1 - i] + 2) >> 2;
        }
        break;
    }
    }
#undef PT
#undef PL
#undef PTL
    return v;
}

// 10-step schedule of the 16 4x4 blocks (x + 2y = step), two blocks max
__constant__ int8_t cI4Sched[10][2] = {{0, -1}, {1, -1}, {4, 2}, {5, 3}, {6, 8},
                                       {7, 9}, {12, 10}, {13, 11}, {14, -1}, {15, -1}};

__device__ void intra_mb(const MbRec &r, const uint8_t *__restrict__ edges, int mb_global, int mbx, int w,
                         const int16_t *res, uint8_t *ty, uint8_t *tu, uint8_t *tv, int lane)
{
    const bool aA = r.avail & AV_A, aB = r.avail & AV_B, aC = r.avail & AV_C, aD = r.avail & AV_D;
    // --- gather neighbours from the edge buffers (unfiltered samples)
    const uint8_t *eA = edges + (size_t)(mb_global - 1) * 64;
    const uint8_t *eB = edges + (size_t)(mb_global - w) * 64;
    const uint8_t *eC = edges + (size_t)(mb_global - w + 1) * 64;
    const uint8_t *eD = edges + (size_t)(mb_global - w - 1) * 64;
    (void)mbx;
    if (lane < 16) {
        if (aB) ty[1 + lane] = eB[lane];                        // top row
        if (aA) ty[(lane + 1) * TY_STRIDE] = eA[32 + lane];     // left column
    } else if (lane < 20) {
        if (aC) ty[1 + lane] = eC[lane - 16];                   // top-right
    } else if (lane < 28) {
        const int i = lane - 20;
        if (aB) { tu[1 + i] = eB[16 + i]; tv[1 + i] = eB[24 + i]; }
        if (aA) { tu[(i + 1) * TC_STRIDE] = eA[48 + i]; tv[(i + 1) * TC_STRIDE] = eA[56 + i]; }
    } else if (lane == 28) {
        if (aD) { ty[0] = eD[15]; tu[0] = eD[23]; tv[0] = eD[31]; }
    }
    __syncthreads();

    if (r.type == MBT_I16) {
        const int mode = r.pred & 3;
        const int y = lane >> 2, x0 = (lane & 3) * 4;
        int dcv = 128, a = 0, b = 0, c = 0;
        if (mode == 2) {
            int st = 0, sl = 0;
            for (int i = 0; i < 16; i++) { st += ty[1 + i]; sl += ty[(i + 1) * TY_STRIDE]; }
            if (aA && aB) dcv = (st + sl + 16) >> 5;
            else if (aA) dcv = (sl + 8) >> 4;
            else if (aB) dcv = (st + 8) >> 4;
        } else if (mode == 3) {
            int H = 0, V = 0;
            for (int i = 0; i < 8; i++) {
                H += (i + 1) * ((int)ty[1 + 8 + i] - (int)ty[1 + 6 - i]);
                V += (i + 1) * ((int)ty[(1 + 8 + i) * TY_STRIDE] - (int)ty[(1 + 6 - i) * TY_STRIDE]);
            }
            a = 16 * ((int)ty[16 * TY_STRIDE] + (int)ty[16]);
            b = (5 * H + 32) >> 6;
            c = (5 * V + 32) >> 6;
        }
        int pv[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int x = x0 + i;
            int p;
            if (mode == 0) p = ty[1 + x];
            else if (mode == 1) p = ty[(y + 1) * TY_STRIDE];
            else if (mode == 2) p = dcv;
            else p = clip255((a + b * (x - 7) + c * (y - 7) + 16) >> 5);
            pv[i] = clip255(p + res[y * 16 + x]);
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 4; i++) ty[(y + 1) * TY_STRIDE + 1 + x0 + i] = (uint8_t)pv[i];
    } else {
        // Intra 4x4: 10 dependency steps, up to two blocks per step
        for (int step = 0; step < 10; step++) {
            const int slot = lane >> 4;
            int v = 0;
            int b = -1;
            if (slot < 2) b = cI4Sched[step][slot];
            const int px = lane & 3, py = (lane >> 2) & 3;
            if (b >= 0) {
                const int bx = blk_x(b), by = blk_y(b);
                const bool avL = bx > 0 || aA;
                const bool avT = by > 0 || aB;
                bool avTR;
                if (b == 3 || b == 7 || b == 11 || b == 13 || b == 15) avTR = false;
                else if (by == 0) avTR = bx == 3 ? aC : aB;
                else avTR = true;
                const int mode = (r.i4[b >> 1] >> ((b & 1) * 4)) & 15;
                const uint8_t *T = ty + (by * 4 + 1) * TY_STRIDE + bx * 4 + 1;
                const int p = i4_pred(T, TY_STRIDE, mode, px, py, avT, avL, avTR);
                v = clip255(p + res[(by * 4 + py) * 16 + bx * 4 + px]);
            }
            __syncthreads();
            if (b >= 0) ty[(blk_y(b) * 4 + py + 1) * TY_STRIDE + blk_x(b) * 4 + px + 1] = (uint8_t)v;
            __syncthreads();
        }
    }
    // chroma: lane -> row (0..7) x comp, 4 samples each
    {
        const int comp = lane >> 5, y = (lane >> 2) & 7, x0 = (lane & 3) * 2;
        uint8_t *T = comp ? tv : tu;
        const int cmode = (r.pred >> 4) & 3;
        int pv[2];
        int a = 0, b = 0, c = 0;
        if (cmode == 3) {
            int H = 0, V = 0;
            for (int i = 0; i < 4; i++) {
                H += (i + 1) * ((int)T[1 + 4 + i] - (int)T[1 + 2 - i]);
                V += (i + 1) * ((int)T[(1 + 4 + i) * TC_STRIDE] - (int)T[(1 + 2 - i) * TC_STRIDE]);
            }
            a = 16 * ((int)T[8 * TC_STRIDE] + (int)T[8]);
            b = (34 * H + 32) >> 6;
            c = (34 * V + 32) >> 6;
        }
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const int x = x0 + i;
            int p;
            if (cmode == 0) {
                const int xo = x & 4, yo = y & 4;
                int st = 0, sl = 0;
                for (int k = 0; k < 4; k++) { st += T[1 + xo + k]; sl += T[(1 + yo + k) * TC_STRIDE]; }
                if ((xo == 0 && yo == 0) || (xo > 0 && yo > 0)) {
                    p = (aA && aB) ? (st + sl + 4) >> 3 : aA ? (sl + 2) >> 2 : aB ? (st + 2) >> 2 : 128;
                } else if (xo > 0) {
                    p = aB ? (st + 2) >> 2 : aA ? (sl + 2) >> 2 : 128;
                } else {
                    p = aA ? (sl + 2) >> 2 : aB ? (st + 2) >> 2 : 128;
                }
            } else if (cmode == 1) p = T[(y + 1) * TC_STRIDE];
            else if (cmode == 2) p = T[1 + x];
            else p = clip255((a + b * (x - 3) + c * (y - 3) + 16) >> 5);
            pv[i] = clip255(p + res[256 + comp * 64 + y * 8 + x]);
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 2; i++) T[(y + 1) * TC_STRIDE + 1 + x0 + i] = (uint8_t)pv[i];
    }
    __syncthreads();
}

// ---------------------------------------------------------------------------
// deblocking of one MB (deblocking.c:574-1736)
// LDS region: luma rows -4..15, cols -4..15 (20x20); chroma rows -2..7,
// cols -4..7 (10x12) per component.
// ---------------------------------------------------------------------------
#define DY_S 20
#define DC_S 12

__device__ __forceinline__ int bs_of(const MbRec &p, int bp, const MbRec &q, int bq, bool mb_edge)
{
    if (p.type >= MBT_I4x4 || q.type >= MBT_I4x4) return mb_edge ? 4 : 3;
    if (((p.cbits >> bp) & 1) | ((q.cbits >> bq) & 1)) return 2;
    if (p.ref[bp >> 2] != q.ref[bq >> 2]) return 1;
    if (abs(p.mv[bp][0] - q.mv[bq][0]) >= 4 || abs(p.mv[bp][1] - q.mv[bq][1]) >= 4) return 1;
    return 0;
}

__device__ __forceinline__ void filt_luma(uint8_t *s, int step, int bS, int alpha, int beta, int tc0)
{
    const int p0 = s[-step], p1 = s[-2 * step], p2 = s[-3 * step], p3 = s[-4 * step];
    const int q0 = s[0], q1 = s[step], q2 = s[2 * step], q3 = s[3 * step];
    if (!(abs(p0 - q0) < alpha && abs(p1 - p0) < beta && abs(q1 - q0) < beta)) return;
    const int ap = abs(p2 - p0), aq = abs(q2 - q0);
    if (bS < 4) {
        const int tc = tc0 + (ap < beta) + (aq < beta);
        const int d = clip3(-tc, tc, (((q0 - p0) << 2) + (p1 - q1) + 4) >> 3);
        s[-step] = (uint8_t)clip255(p0 + d);
        s[0] = (uint8_t)clip255(q0 - d);
        if (ap < beta) s[-2 * step] = (uint8_t)(p1 + clip3(-tc0, tc0, (p2 + ((p0 + q0 + 1) >> 1) - (p1 << 1)) >> 1));
        if (aq < beta) s[step] = (uint8_t)(q1 + clip3(-tc0, tc0, (q2 + ((p0 + q0 + 1) >> 1) - (q1 << 1)) >> 1));
    } else {
        const bool strong = abs(p0 - q0) < ((alpha >> 2) + 2);
        if (ap < beta && strong) {
            s[-step] = (uint8_t)((p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3);
            s[-2 * step] = (uint8_t)((p2 + p1 + p0 + q0 + 2) >> 2);
            s[-3 * step] = (uint8_t)((2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3);
        } else {
            s[-step] = (uint8_t)((2 * p1 + p0 + q1 + 2) >> 2);
        }
        if (aq < beta && strong) {
            s[0] = (uint8_t)((p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3);
            s[step] = (uint8_t)((p0 + q0 + q1 + q2 + 2) >> 2);
            s[2 * step] = (uint8_t)((2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3);
        } else {
            s[0] = (uint8_t)((2 * q1 + q0 + p1 + 2) >> 2);
        }
    }
}

__device__ __forceinline__ void filt_chroma(uint8_t *s, int step, int bS, int alpha, int beta, int tc0)
{
    const int p0 = s[-step], p1 = s[-2 * step], q0 = s[0], q1 = s[step];
    if (!(abs(p0 - q0) < alpha && abs(p1 - p0) < beta && abs(q1 - q0) < beta)) return;
    if (bS < 4) {
        const int tc = tc0 + 1;
        const int d = clip3(-tc, tc, (((q0 - p0) << 2) + (p1 - q1) + 4) >> 3);
        s[-step] = (uint8_t)clip255(p0 + d);
        s[0] = (uint8_t)clip255(q0 - d);
    } else {
        s[-step] = (uint8_t)((2 * p1 + p0 + q1 + 2) >> 2);
        s[0] = (uint8_t)((2 * q1 + q0 + p1 + 2) >> 2);
    }
}

__global__ __launch_bounds__(64) void k_wave(ReconArgs a)
{
    const int p = blockIdx.x / a.diag_len;
    const int k = blockIdx.x - p * a.diag_len;
    if (p >= a.npics) return;
    const int t = a.diag;
    const int r_lo = max(0, (t - (a.w - 1) + 1) >> 1);
    const int mby = r_lo + k;
    const int mbx = t - 2 * mby;
    if (mby >= a.h || mbx < 0 || mbx >= a.w) return;
    const PicDesc pd = a.pics[p];
    const int mb = mby * a.w + mbx;
    const int gmb = pd.rec_base + mb;
    const MbRec &q = a.rec[gmb];
    const bool intra = q.type >= MBT_I4x4;
    const bool dbf = q.avail & DB_INNER;
    if (!intra && !dbf) return;
    const int lane = threadIdx.x;
    const int W16 = a.w * 16, H16 = a.h * 16, CW = W16 / 2, CH = H16 / 2;
    uint8_t *cur = a.frames + (unsigned long long)(pd.frame_base + pd.cur_slot) * a.frame_bytes;
    uint8_t *curU = cur + (size_t)W16 * H16;
    uint8_t *curV = curU + (size_t)CW * CH;

    __shared__ int16_t s_res[384];
    __shared__ int32_t s_dc[24];
    __shared__ uint8_t s_ty[17 * TY_STRIDE];
    __shared__ uint8_t s_tu[9 * TC_STRIDE];
    __shared__ uint8_t s_tv[9 * TC_STRIDE];
    __shared__ uint8_t s_dy[20 * DY_S];
    __shared__ uint8_t s_du[10 * DC_S];
    __shared__ uint8_t s_dv[10 * DC_S];
    __shared__ int8_t s_bs[2][4][4];
    __shared__ int s_err;

    // ---------------------------------------------------------- intra recon
    if (intra) {
        if (lane == 0) s_err = 0;
        if (q.type == MBT_IPCM) {
            const uint8_t *src = (const uint8_t *)(a.coef + ((size_t)pd.coef_base + q.coef) * 16);
            for (int i = lane; i < 256; i += WAVE) s_ty[((i >> 4) + 1) * TY_STRIDE + (i & 15) + 1] = src[i];
            for (int i = lane; i < 64; i += WAVE) {
                s_tu[((i >> 3) + 1) * TC_STRIDE + (i & 7) + 1] = src[256 + i];
                s_tv[((i >> 3) + 1) * TC_STRIDE + (i & 7) + 1] = src[320 + i];
            }
            __syncthreads();
        } else {
            int e = 0;
            if (q.cbits) mb_residual(q, a.coef + (size_t)pd.coef_base * 16, s_res, s_dc, lane, &e);
            else { for (int i = lane; i < 384; i += WAVE) s_res[i] = 0; __syncthreads(); }
            if (e) s_err = 1;
            intra_mb(q, a.edges, gmb, mbx, a.w, s_res, s_ty, s_tu, s_tv, lane);
        }
        // edge buffer of this MB (unfiltered), from the tile
        write_edges(a.edges + (size_t)gmb * 64, s_ty + TY_STRIDE + 1, TY_STRIDE, s_tu + TC_STRIDE + 1,
                    s_tv + TC_STRIDE + 1, TC_STRIDE, lane);
        if (!dbf) {
            // write the MB straight out
            const int row = lane >> 2, qd = lane & 3;
            for (int x = 0; x < 4; x++)
                cur[(size_t)(mby * 16 + row) * W16 + mbx * 16 + qd * 4 + x] = s_ty[(row + 1) * TY_STRIDE + 1 + qd * 4 + x];
            if (lane < 32) {
                const int comp = lane >> 4, crow = (lane >> 1) & 7, cq = lane & 1;
                uint8_t *cp = comp ? curV : curU;
                const uint8_t *T = comp ? s_tv : s_tu;
                for (int x = 0; x < 4; x++)
                    cp[(size_t)(mby * 8 + crow) * CW + mbx * 8 + cq * 4 + x] = T[(crow + 1) * TC_STRIDE + 1 + cq * 4 + x];
            }
            if (lane == 0 && s_err) atomicOr(a.err + p, 1u);
            return;
        }
    }

    // -------------------------------------------------------------- deblock
    const bool fl = q.avail & DB_LEFT, ft = q.avail & DB_TOP;
    // load region into LDS
    for (int i = lane; i < 20 * 20; i += WAVE) {
        const int ry = i / 20 - 4, rx = i % 20 - 4;
        uint8_t v = 0;
        if (ry >= 0 && rx >= 0) {
            v = intra ? s_ty[(ry + 1) * TY_STRIDE + rx + 1] : cur[(size_t)(mby * 16 + ry) * W16 + mbx * 16 + rx];
        } else if (ry < 0 && rx >= 0) {
            if (ft) v = cur[(size_t)(mby * 16 + ry) * W16 + mbx * 16 + rx];
        } else if (rx < 0 && ry >= 0) {
            if (fl) v = cur[(size_t)(mby * 16 + ry) * W16 + mbx * 16 + rx];
        }
        s_dy[(ry + 4) * DY_S + rx + 4] = v;
    }
    for (int i = lane; i < 2 * 10 * 12; i += WAVE) {
        const int comp = i / 120, j = i - comp * 120;
        const int ry = j / 12 - 2, rx = j % 12 - 4;
        uint8_t *cp = comp ? curV : curU;
        const uint8_t *T = comp ? s_tv : s_tu;
        uint8_t v = 0;
        if (ry >= 0 && rx >= 0) v = intra ? T[(ry + 1) * TC_STRIDE + rx + 1] : cp[(size_t)(mby * 8 + ry) * CW + mbx * 8 + rx];
        else if (ry < 0 && rx >= 0) { if (ft) v = cp[(size_t)(mby * 8 + ry) * CW + mbx * 8 + rx]; }
        else if (rx < 0 && ry >= 0) { if (fl) v = cp[(size_t)(mby * 8 + ry) * CW + mbx * 8 + rx]; }
        (comp ? s_dv : s_du)[(ry + 2) * DC_S + rx + 4] = v;
    }
    // boundary strengths: lane -> (dir, edge, segment)
    if (lane < 32) {
        const int dir = lane >> 4, e = (lane >> 2) & 3, kk = lane & 3;
        int bS = 0;
        const bool on = e > 0 || (dir == 0 ? fl : ft);
        if (on) {
            const MbRec &pm = e > 0 ? q : (dir == 0 ? a.rec[gmb - 1] : a.rec[gmb - a.w]);
            const int bq = dir == 0 ? blk_of(e, kk) : blk_of(kk, e);
            const int bp = e == 0 ? (dir == 0 ? blk_of(3, kk) : blk_of(kk, 3)) : (dir == 0 ? blk_of(e - 1, kk) : blk_of(kk, e - 1));
            bS = bs_of(pm, bp, q, bq, e == 0);
        }
        s_bs[dir][e][kk] = (int8_t)bS;
    }
    __syncthreads();

    const int qp_left = fl ? a.rec[gmb - 1].qp : 0, qpc_left = fl ? a.rec[gmb - 1].qpc : 0;
    const int qp_top = ft ? a.rec[gmb - a.w].qp : 0, qpc_top = ft ? a.rec[gmb - a.w].qpc : 0;
    for (int dir = 0; dir < 2; dir++) {
        for (int e = 0; e < 4; e++) {
            if (lane < 16) {
                const int kk = lane >> 2;
                const int bS = s_bs[dir][e][kk];
                if (bS) {
                    const int qpp = e > 0 ? q.qp : (dir == 0 ? qp_left : qp_top);
                    const int qpav = (qpp + q.qp + 1) >> 1;
                    const int ia = clip3(0, 51, qpav + q.offA), ib = clip3(0, 51, qpav + q.offB);
                    const int tc0 = bS < 4 ? cTc0[ia][bS - 1] : 0;
                    uint8_t *s = dir == 0 ? &s_dy[(lane + 4) * DY_S + e * 4 + 4] : &s_dy[(e * 4 + 4) * DY_S + lane + 4];
                    filt_luma(s, dir == 0 ? 1 : DY_S, bS, cAlpha[ia], cBeta[ib], tc0);
                }
            } else if (lane < 32 && !(e & 1)) {
                const int comp = (lane - 16) >> 3, i = (lane - 16) & 7;
                const int bS = s_bs[dir][e][i >> 1];
                if (bS) {
                    const int qpp = e > 0 ? q.qpc : (dir == 0 ? qpc_left : qpc_top);
                    const int qpav = (qpp + q.qpc + 1) >> 1;
                    const int ia = clip3(0, 51, qpav + q.offA), ib = clip3(0, 51, qpav + q.offB);
                    const int tc0 = bS < 4 ? cTc0[ia][bS - 1] : 0;
                    uint8_t *D = comp ? s_dv : s_du;
                    const int ce = e >> 1;
                    uint8_t *s = dir == 0 ? &D[(i + 2) * DC_S + ce * 4 + 4] : &D[(ce * 4 + 2) * DC_S + i + 4];
                    filt_chroma(s, dir == 0 ? 1 : DC_S, bS, cAlpha[ia], cBeta[ib], tc0);
                }
            }
            __syncthreads();
        }
    }
    // write back: MB + modified halo (top 3 rows if ft, left 3 cols if fl)
    for (int i = lane; i < 20 * 20; i += WAVE) {
        const int ry = i / 20 - 4, rx = i % 20 - 4;
        bool w = false;
        if (ry >= 0 && rx >= 0) w = true;
        else if (ry < 0 && rx >= 0) w = ft && ry >= -3;
        else if (rx < 0 && ry >= 0) w = fl && rx >= -3;
        if (w) cur[(size_t)(mby * 16 + ry) * W16 + mbx * 16 + rx] = s_dy[(ry + 4) * DY_S + rx + 4];
    }
    for (int i = lane; i < 2 * 10 * 12; i += WAVE) {
        const int comp = i / 120, j = i - comp * 120;
        const int ry = j / 12 - 2, rx = j % 12 - 4;
        bool w = false;
        if (ry >= 0 && rx >= 0) w = true;
        else if (ry < 0 && rx >= 0) w = ft && ry >= -1;
        else if (rx < 0 && ry >= 0) w = fl && rx >= -1;
        if (w) (comp ? curV : curU)[(size_t)(mby * 8 + ry) * CW + mbx * 8 + rx] = (comp ? s_dv : s_du)[(ry + 2) * DC_S + rx + 4];
    }
    if (intra && lane == 0 && s_err) atomicOr(a.err + p, 1u);
}
