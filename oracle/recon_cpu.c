/* ORACLE -- TEST INFRASTRUCTURE ONLY.  Not part of the product path.
 *
 * Plain-C restatement of the reference's per-macroblock reconstruction and
 * in-loop deblocking (Broadway h264bsd core), operating on the same MbRec
 * batches the HIP kernels consume.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may use it, and only as the checker /
 * CPU baseline -- never as the thing measured or shipped.
 *
 * It follows the reference's structure: macroblocks reconstructed in raster
 * order into the (unfiltered) current picture, then h264bsdFilterPicture over
 * the whole picture.  Anchors (all under /root/reference/Decoder/src):
 *   residual   h264bsd_transform.c:94-231 (ProcessBlock), :252-335 (LumaDc),
 *              :356-398 (ChromaDc); distribution macroblock_layer.c:1343-1424
 *   intra      h264bsd_intra_prediction.c:475-532, 626-686 (16x16),
 *              700-832 (4x4, modes :1492-1831), 844-914 (chroma, :1159-1376),
 *              926-988 (AddResidual)
 *   inter      h264bsd_reconstruct.c:1819-1941 (PredictSamples), luma 6-tap
 *              :491-1600, chroma :110-476, edge fill :2170-2314
 *   write-out  h264bsd_image.c:80-343
 *   deblock    h264bsd_deblocking.c:574-639 (FilterPicture), 288-319 (flags),
 *              1134-1370 (bS), 1381-1532 (thresholds), 1542-1736 (filters),
 *              tables :77-98
 * Parity of this restatement is pinned against the reference decoder itself
 * (oracle/_ref/refdec, built by oracle/Makefile.ref) through the per-frame MD5
 * fixtures in tests/golden/ (tests/golden/make_golden.py).
 */
#include "recon_cpu.h"
#include "../broadway_amd/csrc/common/tables.h"

#include <stdlib.h>
#include <string.h>

typedef struct OracleCtx {
    int w_mbs, h_mbs, nslots;
    size_t frame_bytes;
    uint8_t *frames;
} OracleCtx;

static inline int clip255(int v) { return v < 0 ? 0 : v > 255 ? 255 : v; }
static inline int clip3(int lo, int hi, int v) { return v < lo ? lo : v > hi ? hi : v; }
static inline int iabs(int v) { return v < 0 ? -v : v; }

typedef struct Planes { uint8_t *y, *u, *v; int w, h; } Planes;

static Planes planes_of(const OracleCtx *c, int slot)
{
    Planes p;
    p.w = c->w_mbs * 16;
    p.h = c->h_mbs * 16;
    p.y = c->frames + c->frame_bytes * (size_t)slot;
    p.u = p.y + (size_t)p.w * p.h;
    p.v = p.u + (size_t)p.w * p.h / 4;
    return p;
}

/* ---------------------------------------------------------- residual --- */
static int pos_class(int r)
{
    int x = r & 3, y = r >> 2;
    if (!(x & 1) && !(y & 1)) return 0;
    if ((x & 1) && (y & 1)) return 1;
    return 2;
}

/* 4x4 inverse transform, (x+32)>>6 (transform.c:151-186) */
static void idct4(const int32_t *in, int32_t *out)
{
    int32_t t[16];
    for (int i = 0; i < 4; i++) {
        const int32_t *r = in + 4 * i;
        int32_t a = r[0] + r[2], b = r[0] - r[2];
        int32_t c = (r[1] >> 1) - r[3], d = r[1] + (r[3] >> 1);
        t[4 * i + 0] = a + d; t[4 * i + 1] = b + c; t[4 * i + 2] = b - c; t[4 * i + 3] = a - d;
    }
    for (int j = 0; j < 4; j++) {
        int32_t a = t[j] + t[8 + j], b = t[j] - t[8 + j];
        int32_t c = (t[4 + j] >> 1) - t[12 + j], d = t[4 + j] + (t[12 + j] >> 1);
        out[j] = (a + d + 32) >> 6;
        out[4 + j] = (b + c + 32) >> 6;
        out[8 + j] = (b - c + 32) >> 6;
        out[12 + j] = (a - d + 32) >> 6;
    }
}

/* Residual of one MB: res[0..255] luma (16x16 raster), res[256..383] Cb|Cr
 * (8x8 raster each).  Returns 0, or -1 if any sample leaves [-512,511]
 * (the reference's error, transform.c:181-225). */
static int mb_residual(const MbRec *r, const int16_t *coefs, int32_t *res)
{
    memset(res, 0, 384 * sizeof(int32_t));
    const int16_t *blk[27] = {0};
    const int16_t *p = coefs + (size_t)r->coef * 16;
    for (int b = 0; b < 27; b++) if (r->cbits & (1u << b)) { blk[b] = p; p += 16; }
    int qp = r->qp, qpc = r->qpc;
    int is_i16 = r->type == MBT_I16;
    int32_t dcy[16] = {0};
    int any_dc = 0;
    if (is_i16 && blk[24]) {
        int32_t m[16], t[16];
        for (int s = 0; s < 16; s++) m[kZigzag4x4[s]] = blk[24][s];
        for (int i = 0; i < 4; i++) {
            const int32_t *q = m + 4 * i;
            t[4 * i + 0] = q[0] + q[1] + q[2] + q[3];
            t[4 * i + 1] = q[0] + q[1] - q[2] - q[3];
            t[4 * i + 2] = q[0] - q[1] - q[2] + q[3];
            t[4 * i + 3] = q[0] - q[1] + q[2] - q[3];
        }
        int v = kLevelScale[qp % 6][0], q6 = qp / 6;
        for (int j = 0; j < 4; j++) {
            int32_t a = t[j], b = t[4 + j], c = t[8 + j], d = t[12 + j];
            int32_t f[4] = {a + b + c + d, a + b - c - d, a - b - c + d, a - b + c - d};
            for (int k = 0; k < 4; k++) {
                int32_t x = f[k] * v;
                dcy[4 * k + j] = q6 >= 2 ? x << (q6 - 2) : ((x << q6) + 2) >> 2;
            }
        }
        any_dc = 1;
    }
    for (int b = 0; b < 16; b++) {
        int32_t d[16] = {0}, o[16];
        int nz = 0;
        if (blk[b]) {
            for (int s = is_i16 ? 1 : 0; s < 16; s++) {
                int rr = kZigzag4x4[s];
                d[rr] = (int32_t)blk[b][s] * (kLevelScale[qp % 6][pos_class(rr)] << (qp / 6));
            }
            nz = 1;
        }
        if (any_dc) { d[0] = dcy[kBlkY[b] * 4 + kBlkX[b]]; if (d[0]) nz = 1; }
        if (!nz) continue;
        idct4(d, o);
        int bx = kBlkX[b] * 4, by = kBlkY[b] * 4;
        for (int i = 0; i < 16; i++) {
            if (o[i] < -512 || o[i] > 511) return -1;
            res[(by + (i >> 2)) * 16 + bx + (i & 3)] = o[i];
        }
    }
    int v = kLevelScale[qpc % 6][0], q6 = qpc / 6;
    for (int comp = 0; comp < 2; comp++) {
        int32_t f[4] = {0, 0, 0, 0};
        if (r->cbits & (3u << 25)) {
            const int16_t *x = blk[25 + comp];
            int32_t c0 = x ? x[0] : 0, c1 = x ? x[1] : 0, c2 = x ? x[2] : 0, c3 = x ? x[3] : 0;
            f[0] = c0 + c1 + c2 + c3; f[1] = c0 - c1 + c2 - c3;
            f[2] = c0 + c1 - c2 - c3; f[3] = c0 - c1 - c2 + c3;
            for (int k = 0; k < 4; k++) f[k] = ((f[k] * v) << q6) >> 1;
        }
        for (int b = 0; b < 4; b++) {
            int32_t d[16] = {0}, o[16];
            const int16_t *ac = blk[16 + comp * 4 + b];
            int nz = 0;
            if (ac) {
                for (int s = 1; s < 16; s++) {
                    int rr = kZigzag4x4[s];
                    d[rr] = (int32_t)ac[s] * (kLevelScale[qpc % 6][pos_class(rr)] << q6);
                }
                nz = 1;
            }
            d[0] = f[b];
            if (d[0]) nz = 1;
            if (!nz) continue;
            idct4(d, o);
            int bx = (b & 1) * 4, by = (b >> 1) * 4;
            for (int i = 0; i < 16; i++) {
                if (o[i] < -512 || o[i] > 511) return -1;
                res[256 + comp * 64 + (by + (i >> 2)) * 8 + bx + (i & 3)] = o[i];
            }
        }
    }
    return 0;
}

/* ------------------------------------------------------------- intra --- */
static void intra4x4_pred(int mode, const int *top /* p[0..7,-1] */, const int *left /* p[-1,0..3] */,
                          int tl, int avail_top, int avail_left, int *pred)
{
    /* S[4] = p[-1,-1], S[5+k] = p[k,-1] (k = 0..7), S[3-k] = p[-1,k] (k = 0..3) */
    int S[13];
    S[4] = tl;
    for (int k = 0; k < 8; k++) S[5 + k] = top[k];
    for (int k = 0; k < 4; k++) S[3 - k] = left[k];
    for (int y = 0; y < 4; y++)
        for (int x = 0; x < 4; x++) {
            int v;
            switch (mode) {
            case 0: v = S[5 + x]; break;
            case 1: v = S[3 - y]; break;
            case 2: {
                int st = S[5] + S[6] + S[7] + S[8], sl = S[3] + S[2] + S[1] + S[0];
                if (avail_top && avail_left) v = (st + sl + 4) >> 3;
                else if (avail_left) v = (sl + 2) >> 2;
                else if (avail_top) v = (st + 2) >> 2;
                else v = 128;
                break;
            }
            case 3:
                if (x == 3 && y == 3) v = (S[11] + 3 * S[12] + 2) >> 2;
                else v = (S[5 + x + y] + 2 * S[6 + x + y] + S[7 + x + y] + 2) >> 2;
                break;
            case 4: {
                int d = x - y;
                v = (S[3 + d] + 2 * S[4 + d] + S[5 + d] + 2) >> 2;
                break;
            }
            case 5: {
                int z = 2 * x - y, i = x - (y >> 1);
                if (z >= 0 && !(z & 1)) v = (S[4 + i] + S[5 + i] + 1) >> 1;
                else if (z > 0) v = (S[3 + i] + 2 * S[4 + i] + S[5 + i] + 2) >> 2;
                else if (z == -1) v = (S[3] + 2 * S[4] + S[5] + 2) >> 2;
                else v = (S[4 - y] + 2 * S[5 - y] + S[6 - y] + 2) >> 2;
                break;
            }
            case 6: {
                int z = 2 * y - x, i = y - (x >> 1);
                if (z >= 0 && !(z & 1)) v = (S[4 - i] + S[3 - i] + 1) >> 1;
                else if (z > 0) v = (S[5 - i] + 2 * S[4 - i] + S[3 - i] + 2) >> 2;
                else if (z == -1) v = (S[3] + 2 * S[4] + S[5] + 2) >> 2;
                else v = (S[4 + x] + 2 * S[3 + x] + S[2 + x] + 2) >> 2;
                break;
            }
            case 7: {
                int i = x + (y >> 1);
                if (!(y & 1)) v = (S[5 + i] + S[6 + i] + 1) >> 1;
                else v = (S[5 + i] + 2 * S[6 + i] + S[7 + i] + 2) >> 2;
                break;
            }
            default: {
                int z = x + 2 * y, i = y + (x >> 1);
                if (z > 5) v = S[0];
                else if (z == 5) v = (S[1] + 3 * S[0] + 2) >> 2;
                else if (!(z & 1)) v = (S[3 - i] + S[2 - i] + 1) >> 1;
                else v = (S[3 - i] + 2 * S[2 - i] + S[1 - i] + 2) >> 2;
                break;
            }
            }
            pred[y * 4 + x] = v;
        }
}

static void recon_intra(const OracleCtx *c, Planes *pl, int mbx, int mby, const MbRec *r,
                        const int32_t *res)
{
    int W = pl->w;
    uint8_t *Y = pl->y;
    int aA = !!(r->avail & AV_A), aB = !!(r->avail & AV_B), aC = !!(r->avail & AV_C), aD = !!(r->avail & AV_D);
    int x0 = mbx * 16, y0 = mby * 16;
    (void)c;
    if (r->type == MBT_I16) {
        int mode = r->pred & 3;
        int top[16], left[16], tl = 0;
        for (int i = 0; i < 16; i++) {
            top[i] = aB ? Y[(y0 - 1) * W + x0 + i] : 0;
            left[i] = aA ? Y[(y0 + i) * W + x0 - 1] : 0;
        }
        if (aD) tl = Y[(y0 - 1) * W + x0 - 1];
        int pred[256];
        if (mode == 0) for (int i = 0; i < 256; i++) pred[i] = top[i & 15];
        else if (mode == 1) for (int i = 0; i < 256; i++) pred[i] = left[i >> 4];
        else if (mode == 2) {
            int s = 0, v;
            if (aA && aB) { for (int i = 0; i < 16; i++) s += top[i] + left[i]; v = (s + 16) >> 5; }
            else if (aA) { for (int i = 0; i < 16; i++) s += left[i]; v = (s + 8) >> 4; }
            else if (aB) { for (int i = 0; i < 16; i++) s += top[i]; v = (s + 8) >> 4; }
            else v = 128;
            for (int i = 0; i < 256; i++) pred[i] = v;
        } else {
            int H = 0, V = 0;
            for (int i = 0; i < 8; i++) {
                H += (i + 1) * (top[8 + i] - (6 - i >= 0 ? top[6 - i] : tl));
                V += (i + 1) * (left[8 + i] - (6 - i >= 0 ? left[6 - i] : tl));
            }
            int a = 16 * (left[15] + top[15]);
            int b = (5 * H + 32) >> 6, cc = (5 * V + 32) >> 6;
            for (int y = 0; y < 16; y++)
                for (int x = 0; x < 16; x++) pred[y * 16 + x] = clip255((a + b * (x - 7) + cc * (y - 7) + 16) >> 5);
        }
        for (int y = 0; y < 16; y++)
            for (int x = 0; x < 16; x++)
                Y[(y0 + y) * W + x0 + x] = (uint8_t)clip255(pred[y * 16 + x] + res[y * 16 + x]);
    } else {
        for (int b = 0; b < 16; b++) {
            int bx = kBlkX[b], by = kBlkY[b];
            int px = x0 + bx * 4, py = y0 + by * 4;
            int avL = bx > 0 || aA;
            int avT = by > 0 || aB;
            int avTL = (bx > 0 && by > 0) || (bx == 0 && by > 0 ? aA : (by == 0 && bx > 0 ? aB : aD));
            int avTR;
            if (b == 3 || b == 7 || b == 11 || b == 13 || b == 15) avTR = 0;
            else if (by == 0) avTR = bx == 3 ? aC : aB;
            else avTR = 1;
            int top[8], left[4], tl = 0;
            for (int i = 0; i < 4; i++) {
                top[i] = avT ? Y[(py - 1) * W + px + i] : 0;
                left[i] = avL ? Y[(py + i) * W + px - 1] : 0;
            }
            for (int i = 4; i < 8; i++) top[i] = avT ? (avTR ? Y[(py - 1) * W + px + i] : top[3]) : 0;
            if (avTL) tl = Y[(py - 1) * W + px - 1];
            int mode = (r->i4[b >> 1] >> ((b & 1) * 4)) & 15;
            int pred[16];
            intra4x4_pred(mode, top, left, tl, avT, avL, pred);
            for (int y = 0; y < 4; y++)
                for (int x = 0; x < 4; x++)
                    Y[(py + y) * W + px + x] =
                        (uint8_t)clip255(pred[y * 4 + x] + res[(by * 4 + y) * 16 + bx * 4 + x]);
        }
    }
    /* chroma */
    int cw = W / 2;
    int cmode = (r->pred >> 4) & 3;
    for (int comp = 0; comp < 2; comp++) {
        uint8_t *C = comp ? pl->v : pl->u;
        int cx0 = mbx * 8, cy0 = mby * 8;
        int top[8], left[8], tl = 0;
        for (int i = 0; i < 8; i++) {
            top[i] = aB ? C[(cy0 - 1) * cw + cx0 + i] : 0;
            left[i] = aA ? C[(cy0 + i) * cw + cx0 - 1] : 0;
        }
        if (aD) tl = C[(cy0 - 1) * cw + cx0 - 1];
        int pred[64];
        if (cmode == 0) {
            for (int blk = 0; blk < 4; blk++) {
                int xo = (blk & 1) * 4, yo = (blk >> 1) * 4;
                int st = 0, sl = 0, v;
                for (int i = 0; i < 4; i++) { st += top[xo + i]; sl += left[yo + i]; }
                if ((xo == 0 && yo == 0) || (xo > 0 && yo > 0)) {
                    if (aA && aB) v = (st + sl + 4) >> 3;
                    else if (aA) v = (sl + 2) >> 2;
                    else if (aB) v = (st + 2) >> 2;
                    else v = 128;
                } else if (xo > 0) {
                    if (aB) v = (st + 2) >> 2;
                    else if (aA) v = (sl + 2) >> 2;
                    else v = 128;
                } else {
                    if (aA) v = (sl + 2) >> 2;
                    else if (aB) v = (st + 2) >> 2;
                    else v = 128;
                }
                for (int y = 0; y < 4; y++) for (int x = 0; x < 4; x++) pred[(yo + y) * 8 + xo + x] = v;
            }
        } else if (cmode == 1) {
            for (int i = 0; i < 64; i++) pred[i] = left[i >> 3];
        } else if (cmode == 2) {
            for (int i = 0; i < 64; i++) pred[i] = top[i & 7];
        } else {
            int H = 0, V = 0;
            for (int i = 0; i < 4; i++) {
                H += (i + 1) * (top[4 + i] - (2 - i >= 0 ? top[2 - i] : tl));
                V += (i + 1) * (left[4 + i] - (2 - i >= 0 ? left[2 - i] : tl));
            }
            int a = 16 * (left[7] + top[7]);
            int b = (34 * H + 32) >> 6, cc = (34 * V + 32) >> 6;
            for (int y = 0; y < 8; y++)
                for (int x = 0; x < 8; x++) pred[y * 8 + x] = clip255((a + b * (x - 3) + cc * (y - 3) + 16) >> 5);
        }
        for (int y = 0; y < 8; y++)
            for (int x = 0; x < 8; x++)
                C[(cy0 + y) * cw + cx0 + x] = (uint8_t)clip255(pred[y * 8 + x] + res[256 + comp * 64 + y * 8 + x]);
    }
}

/* ------------------------------------------------------------- inter --- */
static inline int refpix(const uint8_t *p, int w, int h, int x, int y)
{
    return p[clip3(0, h - 1, y) * w + clip3(0, w - 1, x)];
}

static inline int tap6(int a, int b, int c, int d, int e, int f) { return a - 5 * b + 20 * c + 20 * d - 5 * e + f; }

static int luma_sample(const uint8_t *R, int w, int h, int x, int y, int fx, int fy)
{
#define P(dx, dy) refpix(R, w, h, x + (dx), y + (dy))
#define B1(dy) tap6(P(-2, dy), P(-1, dy), P(0, dy), P(1, dy), P(2, dy), P(3, dy))
#define H1(dx) tap6(P(dx, -2), P(dx, -1), P(dx, 0), P(dx, 1), P(dx, 2), P(dx, 3))
    int G = P(0, 0);
    if (!fx && !fy) return G;
    int b = clip255((B1(0) + 16) >> 5);
    int hh = clip255((H1(0) + 16) >> 5);
    int s = clip255((B1(1) + 16) >> 5);
    int m = clip255((H1(1) + 16) >> 5);
    int j1 = tap6(B1(-2), B1(-1), B1(0), B1(1), B1(2), B1(3));
    int j = clip255((j1 + 512) >> 10);
    switch (fy * 4 + fx) {
    case 1: return (G + b + 1) >> 1;
    case 2: return b;
    case 3: return (P(1, 0) + b + 1) >> 1;
    case 4: return (G + hh + 1) >> 1;
    case 5: return (b + hh + 1) >> 1;
    case 6: return (b + j + 1) >> 1;
    case 7: return (b + m + 1) >> 1;
    case 8: return hh;
    case 9: return (hh + j + 1) >> 1;
    case 10: return j;
    case 11: return (j + m + 1) >> 1;
    case 12: return (P(0, 1) + hh + 1) >> 1;
    case 13: return (hh + s + 1) >> 1;
    case 14: return (j + s + 1) >> 1;
    default: return (m + s + 1) >> 1;
    }
#undef P
#undef B1
#undef H1
}

static void recon_inter(const OracleCtx *c, Planes *pl, int mbx, int mby, const MbRec *r,
                        const int32_t *res)
{
    int W = pl->w, H = pl->h;
    for (int b = 0; b < 16; b++) {
        Planes rp = planes_of(c, r->ref[b >> 2]);
        int mvx = r->mv[b][0], mvy = r->mv[b][1];
        int bx = mbx * 16 + kBlkX[b] * 4, by = mby * 16 + kBlkY[b] * 4;
        for (int y = 0; y < 4; y++)
            for (int x = 0; x < 4; x++) {
                int v = luma_sample(rp.y, W, H, bx + x + (mvx >> 2), by + y + (mvy >> 2), mvx & 3, mvy & 3);
                int ly = kBlkY[b] * 4 + y, lx = kBlkX[b] * 4 + x;
                pl->y[(by + y) * W + bx + x] = (uint8_t)clip255(v + res[ly * 16 + lx]);
            }
        int cw = W / 2, ch = H / 2;
        int cbx = bx / 2, cby = by / 2;
        int fx = mvx & 7, fy = mvy & 7;
        for (int comp = 0; comp < 2; comp++) {
            const uint8_t *R = comp ? rp.v : rp.u;
            uint8_t *D = comp ? pl->v : pl->u;
            for (int y = 0; y < 2; y++)
                for (int x = 0; x < 2; x++) {
                    int xi = cbx + x + (mvx >> 3), yi = cby + y + (mvy >> 3);
                    int A = refpix(R, cw, ch, xi, yi), B = refpix(R, cw, ch, xi + 1, yi);
                    int C = refpix(R, cw, ch, xi, yi + 1), D2 = refpix(R, cw, ch, xi + 1, yi + 1);
                    int v = ((8 - fx) * (8 - fy) * A + fx * (8 - fy) * B + (8 - fx) * fy * C + fx * fy * D2 + 32) >> 6;
                    int ly = (cby - mby * 8) + y, lx = (cbx - mbx * 8) + x;
                    D[(cby + y) * cw + cbx + x] = (uint8_t)clip255(v + res[256 + comp * 64 + ly * 8 + lx]);
                }
        }
    }
}

/* ---------------------------------------------------------- deblock --- */
static int bs_edge(const MbRec *p, int bp, const MbRec *q, int bq, int mb_edge)
{
    if (p->type >= MBT_I4x4 || q->type >= MBT_I4x4 || ((p->dbf | q->dbf) & DBF_INTRA)) return mb_edge ? 4 : 3;
    if (((p->cbits >> bp) & 1) || ((q->cbits >> bq) & 1)) return 2;
    if (p->ref[bp >> 2] != q->ref[bq >> 2]) return 1;
    if (iabs(p->mv[bp][0] - q->mv[bq][0]) >= 4 || iabs(p->mv[bp][1] - q->mv[bq][1]) >= 4) return 1;
    return 0;
}

/* filter one line of samples across an edge; s points at q0, step = offset
 * from q0 to q1 (and -step to p0) */
static void filter_luma_line(uint8_t *s, int step, int bS, int alpha, int beta, int tc0)
{
    int p0 = s[-step], p1 = s[-2 * step], p2 = s[-3 * step], p3 = s[-4 * step];
    int q0 = s[0], q1 = s[step], q2 = s[2 * step], q3 = s[3 * step];
    if (!(iabs(p0 - q0) < alpha && iabs(p1 - p0) < beta && iabs(q1 - q0) < beta)) return;
    int ap = iabs(p2 - p0), aq = iabs(q2 - q0);
    if (bS < 4) {
        int tc = tc0 + (ap < beta) + (aq < beta);
        int d = clip3(-tc, tc, (((q0 - p0) << 2) + (p1 - q1) + 4) >> 3);
        s[-step] = (uint8_t)clip255(p0 + d);
        s[0] = (uint8_t)clip255(q0 - d);
        if (ap < beta) s[-2 * step] = (uint8_t)(p1 + clip3(-tc0, tc0, (p2 + ((p0 + q0 + 1) >> 1) - (p1 << 1)) >> 1));
        if (aq < beta) s[step] = (uint8_t)(q1 + clip3(-tc0, tc0, (q2 + ((p0 + q0 + 1) >> 1) - (q1 << 1)) >> 1));
    } else {
        int strong = iabs(p0 - q0) < ((alpha >> 2) + 2);
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

static void filter_chroma_line(uint8_t *s, int step, int bS, int alpha, int beta, int tc0)
{
    int p0 = s[-step], p1 = s[-2 * step], q0 = s[0], q1 = s[step];
    if (!(iabs(p0 - q0) < alpha && iabs(p1 - p0) < beta && iabs(q1 - q0) < beta)) return;
    if (bS < 4) {
        int tc = tc0 + 1;
        int d = clip3(-tc, tc, (((q0 - p0) << 2) + (p1 - q1) + 4) >> 3);
        s[-step] = (uint8_t)clip255(p0 + d);
        s[0] = (uint8_t)clip255(q0 - d);
    } else {
        s[-step] = (uint8_t)((2 * p1 + p0 + q1 + 2) >> 2);
        s[0] = (uint8_t)((2 * q1 + q0 + p1 + 2) >> 2);
    }
}

static void deblock_mb(Planes *pl, const MbRec *rec, int w_mbs, int mbx, int mby)
{
    const MbRec *q = &rec[mby * w_mbs + mbx];
    if (!(q->avail & DB_INNER)) return;
    int W = pl->w, cw = W / 2;
    for (int dir = 0; dir < 2; dir++) {            /* 0: vertical edges, 1: horizontal */
        for (int e = 0; e < 4; e++) {
            const MbRec *p = q;
            if (e == 0) {
                if (!(q->avail & (dir == 0 ? DB_LEFT : DB_TOP))) continue;
                p = dir == 0 ? q - 1 : q - w_mbs;
            }
            int bS[4];
            int any = 0;
            for (int k = 0; k < 4; k++) {
                int bq = dir == 0 ? blk_index(e, k) : blk_index(k, e);
                int bp;
                if (e == 0) bp = dir == 0 ? blk_index(3, k) : blk_index(k, 3);
                else bp = dir == 0 ? blk_index(e - 1, k) : blk_index(k, e - 1);
                bS[k] = bs_edge(p, bp, q, bq, e == 0);
                any |= bS[k];
            }
            if (!any) continue;
            /* luma */
            int qpav = (p->qp + q->qp + 1) >> 1;
            int ia = clip3(0, 51, qpav + q->offA), ib = clip3(0, 51, qpav + q->offB);
            int alpha = kAlpha[ia], beta = kBeta[ib];
            for (int i = 0; i < 16; i++) {
                int k = i >> 2;
                if (!bS[k]) continue;
                int x = mbx * 16 + (dir == 0 ? e * 4 : i), y = mby * 16 + (dir == 0 ? i : e * 4);
                int tc0 = bS[k] < 4 ? kTc0[ia][bS[k] - 1] : 0;
                filter_luma_line(pl->y + y * W + x, dir == 0 ? 1 : W, bS[k], alpha, beta, tc0);
            }
            /* chroma: edges 0 and 2 of luma map to chroma edges 0 and 1 */
            if (e & 1) continue;
            int qpc_av = (p->qpc + q->qpc + 1) >> 1;
            int ca = clip3(0, 51, qpc_av + q->offA), cb = clip3(0, 51, qpc_av + q->offB);
            int calpha = kAlpha[ca], cbeta = kBeta[cb];
            for (int comp = 0; comp < 2; comp++) {
                uint8_t *C = comp ? pl->v : pl->u;
                for (int i = 0; i < 8; i++) {
                    int k = i >> 1;
                    if (!bS[k]) continue;
                    int x = mbx * 8 + (dir == 0 ? e * 2 : i), y = mby * 8 + (dir == 0 ? i : e * 2);
                    int tc0 = bS[k] < 4 ? kTc0[ca][bS[k] - 1] : 0;
                    filter_chroma_line(C + y * cw + x, dir == 0 ? 1 : cw, bS[k], calpha, cbeta, tc0);
                }
            }
        }
    }
}

/* ------------------------------------------------------------ backend --- */
static int oracle_configure(void *vctx, int w_mbs, int h_mbs, int nslots)
{
    OracleCtx *c = (OracleCtx *)vctx;
    free(c->frames);
    c->w_mbs = w_mbs; c->h_mbs = h_mbs; c->nslots = nslots;
    c->frame_bytes = (size_t)w_mbs * h_mbs * 384;
    c->frames = (uint8_t *)calloc((size_t)nslots, c->frame_bytes);
    return c->frames ? 0 : -1;
}

int oracle_recon_picture(void *vctx, const MbRec *rec, const int16_t *coef, int w_mbs, int h_mbs, int cur_slot)
{
    OracleCtx *c = (OracleCtx *)vctx;
    Planes pl = planes_of(c, cur_slot);
    int32_t res[384];
    int errs = 0;
    for (int mby = 0; mby < h_mbs; mby++)
        for (int mbx = 0; mbx < w_mbs; mbx++) {
            const MbRec *r = &rec[mby * w_mbs + mbx];
            if (r->type == MBT_IPCM) {
                const uint8_t *s = (const uint8_t *)(coef + (size_t)r->coef * 16);
                for (int y = 0; y < 16; y++) memcpy(pl.y + (mby * 16 + y) * pl.w + mbx * 16, s + y * 16, 16);
                for (int y = 0; y < 8; y++) {
                    memcpy(pl.u + (mby * 8 + y) * (pl.w / 2) + mbx * 8, s + 256 + y * 8, 8);
                    memcpy(pl.v + (mby * 8 + y) * (pl.w / 2) + mbx * 8, s + 320 + y * 8, 8);
                }
                continue;
            }
            if (mb_residual(r, coef, res)) { errs++; memset(res, 0, sizeof(res)); }
            if (r->type >= MBT_I4x4) recon_intra(c, &pl, mbx, mby, r, res);
            else recon_inter(c, &pl, mbx, mby, r, res);
        }
    for (int mby = 0; mby < h_mbs; mby++)
        for (int mbx = 0; mbx < w_mbs; mbx++) deblock_mb(&pl, rec, w_mbs, mbx, mby);
    return errs;
}

static int oracle_decode(void *vctx, const PicBuild *pb, int cur_slot)
{
    OracleCtx *c = (OracleCtx *)vctx;
    oracle_recon_picture(c, pb->rec, pb->coef, pb->w, pb->h, cur_slot);
    return 0;
}

static int oracle_read(void *vctx, int slot, uint8_t *dst)
{
    OracleCtx *c = (OracleCtx *)vctx;
    memcpy(dst, c->frames + c->frame_bytes * (size_t)slot, c->frame_bytes);
    return 0;
}

static int oracle_copy(void *vctx, int dst, int src)
{
    OracleCtx *c = (OracleCtx *)vctx;
    memcpy(c->frames + c->frame_bytes * (size_t)dst, c->frames + c->frame_bytes * (size_t)src, c->frame_bytes);
    return 0;
}

static void oracle_destroy(void *vctx)
{
    OracleCtx *c = (OracleCtx *)vctx;
    free(c->frames);
    free(c);
}

H264Backend oracle_backend_create(void)
{
    H264Backend be;
    memset(&be, 0, sizeof(be));
    be.ctx = calloc(1, sizeof(OracleCtx));
    be.configure = oracle_configure;
    be.decode = oracle_decode;
    be.read = oracle_read;
    be.copy = oracle_copy;
    be.destroy = oracle_destroy;
    return be;
}

void *oracle_ctx_create(int w_mbs, int h_mbs, int nslots)
{
    OracleCtx *c = (OracleCtx *)calloc(1, sizeof(OracleCtx));
    if (!c) return NULL;
    if (oracle_configure(c, w_mbs, h_mbs, nslots)) { free(c); return NULL; }
    return c;
}

uint8_t *oracle_ctx_frame(void *vctx, int slot)
{
    OracleCtx *c = (OracleCtx *)vctx;
    return c->frames + c->frame_bytes * (size_t)slot;
}

void oracle_ctx_destroy(void *vctx) { oracle_destroy(vctx); }
