/* Neighbour-dependent derivations shared by the parser and the generator
 * (see mbctx.h for the standard / reference anchors). */
#include "mbctx.h"
#include "mbrec.h"
#include "tables.h"

#include <stdlib.h>

static int neighbour_of(const PicCtx *pc, int cur, int n)
{
    int w = pc->w;
    int col = cur % w;
    int a;
    switch (n) {
    case NB_A: if (col == 0) return -1; a = cur - 1; break;
    case NB_B: a = cur - w; break;
    case NB_C: if (col == w - 1) return -1; a = cur - w + 1; break;
    default:   if (col == 0) return -1; a = cur - w - 1; break;
    }
    if (a < 0) return -1;
    if (pc->slice[a] != pc->slice[cur]) return -1;
    return a;
}

int mbctx_neighbour(const PicCtx *pc, int cur, int n)
{
    if (pc->nb_key == cur + 1) return pc->nb[n];
    return neighbour_of(pc, cur, n);
}

static int nn_luma(const MbInfo *m, int blk);
static int nn_chroma(const MbInfo *m, int comp, int blk);

void mbctx_begin_mb(PicCtx *pc, int cur)
{
    pc->nb_key = 0;
    {
        /* neighbour_of for the four, one division */
        const int w = pc->w, col = cur % w;
        const uint16_t sl = pc->slice[cur];
        const int a = col > 0 ? cur - 1 : -1, b = cur - w;
        const int c = col < w - 1 ? cur - w + 1 : -1, d = col > 0 ? cur - w - 1 : -1;
        pc->nb[NB_A] = a >= 0 && pc->slice[a] == sl ? a : -1;
        pc->nb[NB_B] = b >= 0 && pc->slice[b] == sl ? b : -1;
        pc->nb[NB_C] = c >= 0 && pc->slice[c] == sl ? c : -1;
        pc->nb[NB_D] = d >= 0 && pc->slice[d] == sl ? d : -1;
    }
    const MbInfo *A = pc->nb[NB_A] >= 0 ? &pc->mb[pc->nb[NB_A]] : NULL;
    const MbInfo *B = pc->nb[NB_B] >= 0 ? &pc->mb[pc->nb[NB_B]] : NULL;
    for (int i = 0; i < 4; i++) {
        pc->nl[i] = (int8_t)(A ? nn_luma(A, blk_index(3, i)) : -1);
        pc->nt[i] = (int8_t)(B ? nn_luma(B, blk_index(i, 3)) : -1);
    }
    for (int c = 0; c < 2; c++)
        for (int i = 0; i < 2; i++) {
            pc->ncl[c][i] = (int8_t)(A ? nn_chroma(A, c, i * 2 + 1) : -1);
            pc->nct[c][i] = (int8_t)(B ? nn_chroma(B, c, 2 + i) : -1);
        }
    pc->nb_key = cur + 1;
}

/* locate 4x4 block at (x4,y4) relative to MB cur (x4 in -1..4, y4 in -1..3) */
static int blk_nb(const PicCtx *pc, int cur, int x4, int y4, int *addr, int *blk)
{
    int n;
    if (y4 < 0) {
        n = x4 < 0 ? NB_D : (x4 > 3 ? NB_C : NB_B);
    } else {
        if (x4 > 3) return 0;
        if (x4 >= 0) { *addr = cur; *blk = blk_index(x4, y4); return 1; }
        n = NB_A;
    }
    int a = mbctx_neighbour(pc, cur, n);
    if (a < 0) return 0;
    *addr = a;
    *blk = blk_index(x4 & 3, y4 & 3);
    return 1;
}

static int nn_luma(const MbInfo *m, int blk)
{
    if (m->type == MBT_SKIP) return 0;
    if (m->type == MBT_IPCM) return 16;
    return m->tc[blk];
}

static inline int nc_of(int nA, int nB)
{
    if (nA >= 0 && nB >= 0) return (nA + nB + 1) >> 1;
    if (nA >= 0) return nA;
    if (nB >= 0) return nB;
    return 0;
}

int mbctx_nc_luma(const PicCtx *pc, int cur, int blk)
{
    int x = kBlkX[blk], y = kBlkY[blk];
    if (pc->nb_key == cur + 1) {
        /* the current MB's blocks to the left / above precede blk in z-scan
         * and hold their TotalCoeff already (its type is not skip or PCM) */
        const MbInfo *m = &pc->mb[cur];
        const int nA = x > 0 ? m->tc[blk_index(x - 1, y)] : pc->nl[y];
        const int nB = y > 0 ? m->tc[blk_index(x, y - 1)] : pc->nt[x];
        return nc_of(nA, nB);
    }
    int aA, bA, aB, bB;
    int avA = blk_nb(pc, cur, x - 1, y, &aA, &bA);
    int avB = blk_nb(pc, cur, x, y - 1, &aB, &bB);
    int nA = avA ? nn_luma(&pc->mb[aA], bA) : 0;
    int nB = avB ? nn_luma(&pc->mb[aB], bB) : 0;
    if (avA && avB) return (nA + nB + 1) >> 1;
    if (avA) return nA;
    if (avB) return nB;
    return 0;
}

static int nn_chroma(const MbInfo *m, int comp, int blk)
{
    if (m->type == MBT_SKIP) return 0;
    if (m->type == MBT_IPCM) return 16;
    return m->tcc[comp * 4 + blk];
}

int mbctx_nc_chroma(const PicCtx *pc, int cur, int comp, int blk)
{
    int x = blk & 1, y = blk >> 1;
    if (pc->nb_key == cur + 1) {
        const MbInfo *m = &pc->mb[cur];
        const int nA = x > 0 ? m->tcc[comp * 4 + blk - 1] : pc->ncl[comp][y];
        const int nB = y > 0 ? m->tcc[comp * 4 + blk - 2] : pc->nct[comp][x];
        return nc_of(nA, nB);
    }
    int avA, avB, nA = 0, nB = 0;
    if (x > 0) { avA = 1; nA = nn_chroma(&pc->mb[cur], comp, blk - 1); }
    else {
        int a = mbctx_neighbour(pc, cur, NB_A);
        avA = a >= 0;
        if (avA) nA = nn_chroma(&pc->mb[a], comp, y * 2 + 1);
    }
    if (y > 0) { avB = 1; nB = nn_chroma(&pc->mb[cur], comp, blk - 2); }
    else {
        int b = mbctx_neighbour(pc, cur, NB_B);
        avB = b >= 0;
        if (avB) nB = nn_chroma(&pc->mb[b], comp, 2 + x);
    }
    if (avA && avB) return (nA + nB + 1) >> 1;
    if (avA) return nA;
    if (avB) return nB;
    return 0;
}

int mbctx_pred_i4mode(const PicCtx *pc, int cur, int blk)
{
    int x = kBlkX[blk], y = kBlkY[blk];
    int aA, bA, aB, bB;
    int avA = blk_nb(pc, cur, x - 1, y, &aA, &bA);
    int avB = blk_nb(pc, cur, x, y - 1, &aB, &bB);
    if (!avA || !avB) return 2;
    const MbInfo *mA = &pc->mb[aA], *mB = &pc->mb[aB];
    if (pc->cip && (!mb_is_intra(mA) || !mb_is_intra(mB))) return 2;
    int modeA = mA->type == MBT_I4x4 ? mA->i4mode[bA] : 2;
    int modeB = mB->type == MBT_I4x4 ? mB->i4mode[bB] : 2;
    return modeA < modeB ? modeA : modeB;
}

typedef struct { int avail; int ref; int mv[2]; } NbMotion;

static NbMotion nb_motion(const PicCtx *pc, int cur, int x4, int y4, uint32_t done16)
{
    NbMotion r = {0, -1, {0, 0}};
    int a, b;
    if (!blk_nb(pc, cur, x4, y4, &a, &b)) return r;
    if (a == cur && !(done16 & (1u << b))) return r;  /* not yet decoded */
    r.avail = 1;
    const MbInfo *m = &pc->mb[a];
    if (mb_is_intra(m)) return r;                       /* ref -1, mv 0 */
    r.ref = m->refidx[b >> 2];
    r.mv[0] = m->mv[b][0];
    r.mv[1] = m->mv[b][1];
    return r;
}

static int median3(int a, int b, int c)
{
    int mx = a > b ? a : b; if (c > mx) mx = c;
    int mn = a < b ? a : b; if (c < mn) mn = c;
    return a + b + c - mx - mn;
}

void mbctx_mvp(const PicCtx *pc, int cur, int x4, int y4, int w4, int h4,
               int ref, int shape, int part_idx, uint32_t done16, int16_t mvp[2])
{
    (void)h4;
    NbMotion A = nb_motion(pc, cur, x4 - 1, y4, done16);
    NbMotion B = nb_motion(pc, cur, x4, y4 - 1, done16);
    NbMotion C = nb_motion(pc, cur, x4 + w4, y4 - 1, done16);
    if (!C.avail) C = nb_motion(pc, cur, x4 - 1, y4 - 1, done16);

    if (shape == PSHAPE_16x8) {
        if (part_idx == 0 && B.ref == ref) { mvp[0] = B.mv[0]; mvp[1] = B.mv[1]; return; }
        if (part_idx == 1 && A.ref == ref) { mvp[0] = A.mv[0]; mvp[1] = A.mv[1]; return; }
    } else if (shape == PSHAPE_8x16) {
        if (part_idx == 0 && A.ref == ref) { mvp[0] = A.mv[0]; mvp[1] = A.mv[1]; return; }
        if (part_idx == 1 && C.ref == ref) { mvp[0] = C.mv[0]; mvp[1] = C.mv[1]; return; }
    }
    /* §8.4.1.3.1 */
    if (!B.avail && !C.avail && A.avail) { B = A; C = A; }
    int mA = A.ref == ref, mB = B.ref == ref, mC = C.ref == ref;
    if (mA + mB + mC == 1) {
        const NbMotion *s = mA ? &A : (mB ? &B : &C);
        mvp[0] = (int16_t)s->mv[0];
        mvp[1] = (int16_t)s->mv[1];
        return;
    }
    mvp[0] = (int16_t)median3(A.mv[0], B.mv[0], C.mv[0]);
    mvp[1] = (int16_t)median3(A.mv[1], B.mv[1], C.mv[1]);
}

void mbctx_mv_skip(const PicCtx *pc, int cur, int16_t mv[2])
{
    mv[0] = mv[1] = 0;
    if (mbctx_neighbour(pc, cur, NB_A) < 0 || mbctx_neighbour(pc, cur, NB_B) < 0) return;
    NbMotion A = nb_motion(pc, cur, -1, 0, 0);
    NbMotion B = nb_motion(pc, cur, 0, -1, 0);
    if (A.ref == 0 && A.mv[0] == 0 && A.mv[1] == 0) return;
    if (B.ref == 0 && B.mv[0] == 0 && B.mv[1] == 0) return;
    mbctx_mvp(pc, cur, 0, 0, 4, 4, 0, PSHAPE_NORMAL, 0, 0, mv);
}
