/* Per-picture macroblock context and the neighbour-dependent derivations of
 * H.264 that both the host parser and the synthetic-stream generator need:
 *   - neighbour MB availability (§6.4.x; reference h264bsd_neighbour.c:127-175,
 *     h264bsdIsNeighbourAvailable :369)
 *   - nC for CAVLC coeff_token (§9.2.1; reference macroblock_layer.c:807-869)
 *   - Intra4x4PredMode prediction (§8.3.1.1; reference
 *     intra_prediction.c:1885-1936 DetermineIntra4x4PredMode)
 *   - luma motion-vector prediction incl. P_Skip (§8.4.1.1-8.4.1.3; reference
 *     inter_prediction.c:499-1031)
 */
#ifndef H264MI_MBCTX_H
#define H264MI_MBCTX_H

#include <stdint.h>

typedef struct MbInfo {
    uint8_t  type;        /* MBT_* from mbrec.h */
    uint8_t  qp;          /* QPY as stored for deblocking (0 for I_PCM) */
    int8_t   refidx[4];   /* per 8x8, -1 for intra */
    int8_t   i4mode[16];  /* Intra4x4PredMode (z-scan); valid for MBT_I4x4 */
    uint8_t  tc[16];      /* luma TotalCoeff (z-scan) */
    uint8_t  tcc[8];      /* chroma AC TotalCoeff: Cb 0..3, Cr 4..7 */
    int16_t  mv[16][2];
} MbInfo;

#define SLICE_NONE 0xFFFFu

typedef struct PicCtx {
    int      w, h;        /* picture size in MBs */
    int      cip;         /* constrained_intra_pred_flag */
    MbInfo  *mb;          /* w*h entries */
    uint16_t *slice;      /* w*h slice tags, SLICE_NONE if not yet decoded: apart from
                           * the 112-byte MbInfo, so that a picture's reset and a
                           * committed slice touch 2 bytes per MB, not a cache line */
    /* neighbour cache of the MB being parsed (mbctx_begin_mb): nb[n] is
     * mbctx_neighbour(cur, n) while nb_key == cur + 1 (0: no cache; a
     * zero-initialised context has none) */
    int      nb_key;
    int      nb[4];
    /* with it, the neighbours' TotalCoeff next to the MB (-1: neighbour
     * unavailable): luma left column / top row (rows / columns 0..3), chroma
     * per component the left column / top row (0..1) -- nC (§9.2.1) without
     * the per-block neighbour walk */
    int8_t   nl[4], nt[4], ncl[2][2], nct[2][2];
} PicCtx;

enum { NB_A = 0, NB_B = 1, NB_C = 2, NB_D = 3 };

static inline int mb_is_intra(const MbInfo *m) { return m->type >= 2; }

/* address of neighbour MB n of `cur`, or -1 when not available (outside the
 * picture or in another slice) */
int mbctx_neighbour(const PicCtx *pc, int cur, int n);
/* the parser's MB loop: cache the four neighbours of cur once its slice tag
 * is set (every derivation below asks for them several times per MB), and
 * drop the cache when the MB is done (mbctx_end_mb) */
void mbctx_begin_mb(PicCtx *pc, int cur);
static inline void mbctx_end_mb(PicCtx *pc) { pc->nb_key = 0; }

/* nC for luma block `blk` (z-scan) of MB cur */
int mbctx_nc_luma(const PicCtx *pc, int cur, int blk);
/* nC for chroma AC block `blk` (0..3, raster 2x2) of component comp (0 Cb, 1 Cr) */
int mbctx_nc_chroma(const PicCtx *pc, int cur, int comp, int blk);

/* predicted Intra4x4PredMode for block blk; uses modes of blocks already
 * decoded in the current MB (stored in pc->mb[cur].i4mode) */
int mbctx_pred_i4mode(const PicCtx *pc, int cur, int blk);

/* partition shapes for directional prediction */
enum { PSHAPE_NORMAL = 0, PSHAPE_16x8 = 1, PSHAPE_8x16 = 2 };

/* luma MV prediction for a partition at (x4,y4) of w4 x h4 4x4-blocks with
 * reference index ref; done16 = mask of 4x4 blocks of the current MB whose
 * motion is already known (pc->mb[cur].mv/refidx hold it). */
void mbctx_mvp(const PicCtx *pc, int cur, int x4, int y4, int w4, int h4,
               int ref, int shape, int part_idx, uint32_t done16, int16_t mvp[2]);

/* P_Skip motion vector (§8.4.1.1) */
void mbctx_mv_skip(const PicCtx *pc, int cur, int16_t mv[2]);

#endif
