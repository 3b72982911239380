/* slice_data() / macroblock_layer() parsing into MbRec batches (H.264
 * §7.3.4-7.3.5, semantics §7.4.5).  Replaces the parse half of the
 * reference: h264bsdDecodeSliceData (slice_data.c:85-235),
 * h264bsdDecodeMacroblockLayer / DecodeMbPred / DecodeSubMbPred /
 * DecodeResidual (macroblock_layer.c:133-869) and the host-side metadata of
 * h264bsdDecodeMacroblock (:964-1134: QP update, I_PCM), MV prediction
 * (inter_prediction.c:499-1031) and Intra4x4PredMode derivation
 * (intra_prediction.c:1885-1936). */
#include "picbuild.h"
#include "../common/cavlc.h"
#include "../common/resid.h"
#include "../common/tables.h"

#include <stdlib.h>
#include <string.h>

static void picbuild_reset_counts(PicBuild *pb, int cip);

int picbuild_init(PicBuild *pb, int w_mbs, int h_mbs)
{
    return picbuild_init_alloc(pb, w_mbs, h_mbs, NULL, NULL, NULL);
}

static void *pb_alloc(PicBuild *pb, size_t bytes)
{
    return pb->halloc ? pb->halloc(pb->hctx, bytes) : malloc(bytes);
}
static void pb_free(PicBuild *pb, void *p)
{
    if (pb->halloc) { if (p) pb->hfree(pb->hctx, p); }
    else free(p);
}

int picbuild_init_alloc(PicBuild *pb, int w_mbs, int h_mbs, void *(*halloc)(void *, size_t),
                        void (*hfree)(void *, void *), void *hctx)
{
    memset(pb, 0, sizeof(*pb));
    pb->halloc = halloc && hfree ? halloc : NULL;
    pb->hfree = hfree; pb->hctx = hctx;
    pb->pinned = pb->halloc != NULL;
    pb->w = w_mbs; pb->h = h_mbs; pb->nmbs = w_mbs * h_mbs;
    pb->rec = (MbRec *)pb_alloc(pb, (size_t)pb->nmbs * sizeof(MbRec));
    if (pb->rec) memset(pb->rec, 0, (size_t)pb->nmbs * sizeof(MbRec));
    pb->pc.mb = (MbInfo *)calloc((size_t)pb->nmbs, sizeof(MbInfo));
    pb->pc.slice = (uint16_t *)calloc((size_t)pb->nmbs, sizeof(uint16_t));
    pb->decoded = (uint8_t *)calloc((size_t)pb->nmbs, 1);
    pb->cap = (uint32_t)pb->nmbs * 8 + 64;
    pb->coef = (int16_t *)pb_alloc(pb, (size_t)pb->cap * 32);
    pb->pc.w = w_mbs; pb->pc.h = h_mbs;
    if (!pb->rec || !pb->pc.mb || !pb->pc.slice || !pb->coef || !pb->decoded) { picbuild_free(pb); return -1; }
    return 0;
}

void picbuild_free(PicBuild *pb)
{
    pb_free(pb, pb->rec); free(pb->pc.mb); free(pb->pc.slice); pb_free(pb, pb->coef); free(pb->decoded);
    pb->rec = NULL; pb->pc.mb = NULL; pb->pc.slice = NULL; pb->coef = NULL; pb->decoded = NULL;
}

/* a private PicBuild that receives one slice at a time (specparse.c): the
 * slice ids keep counting up instead of every MB's id being cleared, so an
 * MB left from an earlier slice never carries the new slice's id (neighbours
 * outside the slice stay unavailable); a full reset only when the ids wrap */
void picbuild_reuse(PicBuild *pb, int cip)
{
    const int n = pb->nslices;
    if (n >= SLICE_NONE - 2) {
        picbuild_reset(pb, cip);
        return;
    }
    picbuild_reset_counts(pb, cip);
    pb->nslices = n;
}

void picbuild_reset(PicBuild *pb, int cip)
{
    /* h264bsdResetStorage (storage.c:442-462): no MB decoded, no slice id */
    memset(pb->pc.slice, 0xFF, sizeof(uint16_t) * (size_t)pb->nmbs);      /* SLICE_NONE */
    picbuild_reset_counts(pb, cip);
}

static void picbuild_reset_counts(PicBuild *pb, int cip)
{
    memset(pb->decoded, 0, (size_t)pb->nmbs);
    pb->last_mb_addr = 0;
    pb->pc.cip = cip;
    pb->ncoef = 0;
    pb->ndecoded = 0;
    pb->nslices = 0;
    pb->is_p = 0;
    pb->alg_ref_bytes = 0;
    pb->n_inter = pb->n_intra = pb->n_coded_blocks = 0;
}

int16_t *picbuild_coef_alloc(PicBuild *pb, uint32_t nblk)
{
    if (pb->ncoef + nblk > pb->cap) {
        uint32_t nc = pb->cap * 2;
        while (nc < pb->ncoef + nblk) nc *= 2;
        int16_t *p;
        if (pb->halloc) {
            p = (int16_t *)pb->halloc(pb->hctx, (size_t)nc * 32);
            if (!p) return NULL;
            memcpy(p, pb->coef, (size_t)pb->ncoef * 32);
            pb->hfree(pb->hctx, pb->coef);
        } else {
            p = (int16_t *)realloc(pb->coef, (size_t)nc * 32);
            if (!p) return NULL;
        }
        pb->coef = p;
        pb->cap = nc;
    }
    int16_t *r = pb->coef + (size_t)pb->ncoef * 16;
    pb->ncoef += nblk;
    return r;
}

static int clip3(int lo, int hi, int v) { return v < lo ? lo : v > hi ? hi : v; }

/* algorithmic reference-fetch bytes of one partition (SURVEY.md §8d R_alg) */
static uint32_t part_bytes(int w, int h, const int16_t *mv)
{
    int fx = mv[0] & 3, fy = mv[1] & 3, cx = mv[0] & 7, cy = mv[1] & 7;
    uint32_t l = (uint32_t)((w + (fx ? 5 : 0)) * (h + (fy ? 5 : 0)));
    uint32_t c = (uint32_t)((w / 2 + (cx ? 1 : 0)) * (h / 2 + (cy ? 1 : 0)));
    return l + 2 * c;
}

/* fields common to every record: availability, deblocking parameters */
static void finish_rec(PicBuild *pb, int cur, const SliceHdr *sh, const Pps *pps, uint16_t tag)
{
    MbRec *r = &pb->rec[cur];
    const PicCtx *pc = &pb->pc;
    uint8_t av = 0;
    for (int n = 0; n < 4; n++) {
        int a = mbctx_neighbour(pc, cur, n);
        if (a >= 0 && !(pc->cip && !mb_is_intra(&pc->mb[a]))) av |= (uint8_t)(1 << n);
    }
    if (sh->dbf_idc != 1) {
        av |= DB_INNER;
        int col = cur % pb->w;
        if (col > 0 && (sh->dbf_idc != 2 || pc->slice[cur - 1] == tag)) av |= DB_LEFT;
        if (cur >= pb->w && (sh->dbf_idc != 2 || pc->slice[cur - pb->w] == tag)) av |= DB_TOP;
    }
    r->avail = av;
    r->offA = (int8_t)(sh->off_a_div2 * 2);
    r->offB = (int8_t)(sh->off_b_div2 * 2);
    r->qpc = kQpChroma[clip3(0, 51, r->qp + pps->chroma_qp_offset)];
    r->slice = tag;
    r->dbf = 0;
    r->refidx = 0;
    if (r->type == MBT_INTER)
        for (int i = 0; i < 4; i++) r->refidx |= (uint16_t)((pc->mb[cur].refidx[i] & 15) << (4 * i));
}

/* The prediction-stage checks of h264bsdDecodeMacroblock that fail an MB:
 * motion vectors outside [-2048, 2047.75] x [-512, 511.75]
 * (inter_prediction.c:544-549, 620-628, ...) and intra modes that need an
 * unavailable neighbour (intra_prediction.c:656-677 16x16, 770-821 4x4,
 * 878-899 chroma).  Availability is the record's (slice + constrained
 * intra applied). */
static int mb_pred_valid(const MbRec *r)
{
    if (r->type == MBT_INTER || r->type == MBT_SKIP) {
        for (int b = 0; b < 16; b++)
            if ((uint32_t)(r->mv[b][0] + 8192) >= 16384u || (uint32_t)(r->mv[b][1] + 2048) >= 4096u) return 0;
        return 1;
    }
    if (r->type == MBT_IPCM) return 1;
    const int A = r->avail & AV_A, B = r->avail & AV_B, D = r->avail & AV_D;
    if (r->type == MBT_I16) {
        const int mode = r->pred & 3;
        if ((mode == 0 && !B) || (mode == 1 && !A) || (mode == 3 && !(A && B && D))) return 0;
    } else {
        for (int b = 0; b < 16; b++) {
            const int mode = (r->i4[b >> 1] >> ((b & 1) * 4)) & 15;
            const int x = kBlkX[b], y = kBlkY[b];
            const int L = x > 0 || A, T = y > 0 || B;
            const int TL = (x > 0 && y > 0) || (x == 0 && y > 0 ? A : (y == 0 && x > 0 ? B : D));
            if (((mode == 0 || mode == 3 || mode == 7) && !T) || ((mode == 1 || mode == 8) && !L) ||
                ((mode >= 4 && mode <= 6) && !(T && L && TL)))
                return 0;
        }
    }
    const int cm = (r->pred >> 4) & 3;
    return !((cm == 1 && !A) || (cm == 2 && !B) || (cm == 3 && !(A && B && D)));
}

static void decode_skip(PicBuild *pb, int cur, int qp, const int *ref_slot)
{
    /* P_Skip predicts from RefPicList0[0]; a missing picture fails the MB
     * (h264bsdInterPrediction -> h264bsdDecodeMacroblock NOK) */
    if (ref_slot[0] < 0) pb->mb_decode_err = 1;
    MbInfo *m = &pb->pc.mb[cur];
    MbRec *r = &pb->rec[cur];
    int16_t mv[2];
    m->type = MBT_SKIP;
    m->qp = (uint8_t)qp;
    memset(m->refidx, 0, sizeof(m->refidx));
    mbctx_mv_skip(&pb->pc, cur, mv);
    for (int b = 0; b < 16; b++) { m->mv[b][0] = mv[0]; m->mv[b][1] = mv[1]; }
    memset(r, 0, sizeof(*r));
    r->type = MBT_SKIP;
    r->qp = (uint8_t)qp;
    for (int i = 0; i < 4; i++) r->ref[i] = (uint8_t)ref_slot[0];
    memcpy(r->mv, m->mv, sizeof(r->mv));
    r->coef = pb->ncoef;
    pb->alg_ref_bytes += part_bytes(16, 16, mv);
    pb->n_inter++;
}

static int parse_inter_pred(PicBuild *pb, BitReader *br, int cur, int kind, int nref, const int *ref_slot)
{
    MbInfo *m = &pb->pc.mb[cur];
    MbRec *r = &pb->rec[cur];
    int refs[4] = {0, 0, 0, 0};
    int mvd[16][2];
    int nmvd = 0;
    uint32_t done = 0;
    if (kind < 3) {
        int npart = kind == 0 ? 1 : 2;
        for (int i = 0; i < npart; i++) {
            if (nref > 1) {
                uint32_t v = br_te(br, (uint32_t)(nref - 1));
                if ((int)v >= nref) return -1;
                refs[i] = (int)v;
            }
        }
        for (int i = 0; i < npart; i++) { mvd[i][0] = br_se(br); mvd[i][1] = br_se(br); }
        for (int i = 0; i < npart; i++) {
            int x4 = 0, y4 = 0, w4 = 4, h4 = 4, shape = PSHAPE_NORMAL;
            if (kind == 1) { y4 = 2 * i; h4 = 2; shape = PSHAPE_16x8; }
            if (kind == 2) { x4 = 2 * i; w4 = 2; shape = PSHAPE_8x16; }
            for (int b8 = 0; b8 < 4; b8++) {
                int bx = (b8 & 1) * 2, by = (b8 >> 1) * 2;
                if (bx >= x4 && bx < x4 + w4 && by >= y4 && by < y4 + h4) m->refidx[b8] = (int8_t)refs[i];
            }
            int16_t mvp[2];
            mbctx_mvp(&pb->pc, cur, x4, y4, w4, h4, refs[i], shape, i, done, mvp);
            int16_t mv[2] = {(int16_t)(mvp[0] + mvd[i][0]), (int16_t)(mvp[1] + mvd[i][1])};
            for (int y = y4; y < y4 + h4; y++)
                for (int x = x4; x < x4 + w4; x++) {
                    int b = blk_index(x, y);
                    m->mv[b][0] = mv[0]; m->mv[b][1] = mv[1];
                    done |= 1u << b;
                }
            pb->alg_ref_bytes += part_bytes(w4 * 4, h4 * 4, mv);
        }
    } else {
        int sub[4];
        for (int i = 0; i < 4; i++) {
            uint32_t v = br_ue(br);
            if (v > 3) return -1;
            sub[i] = (int)v;
        }
        if (kind == 3 && nref > 1)
            for (int i = 0; i < 4; i++) {
                uint32_t v = br_te(br, (uint32_t)(nref - 1));
                if ((int)v >= nref) return -1;
                refs[i] = (int)v;
            }
        for (int i = 0; i < 4; i++) m->refidx[i] = (int8_t)refs[i];
        static const int nsp[4] = {1, 2, 2, 4};
        for (int i = 0; i < 4; i++)
            for (int s = 0; s < nsp[sub[i]]; s++) { mvd[nmvd][0] = br_se(br); mvd[nmvd][1] = br_se(br); nmvd++; }
        int k = 0;
        for (int i = 0; i < 4; i++) {
            int ox = (i & 1) * 2, oy = (i >> 1) * 2;
            for (int s = 0; s < nsp[sub[i]]; s++, k++) {
                int x4 = ox, y4 = oy, w4 = 2, h4 = 2;
                if (sub[i] == 1) { y4 += s; h4 = 1; }
                if (sub[i] == 2) { x4 += s; w4 = 1; }
                if (sub[i] == 3) { x4 += s & 1; y4 += s >> 1; w4 = h4 = 1; }
                int16_t mvp[2];
                mbctx_mvp(&pb->pc, cur, x4, y4, w4, h4, refs[i], PSHAPE_NORMAL, 0, done, mvp);
                int16_t mv[2] = {(int16_t)(mvp[0] + mvd[k][0]), (int16_t)(mvp[1] + mvd[k][1])};
                for (int y = y4; y < y4 + h4; y++)
                    for (int x = x4; x < x4 + w4; x++) {
                        int b = blk_index(x, y);
                        m->mv[b][0] = mv[0]; m->mv[b][1] = mv[1];
                        done |= 1u << b;
                    }
                pb->alg_ref_bytes += part_bytes(w4 * 4, h4 * 4, mv);
            }
        }
    }
    for (int i = 0; i < 4; i++) {
        int s = ref_slot[m->refidx[i]];
        if (s < 0) pb->mb_decode_err = 1;          /* reference picture missing: fails at reconstruction */
        r->ref[i] = (uint8_t)s;
    }
    memcpy(r->mv, m->mv, sizeof(r->mv));
    return br->err ? -1 : 0;
}

static int parse_mb(PicBuild *pb, BitReader *br, int cur, const SliceHdr *sh, const Pps *pps,
                    const int *ref_slot, int *qp)
{
    MbInfo *m = &pb->pc.mb[cur];
    MbRec *r = &pb->rec[cur];
    int is_p = sh->slice_type == 0;
    uint32_t mbt = br_ue(br);
    int inter = 0;
    memset(r, 0, sizeof(*r));
    memset(m->refidx, -1, sizeof(m->refidx));
    if (is_p) {
        if (mbt < 5) inter = 1; else mbt -= 5;
    }
    if (!inter && mbt > 25) return -1;

    if (!inter && mbt == 25) {                       /* I_PCM, §7.3.5 */
        m->type = MBT_IPCM;
        while (!br_byte_aligned(br)) if (br_u1(br)) return -1;
        int16_t *dst = picbuild_coef_alloc(pb, 12);
        if (!dst) return -1;
        uint8_t *d8 = (uint8_t *)dst;
        for (int i = 0; i < 384; i++) d8[i] = (uint8_t)br_u(br, 8);
        r->type = MBT_IPCM;
        r->coef = pb->ncoef - 12;
        r->cbits = 0;
        m->qp = 0;                                   /* macroblock_layer.c:1003 */
        memset(m->tc, 16, sizeof(m->tc));
        memset(m->tcc, 16, sizeof(m->tcc));
        r->qp = 0;
        pb->n_intra++;
        return br->err ? -1 : 0;
    }

    int cbp = 0, is_i16 = 0;
    if (inter) {
        m->type = MBT_INTER;
        r->type = MBT_INTER;
        if (parse_inter_pred(pb, br, cur, (int)mbt, sh->num_ref_idx_active, ref_slot)) return -1;
        pb->n_inter++;
    } else if (mbt == 0) {                           /* I_NxN (Intra 4x4) */
        m->type = MBT_I4x4;
        r->type = MBT_I4x4;
        for (int b = 0; b < 16; b++) {
            int pred = mbctx_pred_i4mode(&pb->pc, cur, b);
            int mode;
            if (br_u1(br)) mode = pred;
            else {
                int rem = (int)br_u(br, 3);
                mode = rem < pred ? rem : rem + 1;
            }
            m->i4mode[b] = (int8_t)mode;
            r->i4[b >> 1] |= (uint8_t)(mode << ((b & 1) * 4));
        }
        uint32_t cm = br_ue(br);
        if (cm > 3) return -1;
        r->pred = (uint8_t)(cm << 4);
        pb->n_intra++;
    } else {                                          /* I_16x16 */
        m->type = MBT_I16;
        r->type = MBT_I16;
        is_i16 = 1;
        int t = (int)mbt - 1;
        cbp = ((t / 4) % 3) << 4 | (mbt >= 13 ? 15 : 0);
        uint32_t cm = br_ue(br);
        if (cm > 3) return -1;
        r->pred = (uint8_t)((t % 4) | (cm << 4));
        pb->n_intra++;
    }
    if (!is_i16) {
        uint32_t code = br_ue(br);
        if (code > 47) return -1;
        cbp = inter ? kCbpInter[code] : kCbpIntra[code];
    }
    if (cbp || is_i16) {
        int d = br_se(br);
        if (d < -26 || d > 25) return -1;
        *qp = (*qp + d + 52) % 52;
    }
    m->qp = (uint8_t)*qp;
    r->qp = (uint8_t)*qp;

    /* residual(), §7.3.5.3.  Coded blocks are decoded straight into the
     * picture's coefficient pool in bit order (luma 0..15, chroma AC 16..23,
     * then the DC blocks 24..26, which the syntax sends first and which go
     * through a local copy); a block with TotalCoeff 0 leaves no entry. */
    const uint32_t base = pb->ncoef;
    if (!picbuild_coef_alloc(pb, 27)) return -1;     /* room for every block */
    pb->ncoef = base;
    int16_t *nxt = pb->coef + (size_t)base * 16;
    int16_t dcb[3][16];
    memset(dcb, 0, sizeof(dcb));                     /* chroma DC fills 4 of 16 */
    const int16_t *blk[27];
    uint32_t bsum[27];
    uint32_t cbits = 0;
    if (is_i16) {
        int tc = cavlc_decode_block_sum(br, mbctx_nc_luma(&pb->pc, cur, 0), 16, dcb[0], &bsum[24]);
        if (tc < 0) return -1;
        if (tc) { cbits |= 1u << 24; blk[24] = dcb[0]; }
    }
    for (int b = 0; b < 16; b++) {
        if (cbp & (1 << (b >> 2))) {
            int nc = mbctx_nc_luma(&pb->pc, cur, b);
            int tc;
            if (is_i16) { nxt[0] = 0; tc = cavlc_decode_block_sum(br, nc, 15, nxt + 1, &bsum[b]); }
            else tc = cavlc_decode_block_sum(br, nc, 16, nxt, &bsum[b]);
            if (tc < 0) return -1;
            m->tc[b] = (uint8_t)tc;
            if (tc) { cbits |= 1u << b; blk[b] = nxt; nxt += 16; }
        } else {
            m->tc[b] = 0;
        }
    }
    int cc = cbp >> 4;
    if (cc) {
        for (int comp = 0; comp < 2; comp++) {
            int tc = cavlc_decode_block_sum(br, -1, 4, dcb[1 + comp], &bsum[25 + comp]);
            if (tc < 0) return -1;
            if (tc) { cbits |= 1u << (25 + comp); blk[25 + comp] = dcb[1 + comp]; }
        }
    }
    for (int comp = 0; comp < 2; comp++)
        for (int b = 0; b < 4; b++) {
            int idx = 16 + comp * 4 + b;
            if (cc & 2) {
                nxt[0] = 0;
                int tc = cavlc_decode_block_sum(br, mbctx_nc_chroma(&pb->pc, cur, comp, b), 15, nxt + 1, &bsum[idx]);
                if (tc < 0) return -1;
                m->tcc[comp * 4 + b] = (uint8_t)tc;
                if (tc) { cbits |= 1u << idx; blk[idx] = nxt; nxt += 16; }
            } else {
                m->tcc[comp * 4 + b] = 0;
            }
        }
    if (br->err) return -1;
    /* h264bsdDecodeMacroblock -> ProcessResidual: a residual outside
     * [-512, 511] fails the MB, hence the slice (resid.h) */
    if (cbits && !mb_residual_in_range(blk, bsum, cbits, is_i16, *qp,
                                       kQpChroma[clip3(0, 51, *qp + pps->chroma_qp_offset)]))
        pb->mb_decode_err = 1;
    for (int k = 0; k < 3; k++)
        if (cbits & (1u << (24 + k))) { memcpy(nxt, dcb[k], 32); nxt += 16; }
    const int nblk = __builtin_popcount(cbits);
    r->coef = base;
    r->cbits = cbits;
    pb->ncoef = base + (uint32_t)nblk;
    pb->n_coded_blocks += (uint32_t)nblk;
    return br->err ? -1 : 0;
}

/* An MB whose syntax parsed but whose reconstruction fails (residual range,
 * motion vector range, missing reference, intra mode without neighbours):
 * the reference has already counted it decoded (macroblock_layer.c:988) and
 * writes no samples for it.  Unless the slice's un-marking reaches it
 * (slice_data.c:322-338 can stop short of an I slice's second MB) it stays in
 * the picture with the slot's previous samples and its own deblocking
 * parameters: a zero-vector copy of the current slot, filtered as intra if it
 * was intra. */
static void failed_mb(PicBuild *pb, int cur)
{
    MbRec *r = &pb->rec[cur];
    const int intra = r->type >= MBT_I4x4;
    r->type = MBT_SKIP;
    r->cbits = 0;
    memset(r->mv, 0, sizeof(r->mv));
    for (int i = 0; i < 4; i++) r->ref[i] = (uint8_t)pb->cur_slot;
    r->dbf = intra ? DBF_INTRA : 0;
    pb->decoded[cur] = 1;
}

static int slice_data(PicBuild *pb, BitReader *br, const SliceHdr *sh, const Pps *pps, const int *ref_slot);

int parse_slice_data(PicBuild *pb, BitReader *br, const SliceHdr *sh, const Pps *pps,
                     const int *ref_slot)
{
    const int r = slice_data(pb, br, sh, pps, ref_slot);
    mbctx_end_mb(&pb->pc);      /* the neighbour cache lives for one MB of this slice only */
    return r;
}

static int slice_data(PicBuild *pb, BitReader *br, const SliceHdr *sh, const Pps *pps, const int *ref_slot)
{
    int cur = sh->first_mb;
    int qp = sh->slice_qp;
    int is_p = sh->slice_type == 0;
    int more = 1, count = 0;
    const uint16_t tag = (uint16_t)++pb->nslices;     /* sliceId, slice_data.c:120 */
    pb->last_mb_addr = 0;
    if (is_p) pb->is_p = 1;
    while (more) {
        if (is_p) {
            uint32_t run = br_ue(br);
            if (br->err || run > (uint32_t)(pb->nmbs - cur)) return -1;
            for (uint32_t i = 0; i < run; i++, cur++) {
                if (pb->decoded[cur]) return -1;      /* primary picture, already decoded */
                memset(&pb->pc.mb[cur], 0, sizeof(MbInfo));
                pb->pc.slice[cur] = tag;
                mbctx_begin_mb(&pb->pc, cur);
                pb->mb_decode_err = 0;
                decode_skip(pb, cur, qp, ref_slot);
                finish_rec(pb, cur, sh, pps, tag);
                if (pb->mb_decode_err || !mb_pred_valid(&pb->rec[cur])) { failed_mb(pb, cur); return -1; }
                pb->decoded[cur] = 1;
                count++;
            }
            if (run > 0) {
                more = br_more_rbsp_data(br);
                if (!more) break;
            }
        }
        if (cur >= pb->nmbs) return -1;
        if (pb->decoded[cur]) return -1;
        memset(&pb->pc.mb[cur], 0, sizeof(MbInfo));
        pb->pc.slice[cur] = tag;                   /* SetMbParams precedes the parse */
        mbctx_begin_mb(&pb->pc, cur);
        pb->mb_decode_err = 0;
        if (parse_mb(pb, br, cur, sh, pps, ref_slot, &qp)) return -1;
        finish_rec(pb, cur, sh, pps, tag);
        if (pb->mb_decode_err || !mb_pred_valid(&pb->rec[cur])) { failed_mb(pb, cur); return -1; }
        pb->decoded[cur] = 1;
        count++;
        if (!is_p) pb->last_mb_addr = cur;            /* slice_data.c:208-211 */
        cur++;
        more = br_more_rbsp_data(br);
    }
    if (br->err || pb->ndecoded + count > pb->nmbs) return -1;
    pb->ndecoded += count;
    return 0;
}

void picbuild_mark_slice_corrupted(PicBuild *pb, int first_mb)
{
    const uint16_t tag = (uint16_t)pb->nslices;
    int cur = first_mb;
    if (pb->last_mb_addr) {
        /* I slice: keep all but the last max(width, 10) decoded MBs */
        const int keep_back = pb->w > 10 ? pb->w : 10;
        int i = pb->last_mb_addr - 1, n = 0;
        while (i > cur) {
            if (pb->pc.slice[i] == tag && ++n >= keep_back) break;
            i--;
        }
        cur = i;
    }
    for (; cur < pb->nmbs; cur++) {
        if (pb->pc.slice[cur] != tag || !pb->decoded[cur]) break;
        pb->decoded[cur] = 0;
    }
}
