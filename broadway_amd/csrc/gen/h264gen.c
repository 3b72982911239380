/* Seeded synthetic H.264 Baseline stream generator -- see h264gen.h.
 * Syntax per ITU-T H.264 §7.3 (SPS/PPS/slice header/slice data/MB layer),
 * CAVLC per §9.2, predictions per mbctx.c. */
#include "h264gen.h"
#include "../common/bits.h"
#include "../common/cavlc.h"
#include "../common/mbctx.h"
#include "../common/mbrec.h"
#include "../common/tables.h"

#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- rng --- */
typedef struct { uint64_t s; } Rng;
static uint64_t rng_next(Rng *r)
{
    uint64_t z = (r->s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static int rnd(Rng *r, int n) { return n <= 1 ? 0 : (int)(rng_next(r) % (uint64_t)n); }
static int rnd_range(Rng *r, int lo, int hi) { return lo + rnd(r, hi - lo + 1); }
static int pct(Rng *r, int p) { return rnd(r, 100) < p; }

/* ------------------------------------------------------------ params --- */
void h264gen_default_params(GenParams *p, int w_mbs, int h_mbs)
{
    memset(p, 0, sizeof(*p));
    p->w_mbs = w_mbs; p->h_mbs = h_mbs;
    p->nframes = 10; p->gop = 60; p->slices = 1;
    p->pm_skip = 30; p->pm_16x16 = 25; p->pm_16x8 = 10; p->pm_8x16 = 10;
    p->pm_8x8 = 15; p->pm_intra = 10;
    p->p8x8_ref0_pct = 10;
    p->im_i4 = 55; p->im_i16 = 43; p->im_pcm = 2;
    p->i4_rem_pct = 50;
    p->qp_min = 22; p->qp_max = 38; p->qp_delta = 2;
    p->dbf_idc1_pct = 0; p->dbf_idc2_pct = 20; p->dbf_off = 6;
    p->num_ref_frames = 4;
    p->cip = 0; p->chroma_qp_offset = 0; p->poc_type = 2;
    p->coef_pct = 50; p->level_tail_pct = 5;
    p->mv_jitter = 24; p->offpic_pct = 5;
    p->log2_max_frame_num = 8;
    p->poc_swap = 0;
    p->seed = 1;
}

int h264gen_preset(GenParams *p, int config, uint64_t seed)
{
    switch (config) {
    case 0:  /* 640x368 (crop 360) plumbing stream, loop filter off */
        h264gen_default_params(p, 40, 23);
        p->crop_bottom = 8; p->nframes = 300; p->gop = 30;
        p->dbf_idc1_pct = 100; p->dbf_idc2_pct = 0;
        break;
    case 1:  /* 720p I-only */
        h264gen_default_params(p, 80, 45);
        p->nframes = 120; p->gop = 1;
        p->im_i4 = 58; p->im_i16 = 40; p->im_pcm = 2;
        p->qp_min = 20; p->qp_max = 36;
        p->dbf_idc1_pct = 0; p->dbf_idc2_pct = 0;
        break;
    case 2:  /* 1080p I+P */
    case 3:
        h264gen_default_params(p, 120, 68);
        p->crop_bottom = 8; p->nframes = 300; p->gop = 60; p->slices = 4;
        break;
    case 4:  /* 2160p I+P */
        h264gen_default_params(p, 240, 135);
        p->nframes = 120; p->gop = 60; p->slices = 4;
        break;
    default:
        return -1;
    }
    p->seed = seed;
    return 0;
}

/* ------------------------------------------------------------- output --- */
typedef struct { uint8_t *buf; size_t len, cap; } ByteBuf;
static void bb_put(ByteBuf *b, uint8_t v)
{
    if (b->len == b->cap) {
        b->cap = b->cap ? b->cap * 2 : 1 << 16;
        b->buf = (uint8_t *)realloc(b->buf, b->cap);
    }
    b->buf[b->len++] = v;
}

/* Annex-B start code + NAL header + payload with emulation prevention */
static void emit_nal(ByteBuf *out, int ref_idc, int type, const BitWriter *rbsp)
{
    bb_put(out, 0); bb_put(out, 0); bb_put(out, 0); bb_put(out, 1);
    bb_put(out, (uint8_t)((ref_idc << 5) | type));
    int zeros = 0;
    for (size_t i = 0; i < rbsp->nbytes; i++) {
        uint8_t v = rbsp->buf[i];
        if (zeros >= 2 && v <= 3) { bb_put(out, 3); zeros = 0; }
        bb_put(out, v);
        zeros = v == 0 ? zeros + 1 : 0;
    }
}

/* ---------------------------------------------------------- generator --- */
typedef struct Gen {
    GenParams p;
    Rng rng;
    ByteBuf out;
    PicCtx pc;
    int frame_num;
    int idr_id;
    int nref;            /* reference frames available (= nrefs) */
    /* reference model: what the decoder's DPB holds after each picture
     * (sliding window / MMCO, H.264 §8.2.5), for valid modification and
     * marking commands */
    struct { int frame_num, lt; } refs[16];   /* lt: LongTermFrameIdx, -1 short-term */
    int nrefs, max_lt;   /* max_lt: MaxLongTermFrameIdx, -1 "no long-term frame indices" */
    int cur_ref;         /* current picture is a reference picture */
    int prev_ref;        /* previous picture was a reference picture */
    Rng mrng;            /* reference-knob decisions */
    int nops, op[8], opa[8], opb[8];          /* planned MMCO of the current picture */
    int lt_idr;          /* current IDR: long_term_reference_flag */
    int gmx, gmy;        /* global motion, quarter-pel */
    int poc_lsb;
    Rng erng;            /* damage decisions (err_* / drop_* knobs) */
    int cur_mb;          /* MB being generated */
    int range_mb;        /* MB of the current slice given an out-of-range residual, -1: none */
    int drop_pic;        /* current picture's NALs are not emitted */
} Gen;

typedef struct SliceCfg {
    int is_p, qp, idc, offa, offb, nref_active;
    uint16_t tag;
} SliceCfg;

/* ---- residual range check (generator-private restatement of §8.5) ---- */
static int blk_class(int r) { int y = r >> 2, x = r & 3; return ((x & 1) == 0 && (y & 1) == 0) ? 0 : ((x & 1) && (y & 1)) ? 1 : 2; }

static int idct_in_range(const int32_t *d)
{
    int32_t t[16];
    for (int i = 0; i < 4; i++) {
        const int32_t *r = d + 4 * i;
        int32_t e = r[0] + r[2], f = r[0] - r[2];
        int32_t g = (r[1] >> 1) - r[3], h = r[1] + (r[3] >> 1);
        t[4 * i + 0] = e + h; t[4 * i + 1] = f + g;
        t[4 * i + 2] = f - g; t[4 * i + 3] = e - h;
    }
    for (int j = 0; j < 4; j++) {
        int32_t e = t[j] + t[8 + j], f = t[j] - t[8 + j];
        int32_t g = (t[4 + j] >> 1) - t[12 + j], h = t[4 + j] + (t[12 + j] >> 1);
        int32_t o[4] = {e + h, f + g, f - g, e - h};
        for (int k = 0; k < 4; k++) {
            int32_t v = (o[k] + 32) >> 6;
            if (v < -512 || v > 511) return 0;
        }
    }
    return 1;
}

/* levels in scan order; start = first scan position present */
static void dequant_block(const int16_t *lv, int start, int qp, int32_t *d)
{
    memset(d, 0, 16 * sizeof(int32_t));
    for (int s = start; s < 16; s++) {
        int r = kZigzag4x4[s];
        d[r] = (int32_t)lv[s] * (kLevelScale[qp % 6][blk_class(r)] << (qp / 6));
    }
}

typedef struct MbCoefs {
    int16_t luma[16][16];     /* scan order; for I16 position 0 unused */
    int16_t ldc[16];
    int16_t cdc[2][4];
    int16_t cac[2][4][16];    /* position 0 unused */
} MbCoefs;

static int mb_residual_ok(int is_i16, int qp, int qpc, const MbCoefs *c)
{
    int32_t d[16];
    int32_t dcy[16] = {0};
    if (is_i16) {
        int32_t m[16], t[16];
        for (int s = 0; s < 16; s++) m[kZigzag4x4[s]] = c->ldc[s];
        for (int i = 0; i < 4; i++) {
            const int32_t *r = m + 4 * i;
            t[4 * i + 0] = r[0] + r[1] + r[2] + r[3];
            t[4 * i + 1] = r[0] + r[1] - r[2] - r[3];
            t[4 * i + 2] = r[0] - r[1] - r[2] + r[3];
            t[4 * i + 3] = r[0] - r[1] + r[2] - r[3];
        }
        int v = kLevelScale[qp % 6][0], q6 = qp / 6;
        for (int j = 0; j < 4; j++) {
            int32_t a = t[j], b = t[4 + j], cc = t[8 + j], dd = t[12 + j];
            int32_t f[4] = {a + b + cc + dd, a + b - cc - dd, a - b - cc + dd, a - b + cc - dd};
            for (int k = 0; k < 4; k++) {
                int32_t x = f[k] * v;
                dcy[4 * k + j] = q6 >= 2 ? x << (q6 - 2) : ((x << q6) + 2) >> 2;
            }
        }
    }
    for (int b = 0; b < 16; b++) {
        dequant_block(c->luma[b], is_i16 ? 1 : 0, qp, d);
        if (is_i16) d[0] = dcy[kBlkY[b] * 4 + kBlkX[b]];
        if (!idct_in_range(d)) return 0;
    }
    int v = kLevelScale[qpc % 6][0], q6 = qpc / 6;
    for (int comp = 0; comp < 2; comp++) {
        const int16_t *x = c->cdc[comp];
        int32_t f[4] = {x[0] + x[1] + x[2] + x[3], x[0] - x[1] + x[2] - x[3],
                        x[0] + x[1] - x[2] - x[3], x[0] - x[1] - x[2] + x[3]};
        for (int b = 0; b < 4; b++) {
            dequant_block(c->cac[comp][b], 1, qpc, d);
            d[0] = ((f[b] * v) << q6) >> 1;
            if (!idct_in_range(d)) return 0;
        }
    }
    return 1;
}

static int16_t rand_level(Gen *g)
{
    int mag;
    int u = rnd(&g->rng, 100);
    if (pct(&g->rng, g->p.level_tail_pct)) mag = rnd_range(&g->rng, 4, 64);
    else mag = u < 60 ? 1 : (u < 85 ? 2 : 3);
    return (int16_t)(pct(&g->rng, 50) ? -mag : mag);
}

/* fill positions [start, maxpos) with a low-frequency-biased sparse pattern */
static void rand_block(Gen *g, int16_t *lv, int start, int n)
{
    memset(lv, 0, 16 * sizeof(int16_t));
    int k = 1 + rnd(&g->rng, 3);
    if (pct(&g->rng, 20)) k += rnd(&g->rng, 10);
    for (int i = 0; i < k; i++) {
        int span = n - start;
        int pos = start + (pct(&g->rng, 70) ? rnd(&g->rng, span < 6 ? span : 6) : rnd(&g->rng, span));
        lv[pos] = rand_level(g);
    }
}

static void scale_down(MbCoefs *c)
{
    int16_t *v = (int16_t *)c;
    for (size_t i = 0; i < sizeof(*c) / sizeof(int16_t); i++) v[i] = (int16_t)(v[i] / 2);
}

/* ------------------------------------------------------ header writing --- */
static void write_sps(Gen *g)
{
    const GenParams *p = &g->p;
    BitWriter bw; bw_init(&bw);
    bw_put(&bw, 66, 8);            /* profile_idc: Baseline */
    bw_put(&bw, 0xC0, 8);          /* constraint_set0/1 */
    int mbs = p->w_mbs * p->h_mbs;
    int level = mbs <= 1620 ? 30 : mbs <= 3600 ? 31 : mbs <= 8192 ? 40 : 51;
    bw_put(&bw, (uint32_t)level, 8);
    bw_ue(&bw, 0);                 /* seq_parameter_set_id */
    bw_ue(&bw, (uint32_t)(p->log2_max_frame_num - 4));
    bw_ue(&bw, (uint32_t)p->poc_type);
    if (p->poc_type == 0) bw_ue(&bw, 4);   /* log2_max_pic_order_cnt_lsb_minus4 -> 256 */
    bw_ue(&bw, (uint32_t)p->num_ref_frames);
    bw_put(&bw, (uint32_t)(p->gaps_allowed != 0), 1);   /* gaps_in_frame_num_value_allowed_flag */
    bw_ue(&bw, (uint32_t)(p->w_mbs - 1));
    bw_ue(&bw, (uint32_t)(p->h_mbs - 1));
    bw_put(&bw, 1, 1);             /* frame_mbs_only_flag */
    bw_put(&bw, 1, 1);             /* direct_8x8_inference_flag */
    int crop = p->crop_right || p->crop_bottom;
    bw_put(&bw, (uint32_t)crop, 1);
    if (crop) {
        bw_ue(&bw, 0); bw_ue(&bw, (uint32_t)(p->crop_right / 2));
        bw_ue(&bw, 0); bw_ue(&bw, (uint32_t)(p->crop_bottom / 2));
    }
    bw_put(&bw, 0, 1);             /* vui_parameters_present_flag */
    bw_trailing(&bw);
    emit_nal(&g->out, 3, 7, &bw);
    bw_free(&bw);
}

static void write_pps(Gen *g)
{
    const GenParams *p = &g->p;
    BitWriter bw; bw_init(&bw);
    bw_ue(&bw, 0); bw_ue(&bw, 0);  /* pps id, sps id */
    bw_put(&bw, 0, 1);             /* entropy_coding_mode_flag: CAVLC */
    bw_put(&bw, 0, 1);             /* bottom_field_pic_order_in_frame_present */
    bw_ue(&bw, 0);                 /* num_slice_groups_minus1 */
    bw_ue(&bw, (uint32_t)(p->num_ref_frames - 1));
    bw_ue(&bw, 0);
    bw_put(&bw, 0, 1);             /* weighted_pred_flag */
    bw_put(&bw, 0, 2);             /* weighted_bipred_idc */
    bw_se(&bw, 0);                 /* pic_init_qp_minus26 */
    bw_se(&bw, 0);                 /* pic_init_qs_minus26 */
    bw_se(&bw, p->chroma_qp_offset);
    bw_put(&bw, 1, 1);             /* deblocking_filter_control_present_flag */
    bw_put(&bw, (uint32_t)p->cip, 1);
    bw_put(&bw, 0, 1);             /* redundant_pic_cnt_present_flag */
    bw_trailing(&bw);
    emit_nal(&g->out, 3, 8, &bw);
    bw_free(&bw);
}

/* -------------------------------------------------------- MB decisions --- */
typedef struct IntraAv { int a, b, c, d; } IntraAv;

static IntraAv intra_avail(Gen *g, int cur)
{
    IntraAv av;
    int n[4];
    for (int i = 0; i < 4; i++) {
        n[i] = mbctx_neighbour(&g->pc, cur, i);
        if (n[i] >= 0 && g->p.cip && !mb_is_intra(&g->pc.mb[n[i]])) n[i] = -1;
    }
    av.a = n[NB_A] >= 0; av.b = n[NB_B] >= 0; av.c = n[NB_C] >= 0; av.d = n[NB_D] >= 0;
    return av;
}

static int i4_valid(const IntraAv *av, int blk, int mode)
{
    int x = kBlkX[blk], y = kBlkY[blk];
    int L = x > 0 || av->a;
    int T = y > 0 || av->b;
    int TL = (x > 0 && y > 0) || (x == 0 && y > 0 ? av->a : (y == 0 && x > 0 ? av->b : av->d));
    switch (mode) {
    case 2: return 1;
    case 0: case 3: case 7: return T;
    case 1: case 8: return L;
    default: return T && L && TL;
    }
}

static int pick_i4_mode(Gen *g, const IntraAv *av, int blk)
{
    int x = kBlkX[blk], y = kBlkY[blk];
    int L = x > 0 || av->a;
    int T = y > 0 || av->b;
    int TL = (x > 0 && y > 0) || (x == 0 && y > 0 ? av->a : (y == 0 && x > 0 ? av->b : av->d));
    int cand[9], n = 0;
    cand[n++] = 2;
    if (T) { cand[n++] = 0; cand[n++] = 3; cand[n++] = 7; }
    if (L) { cand[n++] = 1; cand[n++] = 8; }
    if (T && L && TL) { cand[n++] = 4; cand[n++] = 5; cand[n++] = 6; }
    return cand[rnd(&g->rng, n)];
}

static int pick_i16_mode(Gen *g, const IntraAv *av)
{
    int cand[4], n = 0;
    cand[n++] = 2;
    if (av->b) cand[n++] = 0;
    if (av->a) cand[n++] = 1;
    if (av->a && av->b && av->d) cand[n++] = 3;
    return cand[rnd(&g->rng, n)];
}

static int pick_chroma_mode(Gen *g, const IntraAv *av)
{
    int cand[4], n = 0;
    cand[n++] = 0;
    if (av->a) cand[n++] = 1;
    if (av->b) cand[n++] = 2;
    if (av->a && av->b && av->d) cand[n++] = 3;
    return cand[rnd(&g->rng, n)];
}

static int clampi(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }

/* choose a motion vector for a partition at pixel (px,py) of size w x h */
static void pick_mv(Gen *g, int px, int py, int w, int h, int base[2], int mv[2])
{
    int W = g->p.w_mbs * 16, H = g->p.h_mbs * 16;
    if (pct(&g->rng, g->p.offpic_pct)) {
        /* reference block partly/fully outside the picture, up to 64 px */
        int rx = pct(&g->rng, 50) ? rnd_range(&g->rng, -64, 0) : rnd_range(&g->rng, W - w, W - w + 64);
        int ry = pct(&g->rng, 50) ? rnd_range(&g->rng, -64, H - h + 64) : (pct(&g->rng, 50) ? rnd_range(&g->rng, -64, 0) : rnd_range(&g->rng, H - h, H - h + 64));
        mv[0] = (rx - px) * 4 + rnd(&g->rng, 4);
        mv[1] = (ry - py) * 4 + rnd(&g->rng, 4);
    } else {
        mv[0] = base[0] + rnd_range(&g->rng, -8, 8);
        mv[1] = base[1] + rnd_range(&g->rng, -8, 8);
        /* keep the reference block within the picture + 64 px margin */
        mv[0] = clampi(mv[0], (-64 - px) * 4, (W - w + 64 - px) * 4);
        mv[1] = clampi(mv[1], (-64 - py) * 4, (H - h + 64 - py) * 4);
    }
    mv[0] = clampi(mv[0], -2048 * 4, 2047 * 4);
    mv[1] = clampi(mv[1], -511 * 4, 511 * 4);
}

/* write the residual() syntax (§7.3.5.3) for MB `cur`; updates tc/tcc */
static void write_residual(Gen *g, BitWriter *bw, int cur, int is_i16, int cbp, const MbCoefs *c)
{
    MbInfo *m = &g->pc.mb[cur];
    if (is_i16) cavlc_encode_block(bw, mbctx_nc_luma(&g->pc, cur, 0), 16, c->ldc);
    for (int b8 = 0; b8 < 4; b8++)
        for (int j = 0; j < 4; j++) {
            int b = b8 * 4 + j;
            if (cbp & (1 << b8)) {
                int nc = mbctx_nc_luma(&g->pc, cur, b);
                int tc = is_i16 ? cavlc_encode_block(bw, nc, 15, c->luma[b] + 1)
                                : cavlc_encode_block(bw, nc, 16, c->luma[b]);
                m->tc[b] = (uint8_t)tc;
            } else {
                m->tc[b] = 0;
            }
        }
    int cc = cbp >> 4;
    if (cc) for (int comp = 0; comp < 2; comp++) cavlc_encode_block(bw, -1, 4, c->cdc[comp]);
    for (int comp = 0; comp < 2; comp++)
        for (int b = 0; b < 4; b++) {
            if (cc & 2) {
                int nc = mbctx_nc_chroma(&g->pc, cur, comp, b);
                m->tcc[comp * 4 + b] = (uint8_t)cavlc_encode_block(bw, nc, 15, c->cac[comp][b] + 1);
            } else {
                m->tcc[comp * 4 + b] = 0;
            }
        }
}

/* random coefficients for a cbp; retried/scaled until in range */
static void make_coefs(Gen *g, int is_i16, int cbp, int qp, MbCoefs *c)
{
    memset(c, 0, sizeof(*c));
    int qpc = kQpChroma[clampi(qp + g->p.chroma_qp_offset, 0, 51)];
    if (is_i16 && pct(&g->rng, 80)) rand_block(g, c->ldc, 0, 16);
    for (int b = 0; b < 16; b++)
        if (cbp & (1 << (b >> 2))) {
            if (pct(&g->rng, 75)) rand_block(g, c->luma[b], is_i16 ? 1 : 0, 16);
        }
    int cc = cbp >> 4;
    if (cc)
        for (int comp = 0; comp < 2; comp++)
            if (pct(&g->rng, 80))
                for (int i = 0; i < 4; i++) if (pct(&g->rng, 50)) c->cdc[comp][i] = rand_level(g);
    if (cc & 2)
        for (int comp = 0; comp < 2; comp++)
            for (int b = 0; b < 4; b++)
                if (pct(&g->rng, 60)) rand_block(g, c->cac[comp][b], 1, 16);
    while (!mb_residual_ok(is_i16, qp, qpc, c)) scale_down(c);
    if (g->cur_mb == g->range_mb) {
        /* one level large enough that the reference's ProcessBlock range
         * check fails (h264bsd_transform.c:181-185, 196-197): the slice is
         * then corrupted and concealed (slice_data.c:302-358, conceal.c) */
        int16_t *lv = is_i16 ? c->ldc : NULL;
        for (int b = 0; !lv && b < 16; b++) if (cbp & (1 << (b >> 2))) lv = c->luma[b];
        if (!lv && (cbp >> 4)) lv = c->cdc[0];
        if (lv) lv[0] = 2000;
    }
}

static int pick_cbp(Gen *g)
{
    int l = 0;
    for (int i = 0; i < 4; i++) if (pct(&g->rng, g->p.coef_pct)) l |= 1 << i;
    int u = rnd(&g->rng, 100);
    int c = u < 100 - g->p.coef_pct ? 0 : (u < 100 - g->p.coef_pct / 2 ? 1 : 2);
    return l | (c << 4);
}

static int cbp_code(int cbp, int intra)
{
    const uint8_t *t = intra ? kCbpIntra : kCbpInter;
    for (int i = 0; i < 48; i++) if (t[i] == cbp) return i;
    return 0;
}

/* pick an mb_qp_delta keeping QP inside [qp_min-? , 51] */
static int pick_qp_delta(Gen *g, int *qp)
{
    int d = rnd_range(&g->rng, -g->p.qp_delta, g->p.qp_delta);
    int nq = *qp + d;
    if (nq < 0 || nq > 51) d = 0;
    *qp += d;
    return d;
}

static void gen_intra_mb(Gen *g, BitWriter *bw, int cur, int is_p, int *qp)
{
    MbInfo *m = &g->pc.mb[cur];
    IntraAv av = intra_avail(g, cur);
    int u = rnd(&g->rng, 100);
    int kind = u < g->p.im_pcm ? MBT_IPCM : (u < g->p.im_pcm + g->p.im_i16 ? MBT_I16 : MBT_I4x4);
    int base = is_p ? 5 : 0;
    memset(m->refidx, -1, sizeof(m->refidx));
    memset(m->mv, 0, sizeof(m->mv));
    m->type = (uint8_t)kind;
    if (kind == MBT_IPCM) {
        bw_ue(bw, (uint32_t)(base + 25));
        while (!bw_aligned(bw)) bw_put(bw, 0, 1);
        for (int i = 0; i < 384; i++) bw_put(bw, (uint32_t)rnd_range(&g->rng, 1, 255), 8);
        m->qp = 0;
        memset(m->tc, 16, sizeof(m->tc));
        memset(m->tcc, 16, sizeof(m->tcc));
        return;
    }
    MbCoefs c;
    if (kind == MBT_I16) {
        int mode = pick_i16_mode(g, &av);
        int cmode = pick_chroma_mode(g, &av);
        int cbp = pick_cbp(g);
        int cl = (cbp & 15) ? 15 : 0, cc = cbp >> 4;
        cbp = cl | (cc << 4);
        bw_ue(bw, (uint32_t)(base + 1 + mode + 4 * cc + (cl ? 12 : 0)));
        bw_ue(bw, (uint32_t)cmode);
        int d = pick_qp_delta(g, qp);
        make_coefs(g, 1, cbp, *qp, &c);
        bw_se(bw, d);
        m->qp = (uint8_t)*qp;
        write_residual(g, bw, cur, 1, cbp, &c);
        return;
    }
    /* I4x4 */
    bw_ue(bw, (uint32_t)base);
    for (int b = 0; b < 16; b++) {
        int pred = mbctx_pred_i4mode(&g->pc, cur, b);
        int mode = (!pct(&g->rng, g->p.i4_rem_pct) && i4_valid(&av, b, pred)) ? pred
                                                                              : pick_i4_mode(g, &av, b);
        if (mode == pred) {
            bw_put(bw, 1, 1);
        } else {
            bw_put(bw, 0, 1);
            bw_put(bw, (uint32_t)(mode < pred ? mode : mode - 1), 3);
        }
        m->i4mode[b] = (int8_t)mode;
    }
    bw_ue(bw, (uint32_t)pick_chroma_mode(g, &av));
    int cbp = pick_cbp(g);
    bw_ue(bw, (uint32_t)cbp_code(cbp, 1));
    if (cbp) {
        int d = pick_qp_delta(g, qp);
        make_coefs(g, 0, cbp, *qp, &c);
        bw_se(bw, d);
        m->qp = (uint8_t)*qp;
        write_residual(g, bw, cur, 0, cbp, &c);
    } else {
        m->qp = (uint8_t)*qp;
    }
}

static void gen_inter_mb(Gen *g, BitWriter *bw, int cur, int kind, const SliceCfg *sc, int *qp, int base_mv[2])
{
    MbInfo *m = &g->pc.mb[cur];
    int W = g->p.w_mbs;
    int mbx = (cur % W) * 16, mby = (cur / W) * 16;
    int nref = sc->nref_active;
    m->type = MBT_INTER;
    uint32_t done = 0;
    int mvd[16][2], nmvd = 0;
    int refs[4];
    if (kind < 3) {
        static const int np[3] = {1, 2, 2};
        int npart = np[kind];
        bw_ue(bw, (uint32_t)kind);
        for (int i = 0; i < npart; i++) refs[i] = rnd(&g->rng, nref);
        if (nref > 1) for (int i = 0; i < npart; i++) bw_te(bw, (uint32_t)refs[i], (uint32_t)(nref - 1));
        for (int i = 0; i < npart; i++) {
            int x4 = 0, y4 = 0, w4 = 4, h4 = 4, shape = PSHAPE_NORMAL;
            if (kind == 1) { y4 = 2 * i; h4 = 2; shape = PSHAPE_16x8; }
            if (kind == 2) { x4 = 2 * i; w4 = 2; shape = PSHAPE_8x16; }
            int mv[2];
            pick_mv(g, mbx + x4 * 4, mby + y4 * 4, w4 * 4, h4 * 4, base_mv, mv);
            int16_t mvp[2];
            for (int b8 = 0; b8 < 4; b8++) {
                int bx = (b8 & 1) * 2, by = (b8 >> 1) * 2;
                if (bx >= x4 && bx < x4 + w4 && by >= y4 && by < y4 + h4) m->refidx[b8] = (int8_t)refs[i];
            }
            mbctx_mvp(&g->pc, cur, x4, y4, w4, h4, refs[i], shape, i, done, mvp);
            mvd[nmvd][0] = mv[0] - mvp[0]; mvd[nmvd][1] = mv[1] - mvp[1]; nmvd++;
            for (int y = y4; y < y4 + h4; y++)
                for (int x = x4; x < x4 + w4; x++) {
                    int b = blk_index(x, y);
                    m->mv[b][0] = (int16_t)mv[0]; m->mv[b][1] = (int16_t)mv[1];
                    done |= 1u << b;
                }
        }
        for (int i = 0; i < nmvd; i++) { bw_se(bw, mvd[i][0]); bw_se(bw, mvd[i][1]); }
    } else {
        int ref0 = nref == 1 ? 0 : pct(&g->rng, g->p.p8x8_ref0_pct);
        bw_ue(bw, ref0 ? 4u : 3u);
        int sub[4];
        for (int i = 0; i < 4; i++) { sub[i] = rnd(&g->rng, 4); bw_ue(bw, (uint32_t)sub[i]); }
        for (int i = 0; i < 4; i++) refs[i] = ref0 ? 0 : rnd(&g->rng, nref);
        if (nref > 1 && !ref0) for (int i = 0; i < 4; i++) bw_te(bw, (uint32_t)refs[i], (uint32_t)(nref - 1));
        for (int i = 0; i < 4; i++) m->refidx[i] = (int8_t)refs[i];
        for (int i = 0; i < 4; i++) {
            int ox = (i & 1) * 2, oy = (i >> 1) * 2;
            static const int nsp[4] = {1, 2, 2, 4};
            for (int s = 0; s < nsp[sub[i]]; s++) {
                int x4 = ox, y4 = oy, w4 = 2, h4 = 2;
                if (sub[i] == 1) { y4 += s; h4 = 1; }
                if (sub[i] == 2) { x4 += s; w4 = 1; }
                if (sub[i] == 3) { x4 += s & 1; y4 += s >> 1; w4 = h4 = 1; }
                int mv[2];
                pick_mv(g, mbx + x4 * 4, mby + y4 * 4, w4 * 4, h4 * 4, base_mv, mv);
                int16_t mvp[2];
                mbctx_mvp(&g->pc, cur, x4, y4, w4, h4, refs[i], PSHAPE_NORMAL, 0, done, mvp);
                mvd[nmvd][0] = mv[0] - mvp[0]; mvd[nmvd][1] = mv[1] - mvp[1]; nmvd++;
                for (int y = y4; y < y4 + h4; y++)
                    for (int x = x4; x < x4 + w4; x++) {
                        int b = blk_index(x, y);
                        m->mv[b][0] = (int16_t)mv[0]; m->mv[b][1] = (int16_t)mv[1];
                        done |= 1u << b;
                    }
            }
        }
        for (int i = 0; i < nmvd; i++) { bw_se(bw, mvd[i][0]); bw_se(bw, mvd[i][1]); }
    }
    int cbp = pick_cbp(g);
    bw_ue(bw, (uint32_t)cbp_code(cbp, 0));
    if (cbp) {
        MbCoefs c;
        int d = pick_qp_delta(g, qp);
        make_coefs(g, 0, cbp, *qp, &c);
        bw_se(bw, d);
        m->qp = (uint8_t)*qp;
        write_residual(g, bw, cur, 0, cbp, &c);
    } else {
        m->qp = (uint8_t)*qp;
    }
}

/* ------------------------------------------------- reference model --- */
static int max_fn(const Gen *g) { return 1 << (g->p.log2_max_frame_num < 4 ? 4 : g->p.log2_max_frame_num); }
/* FrameNumWrap of a short-term reference for the current frame_num */
static int fn_wrap(const Gen *g, int fn) { return fn > g->frame_num ? fn - max_fn(g) : fn; }

static void ref_remove(Gen *g, int i)
{
    for (int k = i; k + 1 < g->nrefs; k++) g->refs[k] = g->refs[k + 1];
    g->nrefs--;
}

static int find_lt(const Gen *g, int idx)
{
    for (int i = 0; i < g->nrefs; i++) if (g->refs[i].lt == idx) return i;
    return -1;
}

/* ref_pic_list_modification() of a P slice (§7.3.3.1): 1..3 commands that
 * move random references to the front, sometimes the same picture twice
 * (two indices then name one picture: bS must compare pictures) */
static void write_ref_mod(Gen *g, BitWriter *bw, int nact)
{
    if (!g->p.ref_mod_pct || !pct(&g->mrng, g->p.ref_mod_pct) || g->nrefs < 1) { bw_put(bw, 0, 1); return; }
    bw_put(bw, 1, 1);
    int ncmd = 1 + rnd(&g->mrng, nact < 3 ? nact : 3);
    int pred = g->frame_num, last = -1;
    for (int c = 0; c < ncmd; c++) {
        int i = (last >= 0 && pct(&g->mrng, 30)) ? last : rnd(&g->mrng, g->nrefs);
        last = i;
        if (g->refs[i].lt >= 0) {
            bw_ue(bw, 2);
            bw_ue(bw, (uint32_t)g->refs[i].lt);
        } else {
            const int M = max_fn(g), t = g->refs[i].frame_num;
            int down = (pred - t + M) % M, up = (t - pred + M) % M;
            if (!down) down = M;
            if (!up) up = M;
            const int use_up = pct(&g->mrng, 50);
            bw_ue(bw, use_up ? 1u : 0u);
            bw_ue(bw, (uint32_t)((use_up ? up : down) - 1));
            pred = t;
        }
    }
    bw_ue(bw, 3);
}

/* decide the current picture's reference marking; the commands are written
 * into every slice header and applied to the model after the picture */
static void plan_marking(Gen *g, int idr)
{
    g->nops = 0;
    g->lt_idr = idr && g->p.lt_idr_pct && pct(&g->mrng, g->p.lt_idr_pct);
    if (idr || !g->cur_ref) return;
    if (!g->p.mmco_pct || !pct(&g->mrng, g->p.mmco_pct)) {
        /* the sliding window needs a short-term picture to drop when the
         * buffer is full (a full buffer of long-term pictures leaves no
         * room, dpb.c:905-940) */
        int nshort = 0;
        for (int j = 0; j < g->nrefs; j++) nshort += g->refs[j].lt < 0;
        if (g->nrefs >= g->p.num_ref_frames && !nshort && g->nrefs) {
            g->op[0] = 2; g->opa[0] = g->refs[0].lt; g->nops = 1;
        }
        return;
    }
    struct { int frame_num, lt; } r[16];       /* the model, as the ops leave it */
    int n = g->nrefs, max_lt = g->max_lt, cur_lt = 0;
    memcpy(r, g->refs, sizeof(r));
    /* MMCO 5: everything unused; the next picture has frame_num 1, so this
     * one must not (the access-unit boundary is found by frame_num) */
    if (g->p.poc_type == 2 && g->frame_num > 1 && pct(&g->mrng, 8)) {
        g->op[0] = 5; g->nops = 1;
        return;
    }
    const int want = 1 + rnd(&g->mrng, 3);
    int n4 = 0;                                          /* at most one MMCO 4 and one MMCO 6 */
    for (int k = 0; k < 8 && g->nops < want && !cur_lt; k++) {
        const int pick = 1 + rnd(&g->mrng, 5);            /* 1,2,3,4 and 5 -> MMCO 6 */
        const int m = g->nops;
        int cs[16], ns = 0, cl[16], nl = 0;
        for (int j = 0; j < n; j++) { if (r[j].lt < 0) cs[ns++] = j; else cl[nl++] = j; }
        if (pick == 1 && ns) {
            const int i = cs[rnd(&g->mrng, ns)];
            g->op[m] = 1; g->opa[m] = g->frame_num - fn_wrap(g, r[i].frame_num) - 1;
            r[i] = r[--n];
        } else if (pick == 2 && nl) {
            const int i = cl[rnd(&g->mrng, nl)];
            g->op[m] = 2; g->opa[m] = r[i].lt;
            r[i] = r[--n];
        } else if (pick == 3 && ns && max_lt >= 0) {
            const int fnum = r[cs[rnd(&g->mrng, ns)]].frame_num;
            const int idx = rnd(&g->mrng, max_lt + 1);
            g->op[m] = 3; g->opa[m] = g->frame_num - fn_wrap(g, fnum) - 1; g->opb[m] = idx;
            for (int j = 0; j < n; j++) if (r[j].lt == idx) { r[j] = r[--n]; break; }
            for (int j = 0; j < n; j++) if (r[j].lt < 0 && r[j].frame_num == fnum) { r[j].lt = idx; break; }
        } else if (pick == 4 && !n4++) {
            const int v = rnd(&g->mrng, (g->p.num_ref_frames < 3 ? g->p.num_ref_frames : 3) + 1);   /* max_long_term_frame_idx_plus1 */
            g->op[m] = 4; g->opa[m] = v;
            max_lt = v - 1;
            for (int j = 0; j < n;) { if (r[j].lt >= 0 && r[j].lt > max_lt) r[j] = r[--n]; else j++; }
        } else if (pick == 5 && max_lt >= 0) {
            const int idx = rnd(&g->mrng, max_lt + 1);
            int nn = n;
            for (int j = 0; j < nn; j++) if (r[j].lt == idx) { nn--; break; }
            if (nn >= g->p.num_ref_frames) continue;     /* no room for the current picture */
            for (int j = 0; j < n; j++) if (r[j].lt == idx) { r[j] = r[--n]; break; }
            g->op[m] = 6; g->opa[m] = idx;
            cur_lt = 1;                                  /* MMCO 6 last */
        } else {
            continue;
        }
        g->nops++;
    }
    /* the current picture needs a free place: adaptive marking has no
     * sliding window (dpb.c:784-801) */
    if (!cur_lt && n >= g->p.num_ref_frames) {
        int i = -1, best = 0;
        for (int j = 0; j < n; j++)
            if (r[j].lt < 0 && (i < 0 || fn_wrap(g, r[j].frame_num) < best)) { i = j; best = fn_wrap(g, r[j].frame_num); }
        if (i >= 0) { g->op[g->nops] = 1; g->opa[g->nops] = g->frame_num - best - 1; }
        else { g->op[g->nops] = 2; g->opa[g->nops] = r[0].lt; }
        g->nops++;
    }
}

/* apply the current picture's marking to the model (after its slices) */
static void apply_marking(Gen *g, int idr)
{
    if (!g->cur_ref) return;
    if (idr) {
        g->nrefs = 1;
        g->refs[0].frame_num = 0;
        g->refs[0].lt = g->lt_idr ? 0 : -1;
        g->max_lt = g->lt_idr ? 0 : -1;
        return;
    }
    int cur_lt = -1, fn = g->frame_num;
    if (g->nops) {
        for (int k = 0; k < g->nops; k++) {
            const int op = g->op[k];
            if (op == 1 || op == 3) {
                const int pn = g->frame_num - (g->opa[k] + 1);
                for (int j = 0; j < g->nrefs; j++)
                    if (g->refs[j].lt < 0 && fn_wrap(g, g->refs[j].frame_num) == pn) {
                        if (op == 1) { ref_remove(g, j); break; }
                        const int o = find_lt(g, g->opb[k]);
                        if (o >= 0) { ref_remove(g, o); if (o < j) j--; }
                        g->refs[j].lt = g->opb[k];
                        break;
                    }
            } else if (op == 2) {
                const int o = find_lt(g, g->opa[k]);
                if (o >= 0) ref_remove(g, o);
            } else if (op == 4) {
                g->max_lt = g->opa[k] - 1;
                for (int j = 0; j < g->nrefs;) { if (g->refs[j].lt >= 0 && g->refs[j].lt > g->max_lt) ref_remove(g, j); else j++; }
            } else if (op == 5) {
                g->nrefs = 0;
                g->max_lt = -1;
                fn = 0;
            } else if (op == 6) {
                const int o = find_lt(g, g->opa[k]);
                if (o >= 0) ref_remove(g, o);
                cur_lt = g->opa[k];
            }
        }
    } else if (g->nrefs >= g->p.num_ref_frames) {
        /* sliding window: the short-term with the smallest FrameNumWrap */
        int i = -1;
        for (int j = 0; j < g->nrefs; j++)
            if (g->refs[j].lt < 0 && (i < 0 || fn_wrap(g, g->refs[j].frame_num) < fn_wrap(g, g->refs[i].frame_num))) i = j;
        if (i >= 0) ref_remove(g, i);
    }
    if (g->nrefs < 16) {
        g->refs[g->nrefs].frame_num = fn;
        g->refs[g->nrefs].lt = cur_lt;
        g->nrefs++;
    }
}

static void gen_slice(Gen *g, int idr, int first, int last, const SliceCfg *sc)
{
    const GenParams *p = &g->p;
    BitWriter bw; bw_init(&bw);
    bw_ue(&bw, (uint32_t)first);
    bw_ue(&bw, sc->is_p ? 0u : 2u);
    bw_ue(&bw, 0);
    bw_put(&bw, (uint32_t)g->frame_num, p->log2_max_frame_num);
    if (idr) bw_ue(&bw, (uint32_t)g->idr_id);
    if (p->poc_type == 0) bw_put(&bw, (uint32_t)g->poc_lsb, 8);
    if (sc->is_p) {
        int override = sc->nref_active != p->num_ref_frames;
        bw_put(&bw, (uint32_t)override, 1);
        if (override) bw_ue(&bw, (uint32_t)(sc->nref_active - 1));
        write_ref_mod(g, &bw, sc->nref_active);
    }
    if (g->cur_ref) {               /* dec_ref_pic_marking() */
        if (idr) { bw_put(&bw, 0, 1); bw_put(&bw, (uint32_t)g->lt_idr, 1); }
        else {
            bw_put(&bw, g->nops > 0, 1);    /* adaptive_ref_pic_marking_mode_flag */
            for (int i = 0; i < g->nops; i++) {
                const int op = g->op[i];
                bw_ue(&bw, (uint32_t)op);
                if (op == 1 || op == 3 || op == 2 || op == 6 || op == 4) bw_ue(&bw, (uint32_t)g->opa[i]);
                if (op == 3) bw_ue(&bw, (uint32_t)g->opb[i]);
            }
            if (g->nops > 0) bw_ue(&bw, 0);
        }
    }
    bw_se(&bw, sc->qp - 26);
    bw_ue(&bw, (uint32_t)sc->idc);
    if (sc->idc != 1) { bw_se(&bw, sc->offa); bw_se(&bw, sc->offb); }

    int qp = sc->qp;
    int skip_run = 0;
    g->range_mb = (p->err_range_pct && pct(&g->erng, p->err_range_pct)) ? rnd_range(&g->erng, first, last) : -1;
    int pm_tot = p->pm_skip + p->pm_16x16 + p->pm_16x8 + p->pm_8x16 + p->pm_8x8 + p->pm_intra;
    for (int cur = first; cur <= last; cur++) {
        MbInfo *m = &g->pc.mb[cur];
        memset(m, 0, sizeof(*m));
        g->pc.slice[cur] = sc->tag;
        g->cur_mb = cur;
        int base_mv[2] = {g->gmx + rnd_range(&g->rng, -p->mv_jitter, p->mv_jitter),
                          g->gmy + rnd_range(&g->rng, -p->mv_jitter, p->mv_jitter)};
        if (sc->is_p) {
            int u = rnd(&g->rng, pm_tot);
            int kind;   /* 0 16x16, 1 16x8, 2 8x16, 3 8x8, 4 intra, 5 skip */
            if (u < p->pm_skip) kind = 5;
            else if ((u -= p->pm_skip) < p->pm_16x16) kind = 0;
            else if ((u -= p->pm_16x16) < p->pm_16x8) kind = 1;
            else if ((u -= p->pm_16x8) < p->pm_8x16) kind = 2;
            else if ((u -= p->pm_8x16) < p->pm_8x8) kind = 3;
            else kind = 4;
            if (kind == 5) {
                int16_t mv[2];
                m->type = MBT_SKIP;
                mbctx_mv_skip(&g->pc, cur, mv);
                for (int b = 0; b < 16; b++) { m->mv[b][0] = mv[0]; m->mv[b][1] = mv[1]; }
                memset(m->refidx, 0, sizeof(m->refidx));
                m->qp = (uint8_t)qp;
                skip_run++;
                continue;
            }
            bw_ue(&bw, (uint32_t)skip_run);
            skip_run = 0;
            if (kind == 4) gen_intra_mb(g, &bw, cur, 1, &qp);
            else gen_inter_mb(g, &bw, cur, kind, sc, &qp, base_mv);
        } else {
            gen_intra_mb(g, &bw, cur, 0, &qp);
        }
    }
    if (skip_run) bw_ue(&bw, (uint32_t)skip_run);
    bw_trailing(&bw);
    int emit = !g->drop_pic;
    if (emit && p->drop_slice_pct && pct(&g->erng, p->drop_slice_pct)) emit = 0;
    if (emit && p->trunc_slice_pct && pct(&g->erng, p->trunc_slice_pct) && bw.nbytes > 4)
        bw.nbytes = (size_t)rnd_range(&g->erng, 2, (int)bw.nbytes - 1);
    if (emit) emit_nal(&g->out, idr ? 3 : g->cur_ref ? 2 : 0, idr ? 5 : 1, &bw);
    bw_free(&bw);
}

static void gen_picture(Gen *g, int idx)
{
    const GenParams *p = &g->p;
    int idr = (idx % p->gop) == 0;
    int nmb = p->w_mbs * p->h_mbs;
    g->drop_pic = !idr && p->drop_pic_pct && pct(&g->erng, p->drop_pic_pct);
    if (idr) {
        write_sps(g);
        write_pps(g);
        g->frame_num = 0;
        g->nref = 0;
        g->nrefs = 0;
        g->poc_lsb = 0;
    }
    /* non-reference pictures: never two in a row with POC type 2 (equal
     * picture order counts) */
    g->cur_ref = idr || !p->nonref_pct || (p->poc_type == 2 && !g->prev_ref) || !pct(&g->mrng, p->nonref_pct);
    plan_marking(g, idr);
    {   /* display order: 2 * index in GOP, optionally swapped in pairs */
        int k = idx % p->gop, d = k;
        int last = p->gop - 1;
        if (p->poc_swap && k >= 1) {
            if ((k & 1) && k + 1 <= last) d = k + 1;
            else if (!(k & 1)) d = k - 1;
        }
        g->poc_lsb = (2 * d) & 255;
    }
    for (int i = 0; i < nmb; i++) g->pc.slice[i] = SLICE_NONE;
    g->gmx += rnd_range(&g->rng, -6, 6);
    g->gmy += rnd_range(&g->rng, -4, 4);
    g->gmx = clampi(g->gmx, -256, 256);
    g->gmy = clampi(g->gmy, -128, 128);

    int ns = p->slices < 1 ? 1 : p->slices;
    if (ns > nmb) ns = nmb;
    int first = 0;
    for (int s = 0; s < ns; s++) {
        int last = (s == ns - 1) ? nmb - 1 : (int)((long)nmb * (s + 1) / ns) - 1 + rnd_range(&g->rng, -3, 3);
        if (last < first) last = first;
        if (last > nmb - 1 - (ns - 1 - s)) last = nmb - 1 - (ns - 1 - s);
        SliceCfg sc;
        sc.is_p = !idr && g->nrefs > 0;
        sc.qp = rnd_range(&g->rng, p->qp_min, p->qp_max);
        int u = rnd(&g->rng, 100);
        sc.idc = u < p->dbf_idc1_pct ? 1 : (u < p->dbf_idc1_pct + p->dbf_idc2_pct ? 2 : 0);
        sc.offa = rnd_range(&g->rng, -p->dbf_off, p->dbf_off);
        sc.offb = rnd_range(&g->rng, -p->dbf_off, p->dbf_off);
        sc.nref_active = g->nrefs < p->num_ref_frames ? g->nrefs : p->num_ref_frames;
        if (sc.nref_active < 1) sc.nref_active = 1;
        sc.tag = (uint16_t)s;
        gen_slice(g, idr, first, last, &sc);
        first = last + 1;
    }
    if (idr) g->idr_id = (g->idr_id + 1) & 0xFFFF;
    apply_marking(g, idr);
    g->nref = g->nrefs;
    /* frame_num: previous reference picture's + 1 (after MMCO 5 that
     * picture counts as frame_num 0) */
    if (g->cur_ref) {
        int mm5 = 0;
        for (int k = 0; k < g->nops; k++) mm5 |= g->op[k] == 5;
        g->frame_num = ((mm5 ? 0 : g->frame_num) + 1) & ((1 << p->log2_max_frame_num) - 1);
    }
    g->prev_ref = g->cur_ref;
}

int h264gen_generate(const GenParams *p, uint8_t **out, size_t *out_len)
{
    h264_tables_init();
    if (p->w_mbs < 1 || p->h_mbs < 1 || p->num_ref_frames < 1 || p->num_ref_frames > 16) return -1;
    Gen g;
    memset(&g, 0, sizeof(g));
    g.p = *p;
    if (g.p.log2_max_frame_num < 4) g.p.log2_max_frame_num = 4;
    g.rng.s = p->seed * 0x2545F4914F6CDD1Dull + 0x1234567ull;
    g.erng.s = p->seed * 0x9E3779B97F4A7C15ull + 0xE770Cull;
    g.mrng.s = p->seed * 0xD6E8FEB86659FD93ull + 0x3EF5ull;
    g.max_lt = -1;
    g.prev_ref = 1;
    g.range_mb = -1;
    g.pc.w = p->w_mbs; g.pc.h = p->h_mbs; g.pc.cip = p->cip;
    g.pc.mb = (MbInfo *)calloc((size_t)p->w_mbs * p->h_mbs, sizeof(MbInfo));
    g.pc.slice = (uint16_t *)calloc((size_t)p->w_mbs * p->h_mbs, sizeof(uint16_t));
    if (!g.pc.mb || !g.pc.slice) { free(g.pc.mb); free(g.pc.slice); return -1; }
    for (int i = 0; i < p->nframes; i++) gen_picture(&g, i);
    free(g.pc.mb);
    free(g.pc.slice);
    *out = g.out.buf;
    *out_len = g.out.len;
    return 0;
}

void h264gen_free(void *ptr) { free(ptr); }

/* CAVLC encode -> decode round trip over random blocks (test hook) */
int h264gen_cavlc_selftest(int iters, uint64_t seed)
{
    h264_tables_init();
    Rng r = {seed * 7919 + 17};
    int bad = 0;
    for (int it = 0; it < iters; it++) {
        static const int maxc[3] = {4, 15, 16};
        int mc = maxc[rnd(&r, 3)];
        int nc = mc == 4 ? -1 : rnd(&r, 17);
        int16_t in[16] = {0}, out[16];
        int k = rnd(&r, mc + 1);
        for (int i = 0; i < k; i++) {
            int pos = rnd(&r, mc);
            int mag = pct(&r, 70) ? 1 + rnd(&r, 3) : (pct(&r, 80) ? 1 + rnd(&r, 100) : 1 + rnd(&r, 2000));
            in[pos] = (int16_t)(pct(&r, 50) ? -mag : mag);
        }
        BitWriter bw;
        bw_init(&bw);
        int tc = cavlc_encode_block(&bw, nc, mc, in);
        if (tc < 0) { bw_free(&bw); continue; }
        bw_put(&bw, 1, 1);                 /* stop bit so more_rbsp_data is sane */
        while (!bw_aligned(&bw)) bw_put(&bw, 0, 1);
        BitReader br;
        br_init(&br, bw.buf, bw.nbytes);
        int tc2 = cavlc_decode_block(&br, nc, mc, out);
        if (tc2 != tc || memcmp(in, out, sizeof(int16_t) * (size_t)mc) || br.pos != bw.nbytes * 8 - 8 + (size_t)0 * 0) {
            /* position check: decoder must stop right before the stop bit */
            size_t stop = br.end_bits;
            if (tc2 != tc || memcmp(in, out, sizeof(int16_t) * (size_t)mc) || br.pos != stop) bad++;
        }
        bw_free(&bw);
    }
    return bad;
}
