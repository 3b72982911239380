/* Seeded synthetic H.264 Baseline (CAVLC) stream generator.
 *
 * There is no encoder in the image and the reference's test media are
 * missing, so every test/bench stream comes from here.
 * The generator makes random *syntax* decisions (MB types, partitions,
 * intra modes valid for the neighbour availability, motion vectors,
 * residual levels, QP deltas, slices, deblocking parameters), derives the
 * predictions the decoder will make (mbctx.c) and writes a conforming
 * Annex-B byte stream.  It never reconstructs pixels; it only keeps the
 * inverse-transformed residual inside the range the reference accepts
 * (h264bsd_transform.c:181-225).
 */
#ifndef H264MI_GEN_H
#define H264MI_GEN_H

#include <stddef.h>
#include <stdint.h>

typedef struct GenParams {
    int w_mbs, h_mbs;
    int crop_right, crop_bottom;   /* luma pixels (even) */
    int nframes, gop;              /* IDR every `gop` frames */
    int slices;                    /* slices per picture */
    /* P-picture MB mix (percent): skip, 16x16, 16x8, 8x16, 8x8, intra */
    int pm_skip, pm_16x16, pm_16x8, pm_8x16, pm_8x8, pm_intra;
    int p8x8_ref0_pct;             /* share of P_8x8 written as P_8x8ref0 */
    /* intra MB mix (percent): I4x4, I16x16, I_PCM */
    int im_i4, im_i16, im_pcm;
    int i4_rem_pct;                /* share of I4x4 blocks coded with rem mode */
    int qp_min, qp_max, qp_delta;  /* slice QP range, |mb_qp_delta| max */
    int dbf_idc1_pct, dbf_idc2_pct, dbf_off;  /* idc mix, offsets in [-off,off] */
    int num_ref_frames;
    int cip;                       /* constrained_intra_pred_flag */
    int chroma_qp_offset;
    int poc_type;                  /* 0 or 2 */
    int coef_pct;                  /* probability (%) a cbp bit is set */
    int level_tail_pct;            /* probability (%) of a large level */
    int mv_jitter;                 /* per-MB motion spread, quarter-pel */
    int offpic_pct;                /* partitions forced to reference off-picture */
    int log2_max_frame_num;        /* 4..16 */
    int poc_swap;                  /* POC type 0: swap display order of picture pairs (1,2),(3,4).. of a GOP */
    /* damaged-stream knobs (error path / concealment); all 0
     * leaves the stream byte-identical.  Decisions come from a second RNG. */
    int err_range_pct;             /* per slice: one MB gets a residual outside [-512,511] */
    int drop_slice_pct;            /* per slice: NAL not emitted */
    int trunc_slice_pct;           /* per slice: NAL payload cut at a random byte */
    int drop_pic_pct;              /* per non-IDR picture: none of its NALs emitted */
    int gaps_allowed;              /* SPS gaps_in_frame_num_value_allowed_flag */
    /* reference-picture knobs (RefPicList0 modification, MMCO, long-term,
     * non-reference pictures; dpb.c / h264bsd_dpb.c paths).  All 0 leaves
     * the stream byte-identical; decisions come from a third RNG. */
    int nonref_pct;                /* per non-IDR picture: nal_ref_idc = 0 */
    int ref_mod_pct;               /* per P slice: ref_pic_list_modification commands */
    int mmco_pct;                  /* per non-IDR reference picture: adaptive marking (MMCO 1-4, 6; 5 with POC type 2) */
    int lt_idr_pct;                /* per IDR: long_term_reference_flag */
    uint64_t seed;
} GenParams;

#ifdef __cplusplus
extern "C" {
#endif

void h264gen_default_params(GenParams *p, int w_mbs, int h_mbs);
/* config presets of BASELINE.json configs[0..4] */
int  h264gen_preset(GenParams *p, int config, uint64_t seed);
/* generate a stream; *out is malloc'ed, caller frees with h264gen_free */
int  h264gen_generate(const GenParams *p, uint8_t **out, size_t *out_len);
/* CAVLC encode/decode round trip self-test; returns mismatches */
int  h264gen_cavlc_selftest(int iters, uint64_t seed);
void h264gen_free(void *ptr);

#ifdef __cplusplus
}
#endif

#endif
