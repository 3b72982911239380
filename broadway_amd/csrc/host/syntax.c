/* NAL / SPS / PPS / VUI / slice header parsing (see syntax.h) */
#include "syntax.h"

#include <string.h>

static int get_dpb_size(int pic_size_mbs, int level)
{
    /* MaxDpbMbs-equivalent byte budgets of Table A-1 (reference
     * GetDpbSize, seq_param_set.c:383-483, incl. its level-5 corrigendum) */
    long bytes; int max_mbs;
    switch (level) {
    case 10: bytes = 152064; max_mbs = 99; break;
    case 11: bytes = 345600; max_mbs = 396; break;
    case 12: case 13: case 20: bytes = 912384; max_mbs = 396; break;
    case 21: bytes = 1824768; max_mbs = 792; break;
    case 22: case 30: bytes = 3110400; max_mbs = 1620; break;
    case 31: bytes = 6912000; max_mbs = 3600; break;
    case 32: bytes = 7864320; max_mbs = 5120; break;
    case 40: case 41: bytes = 12582912; max_mbs = 8192; break;
    case 42: bytes = 34816L * 384; max_mbs = 8704; break;
    case 50: bytes = 42393600; max_mbs = 22080; break;
    case 51: bytes = 70778880; max_mbs = 36864; break;
    default: return -1;
    }
    if (pic_size_mbs > max_mbs) return -1;
    long n = bytes / ((long)pic_size_mbs * 384);
    return (int)(n < 16 ? n : 16);
}

static int parse_hrd(BitReader *br)
{
    uint32_t cnt = br_ue(br);
    if (cnt > 31) return -1;
    br_u(br, 4); br_u(br, 4);
    for (uint32_t i = 0; i <= cnt; i++) { br_ue(br); br_ue(br); br_u1(br); }
    br_u(br, 5); br_u(br, 5); br_u(br, 5); br_u(br, 5);
    return br->err ? -1 : 0;
}

static int parse_vui(BitReader *br, Sps *s)
{
    s->aspect_present = br_u1(br);
    if (s->aspect_present) {
        s->aspect_idc = (int)br_u(br, 8);
        if (s->aspect_idc == 255) { s->sar_w = (int)br_u(br, 16); s->sar_h = (int)br_u(br, 16); }
    }
    if (br_u1(br)) br_u1(br);                         /* overscan */
    if (br_u1(br)) {                                  /* video_signal_type */
        br_u(br, 3);
        s->video_full_range = (int)br_u1(br);
        s->colour_desc_present = (int)br_u1(br);
        if (s->colour_desc_present) {
            br_u(br, 8); br_u(br, 8);
            s->matrix_coeffs = (int)br_u(br, 8);
        }
    }
    if (br_u1(br)) { br_ue(br); br_ue(br); }          /* chroma_loc_info */
    if (br_u1(br)) { br_u(br, 32); br_u(br, 32); br_u1(br); }   /* timing */
    int nal_hrd = (int)br_u1(br);
    if (nal_hrd && parse_hrd(br)) return -1;
    int vcl_hrd = (int)br_u1(br);
    if (vcl_hrd && parse_hrd(br)) return -1;
    if (nal_hrd || vcl_hrd) br_u1(br);
    br_u1(br);                                         /* pic_struct_present */
    s->bitstream_restriction = (int)br_u1(br);
    if (s->bitstream_restriction) {
        br_u1(br); br_ue(br); br_ue(br); br_ue(br); br_ue(br);
        s->num_reorder_frames = (int)br_ue(br);
        s->max_dec_frame_buffering = (int)br_ue(br);
    } else {
        s->num_reorder_frames = 16;
        s->max_dec_frame_buffering = 16;
    }
    return br->err ? -1 : 0;
}

int parse_sps(BitReader *br, Sps *s)
{
    memset(s, 0, sizeof(*s));
    s->matrix_coeffs = 2;
    s->profile_idc = (int)br_u(br, 8);
    br_u(br, 8);                                       /* constraint flags */
    s->level_idc = (int)br_u(br, 8);
    uint32_t id = br_ue(br);
    if (id >= MAX_SPS) return -1;
    s->id = (int)id;
    uint32_t l2 = br_ue(br);
    if (l2 > 12) return -1;
    s->log2_max_frame_num = (int)l2 + 4;
    uint32_t pt = br_ue(br);
    if (pt > 2) return -1;
    s->poc_type = (int)pt;
    if (pt == 0) {
        uint32_t l = br_ue(br);
        if (l > 12) return -1;
        s->log2_max_poc_lsb = (int)l + 4;
    } else if (pt == 1) {
        s->delta_pic_order_always_zero = (int)br_u1(br);
        s->offset_for_non_ref_pic = br_se(br);
        s->offset_for_top_to_bottom = br_se(br);
        uint32_t n = br_ue(br);
        if (n > 255) return -1;
        s->num_ref_frames_in_poc_cycle = (int)n;
        for (uint32_t i = 0; i < n; i++) s->offset_for_ref_frame[i] = br_se(br);
    }
    uint32_t nref = br_ue(br);
    if (nref > MAX_REFS) return -1;
    s->num_ref_frames = (int)nref;
    s->gaps_allowed = (int)br_u1(br);
    s->w_mbs = (int)br_ue(br) + 1;
    s->h_mbs = (int)br_ue(br) + 1;
    s->frame_mbs_only = (int)br_u1(br);
    if (!s->frame_mbs_only) return -1;                 /* interlace not in Baseline */
    br_u1(br);                                         /* direct_8x8_inference */
    s->crop = (int)br_u1(br);
    if (s->crop) {
        s->crop_l = (int)br_ue(br); s->crop_r = (int)br_ue(br);
        s->crop_t = (int)br_ue(br); s->crop_b = (int)br_ue(br);
        if (s->crop_l > 8 * s->w_mbs - (s->crop_r + 1) || s->crop_t > 8 * s->h_mbs - (s->crop_b + 1))
            return -1;
    }
    if (s->w_mbs > 1024 || s->h_mbs > 1024) return -1;
    int dpb = get_dpb_size(s->w_mbs * s->h_mbs, s->level_idc);
    if (dpb < 0 || s->num_ref_frames > dpb) dpb = s->num_ref_frames;
    s->max_dpb = dpb;
    s->vui_present = (int)br_u1(br);
    if (s->vui_present) {
        if (parse_vui(br, s)) return -1;
        if (s->bitstream_restriction) {
            /* reference seq_param_set.c:331-347 */
            if (s->num_reorder_frames > s->max_dec_frame_buffering ||
                s->max_dec_frame_buffering < s->num_ref_frames ||
                s->max_dec_frame_buffering > s->max_dpb)
                return -1;
            s->max_dpb = s->max_dec_frame_buffering > 1 ? s->max_dec_frame_buffering : 1;
        }
    }
    if (br->err) return -1;
    s->valid = 1;
    return 0;
}

int sps_equal(const Sps *a, const Sps *b)
{
    return a->profile_idc == b->profile_idc && a->level_idc == b->level_idc &&
           a->log2_max_frame_num == b->log2_max_frame_num && a->poc_type == b->poc_type &&
           a->log2_max_poc_lsb == b->log2_max_poc_lsb &&
           a->delta_pic_order_always_zero == b->delta_pic_order_always_zero &&
           a->offset_for_non_ref_pic == b->offset_for_non_ref_pic &&
           a->offset_for_top_to_bottom == b->offset_for_top_to_bottom &&
           a->num_ref_frames_in_poc_cycle == b->num_ref_frames_in_poc_cycle &&
           !memcmp(a->offset_for_ref_frame, b->offset_for_ref_frame,
                   sizeof(int) * (size_t)a->num_ref_frames_in_poc_cycle) &&
           a->num_ref_frames == b->num_ref_frames && a->gaps_allowed == b->gaps_allowed &&
           a->w_mbs == b->w_mbs && a->h_mbs == b->h_mbs && a->crop == b->crop &&
           a->crop_l == b->crop_l && a->crop_r == b->crop_r && a->crop_t == b->crop_t &&
           a->crop_b == b->crop_b && a->vui_present == b->vui_present &&
           a->max_dpb == b->max_dpb && a->num_reorder_frames == b->num_reorder_frames &&
           a->bitstream_restriction == b->bitstream_restriction;
}

int parse_pps(BitReader *br, const Sps *sps_table, Pps *p)
{
    memset(p, 0, sizeof(*p));
    uint32_t id = br_ue(br);
    if (id >= MAX_PPS) return -1;
    p->id = (int)id;
    uint32_t sid = br_ue(br);
    if (sid >= MAX_SPS) return -1;
    p->sps_id = (int)sid;
    p->entropy_coding = (int)br_u1(br);
    p->bottom_field_poc_present = (int)br_u1(br);
    p->num_slice_groups = (int)br_ue(br) + 1;
    if (p->num_slice_groups != 1) return -1;           /* FMO: not supported */
    uint32_t n0 = br_ue(br);
    if (n0 > 31) return -1;
    p->num_ref_idx_default = (int)n0 + 1;
    uint32_t n1 = br_ue(br);
    if (n1 > 31) return -1;
    p->weighted_pred = (int)br_u1(br);
    p->weighted_bipred = (int)br_u(br, 2);
    int qp = br_se(br);
    if (qp < -26 || qp > 25) return -1;
    p->pic_init_qp = 26 + qp;
    int qs = br_se(br);
    if (qs < -26 || qs > 25) return -1;
    int off = br_se(br);
    if (off < -12 || off > 12) return -1;
    p->chroma_qp_offset = off;
    p->deblocking_ctrl = (int)br_u1(br);
    p->cip = (int)br_u1(br);
    p->redundant_pic_cnt_present = (int)br_u1(br);
    (void)sps_table;
    if (br->err) return -1;
    p->valid = 1;
    return 0;
}

int peek_slice_pps_id(const BitReader *br0, int *pps_id)
{
    BitReader br = *br0;
    br_ue(&br); br_ue(&br);
    uint32_t id = br_ue(&br);
    if (br.err || id >= MAX_PPS) return -1;
    *pps_id = (int)id;
    return 0;
}

int parse_slice_header(BitReader *br, const NalHdr *nal, const Sps *sps, const Pps *pps, SliceHdr *h)
{
    memset(h, 0, sizeof(*h));
    h->nal_type = nal->type;
    h->nal_ref_idc = nal->ref_idc;
    int idr = nal->type == NAL_IDR;
    uint32_t first = br_ue(br);
    if (first >= (uint32_t)(sps->w_mbs * sps->h_mbs)) return -1;
    h->first_mb = (int)first;
    uint32_t st = br_ue(br);
    if (st > 9) return -1;
    st %= 5;
    if (st != 0 && st != 2) return -1;                 /* P and I only (Baseline) */
    if (idr && st != 2) return -1;
    h->slice_type = (int)st;
    h->pps_id = (int)br_ue(br);
    h->frame_num = (int)br_u(br, sps->log2_max_frame_num);
    if (idr && h->frame_num != 0) return -1;
    if (idr) {
        uint32_t v = br_ue(br);
        if (v > 65535) return -1;
        h->idr_pic_id = (int)v;
    }
    if (sps->poc_type == 0) {
        h->poc_lsb = (int)br_u(br, sps->log2_max_poc_lsb);
        if (pps->bottom_field_poc_present) h->delta_poc_bottom = br_se(br);
    } else if (sps->poc_type == 1 && !sps->delta_pic_order_always_zero) {
        h->delta_poc[0] = br_se(br);
        if (pps->bottom_field_poc_present) h->delta_poc[1] = br_se(br);
    }
    if (pps->redundant_pic_cnt_present) h->redundant_pic_cnt = (int)br_ue(br);
    h->num_ref_idx_active = pps->num_ref_idx_default;
    if (st == 0) {
        if (br_u1(br)) {
            uint32_t n = br_ue(br);
            if (n > 15) return -1;
            h->num_ref_idx_active = (int)n + 1;
        }
        if (h->num_ref_idx_active > MAX_REFS) return -1;
        h->ref_mod_flag = (int)br_u1(br);
        if (h->ref_mod_flag) {
            int i = 0;
            for (;;) {
                uint32_t idc = br_ue(br);
                if (idc > 3 || i > h->num_ref_idx_active) return -1;
                h->ref_mod[i].idc = (int)idc;
                if (idc == 3) break;
                h->ref_mod[i].val = br_ue(br);
                if (br->err) return -1;
                /* abs_diff_pic_num_minus1 < MaxPicNum (slice_header.c:RefPicListReordering) */
                if (idc < 2 && h->ref_mod[i].val >= (uint32_t)(1u << sps->log2_max_frame_num)) return -1;
                i++;
            }
            if (i == 0) return -1;
        }
    }
    if (nal->ref_idc) {
        /* dec_ref_pic_marking() with the reference's checks (slice_header.c
         * DecRefPicMarking): long-term IDR needs reference frames, at most
         * 2 * num_ref_frames + 3 operations, max_long_term_frame_idx_plus1
         * <= num_ref_frames, one each of MMCO 4, 5, 6, no MMCO 5 with 1-3 */
        if (idr) {
            h->no_output_prior = (int)br_u1(br);
            h->long_term_ref = (int)br_u1(br);
            if (!sps->num_ref_frames && h->long_term_ref) return -1;
        } else {
            h->adaptive_marking = (int)br_u1(br);
            if (h->adaptive_marking) {
                int i = 0, n4 = 0, n5 = 0, n6 = 0, n13 = 0;
                for (;;) {
                    if (i > 2 * sps->num_ref_frames + 2 || i >= 65) return -1;
                    uint32_t op = br_ue(br);
                    if (br->err || op > 6) return -1;
                    h->mmco[i].op = (int)op;
                    if (op == 0) break;
                    if (op == 1 || op == 3) h->mmco[i].diff = br_ue(br) + 1;
                    if (op == 2) h->mmco[i].lt_pic_num = br_ue(br);
                    if (op == 3 || op == 6) h->mmco[i].lt_idx = br_ue(br);
                    if (op == 4) {
                        h->mmco[i].max_lt_idx = br_ue(br);
                        if (h->mmco[i].max_lt_idx > (uint32_t)sps->num_ref_frames) return -1;
                        n4++;
                    }
                    if (br->err) return -1;
                    n5 += op == 5;
                    n6 += op == 6;
                    n13 += op <= 3;
                    i++;
                }
                h->nmmco = i;
                if (n4 > 1 || n5 > 1 || n6 > 1 || (n13 && n5)) return -1;
            }
        }
    }
    int dqp = br_se(br);
    h->slice_qp = pps->pic_init_qp + dqp;
    if (h->slice_qp < 0 || h->slice_qp > 51) return -1;
    if (pps->deblocking_ctrl) {
        uint32_t idc = br_ue(br);
        if (idc > 2) return -1;
        h->dbf_idc = (int)idc;
        if (idc != 1) {
            h->off_a_div2 = br_se(br);
            h->off_b_div2 = br_se(br);
            if (h->off_a_div2 < -6 || h->off_a_div2 > 6 || h->off_b_div2 < -6 || h->off_b_div2 > 6)
                return -1;
        }
    }
    return br->err ? -1 : 0;
}
