/* High-level syntax of H.264 Baseline: NAL unit header, sequence / picture
 * parameter sets (incl. VUI) and slice header, parsed on the host.
 * Replaces reference h264bsd_nal_unit.c, h264bsd_seq_param_set.c,
 * h264bsd_pic_param_set.c, h264bsd_vui.c, h264bsd_slice_header.c with the
 * same validity rules where they affect behaviour (e.g. GetDpbSize,
 * seq_param_set.c:383-470; VUI dpb override, seq_param_set.c:331-347). */
#ifndef H264MI_SYNTAX_H
#define H264MI_SYNTAX_H

#include <stdint.h>
#include "../common/bits.h"

#define MAX_SPS 32
#define MAX_PPS 256
#define MAX_REFS 16

enum { NAL_SLICE = 1, NAL_IDR = 5, NAL_SEI = 6, NAL_SPS = 7, NAL_PPS = 8, NAL_AUD = 9,
       NAL_EOSEQ = 10, NAL_EOSTREAM = 11, NAL_FILLER = 12 };

typedef struct Sps {
    int valid;
    int profile_idc, level_idc, id;
    int log2_max_frame_num;            /* MaxFrameNum = 1 << this */
    int poc_type;
    int log2_max_poc_lsb;
    int delta_pic_order_always_zero;
    int offset_for_non_ref_pic, offset_for_top_to_bottom;
    int num_ref_frames_in_poc_cycle;
    int offset_for_ref_frame[256];
    int num_ref_frames;
    int gaps_allowed;
    int w_mbs, h_mbs;
    int frame_mbs_only;
    int crop, crop_l, crop_r, crop_t, crop_b;   /* in SPS units (2 px) */
    int vui_present;
    /* VUI items that affect behaviour / GetInfo */
    int video_full_range, matrix_coeffs, colour_desc_present;
    int aspect_present, aspect_idc, sar_w, sar_h;
    int bitstream_restriction, num_reorder_frames, max_dec_frame_buffering;
    int max_dpb;                       /* derived (GetDpbSize + VUI rule) */
} Sps;

typedef struct Pps {
    int valid;
    int id, sps_id;
    int entropy_coding;
    int bottom_field_poc_present;
    int num_slice_groups;
    int num_ref_idx_default;           /* num_ref_idx_l0_default_active_minus1 + 1 */
    int weighted_pred, weighted_bipred;
    int pic_init_qp;
    int chroma_qp_offset;
    int deblocking_ctrl;
    int cip;                           /* constrained_intra_pred_flag */
    int redundant_pic_cnt_present;
} Pps;

typedef struct RefMod { int idc; uint32_t val; } RefMod;
typedef struct Mmco { int op; uint32_t diff, lt_pic_num, lt_idx, max_lt_idx; } Mmco;

typedef struct SliceHdr {
    int nal_type, nal_ref_idc;
    int first_mb;
    int slice_type;                    /* 0 P, 2 I (mod 5) */
    int pps_id;
    int frame_num;
    int idr_pic_id;
    int poc_lsb, delta_poc_bottom;
    int delta_poc[2];
    int redundant_pic_cnt;
    int num_ref_idx_active;
    int ref_mod_flag;
    RefMod ref_mod[MAX_REFS + 2];
    int no_output_prior, long_term_ref;     /* IDR marking */
    int adaptive_marking;
    Mmco mmco[66];
    int nmmco;
    int slice_qp;                      /* SliceQPY */
    int dbf_idc, off_a_div2, off_b_div2;
} SliceHdr;

typedef struct NalHdr { int ref_idc, type; } NalHdr;

/* all return 0 on success, -1 on syntax error */
int parse_sps(BitReader *br, Sps *s);
int parse_pps(BitReader *br, const Sps *sps_table, Pps *p);
/* peek the PPS id of a slice header without consuming the reader */
int peek_slice_pps_id(const BitReader *br, int *pps_id);
int parse_slice_header(BitReader *br, const NalHdr *nal, const Sps *sps, const Pps *pps, SliceHdr *h);
int sps_equal(const Sps *a, const Sps *b);

#endif
