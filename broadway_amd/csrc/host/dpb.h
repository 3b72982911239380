/* Decoded picture buffer bookkeeping (host side).  The frame data itself
 * lives in device memory slots; this module decides which slot holds which
 * picture, builds RefPicList0, applies sliding-window / MMCO marking and
 * produces the output (display) queue.  Behaviour follows the reference
 * h264bsd_dpb.c: h264bsdInitDpb :980-1045 (dpbSize / noReordering rule),
 * h264bsdMarkDecRefPic :628-833, Mmcop1-6 :330-627, SlidingWindow :902,
 * h264bsdCheckGapsInFrameNum :1226-1350, OutputPicture :1423,
 * h264bsdFlushDpb :1500, h264bsdReorderRefPicList :224-300. */
#ifndef H264MI_DPB_H
#define H264MI_DPB_H

#include "syntax.h"

#define DPB_MAX (MAX_REFS + 1)

enum { PIC_UNUSED = 0, PIC_NONEXIST = 1, PIC_SHORT = 2, PIC_LONG = 3 };

typedef struct DpbPic {
    int slot;
    int status;
    int frame_num;
    int pic_num;          /* FrameNumWrap (short-term) or LongTermFrameIdx */
    int poc;
    int to_display;
    int is_idr, pic_id, err_mbs;
} DpbPic;

typedef struct DpbOut { int slot, is_idr, pic_id, err_mbs; } DpbOut;

typedef struct Dpb {
    DpbPic pic[DPB_MAX];
    int    npic;            /* dpbSize + 1 entries */
    int    size;            /* dpbSize */
    int    max_ref, num_ref, fullness;
    int    max_frame_num;
    int    no_reorder;
    int    max_lt_idx;      /* -1: no long-term frame indices */
    int    prev_ref_frame_num;
    int    cur;             /* entry holding the picture being decoded */
    int    flushed;
    int    last_mmco5;
    DpbOut out[DPB_MAX + 1];
    int    num_out, out_index;
    int    list[MAX_REFS + 1];  /* RefPicList0 -> entry index, -1 if none */
} Dpb;

void dpb_init(Dpb *d, int dpb_size, int max_ref_frames, int max_frame_num, int no_reorder);
int  dpb_alloc_current(Dpb *d);               /* returns slot of current picture */
int  dpb_check_gaps(Dpb *d, int frame_num, int is_ref, int gaps_allowed);
/* RefPicList0 construction + modification; fills ref_slot[0..n-1] */
int  dpb_build_list(Dpb *d, const SliceHdr *sh, int *ref_slot);
/* mark the current picture (sh == NULL: non-reference) */
int  dpb_mark(Dpb *d, const SliceHdr *sh, int is_ref, int frame_num, int poc, int is_idr,
              int pic_id, int err_mbs);
void dpb_flush(Dpb *d);
const DpbOut *dpb_next_output(Dpb *d);

#endif
