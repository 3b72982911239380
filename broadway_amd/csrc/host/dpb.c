/* Host DPB bookkeeping -- see dpb.h.
 *
 * The entries are kept the way the reference keeps its dpbPicture_t buffer:
 * an array of dpbSize + 1 positions re-sorted after every marking (and per
 * inserted non-existing frame) by the same diminishing-increment sort and
 * ordering -- short-term references by descending PicNum, long-term by
 * ascending LongTermPicNum, then pictures waiting for display, then the rest
 * (ShellSort / ComparePictures, h264bsd_dpb.c:138-196, 1612-1640).  The
 * current picture always takes the last position (h264bsdAllocateDpbImage,
 * :877-893), RefPicList0 starts as the first numRefFrames positions
 * (h264bsdInitRefPicList, :1104-1116), and every scan runs over the same
 * range as the reference's.  Each position carries the device frame slot its
 * samples live in, moving with the entry as the reference's data pointer
 * does, so slot reuse -- what an unwritten or partly written picture shows --
 * is the reference's buffer reuse. */
#include "dpb.h"

#include <string.h>

#define IS_REF(p) ((p)->status != PIC_UNUSED)
#define IS_SHORT(p) ((p)->status == PIC_SHORT || (p)->status == PIC_NONEXIST)
#define IS_LONG(p) ((p)->status == PIC_LONG)
#define IS_EXISTING(p) ((p)->status > PIC_NONEXIST)

void dpb_init(Dpb *d, int dpb_size, int max_ref_frames, int max_frame_num, int no_reorder)
{
    memset(d, 0, sizeof(*d));
    d->max_ref = max_ref_frames > 1 ? max_ref_frames : 1;
    d->size = no_reorder ? d->max_ref : dpb_size;
    if (d->size > MAX_REFS) d->size = MAX_REFS;
    if (d->size < 1) d->size = 1;
    d->npic = d->size + 1;
    for (int i = 0; i < d->npic; i++) d->pic[i].slot = i;
    d->max_frame_num = max_frame_num;
    d->no_reorder = no_reorder;
    d->max_lt_idx = -1;
    d->cur = -1;
    for (int i = 0; i <= MAX_REFS; i++) d->list[i] = -1;
}

/* ComparePictures (:138-196): < 0 if a sorts before b */
static int compare(const DpbPic *a, const DpbPic *b)
{
    if (!IS_REF(a) && !IS_REF(b)) return (a->to_display && !b->to_display) ? -1 : (!a->to_display && b->to_display) ? 1 : 0;
    if (!IS_REF(b)) return -1;
    if (!IS_REF(a)) return 1;
    if (IS_SHORT(a) && IS_SHORT(b)) return a->pic_num > b->pic_num ? -1 : a->pic_num < b->pic_num ? 1 : 0;
    if (IS_SHORT(a)) return -1;
    if (IS_SHORT(b)) return 1;
    return a->pic_num > b->pic_num ? 1 : a->pic_num < b->pic_num ? -1 : 0;
}

/* ShellSort (:1612-1640): increments 7, 3, 1 -- not stable, so equal
 * entries end where the reference's do only with the same increments */
static void sort_entries(Dpb *d)
{
    for (int step = 7; step; step >>= 1)
        for (int i = step; i < d->npic; i++) {
            const DpbPic t = d->pic[i];
            int j = i;
            while (j >= step && compare(&d->pic[j - step], &t) > 0) {
                d->pic[j] = d->pic[j - step];
                j -= step;
            }
            d->pic[j] = t;
        }
}

int dpb_alloc_current(Dpb *d)
{
    d->cur = d->size;
    return d->pic[d->cur].slot;
}

/* SetPicNums (:1189-1210) */
static void set_pic_nums(Dpb *d, int curr_frame_num)
{
    for (int i = 0; i < d->num_ref; i++) {
        DpbPic *p = &d->pic[i];
        if (IS_SHORT(p))
            p->pic_num = p->frame_num > curr_frame_num ? p->frame_num - d->max_frame_num : p->frame_num;
    }
}

static void unmark(Dpb *d, DpbPic *p)
{
    p->status = PIC_UNUSED;
    d->num_ref--;
    if (!p->to_display) d->fullness--;
}

/* OutputPicture + FindSmallestPicOrderCnt (:1398-1460): the first position
 * with the smallest POC */
static int output_picture(Dpb *d)
{
    if (d->no_reorder) return -1;
    int best = -1;
    for (int i = 0; i < d->npic; i++)
        if (d->pic[i].to_display && (best < 0 || d->pic[i].poc < d->pic[best].poc)) best = i;
    if (best < 0) return -1;
    DpbPic *p = &d->pic[best];
    if (d->num_out <= DPB_MAX) {
        DpbOut *o = &d->out[d->num_out++];
        o->slot = p->slot; o->is_idr = p->is_idr; o->pic_id = p->pic_id; o->err_mbs = p->err_mbs;
    }
    p->to_display = 0;
    if (!IS_REF(p)) d->fullness--;
    return 0;
}

/* SlidingWindowRefPicMarking (:905-940): oldest short-term among the first
 * numRefFrames positions */
static int sliding_window(Dpb *d)
{
    if (d->num_ref < d->max_ref) return 0;
    int best = -1;
    for (int i = 0; i < d->num_ref; i++)
        if (IS_SHORT(&d->pic[i]) && (best < 0 || d->pic[i].pic_num < d->pic[best].pic_num)) best = i;
    if (best < 0) return -1;
    unmark(d, &d->pic[best]);
    return 0;
}

/* FindDpbPic (:1132-1170): the first maxRefFrames positions */
static int find_pic(Dpb *d, int pic_num, int short_term)
{
    for (int i = 0; i < d->max_ref && i < d->npic; i++) {
        DpbPic *p = &d->pic[i];
        if ((short_term ? IS_SHORT(p) : IS_LONG(p)) && p->pic_num == pic_num) return i;
    }
    return -1;
}

/* h264bsdCheckGapsInFrameNum (:1245-1350) */
int dpb_check_gaps(Dpb *d, int frame_num, int is_ref, int gaps_allowed)
{
    d->num_out = 0;
    d->out_index = 0;
    if (!gaps_allowed) return 0;
    if (frame_num != d->prev_ref_frame_num &&
        frame_num != (d->prev_ref_frame_num + 1) % d->max_frame_num) {
        int fn = (d->prev_ref_frame_num + 1) % d->max_frame_num;
        /* the last position's slot is what the current picture would get;
         * it must not be a slot placed in the output queue below */
        const int keep = d->pic[d->size].slot;
        do {
            set_pic_nums(d, fn);
            if (sliding_window(d)) return -1;
            while (d->fullness >= d->size) if (output_picture(d)) break;
            DpbPic *p = &d->pic[d->size];
            p->status = PIC_NONEXIST;
            p->frame_num = fn;
            p->pic_num = fn;
            p->poc = 0;
            p->to_display = 0;
            d->fullness++;
            d->num_ref++;
            sort_entries(d);
            fn = (fn + 1) % d->max_frame_num;
        } while (fn != frame_num);
        for (int i = 0; i < d->num_out; i++)
            if (d->out[i].slot == d->pic[d->size].slot) {
                for (int k = 0; k < d->size; k++)
                    if (d->pic[k].slot == keep) {
                        d->pic[k].slot = d->pic[d->size].slot;
                        d->pic[d->size].slot = keep;
                        break;
                    }
                break;
            }
    } else if (is_ref && frame_num == d->prev_ref_frame_num) {
        return -1;
    }
    if (is_ref) d->prev_ref_frame_num = frame_num;
    else if (frame_num != d->prev_ref_frame_num)
        d->prev_ref_frame_num = (frame_num + d->max_frame_num - 1) % d->max_frame_num;
    return 0;
}

/* h264bsdInitRefPicList (:1104-1116) + h264bsdReorderRefPicList (:224-300) */
int dpb_build_list(Dpb *d, const SliceHdr *sh, int *ref_slot)
{
    for (int i = 0; i < d->num_ref; i++) d->list[i] = i;
    set_pic_nums(d, sh->frame_num);
    if (sh->slice_type == 0 && sh->ref_mod_flag) {
        const int nact = sh->num_ref_idx_active;
        int pred = sh->frame_num, ref_idx = 0;
        for (int k = 0; sh->ref_mod[k].idc != 3; k++) {
            int pn, st;
            if (sh->ref_mod[k].idc < 2) {
                int nw;
                const int diff = (int)sh->ref_mod[k].val + 1;
                if (sh->ref_mod[k].idc == 0) { nw = pred - diff; if (nw < 0) nw += d->max_frame_num; }
                else { nw = pred + diff; if (nw >= d->max_frame_num) nw -= d->max_frame_num; }
                pred = nw;
                pn = nw > sh->frame_num ? nw - d->max_frame_num : nw;
                st = 1;
            } else {
                pn = (int)sh->ref_mod[k].val;
                st = 0;
            }
            const int e = find_pic(d, pn, st);
            if (e < 0 || !IS_EXISTING(&d->pic[e])) return -1;
            for (int j = nact; j > ref_idx; j--) d->list[j] = d->list[j - 1];
            d->list[ref_idx++] = e;
            int w = ref_idx;
            for (int j = ref_idx; j <= nact; j++) if (d->list[j] != e) d->list[w++] = d->list[j];
        }
    }
    /* h264bsdGetRefPicData (:846-860) */
    for (int i = 0; i < MAX_REFS; i++) {
        const int e = i < sh->num_ref_idx_active ? d->list[i] : -1;
        ref_slot[i] = (e >= 0 && IS_EXISTING(&d->pic[e])) ? d->pic[e].slot : -1;
    }
    return 0;
}

/* Mmcop5 (:520-545): every reference unused, everything displayable queued */
static void mmco5(Dpb *d)
{
    for (int i = 0; i < d->npic; i++) {
        DpbPic *p = &d->pic[i];
        if (IS_REF(p)) {
            p->status = PIC_UNUSED;
            if (!p->to_display) d->fullness--;
        }
    }
    while (output_picture(d) == 0) {}
    d->num_ref = 0;
    d->max_lt_idx = -1;
    d->prev_ref_frame_num = 0;
}

/* a long-term picture holding LongTermFrameIdx idx among the first
 * maxRefFrames positions becomes unused (Mmcop3 / Mmcop6 :424-432, 582-590) */
static void free_lt_idx(Dpb *d, int idx)
{
    for (int i = 0; i < d->max_ref && i < d->npic; i++)
        if (IS_LONG(&d->pic[i]) && d->pic[i].pic_num == idx) {
            unmark(d, &d->pic[i]);
            break;
        }
}

/* h264bsdMarkDecRefPic (:650-833) */
int dpb_mark(Dpb *d, const SliceHdr *sh, int is_ref, int frame_num, int poc, int is_idr,
             int pic_id, int err_mbs)
{
    DpbPic *c = &d->pic[d->cur];
    int status = 0;
    const int to_disp = !d->no_reorder;
    d->last_mmco5 = 0;
    if (!is_ref) {
        c->status = PIC_UNUSED;
        c->frame_num = frame_num;
        c->pic_num = frame_num;
        c->poc = poc;
        c->to_display = to_disp;
        if (!d->no_reorder) d->fullness++;
    } else if (is_idr) {
        d->num_out = d->out_index = 0;
        mmco5(d);
        if (sh->no_output_prior || d->no_reorder) d->num_out = d->out_index = 0;
        if (sh->long_term_ref) { c->status = PIC_LONG; d->max_lt_idx = 0; }
        else { c->status = PIC_SHORT; d->max_lt_idx = -1; }
        c->frame_num = 0;
        c->pic_num = 0;
        c->poc = 0;
        c->to_display = to_disp;
        d->fullness = 1;
        d->num_ref = 1;
    } else {
        int marked_long = 0;
        if (sh->adaptive_marking) {
            for (int k = 0; k < sh->nmmco && status == 0; k++) {
                const Mmco *m = &sh->mmco[k];
                int e;
                switch (m->op) {
                case 1:
                    e = find_pic(d, frame_num - (int)m->diff, 1);
                    if (e < 0) { status = -1; break; }
                    unmark(d, &d->pic[e]);
                    break;
                case 2:
                    e = find_pic(d, (int)m->lt_pic_num, 0);
                    if (e < 0) { status = -1; break; }
                    unmark(d, &d->pic[e]);
                    break;
                case 3:
                    if (d->max_lt_idx < 0 || (int)m->lt_idx > d->max_lt_idx) { status = -1; break; }
                    free_lt_idx(d, (int)m->lt_idx);
                    e = find_pic(d, frame_num - (int)m->diff, 1);
                    if (e < 0 || !IS_EXISTING(&d->pic[e])) { status = -1; break; }
                    d->pic[e].status = PIC_LONG;
                    d->pic[e].pic_num = (int)m->lt_idx;
                    break;
                case 4:
                    d->max_lt_idx = (int)m->max_lt_idx - 1;
                    for (int i = 0; i < d->max_ref && i < d->npic; i++)
                        if (IS_LONG(&d->pic[i]) && (d->max_lt_idx < 0 || d->pic[i].pic_num > d->max_lt_idx))
                            unmark(d, &d->pic[i]);
                    break;
                case 5:
                    mmco5(d);
                    d->last_mmco5 = 1;
                    frame_num = 0;
                    break;
                case 6:
                    if (d->max_lt_idx < 0 || (int)m->lt_idx > d->max_lt_idx) { status = -1; break; }
                    free_lt_idx(d, (int)m->lt_idx);
                    if (d->num_ref < d->max_ref) {
                        c->frame_num = frame_num;
                        c->pic_num = (int)m->lt_idx;
                        c->poc = poc;
                        c->status = PIC_LONG;
                        c->to_display = to_disp;
                        d->num_ref++;
                        d->fullness++;
                        marked_long = 1;
                    } else status = -1;
                    break;
                default:
                    status = -1;
                }
            }
        } else {
            status = sliding_window(d);
        }
        if (!marked_long) {
            if (d->num_ref < d->max_ref) {
                c->frame_num = frame_num;
                c->pic_num = frame_num;
                c->poc = poc;
                c->status = PIC_SHORT;
                c->to_display = to_disp;
                d->fullness++;
                d->num_ref++;
            } else {
                status = -1;
            }
        }
    }
    c->is_idr = is_idr;
    c->pic_id = pic_id;
    c->err_mbs = err_mbs;
    if (d->no_reorder) {
        if (d->num_out <= DPB_MAX) {
            DpbOut *o = &d->out[d->num_out++];
            o->slot = c->slot; o->is_idr = is_idr; o->pic_id = pic_id; o->err_mbs = err_mbs;
        }
    } else {
        while (d->fullness > d->size) if (output_picture(d)) break;
    }
    sort_entries(d);
    return status;
}

void dpb_flush(Dpb *d)
{
    d->flushed = 1;
    while (output_picture(d) == 0) {}
}

const DpbOut *dpb_next_output(Dpb *d)
{
    if (d->out_index < d->num_out) return &d->out[d->out_index++];
    return NULL;
}
