/* Host DPB bookkeeping -- see dpb.h for the reference behaviour it keeps. */
#include "dpb.h"

#include <string.h>

#define IS_REF(p) ((p)->status != PIC_UNUSED)
#define IS_SHORT(p) ((p)->status == PIC_SHORT || (p)->status == PIC_NONEXIST)
#define IS_LONG(p) ((p)->status == PIC_LONG)

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

static int slot_pending_output(const Dpb *d, int slot)
{
    for (int i = d->out_index; i < d->num_out; i++) if (d->out[i].slot == slot) return 1;
    return 0;
}

static int find_free(const Dpb *d)
{
    int fallback = -1;
    for (int i = 0; i < d->npic; i++) {
        const DpbPic *p = &d->pic[i];
        if (IS_REF(p) || p->to_display || i == d->cur) continue;
        if (!slot_pending_output(d, p->slot)) return i;
        if (fallback < 0) fallback = i;
    }
    if (fallback < 0)      /* the current entry may be reused */
        for (int i = 0; i < d->npic; i++)
            if (!IS_REF(&d->pic[i]) && !d->pic[i].to_display) return i;
    return fallback;
}

int dpb_alloc_current(Dpb *d)
{
    int saved = d->cur;
    d->cur = -1;
    int i = find_free(d);
    if (i < 0) { d->cur = saved; return -1; }
    d->cur = i;
    return d->pic[i].slot;
}

static void set_pic_nums(Dpb *d, int curr_frame_num)
{
    for (int i = 0; i < d->npic; i++) {
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

static int sliding_window(Dpb *d)
{
    if (d->num_ref < d->max_ref) return 0;
    int best = -1;
    for (int i = 0; i < d->npic; i++)
        if (IS_SHORT(&d->pic[i]) && (best < 0 || d->pic[i].pic_num < d->pic[best].pic_num)) best = i;
    if (best < 0) return -1;
    unmark(d, &d->pic[best]);
    return 0;
}

static int find_pic(Dpb *d, int pic_num, int short_term)
{
    for (int i = 0; i < d->npic; i++) {
        DpbPic *p = &d->pic[i];
        if (short_term ? IS_SHORT(p) : IS_LONG(p))
            if (p->pic_num == pic_num) return i;
    }
    return -1;
}

int dpb_check_gaps(Dpb *d, int frame_num, int is_ref, int gaps_allowed)
{
    d->num_out = 0;
    d->out_index = 0;
    if (!gaps_allowed) return 0;
    if (frame_num != d->prev_ref_frame_num &&
        frame_num != (d->prev_ref_frame_num + 1) % d->max_frame_num) {
        int fn = (d->prev_ref_frame_num + 1) % d->max_frame_num;
        do {
            set_pic_nums(d, fn);
            if (sliding_window(d)) return -1;
            while (d->fullness >= d->size) if (output_picture(d)) break;
            int saved = d->cur;
            d->cur = -1;
            int e = find_free(d);
            d->cur = saved;
            if (e < 0) return -1;
            DpbPic *p = &d->pic[e];
            p->status = PIC_NONEXIST;
            p->frame_num = fn;
            p->pic_num = fn;
            p->poc = 0;
            p->to_display = 0;
            d->fullness++;
            d->num_ref++;
            fn = (fn + 1) % d->max_frame_num;
        } while (fn != frame_num);
    } else if (is_ref && frame_num == d->prev_ref_frame_num) {
        return -1;
    }
    if (is_ref) d->prev_ref_frame_num = frame_num;
    else if (frame_num != d->prev_ref_frame_num)
        d->prev_ref_frame_num = (frame_num + d->max_frame_num - 1) % d->max_frame_num;
    return 0;
}

int dpb_build_list(Dpb *d, const SliceHdr *sh, int *ref_slot)
{
    int n = 0;
    set_pic_nums(d, sh->frame_num);
    /* short-term by descending PicNum, then long-term by ascending LongTermPicNum */
    int idx[DPB_MAX];
    for (int i = 0; i < d->npic; i++) if (IS_SHORT(&d->pic[i])) idx[n++] = i;
    for (int a = 1; a < n; a++)
        for (int b = a; b > 0 && d->pic[idx[b]].pic_num > d->pic[idx[b - 1]].pic_num; b--) {
            int t = idx[b]; idx[b] = idx[b - 1]; idx[b - 1] = t;
        }
    int ns = n;
    for (int i = 0; i < d->npic; i++) if (IS_LONG(&d->pic[i])) idx[n++] = i;
    for (int a = ns + 1; a < n; a++)
        for (int b = a; b > ns && d->pic[idx[b]].pic_num < d->pic[idx[b - 1]].pic_num; b--) {
            int t = idx[b]; idx[b] = idx[b - 1]; idx[b - 1] = t;
        }
    for (int i = 0; i <= MAX_REFS; i++) d->list[i] = i < n ? idx[i] : -1;

    if (sh->slice_type == 0 && sh->ref_mod_flag) {
        int nact = sh->num_ref_idx_active;
        int pred = sh->frame_num, ref_idx = 0;
        for (int k = 0; sh->ref_mod[k].idc != 3; k++) {
            int pn, st;
            if (sh->ref_mod[k].idc < 2) {
                int nw;
                int diff = (int)sh->ref_mod[k].val + 1;
                if (sh->ref_mod[k].idc == 0) { nw = pred - diff; if (nw < 0) nw += d->max_frame_num; }
                else { nw = pred + diff; if (nw >= d->max_frame_num) nw -= d->max_frame_num; }
                pred = nw;
                pn = nw > sh->frame_num ? nw - d->max_frame_num : nw;
                st = 1;
            } else {
                pn = (int)sh->ref_mod[k].val;
                st = 0;
            }
            int e = find_pic(d, pn, st);
            if (e < 0 || d->pic[e].status == PIC_NONEXIST) return -1;
            for (int j = nact; j > ref_idx; j--) d->list[j] = d->list[j - 1];
            d->list[ref_idx++] = e;
            int w = ref_idx;
            for (int j = ref_idx; j <= nact; j++) if (d->list[j] != e) d->list[w++] = d->list[j];
            for (; w <= nact; w++) d->list[w] = -1;
        }
    }
    for (int i = 0; i < MAX_REFS; i++) {
        int e = i < sh->num_ref_idx_active ? d->list[i] : -1;
        ref_slot[i] = (e >= 0 && d->pic[e].status > PIC_NONEXIST) ? d->pic[e].slot : -1;
    }
    return 0;
}

static void mmco5(Dpb *d)
{
    for (int i = 0; i < d->npic; i++) {
        DpbPic *p = &d->pic[i];
        if (i == d->cur) continue;
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

int dpb_mark(Dpb *d, const SliceHdr *sh, int is_ref, int frame_num, int poc, int is_idr,
             int pic_id, int err_mbs)
{
    DpbPic *c = &d->pic[d->cur];
    int status = 0;
    int to_disp = !d->no_reorder;
    d->last_mmco5 = 0;
    set_pic_nums(d, frame_num);
    if (!is_ref) {
        c->status = PIC_UNUSED;
        c->frame_num = frame_num;
        c->pic_num = frame_num;
        c->poc = poc;
        c->to_display = to_disp;
        if (!d->no_reorder) d->fullness++;
    } else if (is_idr) {
        d->num_out = d->out_index = 0;
        c->to_display = 0;
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
                    e = find_pic(d, (int)m->lt_idx, 0);
                    if (e >= 0) unmark(d, &d->pic[e]);
                    e = find_pic(d, frame_num - (int)m->diff, 1);
                    if (e < 0 || d->pic[e].status == PIC_NONEXIST) { status = -1; break; }
                    d->pic[e].status = PIC_LONG;
                    d->pic[e].pic_num = (int)m->lt_idx;
                    break;
                case 4:
                    d->max_lt_idx = (int)m->max_lt_idx - 1;
                    for (int i = 0; i < d->npic; i++)
                        if (IS_LONG(&d->pic[i]) && (d->max_lt_idx < 0 || d->pic[i].pic_num > d->max_lt_idx))
                            unmark(d, &d->pic[i]);
                    break;
                case 5:
                    c->to_display = 0;
                    mmco5(d);
                    d->last_mmco5 = 1;
                    frame_num = 0;
                    break;
                case 6:
                    if (d->max_lt_idx < 0 || (int)m->lt_idx > d->max_lt_idx) { status = -1; break; }
                    e = find_pic(d, (int)m->lt_idx, 0);
                    if (e >= 0) unmark(d, &d->pic[e]);
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
