/* Host decoder control -- see decoder.h. */
#include "decoder.h"
#include "../common/tables.h"

#include <stdlib.h>
#include <stdatomic.h>
#include <string.h>

#include <stdio.h>
#include <time.h>

double h264dec_now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* H264MI_DEBUG, read once; instances on several threads may ask first */
static int dbg_enabled(void)
{
    static _Atomic int e = -1;
    int v = atomic_load_explicit(&e, memory_order_relaxed);
    if (v < 0) {
        v = getenv("H264MI_DEBUG") != NULL;
        atomic_store_explicit(&e, v, memory_order_relaxed);
    }
    return v;
}
#define DEC_FAIL(code) (dbg_enabled() ? (fprintf(stderr, "h264mi: %s:%d -> %d\n", __FILE__, __LINE__, (code)), (code)) : (code))
#define SPS_FORCE (MAX_SPS + 1)
#define PPS_FORCE (MAX_PPS + 1)

int h264dec_init(H264Dec *d, int no_output_reordering, H264Backend be)
{
    h264_tables_init();
    memset(d, 0, sizeof(*d));
    d->active_sps = -1;
    d->active_pps = -1;
    d->old_sps_id = -1;
    d->no_reorder_app = no_output_reordering;
    d->be = be;
    d->aub_first_call = 1;
    d->cur_slot = -1;
    /* worker threads for speculative slice parsing: H264MI_PARSE_THREADS
     * (default 3; 0 = none).  H264MI_PARSE_HELP (default 1): the calling
     * thread, about to wait for a picture's reconstruction, parses the next
     * picture's slices ahead itself (spec_help) -- with no workers too */
    const char *pt = getenv("H264MI_PARSE_THREADS"), *ph = getenv("H264MI_PARSE_HELP");
    const int nth = pt ? atoi(pt) : 3;
    d->spec_help = ph ? atoi(ph) != 0 : 1;
    d->spec = nth > 0 || d->spec_help ? spec_create(nth > 16 ? 16 : nth < 0 ? 0 : nth) : NULL;
    return 0;
}

/* the backend may still be uploading the last picture's records from d->pb
 * (H264Backend.records_wait): wait before writing them */
void h264dec_pb_writable(H264Dec *d)
{
    if (d->pb.pinned && d->be.records_wait) (void)d->be.records_wait(d->be.ctx);
}

static void out_frames_free(H264Dec *d)
{
    if (d->out_frames && d->be.host_free) d->be.host_free(d->be.ctx, d->out_frames);
    else free(d->out_frames);
    d->out_frames = NULL;
}

void h264dec_release(H264Dec *d)
{
    spec_destroy(d->spec);
    d->spec = NULL;
    if (d->pb_ready) {
        h264dec_pb_writable(d);
        picbuild_free(&d->pb);
    }
    free(d->rbsp);
    out_frames_free(d);
    if (d->be.destroy) d->be.destroy(d->be.ctx);
    memset(d, 0, sizeof(*d));
}

const Sps *h264dec_active_sps(const H264Dec *d)
{
    if (d->active_sps < 0 || d->active_sps >= MAX_SPS) return NULL;
    return &d->sps[d->active_sps];
}

int h264dec_valid_param_sets(const H264Dec *d)
{
    for (int i = 0; i < MAX_PPS; i++)
        if (d->pps[i].valid && d->sps[d->pps[i].sps_id].valid) return 1;
    return 0;
}

/* ---- byte stream: reference byte_stream.c:80-236 semantics ----------- */
/* locate the next NAL unit: payload at bs + *init, *size bytes; *emul: an
 * emulation-prevention pattern was seen (or raw NAL mode) */
int nal_scan(const uint8_t *bs, uint32_t len, uint32_t *init_out, uint32_t *size_out, uint32_t *read_bytes,
             int *emul_out)
{
    uint32_t init = 0, size, zeros = 0;
    int emul = 0;
    if (len > 3 && bs[0] == 0 && bs[1] == 0 && (bs[2] & 0xFE) == 0) {
        uint32_t cnt = 2;
        zeros = 2;
        const uint8_t *p = bs + 2;
        for (;;) {
            uint8_t b = *p++;
            cnt++;
            if (cnt == len) { *read_bytes = len; return -1; }
            if (!b) zeros++;
            else if (b == 1 && zeros >= 2) break;
            else zeros = 0;
        }
        init = cnt;
        zeros = 0;
        int invalid = 0;
        for (;;) {
            if (zeros == 0) {
                /* runs of non-zero bytes change nothing but the position */
                const uint8_t *z = (const uint8_t *)memchr(p, 0, len - cnt);
                if (!z) { p += len - cnt; cnt = len; size = cnt - init; break; }
                cnt += (uint32_t)(z - p);
                p = z;
            }
            uint8_t b = *p++;
            cnt++;
            if (!b) zeros++;
            if (b == 3 && zeros == 2) emul = 1;      /* hasEmulation (byte_stream.c:142-145) */
            if (b == 1 && zeros >= 2) {
                size = cnt - init - zeros - 1;
                zeros -= zeros < 3 ? zeros : 3;
                break;
            } else if (b) {
                if (zeros >= 3) invalid = 1;
                zeros = 0;
            }
            if (cnt == len) { size = cnt - init - zeros; break; }
        }
        *read_bytes = size + init + zeros;
        if (invalid) return -1;
    } else {
        size = len;
        *read_bytes = len;
        emul = 1;
    }
    *init_out = init;
    *size_out = size;
    *emul_out = emul;
    return 0;
}

/* emulation-prevention removal (byte_stream.c:191-229) into dst (>= size
 * bytes); returns the RBSP length or -1 on an invalid sequence */
int nal_unescape(const uint8_t *src, uint32_t size, int emul, uint8_t *dst)
{
    uint32_t w = 0;
    if (!emul) {
        memcpy(dst, src, size);
        return (int)size;
    }
    int zc = 0;
    for (uint32_t i = 0; i < size; i++) {
        if (zc == 0) {
            /* copy up to the next zero byte in one go */
            const uint8_t *z = (const uint8_t *)memchr(src + i, 0, size - i);
            const uint32_t n = z ? (uint32_t)(z - (src + i)) : size - i;
            memcpy(dst + w, src + i, n);
            w += n;
            i += n;
            if (i == size) break;
        }
        uint8_t b = src[i];
        if (zc == 2 && b == 3) {
            if (i == size - 1 || src[i + 1] > 3) return -1;
            zc = 0;
            continue;
        }
        if (zc == 2 && b <= 2) return -1;
        zc = b == 0 ? zc + 1 : 0;
        dst[w++] = b;
    }
    return (int)w;
}

static int extract_nal(H264Dec *d, const uint8_t *bs, uint32_t len, const uint8_t **nal,
                       uint32_t *nal_len, uint32_t *read_bytes)
{
    uint32_t init, size;
    int emul;
    if (nal_scan(bs, len, &init, &size, read_bytes, &emul)) return -1;
    if (d->rbsp_cap < size + 8) {
        size_t nc = size + 64 + size / 2;
        uint8_t *r = (uint8_t *)realloc(d->rbsp, nc);
        if (!r) return -1;
        d->rbsp = r;
        d->rbsp_cap = nc;
    }
    int w = nal_unescape(bs + init, size, emul, d->rbsp);
    if (w < 0) return -1;
    *nal = d->rbsp;
    *nal_len = (uint32_t)w;
    return 0;
}

/* ---- picture order count, H.264 §8.2.1 -------------------------------- */
static int decode_poc(H264Dec *d, const Sps *sps, const SliceHdr *sh)
{
    PocState *s = &d->poc;
    int idr = sh->nal_type == NAL_IDR;
    int max_fn = 1 << sps->log2_max_frame_num;
    int poc = 0;
    if (sps->poc_type == 0) {
        if (idr) { s->prev_msb = 0; s->prev_lsb = 0; }
        else if (s->prev_mmco5) { s->prev_msb = 0; s->prev_lsb = 0; }
        int max_lsb = 1 << sps->log2_max_poc_lsb;
        int msb;
        if (sh->poc_lsb < s->prev_lsb && s->prev_lsb - sh->poc_lsb >= max_lsb / 2) msb = s->prev_msb + max_lsb;
        else if (sh->poc_lsb > s->prev_lsb && sh->poc_lsb - s->prev_lsb > max_lsb / 2) msb = s->prev_msb - max_lsb;
        else msb = s->prev_msb;
        int top = msb + sh->poc_lsb;
        int bot = top + sh->delta_poc_bottom;
        poc = top < bot ? top : bot;
        if (sh->nal_ref_idc) { s->prev_msb = msb; s->prev_lsb = sh->poc_lsb; }
    } else {
        int fno;
        if (idr) fno = 0;
        else if (s->prev_mmco5) fno = s->prev_frame_num > sh->frame_num ? max_fn : 0;
        else if (s->prev_frame_num > sh->frame_num) fno = s->prev_frame_num_offset + max_fn;
        else fno = s->prev_frame_num_offset;
        if (sps->poc_type == 2) {
            if (idr) poc = 0;
            else if (!sh->nal_ref_idc) poc = 2 * (fno + sh->frame_num) - 1;
            else poc = 2 * (fno + sh->frame_num);
        } else {
            int abs_fn = sps->num_ref_frames_in_poc_cycle ? fno + sh->frame_num : 0;
            if (!sh->nal_ref_idc && abs_fn > 0) abs_fn--;
            int exp = 0;
            if (abs_fn > 0) {
                int delta_cycle = 0;
                for (int i = 0; i < sps->num_ref_frames_in_poc_cycle; i++) delta_cycle += sps->offset_for_ref_frame[i];
                int cyc = (abs_fn - 1) / sps->num_ref_frames_in_poc_cycle;
                int in_cyc = (abs_fn - 1) % sps->num_ref_frames_in_poc_cycle;
                exp = cyc * delta_cycle;
                for (int i = 0; i <= in_cyc; i++) exp += sps->offset_for_ref_frame[i];
            }
            if (!sh->nal_ref_idc) exp += sps->offset_for_non_ref_pic;
            int top = exp + sh->delta_poc[0];
            int bot = top + sps->offset_for_top_to_bottom + sh->delta_poc[1];
            poc = top < bot ? top : bot;
        }
        s->prev_frame_num_offset = fno;
        s->prev_frame_num = sh->frame_num;
    }
    s->prev_mmco5 = 0;
    for (int i = 0; i < sh->nmmco; i++) if (sh->mmco[i].op == 5) s->prev_mmco5 = 1;
    if (s->prev_mmco5) {
        /* tempPicOrderCnt handling (§8.2.1): the picture is treated as POC 0 */
        s->prev_frame_num_offset = 0;
        s->prev_frame_num = 0;
        if (sps->poc_type == 0) { s->prev_msb = 0; s->prev_lsb = 0; }
        poc = 0;
    }
    return poc;
}

/* ---- access unit boundary (reference storage.c:632-760) --------------- */
static int check_au_boundary(H264Dec *d, const NalHdr *nal, const BitReader *br, int *boundary)
{
    *boundary = 0;
    if ((nal->type > 5 && nal->type < 12) || (nal->type > 12 && nal->type <= 18)) {
        *boundary = 1;
        return 0;
    }
    if (nal->type != NAL_SLICE && nal->type != NAL_IDR) return 0;
    if (d->aub_first_call) { *boundary = 1; d->aub_first_call = 0; }
    int pps_id;
    if (peek_slice_pps_id(br, &pps_id)) return DEC_FAIL(DEC_ERROR);
    const Pps *pps = &d->pps[pps_id];
    if (!pps->valid || !d->sps[pps->sps_id].valid ||
        (d->active_sps >= 0 && d->active_sps < MAX_SPS && pps->sps_id != d->active_sps && nal->type != NAL_IDR))
        return DEC_FAIL(DEC_PARAM_SET_ERROR);
    const Sps *sps = &d->sps[pps->sps_id];
    if (d->aub_prev_nal.ref_idc != nal->ref_idc && (d->aub_prev_nal.ref_idc == 0 || nal->ref_idc == 0)) *boundary = 1;
    if ((d->aub_prev_nal.type == NAL_IDR) != (nal->type == NAL_IDR)) *boundary = 1;
    /* each field is checked as the reference's h264bsdCheck* re-parse
     * reads it: state updated before a failing read stays updated, and the
     * previous NAL is only replaced when every read succeeded */
    BitReader b = *br;
    br_ue(&b); br_ue(&b); br_ue(&b);
    int fn = (int)br_u(&b, sps->log2_max_frame_num);
    if (b.err) return DEC_FAIL(DEC_ERROR);
    if (d->aub_prev_frame_num != fn) { d->aub_prev_frame_num = fn; *boundary = 1; }
    if (nal->type == NAL_IDR) {
        int id = (int)br_ue(&b);
        if (b.err) return DEC_FAIL(DEC_ERROR);
        if (d->aub_prev_nal.type == NAL_IDR && d->aub_prev_idr_id != id) *boundary = 1;
        d->aub_prev_idr_id = id;
    }
    if (sps->poc_type == 0) {
        int lsb = (int)br_u(&b, sps->log2_max_poc_lsb);
        if (b.err) return DEC_FAIL(DEC_ERROR);
        if (d->aub_prev_poc_lsb != lsb) { d->aub_prev_poc_lsb = lsb; *boundary = 1; }
        if (pps->bottom_field_poc_present) {
            int db = br_se(&b);
            if (b.err) return DEC_FAIL(DEC_ERROR);
            if (d->aub_prev_dpoc_bottom != db) { d->aub_prev_dpoc_bottom = db; *boundary = 1; }
        }
    } else if (sps->poc_type == 1 && !sps->delta_pic_order_always_zero) {
        int d0 = br_se(&b), d1 = pps->bottom_field_poc_present ? br_se(&b) : 0;
        if (b.err) return DEC_FAIL(DEC_ERROR);
        if (d->aub_prev_dpoc[0] != d0) { d->aub_prev_dpoc[0] = d0; *boundary = 1; }
        if (pps->bottom_field_poc_present && d->aub_prev_dpoc[1] != d1) { d->aub_prev_dpoc[1] = d1; *boundary = 1; }
    }
    d->aub_prev_nal = *nal;      /* aub->nuPrev (storage.c:774); prevNalUnit is set per decoded slice header */
    return 0;
}

/* ---- parameter-set activation (reference storage.c:298-420) ----------- */
static int ensure_picbuild(H264Dec *d, const Sps *sps)
{
    if (d->pb_ready && d->pb.w == sps->w_mbs && d->pb.h == sps->h_mbs) return 0;
    if (d->pb_ready) {
        h264dec_pb_writable(d);
        picbuild_free(&d->pb);
    }
    d->pb_ready = 0;
    /* pinned records when the backend uploads from them (records_wait) */
    const int pinned = d->be.records_wait && d->be.host_alloc && d->be.host_free;
    if (picbuild_init_alloc(&d->pb, sps->w_mbs, sps->h_mbs, pinned ? d->be.host_alloc : NULL,
                            pinned ? d->be.host_free : NULL, d->be.ctx)) return -1;
    d->pb_ready = 1;
    return 0;
}

static int activate(H264Dec *d, int pps_id, int is_idr)
{
    const Pps *pps = &d->pps[pps_id];
    if (!pps->valid || !d->sps[pps->sps_id].valid) return DEC_FAIL(DEC_PARAM_SET_ERROR);
    if (pps->entropy_coding || pps->weighted_pred) return DEC_FAIL(DEC_PARAM_SET_ERROR);
    if (d->active_pps == -1) {
        d->active_pps = pps_id;
        d->active_sps = pps->sps_id;
        d->pending_activation = 1;
    } else if (d->pending_activation) {
        d->pending_activation = 0;
        const Sps *sps = &d->sps[d->active_sps];
        if (ensure_picbuild(d, sps)) return DEC_MEMALLOC_ERROR;
        int no_reorder = d->no_reorder_app || sps->poc_type == 2 ||
                         (sps->vui_present && sps->bitstream_restriction && !sps->num_reorder_frames);
        dpb_init(&d->dpb, sps->max_dpb, sps->num_ref_frames, 1 << sps->log2_max_frame_num, no_reorder);
        d->nslots = d->dpb.npic;
        d->frame_bytes = (size_t)sps->w_mbs * sps->h_mbs * 384;
        out_frames_free(d);
        d->out_frames = (uint8_t *)(d->be.host_alloc ? d->be.host_alloc(d->be.ctx, d->frame_bytes * (size_t)d->nslots)
                                                     : malloc(d->frame_bytes * (size_t)d->nslots));
        if (!d->out_frames) return DEC_MEMALLOC_ERROR;
        if (d->be.configure(d->be.ctx, sps->w_mbs, sps->h_mbs, d->nslots)) return DEC_MEMALLOC_ERROR;
    } else if (pps_id != d->active_pps) {
        if (pps->sps_id != d->active_sps) {
            if (!is_idr) return DEC_FAIL(DEC_PARAM_SET_ERROR);
            d->active_pps = pps_id;
            d->active_sps = pps->sps_id;
            d->pending_activation = 1;
        } else {
            d->active_pps = pps_id;
        }
    }
    return 0;
}

static void store_sps(H264Dec *d, const Sps *s)
{
    int id = s->id;
    if (d->sps[id].valid && id == d->active_sps) {
        if (!sps_equal(s, &d->sps[id])) {
            d->active_sps = SPS_FORCE;
            d->active_pps = PPS_FORCE;
        } else {
            return;
        }
    }
    d->sps[id] = *s;
}

static void store_pps(H264Dec *d, const Pps *p)
{
    int id = p->id;
    if (d->pps[id].valid && id == d->active_pps && p->sps_id != d->active_sps)
        d->active_pps = PPS_FORCE;
    d->pps[id] = *p;
}

static int finish_picture(H264Dec *d, int concealed_mbs)
{
    const Sps *sps = &d->sps[d->active_sps];
    const double t0 = h264dec_now();
    int rc = d->be.decode(d->be.ctx, &d->pb, d->cur_slot);
    /* the picture's output copy starts now, behind its reconstruction */
    if (!rc && d->be.prefetch && d->out_frames)
        rc = d->be.prefetch(d->be.ctx, d->cur_slot, d->out_frames + d->frame_bytes * (size_t)d->cur_slot);
    d->t_submit += h264dec_now() - t0;
    if (rc) return DEC_FAIL(DEC_ERROR);
    d->pics_decoded++;
    d->alg_ref_bytes += d->pb.alg_ref_bytes;
    d->coded_blocks += d->pb.n_coded_blocks;
    int poc = decode_poc(d, sps, &d->sh);
    if (d->valid_slice_in_au) {
        int is_idr = d->prev_nal.type == NAL_IDR;
        dpb_mark(&d->dpb, &d->sh, d->prev_nal.ref_idc != 0, d->sh.frame_num, poc, is_idr,
                 d->cur_pic_id, concealed_mbs);
    }
    d->pic_started = 0;
    d->valid_slice_in_au = 0;
    return DEC_PIC_RDY;
}

static int decode_nal(H264Dec *d, const uint8_t *buf, uint32_t len, uint32_t pic_id, uint32_t *read_bytes);

int h264dec_decode(H264Dec *d, const uint8_t *buf, uint32_t len, uint32_t pic_id, uint32_t *read_bytes)
{
    const double t0 = h264dec_now(), s0 = d->t_submit;
    const int st = spec_stats_on(d->spec);
    const double c0 = st ? spec_thread_cpu() : 0.0;
    const int r = decode_nal(d, buf, len, pic_id, read_bytes);
    if (st) spec_account_caller(d->spec, spec_thread_cpu() - c0);
    d->t_parse += h264dec_now() - t0 - (d->t_submit - s0);
    return r;
}

static int decode_nal(H264Dec *d, const uint8_t *buf, uint32_t len, uint32_t pic_id, uint32_t *read_bytes)
{
    const uint8_t *nal;
    uint32_t nal_len;
    if (extract_nal(d, buf, len, &nal, &nal_len, read_bytes)) return DEC_FAIL(DEC_ERROR);
    if (d->prev_buf_not_finished && buf == d->prev_buf_ptr) *read_bytes = d->prev_bytes;
    d->prev_bytes = *read_bytes;
    d->prev_buf_ptr = buf;
    d->prev_buf_not_finished = 0;
    if (nal_len < 1) return DEC_FAIL(DEC_ERROR);
    if (nal[0] & 0x80) return DEC_FAIL(DEC_ERROR);
    NalHdr nh = {(nal[0] >> 5) & 3, nal[0] & 31};
    if ((nh.type == NAL_IDR && nh.ref_idc == 0) ||
        ((nh.type == NAL_SPS || nh.type == NAL_PPS) && nh.ref_idc == 0)) return DEC_FAIL(DEC_ERROR);
    BitReader br;
    br_init(&br, nal + 1, nal_len - 1);
    if (nh.type == 0 || nh.type >= 13) return DEC_RDY;

    int boundary = 0;
    int r = check_au_boundary(d, &nh, &br, &boundary);
    if (r) return r;
    if (boundary) {
        if (d->pic_started && d->active_sps >= 0 && d->active_sps < MAX_SPS) {
            if (d->pending_activation) return DEC_FAIL(DEC_ERROR);
            /* conceal what the picture is missing (decoder.c:240-268): as P
             * after a fresh allocation and RefPicList0 init when no slice
             * header was valid, else by the last valid slice's type */
            int is_i;
            if (!d->valid_slice_in_au) {
                d->cur_slot = dpb_alloc_current(&d->dpb);
                if (d->cur_slot < 0) return DEC_FAIL(DEC_ERROR);
                h264dec_pb_writable(d), picbuild_reset(&d->pb, 0);
                d->pb.cur_slot = d->cur_slot;
                SliceHdr tmp = d->sh;
                int ref_slot[MAX_REFS];
                tmp.slice_type = 0;
                tmp.ref_mod_flag = 0;
                if (tmp.num_ref_idx_active < 1) tmp.num_ref_idx_active = 1;
                dpb_build_list(&d->dpb, &tmp, ref_slot);
                is_i = 0;
            } else {
                is_i = d->sh.slice_type == 2;
            }
            int n = h264dec_conceal(d, is_i);
            if (n < 0) return DEC_FAIL(DEC_ERROR);
            d->num_concealed += n;
            *read_bytes = 0;
            d->prev_buf_not_finished = 1;
            return finish_picture(d, d->num_concealed);
        }
        d->valid_slice_in_au = 0;
        d->skip_redundant = 0;
    }

    switch (nh.type) {
    case NAL_SPS: {
        Sps s;
        if (parse_sps(&br, &s)) return DEC_FAIL(DEC_ERROR);
        store_sps(d, &s);
        return DEC_RDY;
    }
    case NAL_PPS: {
        Pps p;
        if (parse_pps(&br, d->sps, &p)) return DEC_FAIL(DEC_ERROR);
        store_pps(d, &p);
        return DEC_RDY;
    }
    case NAL_SLICE:
    case NAL_IDR: {
        if (d->skip_redundant) return DEC_RDY;
        d->pic_started = 1;
        int is_idr = nh.type == NAL_IDR;
        if (!d->valid_slice_in_au) {
            d->num_concealed = 0;
            d->cur_pic_id = (int)pic_id;
            int pps_id;
            if (peek_slice_pps_id(&br, &pps_id)) return DEC_FAIL(DEC_ERROR);
            int old = d->active_sps;
            int rr = activate(d, pps_id, is_idr);
            if (rr) {
                d->active_pps = -1; d->active_sps = -1; d->pending_activation = 0;
                return rr;
            }
            if (old != d->active_sps) {
                const Sps *nsps = &d->sps[d->active_sps];
                const Sps *osps = (d->old_sps_id >= 0 && d->old_sps_id < MAX_SPS) ? &d->sps[d->old_sps_id] : NULL;
                *read_bytes = 0;
                d->prev_buf_not_finished = 1;
                int no_out_prior = 1;
                if (is_idr) {
                    SliceHdr t;
                    BitReader b2 = br;
                    if (!parse_slice_header(&b2, &nh, nsps, &d->pps[d->active_pps], &t)) no_out_prior = t.no_output_prior;
                }
                if (no_out_prior || d->dpb.no_reorder || !osps || osps->w_mbs != nsps->w_mbs ||
                    osps->h_mbs != nsps->h_mbs || osps->max_dpb != nsps->max_dpb)
                    d->dpb.flushed = 0;
                else
                    dpb_flush(&d->dpb);
                d->old_sps_id = d->active_sps;
                return DEC_HDRS_RDY;
            }
        }
        if (d->pending_activation) return DEC_FAIL(DEC_ERROR);
        const Sps *sps = &d->sps[d->active_sps];
        const Pps *pps = &d->pps[d->active_pps];
        SliceHdr sh;
        if (parse_slice_header(&br, &nh, sps, pps, &sh)) return DEC_FAIL(DEC_ERROR);
        if (sh.pps_id != d->active_pps) {
            /* a later slice of the picture may name another PPS of the same SPS */
            if (!d->pps[sh.pps_id].valid || d->pps[sh.pps_id].sps_id != d->active_sps) return DEC_FAIL(DEC_ERROR);
            pps = &d->pps[sh.pps_id];
        }
        const int first_slice = !d->valid_slice_in_au;
        if (first_slice) {
            if (!is_idr && dpb_check_gaps(&d->dpb, sh.frame_num, nh.ref_idc != 0, sps->gaps_allowed))
                return DEC_FAIL(DEC_ERROR);
            d->cur_slot = dpb_alloc_current(&d->dpb);
            if (d->cur_slot < 0) return DEC_FAIL(DEC_ERROR);
            h264dec_pb_writable(d), picbuild_reset(&d->pb, pps->cip);
            d->pb.cur_slot = d->cur_slot;
        }
        d->sh = sh;
        d->valid_slice_in_au = 1;
        d->prev_nal = nh;
        int ref_slot[MAX_REFS];
        if (dpb_build_list(&d->dpb, &sh, ref_slot)) return DEC_FAIL(DEC_ERROR);
        d->pb.pc.cip = pps->cip;
        /* the picture's later slices already in the buffer are parsed ahead
         * on worker threads; this thread takes their results when it gets
         * there (specparse.c), else parses them itself */
        if (first_slice && !spec_active_for(d->spec, buf))
            spec_launch(d->spec, d, sps, pps, &nh, &sh, buf, *read_bytes, len);
        const int st = spec_stats_on(d->spec);
        const double c0 = st ? spec_thread_cpu() : 0.0;
        const int nd0 = d->pb.ndecoded;
        int taken = 0, perr = 0;
        if (spec_take(d->spec, d, buf, *read_bytes, &sh, pps, ref_slot)) taken = 1;   /* identical to parsing it here */
        else perr = parse_slice_data(&d->pb, &br, &sh, pps, ref_slot);
        if (st && !taken) spec_account_main(d->spec, spec_thread_cpu() - c0, d->pb.ndecoded - nd0);
        if (perr) {
            /* the slice is un-marked (decoder.c:462-467, slice_data.c:302-358);
             * its MBs are concealed at the next access-unit boundary */
            picbuild_mark_slice_corrupted(&d->pb, sh.first_mb);
            return DEC_FAIL(DEC_ERROR);
        }
        if (d->pb.ndecoded == d->pb.nmbs) {
            d->skip_redundant = 1;
            const int r = finish_picture(d, d->num_concealed);
            /* the next picture's slices, if the buffer holds them, are parsed
             * while the caller fetches this one */
            if (r == DEC_PIC_RDY && *read_bytes < len) spec_launch_ahead(d->spec, d, buf + *read_bytes, len - *read_bytes);
            return r;
        }
        return DEC_RDY;
    }
    default:
        return DEC_RDY;
    }
}

void h264dec_flush(H264Dec *d)
{
    if (d->dpb.npic) dpb_flush(&d->dpb);
}

const uint8_t *h264dec_next_output(H264Dec *d, uint32_t *pic_id, uint32_t *is_idr, uint32_t *err_mbs)
{
    return h264dec_next_output_rgba(d, pic_id, is_idr, err_mbs, NULL);
}

/* rgba != NULL: the picture as RGBA (w*h*4 bytes) into rgba, converted by
 * the backend (returns rgba) */
const uint8_t *h264dec_next_output_rgba(H264Dec *d, uint32_t *pic_id, uint32_t *is_idr, uint32_t *err_mbs,
                                        uint8_t *rgba)
{
    if (rgba && !d->be.read_rgba) return NULL;
    const DpbOut *o = dpb_next_output(&d->dpb);
    if (!o) return NULL;
    uint8_t *dst = rgba ? rgba : d->out_frames + d->frame_bytes * (size_t)o->slot;
    /* rather than wait for the GPU, parse the next picture's slices that
     * spec_launch_ahead queued (the buffer already holds them); the core
     * stays busy and warm, and the decode call that follows takes them */
    if (d->spec_help) {
        const double h0 = h264dec_now();
        spec_help(d->spec);
        d->t_parse += h264dec_now() - h0;
    }
    const double t0 = h264dec_now();
    if (d->be.sync && d->be.sync(d->be.ctx)) return NULL;
    const double t1 = h264dec_now();
    const int rr = rgba ? d->be.read_rgba(d->be.ctx, o->slot, dst) : d->be.read(d->be.ctx, o->slot, dst);
    d->t_wait += t1 - t0;
    d->t_copy += h264dec_now() - t1;
    d->n_output++;
    if (rr < 0) return NULL;
    if (pic_id) *pic_id = (uint32_t)o->pic_id;
    if (is_idr) *is_idr = (uint32_t)o->is_idr;
    /* rr > 0: the device flagged the reconstruction (a bounded wait that
     * expired, or a residual range error the host check did not predict):
     * the whole picture counts as erroneous */
    if (err_mbs) *err_mbs = rr > 0 ? (uint32_t)d->pb.nmbs : (uint32_t)o->err_mbs;
    return dst;
}
