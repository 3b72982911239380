/* Error concealment of the MBs a picture is missing -- clean-room
 * restatement of the reference's h264bsdConceal / ConcealMb / Transform
 * (h264bsd_conceal.c:125-245, 257-579, 592-629), producing MB records for the
 * reconstruction backend instead of writing pixels:
 *
 *  - P concealment with a reference picture: each missing MB is a copy of
 *    the co-located MB of the first existing picture of RefPicList0
 *    (:149-159, 310-332) -- a P_Skip-shaped record with a zero vector.
 *  - otherwise (I slices, or no reference): every missing MB is predicted
 *    from the decoded (unfiltered) neighbour samples above, below, left and
 *    right, in the reference's order (first decoded MB's row leftwards then
 *    rightwards, the rows above bottom-up column by column, then the rows
 *    below), each concealed MB becoming a neighbour of the next (:192-241).
 *    The backend first reconstructs the decoded MBs with the loop filter off
 *    and returns the picture; the concealed samples then travel as I_PCM
 *    records.
 *  - nothing decoded: grey (128) or a copy of the reference picture, with no
 *    loop filtering (:174-190).
 * A concealed MB is filtered as an intra MB with QP 40 and zero filter /
 * chroma QP offsets (:300-308). */
#include "decoder.h"
#include "../common/tables.h"

#include <stdlib.h>
#include <string.h>

#define CONCEAL_QP 40

static inline int clip1(int v) { return v < 0 ? 0 : v > 255 ? 255 : v; }

/* the reference's reduced 4x4 transform: only data[0], data[1] (first row)
 * and data[4] (first column) can be non-zero (:592-629) */
static void low_transform(int32_t *d)
{
    if (!d[1] && !d[4]) {
        for (int i = 1; i < 16; i++) d[i] = d[0];
        return;
    }
    const int32_t t0 = d[0], t1 = d[1];
    d[0] = t0 + t1;
    d[1] = t0 + (t1 >> 1);
    d[2] = t0 - (t1 >> 1);
    d[3] = t0 - t1;
    d[5] = d[6] = d[7] = d[4];
    for (int c = 0; c < 4; c++) {
        const int32_t a = d[c], b = d[4 + c];
        d[c] = a + b;
        d[4 + c] = a + (b >> 1);
        d[8 + c] = a - (b >> 1);
        d[12 + c] = a - b;
    }
}

/* one plane of ConcealMb's neighbour prediction (:337-457 luma, :459-572
 * chroma); n = MB size (16 or 8), s = samples summed per group (4 or 2) */
static void conceal_plane(uint8_t *plane, int stride, int n, int x0, int y0, int A, int B, int L, int R)
{
    const int s = n / 4;
    int32_t a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0}, l[4] = {0, 0, 0, 0}, r[4] = {0, 0, 0, 0};
    int32_t fp[16];
    memset(fp, 0, sizeof(fp));
    int j = 0, hor = 0, ver = 0;
    const uint8_t *mb = plane + (size_t)y0 * stride + x0;
    if (A) {
        for (int k = 0; k < 4; k++) for (int i = 0; i < s; i++) a[k] += mb[-stride + k * s + i];
        j++; hor++;
        fp[0] += a[0] + a[1] + a[2] + a[3];
        fp[1] += a[0] + a[1] - a[2] - a[3];
    }
    if (B) {
        for (int k = 0; k < 4; k++) for (int i = 0; i < s; i++) b[k] += mb[(size_t)n * stride + k * s + i];
        j++; hor++;
        fp[0] += b[0] + b[1] + b[2] + b[3];
        fp[1] += b[0] + b[1] - b[2] - b[3];
    }
    if (L) {
        for (int k = 0; k < 4; k++) for (int i = 0; i < s; i++) l[k] += mb[(size_t)(k * s + i) * stride - 1];
        j++; ver++;
        fp[0] += l[0] + l[1] + l[2] + l[3];
        fp[4] += l[0] + l[1] - l[2] - l[3];
    }
    if (R) {
        for (int k = 0; k < 4; k++) for (int i = 0; i < s; i++) r[k] += mb[(size_t)(k * s + i) * stride + n];
        j++; ver++;
        fp[0] += r[0] + r[1] + r[2] + r[3];
        fp[4] += r[0] + r[1] - r[2] - r[3];
    }
    /* luma: shifts 5 / 3+k and j -> 4,5,(21x)>>10,6; chroma one less */
    const int c = n == 16 ? 0 : 1;
    if (!hor && L && R) fp[1] = (l[0] + l[1] + l[2] + l[3] - r[0] - r[1] - r[2] - r[3]) >> (5 - c);
    else if (hor) fp[1] >>= (3 - c + hor);
    if (!ver && A && B) fp[4] = (a[0] + a[1] + a[2] + a[3] - b[0] - b[1] - b[2] - b[3]) >> (5 - c);
    else if (ver) fp[4] >>= (3 - c + ver);
    switch (j) {
    case 1: fp[0] >>= 4 - c; break;
    case 2: fp[0] >>= 5 - c; break;
    case 3: fp[0] = (21 * fp[0]) >> (10 - c); break;
    default: fp[0] >>= 6 - c; break;
    }
    low_transform(fp);
    uint8_t *o = plane + (size_t)y0 * stride + x0;
    for (int y = 0; y < n; y++)
        for (int x = 0; x < n; x++) o[(size_t)y * stride + x] = (uint8_t)clip1(fp[(y / s) * 4 + x / s]);
}

/* ConcealMb, neighbour-based branch, on an I420 picture of w x h MBs */
void h264dec_conceal_mb_intra(uint8_t *img, int w, int h, int row, int col, const uint8_t *dec)
{
    const int mb = row * w + col;
    const int A = row && dec[mb - w], B = row != h - 1 && dec[mb + w];
    const int L = col && dec[mb - 1], R = col != w - 1 && dec[mb + 1];
    const int W = w * 16, H = h * 16;
    conceal_plane(img, W, 16, col * 16, row * 16, A, B, L, R);
    conceal_plane(img + (size_t)W * H, W / 2, 8, col * 8, row * 8, A, B, L, R);
    conceal_plane(img + (size_t)W * H + (size_t)(W / 2) * (H / 2), W / 2, 8, col * 8, row * 8, A, B, L, R);
}

/* fields every concealed MB gets (:300-308): filtered as intra, QP 40,
 * deblocking idc 0 -- left / top MB edges wherever the neighbour exists */
static void conceal_fields(MbRec *r, int w, int mb)
{
    r->qp = CONCEAL_QP;
    r->qpc = kQpChroma[CONCEAL_QP];
    r->offA = r->offB = 0;
    r->avail = (uint8_t)(DB_INNER | (mb % w ? DB_LEFT : 0) | (mb >= w ? DB_TOP : 0));
}

static void copy_record(MbRec *r, int ref_slot)
{
    const uint16_t slice = r->slice;
    memset(r, 0, sizeof(*r));
    r->type = MBT_SKIP;
    for (int i = 0; i < 4; i++) r->ref[i] = (uint8_t)ref_slot;
    r->dbf = DBF_INTRA;
    r->slice = slice;
}

static void pcm_record(MbRec *r, uint32_t coef)
{
    const uint16_t slice = r->slice;
    memset(r, 0, sizeof(*r));
    r->type = MBT_IPCM;
    r->coef = coef;
    r->slice = slice;
}

/* 12 coefficient blocks = one MB of samples (I_PCM layout) */
static int pcm_alloc(PicBuild *pb, uint32_t *coef)
{
    if (!picbuild_coef_alloc(pb, 12)) return -1;
    *coef = pb->ncoef - 12;
    return 0;
}

int h264dec_conceal(H264Dec *d, int is_i)
{
    PicBuild *pb = &d->pb;
    const int w = pb->w, h = pb->h, nmbs = pb->nmbs;
    /* reference picture: the first existing entry of the list (:149-159) */
    int ref = -1;
    if (!is_i || d->intra_conceal)
        for (int i = 0; i < 16 && ref < 0; i++) {
            const int e = d->dpb.list[i];
            if (e >= 0 && d->dpb.pic[e].status > PIC_NONEXIST) ref = d->dpb.pic[e].slot;
        }
    int first = 0;
    while (first < nmbs && !pb->decoded[first]) first++;
    h264dec_pb_writable(d);
    for (int i = 0; i < nmbs; i++) pb->rec[i].slice = pb->pc.slice[i];

    if (first == nmbs) {
        /* whole picture lost: grey, or a copy of the reference; no filtering */
        uint32_t grey = 0;
        const int copy = !(is_i && !d->intra_conceal) && ref >= 0;
        if (!copy) {
            if (pcm_alloc(pb, &grey)) return -1;
            memset(pb->coef + (size_t)grey * 16, 128, 384);
        }
        for (int i = 0; i < nmbs; i++) {
            if (copy) copy_record(&pb->rec[i], ref);
            else pcm_record(&pb->rec[i], grey);
            pb->rec[i].dbf = 0;
            pb->decoded[i] = 1;
        }
        return nmbs;
    }

    int n = 0;
    if (!is_i && ref >= 0) {
        for (int i = 0; i < nmbs; i++)
            if (!pb->decoded[i]) {
                copy_record(&pb->rec[i], ref);
                conceal_fields(&pb->rec[i], w, i);
                pb->decoded[i] = 1;
                n++;
            }
        return n;
    }

    /* neighbour-based: pass 1 reconstructs the decoded MBs unfiltered */
    const int on_backend = d->be.conceal != NULL && (!d->be.conceal_ok || d->be.conceal_ok(d->be.ctx));
    uint8_t *saved = (uint8_t *)malloc((size_t)nmbs);
    uint8_t *img = on_backend ? NULL : (uint8_t *)malloc(d->frame_bytes);
    uint32_t grey = 0;
    if (!saved || (!on_backend && !img) || pcm_alloc(pb, &grey)) { free(saved); free(img); return -1; }
    memset(pb->coef + (size_t)grey * 16, 128, 384);
    for (int i = 0; i < nmbs; i++) {
        saved[i] = pb->rec[i].avail;
        if (!pb->decoded[i]) pcm_record(&pb->rec[i], grey);
        else pb->rec[i].avail &= (uint8_t)~(DB_LEFT | DB_TOP | DB_INNER);
    }
    int rc = d->be.decode(d->be.ctx, pb, d->cur_slot);
    if (!rc && !on_backend) rc = d->be.read(d->be.ctx, d->cur_slot, img) < 0 ? -1 : 0;
    h264dec_pb_writable(d);                 /* pass 1's records are uploaded */
    for (int i = 0; i < nmbs; i++) if (pb->decoded[i]) pb->rec[i].avail = saved[i];
    free(saved);
    if (rc) { free(img); return -1; }

    /* the reference's order (:192-241); dec[] grows as MBs are concealed */
    uint8_t *dec = pb->decoded;
    const int row = first / w, col = first % w;
    int *order = (int *)malloc(sizeof(int) * (size_t)nmbs);
    if (!order) { free(img); return -1; }
    for (int j = col - 1; j >= 0; j--) order[n++] = row * w + j;
    for (int j = col + 1; j < w; j++) if (!dec[row * w + j]) order[n++] = row * w + j;
    for (int j = 0; j < w; j++) for (int i = row - 1; i >= 0; i--) order[n++] = i * w + j;
    for (int i = row + 1; i < h; i++) for (int j = 0; j < w; j++) if (!dec[i * w + j]) order[n++] = i * w + j;
    if (on_backend) {
        /* the backend conceals in place (k_conceal); pass 2 copies each
         * concealed MB from the slot itself (zero-vector skip records read
         * only the MB's own samples, which nothing else writes before) and
         * filters it as intra */
        if (d->be.conceal(d->be.ctx, d->cur_slot, order, n, dec)) { free(order); return -1; }
        for (int k = 0; k < n; k++) {
            const int mb = order[k];
            copy_record(&pb->rec[mb], d->cur_slot);
            conceal_fields(&pb->rec[mb], w, mb);
            dec[mb] = 1;
        }
        free(order);
        return n;
    }
    for (int k = 0; k < n; k++) {
        const int mb = order[k];
        h264dec_conceal_mb_intra(img, w, h, mb / w, mb % w, dec);
        dec[mb] = 1;
    }
    /* pass 2 records: the concealed samples as I_PCM */
    const int W = w * 16, H = h * 16;
    for (int k = 0; k < n; k++) {
        const int mb = order[k], mx = mb % w, my = mb / w;
        uint32_t c;
        if (pcm_alloc(pb, &c)) { free(order); free(img); return -1; }
        uint8_t *s = (uint8_t *)(pb->coef + (size_t)c * 16);
        for (int y = 0; y < 16; y++) memcpy(s + y * 16, img + (size_t)(my * 16 + y) * W + mx * 16, 16);
        for (int y = 0; y < 8; y++) {
            memcpy(s + 256 + y * 8, img + (size_t)W * H + (size_t)(my * 8 + y) * (W / 2) + mx * 8, 8);
            memcpy(s + 320 + y * 8, img + (size_t)W * H * 5 / 4 + (size_t)(my * 8 + y) * (W / 2) + mx * 8, 8);
        }
        pcm_record(&pb->rec[mb], c);
        conceal_fields(&pb->rec[mb], w, mb);
    }
    free(order);
    free(img);
    return n;
}
