/* MB-record capture: run the host parser over a whole stream and keep every
 * picture's MB-record batch (records, coefficient blocks, target slot) in
 * host memory instead of reconstructing it.  This is the "pre-parsed record
 * batch" producer of SURVEY.md §8d (kernel-only timing uploads these to HBM
 * once) and the record source for kernel-level parity tests. */
#include "../../../include/h264mi.h"
#include "decoder.h"

#include <stdlib.h>
#include <string.h>

typedef struct CapPic {
    size_t   rec_off;
    size_t   coef_off;       /* in 16-coefficient blocks */
    uint32_t ncoef;
    int      cur_slot;
    uint64_t alg_ref_bytes;
    uint64_t ref_line_bytes;
    uint32_t n_inter, n_intra, n_coded;
} CapPic;

struct h264mi_capture {
    int w, h, nslots;
    MbRec *recs;
    size_t nrec, rec_cap;
    int16_t *coefs;
    size_t ncoef, coef_cap;
    CapPic *pics;
    int npics, pic_cap;
    int errors;
    int reconfigured;
};

static uint64_t ref_line_bytes(const MbRec *rec, int w, int h);

static int cap_configure(void *vctx, int w_mbs, int h_mbs, int nslots)
{
    struct h264mi_capture *c = (struct h264mi_capture *)vctx;
    if (c->w && (c->w != w_mbs || c->h != h_mbs)) c->reconfigured = 1;
    c->w = w_mbs; c->h = h_mbs;
    if (nslots > c->nslots) c->nslots = nslots;
    return 0;
}

/* Test hooks (H264MI_CHECK_INJECT*, H264MI_DEBUG_FLAG_PICTURE) break a hand-off
 * or force a device flag on purpose; the library honours them only when
 * H264MI_TEST=1 is set as well, so that a shipped decoder never produces wrong
 * pictures because of one stray environment variable (tests/test_knobs.py). */
int h264mi_test_hooks(void)
{
    static int cached = -1;
    int v = __atomic_load_n(&cached, __ATOMIC_RELAXED);
    if (v < 0) {
        const char *t = getenv("H264MI_TEST");
        v = t && atoi(t) == 1;
        __atomic_store_n(&cached, v, __ATOMIC_RELAXED);
    }
    return v;
}

/* Frame-pipelined launches with whole-row waits (recon_kernels.hip
 * dep_wait_rows): per inter MB and 8x8 partition, the last MB row of its
 * reference slot that a 128-B line read by its motion compensation touches,
 * as four uint16 in MbRec.i4 (luma 9 rows x 12 bytes per 4x4 block, chroma 3
 * rows x 8 bytes per 2x2 block and plane, windows clamped as in the kernel's
 * mc_issue).  Slot layout H264MI_SLOT_BYTES: no line crosses a plane
 * boundary, chroma lines hold one row; a luma line can reach into the next
 * row (w % 8 != 0), so the row is that of the line's last byte.  The
 * column-granular mode (dep_wait_cols) takes the geometry in the kernel. */
static int line_row(long long last, long long pbase, long long pbytes, int pitch, int mbh)
{
    long long le = last | 127;
    if (le > pbase + pbytes - 1) le = pbase + pbytes - 1;
    return (int)((le - pbase) / pitch) / mbh;
}

static int clampi(int lo, int hi, int v) { return v < lo ? lo : v > hi ? hi : v; }

static void set_ref_rows(MbRec *recs, int w, int h)
{
    static const int bx[16] = {0, 1, 0, 1, 2, 3, 2, 3, 0, 1, 0, 1, 2, 3, 2, 3};
    static const int by[16] = {0, 0, 1, 1, 0, 0, 1, 1, 2, 2, 3, 3, 2, 2, 3, 3};
    const int W16 = w * 16, H16 = h * 16, CW = W16 / 2, CH = H16 / 2, CP = H264MI_CPITCH(w);
    const long long ysz = (long long)W16 * H16, csz = (long long)CP * CH;
    for (int mb = 0; mb < w * h; mb++) {
        MbRec *r = &recs[mb];
        if (r->type != MBT_INTER && r->type != MBT_SKIP) continue;
        const int mbx = mb % w, mby = mb / w;
        uint16_t rows[4] = {0, 0, 0, 0};
        for (int b = 0; b < 16; b++) {
            const int mvx = r->mv[b][0], mvy = r->mv[b][1];
            const int lax = clampi(0, W16 - 12, (mbx * 16 + bx[b] * 4 + (mvx >> 2) - 2) & ~3);
            const int ly = clampi(0, H16 - 1, mby * 16 + by[b] * 4 + (mvy >> 2) - 2 + 8);
            int n = line_row((long long)ly * W16 + lax + 11, 0, ysz, W16, 16);
            const int cax = clampi(0, CW - 8, (mbx * 8 + bx[b] * 2 + (mvx >> 3)) & ~3);
            const int cy = clampi(0, CH - 1, mby * 8 + by[b] * 2 + (mvy >> 3) + 2);
            for (int comp = 0; comp < 2; comp++) {
                const long long pb = ysz + comp * csz;
                const int nc = line_row(pb + (long long)cy * CP + cax + 7, pb, csz, CP, 8);
                if (nc > n) n = nc;
            }
            if (n > rows[b >> 2]) rows[b >> 2] = (uint16_t)n;
        }
        memcpy(r->i4, rows, 8);
    }
}

static int cap_decode(void *vctx, const PicBuild *pb, int cur_slot)
{
    struct h264mi_capture *c = (struct h264mi_capture *)vctx;
    if (c->npics == c->pic_cap) {
        c->pic_cap = c->pic_cap ? c->pic_cap * 2 : 64;
        CapPic *np = (CapPic *)realloc(c->pics, sizeof(CapPic) * (size_t)c->pic_cap);
        if (!np) return -1;
        c->pics = np;
    }
    size_t nmbs = (size_t)pb->nmbs;
    if (c->nrec + nmbs > c->rec_cap) {
        size_t nc = c->rec_cap ? c->rec_cap * 2 : nmbs * 16;
        while (nc < c->nrec + nmbs) nc *= 2;
        MbRec *nr = (MbRec *)realloc(c->recs, sizeof(MbRec) * nc);
        if (!nr) return -1;
        c->recs = nr;
        c->rec_cap = nc;
    }
    if (c->ncoef + pb->ncoef > c->coef_cap) {
        size_t nc = c->coef_cap ? c->coef_cap * 2 : (size_t)pb->ncoef * 16 + 1024;
        while (nc < c->ncoef + pb->ncoef) nc *= 2;
        int16_t *ncf = (int16_t *)realloc(c->coefs, nc * 32);
        if (!ncf) return -1;
        c->coefs = ncf;
        c->coef_cap = nc;
    }
    CapPic *p = &c->pics[c->npics++];
    p->rec_off = c->nrec;
    p->coef_off = c->ncoef;
    p->ncoef = pb->ncoef;
    p->cur_slot = cur_slot;
    p->alg_ref_bytes = pb->alg_ref_bytes;
    p->n_inter = pb->n_inter;
    p->n_intra = pb->n_intra;
    p->n_coded = pb->n_coded_blocks;
    memcpy(c->recs + c->nrec, pb->rec, sizeof(MbRec) * nmbs);
    set_ref_rows(c->recs + c->nrec, c->w, c->h);
    p->ref_line_bytes = ref_line_bytes(c->recs + c->nrec, c->w, c->h);
    if (pb->ncoef) memcpy(c->coefs + c->ncoef * 16, pb->coef, (size_t)pb->ncoef * 32);
    c->nrec += nmbs;
    c->ncoef += pb->ncoef;
    return 0;
}

/* Distinct 128-B lines of the reference slots that k_wgpp's MC loads touch
 * for one picture, times 128: the line-granular (compulsory) part of its
 * reference traffic, beside R_alg's bytes actually used (part_bytes).  The
 * windows are mc_issue's (recon_kernels.hip): per 4x4 luma block 9 rows of
 * 12 bytes from (x0 & ~3) clamped to [0, W16 - 12], per 2x2 chroma block and
 * component 3 rows of 8 bytes from (x0 & ~3) clamped to [0, CW - 8], rows
 * clamped to the plane, chroma rows CP = H264MI_CPITCH apart.  Slots are
 * H264MI_SLOT_BYTES apart, a multiple of 128, so line ids never straddle
 * slots. */
static uint64_t ref_line_bytes(const MbRec *rec, int w, int h)
{
    const int W16 = w * 16, H16 = h * 16, CW = W16 / 2, CH = H16 / 2, CP = H264MI_CPITCH(w);
    const size_t lines = H264MI_SLOT_BYTES(w, h) / 128;
    int maxslot = -1;
    for (int i = 0; i < w * h; i++)
        if (rec[i].type == MBT_INTER || rec[i].type == MBT_SKIP)
            for (int k = 0; k < 4; k++) maxslot = rec[i].ref[k] > maxslot ? rec[i].ref[k] : maxslot;
    if (maxslot < 0) return 0;
    uint8_t *mark = (uint8_t *)calloc((size_t)(maxslot + 1) * lines, 1);
    if (!mark) return 0;
    uint64_t n = 0;
#define MARK(slot, off, len) do {                                                   \
        const size_t a_ = (off) / 128, b_ = ((off) + (len) - 1) / 128;             \
        for (size_t l_ = a_; l_ <= b_; l_++) {                                     \
            uint8_t *m_ = mark + (size_t)(slot) * lines + l_;                      \
            if (!*m_) { *m_ = 1; n++; }                                            \
        }                                                                          \
    } while (0)
    for (int i = 0; i < w * h; i++) {
        const MbRec *r = &rec[i];
        if (r->type != MBT_INTER && r->type != MBT_SKIP) continue;
        const int mbx = i % w, mby = i / w;
        for (int b = 0; b < 16; b++) {
            const int bx = ((b >> 2) & 1) * 2 + (b & 1), by = ((b >> 3) & 1) * 2 + ((b >> 1) & 1);
            const int slot = r->ref[b >> 2];
            const int mvx = r->mv[b][0], mvy = r->mv[b][1];
            int x0 = mbx * 16 + bx * 4 + (mvx >> 2) - 2, y0 = mby * 16 + by * 4 + (mvy >> 2) - 2;
            int ax = x0 & ~3;
            ax = ax < 0 ? 0 : ax > W16 - 12 ? W16 - 12 : ax;
            for (int k = 0; k < 9; k++) {
                int y = y0 + k;
                y = y < 0 ? 0 : y > H16 - 1 ? H16 - 1 : y;
                MARK(slot, (size_t)y * W16 + ax, 12);
            }
            int cx0 = mbx * 8 + bx * 2 + (mvx >> 3), cy0 = mby * 8 + by * 2 + (mvy >> 3);
            int cax = cx0 & ~3;
            cax = cax < 0 ? 0 : cax > CW - 8 ? CW - 8 : cax;
            for (int comp = 0; comp < 2; comp++)
                for (int k = 0; k < 3; k++) {
                    int y = cy0 + k;
                    y = y < 0 ? 0 : y > CH - 1 ? CH - 1 : y;
                    MARK(slot, (size_t)W16 * H16 + (size_t)comp * CP * CH + (size_t)y * CP + cax, 8);
                }
        }
    }
#undef MARK
    free(mark);
    return n * 128;
}

static int cap_read(void *vctx, int slot, uint8_t *dst)
{
    struct h264mi_capture *c = (struct h264mi_capture *)vctx;
    (void)slot;
    memset(dst, 0, (size_t)c->w * c->h * 384);
    return 0;
}

static int cap_copy(void *vctx, int dst, int src) { (void)vctx; (void)dst; (void)src; return 0; }
static void cap_destroy(void *vctx) { (void)vctx; }

h264mi_capture *h264mi_capture_stream(const uint8_t *buf, size_t len, int no_reorder)
{
    h264mi_capture *c = (h264mi_capture *)calloc(1, sizeof(*c));
    H264Dec *d = (H264Dec *)calloc(1, sizeof(H264Dec));
    if (!c || !d) { free(c); free(d); return NULL; }
    H264Backend be;
    memset(&be, 0, sizeof(be));
    be.ctx = c;
    be.configure = cap_configure;
    be.decode = cap_decode;
    be.read = cap_read;
    be.copy = cap_copy;
    be.destroy = cap_destroy;
    h264dec_init(d, no_reorder, be);
    const uint8_t *p = buf;
    uint32_t left = (uint32_t)len, pic_id = 0;
    while (left > 0) {
        uint32_t rb = 0;
        int r = h264dec_decode(d, p, left, pic_id, &rb);
        if (r == DEC_PIC_RDY) pic_id++;
        if (r == DEC_ERROR || r == DEC_PARAM_SET_ERROR) c->errors++;
        if (r == DEC_PIC_RDY || r == DEC_HDRS_RDY)
            while (h264dec_next_output(d, NULL, NULL, NULL)) {}
        if (rb > left) rb = left;
        p += rb;
        left -= rb;
    }
    h264dec_release(d);
    free(d);
    return c;
}

int h264mi_capture_info(const h264mi_capture *c, int *w_mbs, int *h_mbs, int *nslots, int *npics, int *errors)
{
    if (!c) return -1;
    if (w_mbs) *w_mbs = c->w;
    if (h_mbs) *h_mbs = c->h;
    if (nslots) *nslots = c->nslots;
    if (npics) *npics = c->npics;
    if (errors) *errors = c->errors + (c->reconfigured ? 1 : 0);
    return 0;
}

int h264mi_capture_picture(const h264mi_capture *c, int i, const void **rec, const int16_t **coef,
                           uint32_t *ncoef, int *cur_slot, uint64_t *alg_ref_bytes)
{
    if (!c || i < 0 || i >= c->npics) return -1;
    const CapPic *p = &c->pics[i];
    if (rec) *rec = c->recs + p->rec_off;
    if (coef) *coef = c->coefs + p->coef_off * 16;
    if (ncoef) *ncoef = p->ncoef;
    if (cur_slot) *cur_slot = p->cur_slot;
    if (alg_ref_bytes) *alg_ref_bytes = p->alg_ref_bytes;
    return 0;
}

int h264mi_capture_ref_lines(const h264mi_capture *c, int i, uint64_t *ref_line_bytes)
{
    if (!c || i < 0 || i >= c->npics || !ref_line_bytes) return -1;
    *ref_line_bytes = c->pics[i].ref_line_bytes;
    return 0;
}

int h264mi_capture_stats(const h264mi_capture *c, int i, uint32_t *n_inter, uint32_t *n_intra, uint32_t *n_coded)
{
    if (!c || i < 0 || i >= c->npics) return -1;
    const CapPic *p = &c->pics[i];
    *n_inter = p->n_inter; *n_intra = p->n_intra; *n_coded = p->n_coded;
    return 0;
}

void h264mi_capture_free(h264mi_capture *c)
{
    if (!c) return;
    free(c->recs); free(c->coefs); free(c->pics);
    free(c);
}
