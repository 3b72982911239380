/* ORACLE -- TEST INFRASTRUCTURE ONLY.
 * ctypes-friendly entry points of liboracle.so for tests/ and bench.py's
 * cpu_baseline leg.  Decodes a whole Annex-B buffer the way the reference
 * testbench does (DecTestBench.c:230-410: drain NextPicture after every
 * PIC_RDY, flush at end) with the CPU restatement of the reconstruction. */
#include "recon_cpu.h"

#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef struct OracleOut {
    uint8_t *data;
    size_t   len, cap;
    int      npics, errors;
    int      w, h;
    int     *info;           /* per output picture: pic_id, is_idr, err_mbs */
    int      info_cap;
} OracleOut;

static void out_append(OracleOut *o, const uint8_t *p, size_t n)
{
    if (o->len + n > o->cap) {
        size_t nc = o->cap ? o->cap * 2 : (n * 8);
        while (nc < o->len + n) nc *= 2;
        o->data = (uint8_t *)realloc(o->data, nc);
        o->cap = nc;
    }
    memcpy(o->data + o->len, p, n);
    o->len += n;
}

static void drain(H264Dec *d, OracleOut *o)
{
    const uint8_t *pic;
    uint32_t id, idr, em;
    while ((pic = h264dec_next_output(d, &id, &idr, &em)) != NULL) {
        out_append(o, pic, d->frame_bytes);
        if (o->npics >= o->info_cap) {
            o->info_cap = o->info_cap ? o->info_cap * 2 : 64;
            o->info = (int *)realloc(o->info, sizeof(int) * 3 * (size_t)o->info_cap);
        }
        o->info[3 * o->npics] = (int)id;
        o->info[3 * o->npics + 1] = (int)idr;
        o->info[3 * o->npics + 2] = (int)em;
        o->npics++;
        o->errors += (int)em;
    }
}

/* Decode buf; returns an opaque result (frames concatenated, I420 MB-aligned). */
void *oracle_decode_stream(const uint8_t *buf, size_t len, int no_reorder, double *seconds)
{
    /* DecTestBench feeds the whole remaining buffer and passes
     * intraConcealmentMethod = 0 (DecTestBench.c:211) */
    OracleOut *o = (OracleOut *)calloc(1, sizeof(OracleOut));
    H264Dec *d = (H264Dec *)calloc(1, sizeof(H264Dec));
    if (!o || !d) { free(o); free(d); return NULL; }
    h264dec_init(d, no_reorder, oracle_backend_create());
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    const uint8_t *p = buf;
    uint32_t left = (uint32_t)len, pic_id = 1;   /* picDecodeNumber starts at 1 (DecTestBench.c:218) */
    while (left > 0) {
        uint32_t rb = 0;
        int r = h264dec_decode(d, p, left, pic_id, &rb);
        if (r == DEC_PIC_RDY) pic_id++;
        if (r == DEC_ERROR || r == DEC_PARAM_SET_ERROR) o->errors++;
        if (r == DEC_PIC_RDY || r == DEC_HDRS_RDY) drain(d, o);
        if (rb > left) rb = left;
        p += rb;
        left -= rb;
    }
    h264dec_flush(d);
    drain(d, o);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (seconds) *seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    const Sps *s = h264dec_active_sps(d);
    if (s) { o->w = s->w_mbs * 16; o->h = s->h_mbs * 16; }
    h264dec_release(d);
    free(d);
    return o;
}

/* SoftAVC protocol (Decoder/SoftAVC.cpp:289-400): one input buffer per NAL
 * unit (start code included), picId counting input buffers, the buffer
 * re-fed until consumed, intraConcealmentMethod = intra_conceal
 * (SoftAVC.cpp:335 sets 1), NextPicture drained after every buffer and
 * flushed at end of stream. */
static size_t next_start(const uint8_t *b, size_t n, size_t from)
{
    for (size_t i = from; i + 3 < n; i++)
        if (b[i] == 0 && b[i + 1] == 0 && b[i + 2] == 1) return i > 0 && b[i - 1] == 0 ? i - 1 : i;
    return n;
}

/* host/api.c's H264SwDecDecode loop over the decoder core (the oracle has
 * no HIP backend, so api.c itself cannot link here): returns the
 * H264SwDecRet code, *consumed = bytes up to pStrmCurrPos */
enum { R_STRM_PROCESSED = 1, R_PIC_RDY = 2, R_PIC_RDY_BNE = 3, R_HDRS_RDY_BNE = 4, R_STRM_ERR = -2, R_MEMFAIL = -4 };
static int api_decode(H264Dec *d, int *new_headers, const uint8_t *p0, uint32_t len, uint32_t pic_id, uint32_t *consumed)
{
    int ret = R_STRM_PROCESSED;
    const uint8_t *p = p0;
    do {
        int r;
        uint32_t nread = 0;
        if (*new_headers) {
            r = DEC_HDRS_RDY;
            *new_headers = 0;
        } else {
            r = h264dec_decode(d, p, len, pic_id, &nread);
        }
        p += nread;
        len = ((int32_t)(len - nread) >= 0) ? len - nread : 0;
        switch (r) {
        case DEC_HDRS_RDY:
            if (d->dpb.flushed && d->dpb.num_out != d->dpb.out_index) {
                d->dpb.flushed = 0;
                *new_headers = 1;
                ret = R_PIC_RDY_BNE;
            } else {
                ret = R_HDRS_RDY_BNE;
            }
            len = 0;
            break;
        case DEC_PIC_RDY:
            ret = len == 0 ? R_PIC_RDY : R_PIC_RDY_BNE;
            len = 0;
            break;
        case DEC_PARAM_SET_ERROR:
            if (!h264dec_valid_param_sets(d) && len == 0) ret = R_STRM_ERR;
            break;
        case DEC_MEMALLOC_ERROR:
            ret = R_MEMFAIL;
            len = 0;
            break;
        default:
            break;
        }
    } while (len);
    *consumed = (uint32_t)(p - p0);
    return ret;
}

void *oracle_decode_stream_nals(const uint8_t *buf, size_t len, int intra_conceal, double *seconds)
{
    OracleOut *o = (OracleOut *)calloc(1, sizeof(OracleOut));
    H264Dec *d = (H264Dec *)calloc(1, sizeof(H264Dec));
    if (!o || !d) { free(o); free(d); return NULL; }
    h264dec_init(d, 0, oracle_backend_create());
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    uint32_t pic_id = 0;
    int new_headers = 0, headers = 0;
    size_t pos = next_start(buf, len, 0);
    while (pos < len) {
        const size_t end = next_start(buf, len, pos + 3);
        const uint8_t *p = buf + pos;
        uint32_t left = (uint32_t)(end - pos);
        pic_id++;
        while (left > 0) {
            uint32_t used = 0;
            d->intra_conceal = intra_conceal;
            const int r = api_decode(d, &new_headers, p, left, pic_id, &used);
            if (r == R_HDRS_RDY_BNE) headers = 1;
            if (r == R_HDRS_RDY_BNE || r == R_PIC_RDY_BNE) {
                p += used;
                left -= used < left ? used : left;
            } else {
                if (r < 0) o->errors++;
                left = 0;
            }
        }
        if (headers) drain(d, o);
        pos = end;
    }
    h264dec_flush(d);
    drain(d, o);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (seconds) *seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    const Sps *s = h264dec_active_sps(d);
    if (s) { o->w = s->w_mbs * 16; o->h = s->h_mbs * 16; }
    h264dec_release(d);
    free(d);
    return o;
}

int oracle_result_info(void *res, int *npics, int *errors, int *w, int *h, size_t *bytes)
{
    OracleOut *o = (OracleOut *)res;
    if (!o) return -1;
    *npics = o->npics; *errors = o->errors; *w = o->w; *h = o->h; *bytes = o->len;
    return 0;
}

int oracle_result_copy(void *res, uint8_t *dst, size_t cap)
{
    OracleOut *o = (OracleOut *)res;
    if (!o || cap < o->len) return -1;
    memcpy(dst, o->data, o->len);
    return 0;
}

/* per output picture (pic_id, is_idr, nbrOfErrMBs), 3 ints each */
int oracle_result_pics(void *res, int *dst, int cap)
{
    OracleOut *o = (OracleOut *)res;
    if (!o || cap < 3 * o->npics) return -1;
    if (o->npics) memcpy(dst, o->info, sizeof(int) * 3 * (size_t)o->npics);
    return o->npics;
}

void oracle_result_free(void *res)
{
    OracleOut *o = (OracleOut *)res;
    if (!o) return;
    free(o->info);
    free(o->data);
    free(o);
}

/* Reconstruct a sequence of captured MB-record pictures (as produced by the
 * product's h264mi_capture_*) into CPU frame slots, for record-level parity
 * checks of the HIP kernels.  frames_out receives nslots*w*h*384 bytes. */
void *oracle_replay_create(int w_mbs, int h_mbs, int nslots) { return oracle_ctx_create(w_mbs, h_mbs, nslots); }
int oracle_replay_picture(void *ctx, const void *rec, const int16_t *coef, int w_mbs, int h_mbs, int cur_slot)
{
    return oracle_recon_picture(ctx, (const MbRec *)rec, coef, w_mbs, h_mbs, cur_slot);
}
const uint8_t *oracle_replay_frame(void *ctx, int slot) { return oracle_ctx_frame(ctx, slot); }
void oracle_replay_free(void *ctx) { oracle_ctx_destroy(ctx); }

/* I420 -> RGBA of Decoder.js's `rgb: true` output, restated from the
 * reference's asm.js converter: per pixel yuv2rgbcalc
 * (templates/DecoderPost.js:514-560) -- a0 = 1192 (y-16), R = (a0 + 1634
 * (v-128)) >> 10, G = (a0 - 832 (v-128) - 400 (u-128)) >> 10, B = (a0 + 2066
 * (u-128)) >> 10, each clamped to [0,255] (:541-549), stored as the word
 * 255 << 24 | B << 16 | G << 8 | R (:551-558) -- over the picture in 2x2
 * blocks sharing one (u, v) (doit, :420-505).  Plain scalar loops; the
 * (y, u, v) result cache of the reference changes no value. */
void oracle_yuv2rgba(const uint8_t *i420, int width, int height, uint8_t *rgba)
{
    const uint8_t *Y = i420, *U = i420 + (size_t)width * height;
    const uint8_t *V = U + (size_t)(width / 2) * (height / 2);
    for (int r = 0; r < height; r++)
        for (int c = 0; c < width; c++) {
            const int y = Y[(size_t)r * width + c];
            const int u = U[(size_t)(r / 2) * (width / 2) + c / 2] - 128;
            const int v = V[(size_t)(r / 2) * (width / 2) + c / 2] - 128;
            const int a0 = 1192 * (y - 16);
            int R = (a0 + 1634 * v) >> 10, G = (a0 - 832 * v - 400 * u) >> 10, B = (a0 + 2066 * u) >> 10;
            R = R < 0 ? 0 : R > 255 ? 255 : R;
            G = G < 0 ? 0 : G > 255 ? 255 : G;
            B = B < 0 ? 0 : B > 255 ? 255 : B;
            uint8_t *o = rgba + ((size_t)r * width + c) * 4;
            o[0] = (uint8_t)R; o[1] = (uint8_t)G; o[2] = (uint8_t)B; o[3] = 255;
        }
}
