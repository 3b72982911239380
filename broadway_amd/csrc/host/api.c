/* Broadway decoder API (H264SwDec*) and wasm/JS glue (broadway*) on top of
 * the host decoder + HIP reconstruction backend.
 *
 * H264SwDec*: same structures, return codes and call protocol as the
 * reference Decoder/src/H264SwDecApi.c (Init :124-180, GetInfo :204-257,
 * Release :259-290, Decode :338-473, GetAPIVersion :487-500,
 * NextPicture :524-569).  broadway*: same behaviour as Decoder/src/Decoder.c
 * (playStream loop :44-53, broadwayDecode :100-162 incl. dropping the rest of
 * the buffer after a picture, :122-134), with the emscripten imports
 * broadwayOnHeadersDecoded / broadwayOnPictureDecoded delivered through
 * callbacks registered by broadwaySetCallbacks.
 *
 * The product path has no CPU reconstruction: if the HIP backend cannot be
 * created the API fails (H264SWDEC_INITFAIL / MEMFAIL) instead of falling
 * back. */
#include "../../../include/h264mi.h"
#include "decoder.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

H264Backend h264mi_hip_backend_create(int device);

/* ---- application hooks (reference inc/H264SwDecApi.h:160-173) ----------
 * The library allocates and frees its instances through H264SwDecMalloc /
 * H264SwDecFree and fills them with H264SwDecMemset, as H264SwDecApi.c:147,
 * :301 does; H264SwDecTrace receives the API trace strings when built with
 * -DH264DEC_TRACE (H264SwDecApi.c:66-72).  These are the reference's default
 * definitions (H264SwDecApi.c:78-96): an application that defines its own
 * (DecTestBench.c:678-760, TestBenchMultipleInstance.c:396-446) overrides them
 * by ordinary ELF symbol interposition -- the library calls them through its
 * PLT. */
void H264SwDecTrace(char *string) { (void)string; }
void *H264SwDecMalloc(u32 size) { return malloc(size); }
void H264SwDecFree(void *ptr) { free(ptr); }
void H264SwDecMemcpy(void *dest, void *src, u32 count) { memcpy(dest, src, count); }
void H264SwDecMemset(void *ptr, i32 value, u32 count) { memset(ptr, value, count); }

#ifdef H264DEC_TRACE
#define DEC_API_TRC(str) H264SwDecTrace((char *)(str))
#else
#define DEC_API_TRC(str) ((void)0)
#endif

enum { ST_UNINIT = 0, ST_INIT = 1, ST_NEW_HEADERS = 2 };

typedef struct DecContainer {
    H264Dec dec;
    int     stat;
    u32     pic_number;
} DecContainer;

static int backend_device(void)
{
    const char *s = getenv("H264MI_DEVICE");
    return s ? atoi(s) : 0;
}

H264SwDecRet H264SwDecInit(H264SwDecInst *decInst, u32 noOutputReordering)
{
    DEC_API_TRC("H264SwDecInit#");
    if (decInst == NULL) {
        DEC_API_TRC("H264SwDecInit# ERROR: decInst == NULL");
        return H264SWDEC_PARAM_ERR;
    }
    *decInst = NULL;
    DecContainer *c = (DecContainer *)H264SwDecMalloc((u32)sizeof(DecContainer));
    if (!c) {
        DEC_API_TRC("H264SwDecInit# ERROR: Memory allocation failed");
        return H264SWDEC_MEMFAIL;
    }
    H264SwDecMemset(c, 0, (u32)sizeof(DecContainer));
    H264Backend be = h264mi_hip_backend_create(backend_device());
    if (!be.ctx) { H264SwDecFree(c); return H264SWDEC_MEMFAIL; }
    if (h264dec_init(&c->dec, (int)noOutputReordering, be)) {
        be.destroy(be.ctx);
        H264SwDecFree(c);
        return H264SWDEC_INITFAIL;
    }
    c->stat = ST_INIT;
    *decInst = c;
    DEC_API_TRC("H264SwDecInit# OK");
    return H264SWDEC_OK;
}

H264SwDecRet H264SwDecGetInfo(H264SwDecInst decInst, H264SwDecInfo *pDecInfo)
{
    DEC_API_TRC("H264SwDecGetInfo#");
    if (decInst == NULL || pDecInfo == NULL) return H264SWDEC_PARAM_ERR;
    DecContainer *c = (DecContainer *)decInst;
    const Sps *s = h264dec_active_sps(&c->dec);
    if (!s || c->dec.active_pps < 0 || c->dec.active_pps >= MAX_PPS) return H264SWDEC_HDRS_NOT_RDY;
    memset(pDecInfo, 0, sizeof(*pDecInfo));
    pDecInfo->picWidth = (u32)s->w_mbs << 4;
    pDecInfo->picHeight = (u32)s->h_mbs << 4;
    pDecInfo->videoRange = (s->vui_present && s->video_full_range) ? 1 : 0;
    pDecInfo->matrixCoefficients = (s->vui_present && s->colour_desc_present) ? (u32)s->matrix_coeffs : 2;
    if (s->crop) {
        pDecInfo->croppingFlag = 1;
        pDecInfo->cropParams.cropLeftOffset = 2u * (u32)s->crop_l;
        pDecInfo->cropParams.cropOutWidth = 16u * (u32)s->w_mbs - 2u * (u32)(s->crop_l + s->crop_r);
        pDecInfo->cropParams.cropTopOffset = 2u * (u32)s->crop_t;
        pDecInfo->cropParams.cropOutHeight = 16u * (u32)s->h_mbs - 2u * (u32)(s->crop_t + s->crop_b);
    }
    u32 w = 1, h = 1;
    if (s->vui_present && s->aspect_present) {
        static const u8 sar[17][2] = {{0, 0}, {1, 1}, {12, 11}, {10, 11}, {16, 11}, {40, 33}, {24, 11},
                                      {20, 11}, {32, 11}, {80, 33}, {18, 11}, {15, 11}, {64, 33},
                                      {160, 99}, {0, 0}, {0, 0}, {0, 0}};
        if (s->aspect_idc == 255) {
            w = (u32)s->sar_w; h = (u32)s->sar_h;
            if (!w || !h) w = h = 0;
        } else if (s->aspect_idc < 14) {
            w = sar[s->aspect_idc][0]; h = sar[s->aspect_idc][1];
        } else {
            w = h = 0;
        }
    }
    pDecInfo->parWidth = w;
    pDecInfo->parHeight = h;
    pDecInfo->profile = (u32)s->profile_idc;
    return H264SWDEC_OK;
}

void H264SwDecRelease(H264SwDecInst decInst)
{
    if (!decInst) return;
    DEC_API_TRC("H264SwDecRelease#");
    DecContainer *c = (DecContainer *)decInst;
    h264dec_release(&c->dec);
    H264SwDecFree(c);
}

H264SwDecRet H264SwDecDecode(H264SwDecInst decInst, H264SwDecInput *pInput, H264SwDecOutput *pOutput)
{
    DEC_API_TRC("H264SwDecDecode#");
    if (pInput == NULL || pOutput == NULL) return H264SWDEC_PARAM_ERR;
    if (pInput->pStream == NULL || pInput->dataLen == 0) return H264SWDEC_PARAM_ERR;
    DecContainer *c = (DecContainer *)decInst;
    if (decInst == NULL || c->stat == ST_UNINIT) return H264SWDEC_NOT_INITIALIZED;

    H264SwDecRet ret = H264SWDEC_STRM_PROCESSED;
    u32 len = pInput->dataLen;
    u8 *p = pInput->pStream;
    pOutput->pStrmCurrPos = NULL;
    c->dec.intra_conceal = (int)pInput->intraConcealmentMethod;
    do {
        int r;
        uint32_t nread = 0;
        if (c->stat == ST_NEW_HEADERS) {
            r = DEC_HDRS_RDY;
            c->stat = ST_INIT;
        } else {
            r = h264dec_decode(&c->dec, p, len, pInput->picId, &nread);
        }
        p += nread;
        len = ((int32_t)(len - nread) >= 0) ? len - nread : 0;
        pOutput->pStrmCurrPos = p;
        switch (r) {
        case DEC_HDRS_RDY:
            if (c->dec.dpb.flushed && c->dec.dpb.num_out != c->dec.dpb.out_index) {
                c->dec.dpb.flushed = 0;
                c->stat = ST_NEW_HEADERS;
                ret = H264SWDEC_PIC_RDY_BUFF_NOT_EMPTY;
            } else {
                ret = H264SWDEC_HDRS_RDY_BUFF_NOT_EMPTY;
            }
            len = 0;
            break;
        case DEC_PIC_RDY:
            c->pic_number++;
            ret = len == 0 ? H264SWDEC_PIC_RDY : H264SWDEC_PIC_RDY_BUFF_NOT_EMPTY;
            len = 0;
            break;
        case DEC_PARAM_SET_ERROR:
            if (!h264dec_valid_param_sets(&c->dec) && len == 0) ret = H264SWDEC_STRM_ERR;
            break;
        case DEC_MEMALLOC_ERROR:
            ret = H264SWDEC_MEMFAIL;
            len = 0;
            break;
        default:
            break;
        }
    } while (len);
    return ret;
}

H264SwDecApiVersion H264SwDecGetAPIVersion(void)
{
    H264SwDecApiVersion v;
    v.major = 2;
    v.minor = 3;
    return v;
}

H264SwDecRet H264SwDecNextPicture(H264SwDecInst decInst, H264SwDecPicture *pOutput, u32 flushBuffer)
{
    DEC_API_TRC("H264SwDecNextPicture#");
    if (decInst == NULL || pOutput == NULL) return H264SWDEC_PARAM_ERR;
    DecContainer *c = (DecContainer *)decInst;
    if (flushBuffer) h264dec_flush(&c->dec);
    uint32_t id, idr, em;
    const uint8_t *pic = h264dec_next_output(&c->dec, &id, &idr, &em);
    if (!pic) return H264SWDEC_OK;
    pOutput->pOutputPicture = (u32 *)(void *)pic;
    pOutput->picId = id;
    pOutput->isIdrPicture = idr;
    pOutput->nbrOfErrMBs = em;
    return H264SWDEC_PIC_RDY;
}

/* NextPicture with the picture converted to RGBA on the GPU (Decoder.js
 * `rgb: true`, DecoderPost.js:82-97 + :420-560): rgba receives
 * picWidth * picHeight * 4 bytes and pOutputPicture points to it. */
H264SwDecRet H264SwDecNextPictureRGBA(H264SwDecInst decInst, H264SwDecPicture *pOutput, u32 flushBuffer, u8 *rgba)
{
    if (decInst == NULL || pOutput == NULL || rgba == NULL) return H264SWDEC_PARAM_ERR;
    DecContainer *c = (DecContainer *)decInst;
    if (flushBuffer) h264dec_flush(&c->dec);
    uint32_t id, idr, em;
    const uint8_t *pic = h264dec_next_output_rgba(&c->dec, &id, &idr, &em, rgba);
    if (!pic) return H264SWDEC_OK;
    pOutput->pOutputPicture = (u32 *)(void *)pic;
    pOutput->picId = id;
    pOutput->isIdrPicture = idr;
    pOutput->nbrOfErrMBs = em;
    return H264SWDEC_PIC_RDY;
}

H264SwDecRet H264SwDecGetTiming(H264SwDecInst decInst, double *parse_s, double *submit_s, double *wait_s,
                                double *copy_s, u32 *pictures)
{
    if (decInst == NULL) return H264SWDEC_PARAM_ERR;
    const DecContainer *c = (const DecContainer *)decInst;
    if (parse_s) *parse_s = c->dec.t_parse;
    if (submit_s) *submit_s = c->dec.t_submit;
    if (wait_s) *wait_s = c->dec.t_wait;
    if (copy_s) *copy_s = c->dec.t_copy;
    if (pictures) *pictures = (u32)c->dec.n_output;
    return H264SWDEC_OK;
}

/* ------------------------------------------------------------------------ */
/* wasm / JS glue (Decoder.c): one global instance per process               */
/* ------------------------------------------------------------------------ */
static H264SwDecInst g_inst;
static H264SwDecInput g_in;
static H264SwDecOutput g_out;
static H264SwDecPicture g_pic;
static H264SwDecInfo g_info;
static u32 g_pic_decode, g_pic_display;
static struct { u32 length; u8 *buffer; } g_stream;
static broadway_headers_cb g_on_headers;
static broadway_picture_cb g_on_picture;
static void *g_user;

void broadwaySetCallbacks(broadway_headers_cb on_headers, broadway_picture_cb on_picture, void *user)
{
    g_on_headers = on_headers;
    g_on_picture = on_picture;
    g_user = user;
}

u32 broadwayInit(void)
{
    if (H264SwDecInit(&g_inst, 0) != H264SWDEC_OK) {
        fprintf(stderr, "DECODER INITIALIZATION FAILED\n");
        broadwayExit();
        return (u32)-1;
    }
    g_pic_decode = g_pic_display = 1;
    return 0;
}

u8 *broadwayCreateStream(u32 length)
{
    free(g_stream.buffer);
    g_stream.buffer = (u8 *)malloc(length ? length : 1);
    g_stream.length = length;
    return g_stream.buffer;
}

static u32 broadway_decode(void)
{
    g_in.picId = g_pic_decode;
    H264SwDecRet ret = H264SwDecDecode(g_inst, &g_in, &g_out);
    switch ((int)ret) {
    case H264SWDEC_HDRS_RDY_BUFF_NOT_EMPTY:
        if (H264SwDecGetInfo(g_inst, &g_info) != H264SWDEC_OK) return (u32)-1;
        if (g_on_headers) g_on_headers(g_user);
        g_in.dataLen -= (u32)(g_out.pStrmCurrPos - g_in.pStream);
        g_in.pStream = g_out.pStrmCurrPos;
        break;
    case H264SWDEC_PIC_RDY_BUFF_NOT_EMPTY:
        g_in.dataLen -= (u32)(g_out.pStrmCurrPos - g_in.pStream);
        g_in.pStream = g_out.pStrmCurrPos;
        /* fall through */
    case H264SWDEC_PIC_RDY:
        g_in.dataLen = 0;           /* Decoder.c:130: rest of the buffer is dropped */
        g_pic_decode++;
        while (H264SwDecNextPicture(g_inst, &g_pic, 0) == H264SWDEC_PIC_RDY) {
            g_pic_display++;
            if (g_on_picture) g_on_picture(g_user, (u8 *)g_pic.pOutputPicture, g_info.picWidth, g_info.picHeight);
        }
        break;
    case H264SWDEC_STRM_PROCESSED:
    case H264SWDEC_STRM_ERR:
        g_in.dataLen = 0;
        break;
    default:
        break;
    }
    return (u32)ret;
}

void broadwayPlayStream(u32 length)
{
    g_stream.length = length;
    g_in.pStream = g_stream.buffer;
    g_in.dataLen = length;
    do {
        broadway_decode();
    } while (g_in.dataLen > 0);
}

void broadwayExit(void)
{
    if (g_inst) H264SwDecRelease(g_inst);
    g_inst = NULL;
    free(g_stream.buffer);
    g_stream.buffer = NULL;
}

u32 broadwayGetMajorVersion(void) { return H264SwDecGetAPIVersion().major; }
u32 broadwayGetMinorVersion(void) { return H264SwDecGetAPIVersion().minor; }
