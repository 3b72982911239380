/* h264mi -- MI355X-native H.264 Baseline macroblock-reconstruction engine.
 *
 * C-ABI of libh264mi.so (plain pointers and sizes only).  Three layers:
 *
 * 1. The Broadway decoder API (drop-in for Decoder/inc/H264SwDecApi.h):
 *    H264SwDecInit / Decode / NextPicture / GetInfo / Release /
 *    GetAPIVersion with the same structures, return codes and call
 *    protocol.  Replaces reference H264SwDecApi.c:124-569.
 * 2. The wasm/JS glue API (drop-in for Decoder/src/Decoder.c:44-185):
 *    broadwayInit / broadwayCreateStream / broadwayPlayStream / broadwayExit /
 *    broadwayGetMajorVersion / broadwayGetMinorVersion, calling back into
 *    broadwayOnHeadersDecoded / broadwayOnPictureDecoded, which the embedder
 *    registers with broadwaySetCallbacks (the emscripten library.js:1-13
 *    bridge becomes a function-pointer registration).
 * 3. The batched engine API used for multi-stream throughput (one picture
 *    from each of S streams per launch): h264mi_engine_*.
 *    This is the hot path the reference has no equivalent for; its unit of
 *    work is the MB-record batch of include/h264mi_records.h.
 */
#ifndef H264MI_H
#define H264MI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------------- */
/* 1. H264SwDec API  (reference Decoder/inc/H264SwDecApi.h:53-173)         */
/* ---------------------------------------------------------------------- */
typedef uint8_t  u8;
typedef uint32_t u32;
typedef int32_t  i32;

typedef enum {
    H264SWDEC_OK = 0,
    H264SWDEC_STRM_PROCESSED = 1,
    H264SWDEC_PIC_RDY,
    H264SWDEC_PIC_RDY_BUFF_NOT_EMPTY,
    H264SWDEC_HDRS_RDY_BUFF_NOT_EMPTY,
    H264SWDEC_PARAM_ERR = -1,
    H264SWDEC_STRM_ERR = -2,
    H264SWDEC_NOT_INITIALIZED = -3,
    H264SWDEC_MEMFAIL = -4,
    H264SWDEC_INITFAIL = -5,
    H264SWDEC_HDRS_NOT_RDY = -6,
    H264SWDEC_EVALUATION_LIMIT_EXCEEDED = -7
} H264SwDecRet;

typedef void *H264SwDecInst;

typedef struct {
    u8  *pStream;
    u32  dataLen;
    u32  picId;
    u32  intraConcealmentMethod;
} H264SwDecInput;

typedef struct {
    u8  *pStrmCurrPos;
} H264SwDecOutput;

typedef struct {
    u32 *pOutputPicture;     /* planar I420, picWidth*picHeight*3/2 bytes */
    u32 picId;
    u32 isIdrPicture;
    u32 nbrOfErrMBs;
} H264SwDecPicture;

typedef struct {
    u32 cropLeftOffset;
    u32 cropOutWidth;
    u32 cropTopOffset;
    u32 cropOutHeight;
} CropParams;

typedef struct {
    u32 profile;
    u32 picWidth;            /* MB-aligned, pixels */
    u32 picHeight;
    u32 videoRange;
    u32 matrixCoefficients;
    u32 parWidth;
    u32 parHeight;
    u32 croppingFlag;
    CropParams cropParams;
} H264SwDecInfo;

typedef struct {
    u32 major;
    u32 minor;
} H264SwDecApiVersion;

H264SwDecRet H264SwDecInit(H264SwDecInst *decInst, u32 noOutputReordering);   /* H264SwDecApi.c:124 */
H264SwDecRet H264SwDecDecode(H264SwDecInst decInst, H264SwDecInput *pInput,
                             H264SwDecOutput *pOutput);                          /* :338 */
H264SwDecRet H264SwDecNextPicture(H264SwDecInst decInst, H264SwDecPicture *pOutput,
                                  u32 endOfStream);                              /* :524 */
H264SwDecRet H264SwDecGetInfo(H264SwDecInst decInst, H264SwDecInfo *pDecInfo);  /* :204 */
void H264SwDecRelease(H264SwDecInst decInst);                                    /* :259 */
H264SwDecApiVersion H264SwDecGetAPIVersion(void);                                /* :487 */
/* NextPicture, the picture converted to RGBA on the GPU: what Decoder.js
 * delivers with `rgb: true` (templates/DecoderPost.js:82-97, the asm.js
 * converter :322-560, per pixel yuv2rgbcalc :514-560).  rgba: picWidth *
 * picHeight * 4 bytes; pOutput->pOutputPicture = rgba.  No reference C
 * counterpart: the reference converts in JavaScript. */
H264SwDecRet H264SwDecNextPictureRGBA(H264SwDecInst decInst, H264SwDecPicture *pOutput, u32 flushBuffer, u8 *rgba);

/* ---------------------------------------------------------------------- */
/* 2. Broadway glue (reference Decoder/src/Decoder.c:44-185, make.py:39)   */
/* ---------------------------------------------------------------------- */
typedef void (*broadway_headers_cb)(void *user);
typedef void (*broadway_picture_cb)(void *user, u8 *buffer, u32 width, u32 height);

void broadwaySetCallbacks(broadway_headers_cb on_headers, broadway_picture_cb on_picture, void *user);
u32  broadwayInit(void);                    /* Decoder.c:178 */
u8  *broadwayCreateStream(u32 length);      /* Decoder.c:58  */
void broadwayPlayStream(u32 length);        /* Decoder.c:67  */
void broadwayExit(void);                    /* Decoder.c:88  */
u32  broadwayGetMajorVersion(void);         /* Decoder.c:164 */
u32  broadwayGetMinorVersion(void);         /* Decoder.c:169 */

/* ---------------------------------------------------------------------- */
/* 3. Batched reconstruction engine (MI355X hot path)                      */
/* ---------------------------------------------------------------------- */
typedef struct h264mi_engine h264mi_engine;

/* Reconstruction engine for `nstreams` independent streams of one size
 * (w_mbs x h_mbs macroblocks), each with `nslots` frame slots in HBM. */
h264mi_engine *h264mi_engine_create(int device, int w_mbs, int h_mbs, int nstreams, int nslots);
void h264mi_engine_destroy(h264mi_engine *e);

/* Reconstruct one picture per listed stream (host-resident record batches):
 * recs[i] -> w*h MbRec (96 B each), coefs[i] -> ncoef[i] int16x16 blocks. */
int h264mi_engine_decode(h264mi_engine *e, int npics, const int *stream, const int *cur_slot,
                         const void *const *recs, const int16_t *const *coefs, const uint32_t *ncoef);

/* Device-resident variant (records already in HBM; kernel-only timing):
 * d_recs = npics*w*h MbRec in batch order with coefficient offsets relative
 * to d_coef, d_pics = npics PicDesc. */
int h264mi_engine_decode_device(h264mi_engine *e, int npics, const void *d_recs, const int16_t *d_coef,
                                const void *d_pics);

int  h264mi_engine_read(h264mi_engine *e, int stream, int slot, uint8_t *dst);   /* D2H I420 */
/* D2H of a slot as RGBA (w*16 * h*16 * 4 bytes), converted on the GPU
 * (DecoderPost.js yuv2rgbcalc :514-560 per pixel) */
int  h264mi_engine_read_rgba(h264mi_engine *e, int stream, int slot, uint8_t *dst);
/* the conversion kernel on device buffers: npics MB-aligned I420 pictures
 * of width x height (multiples of 16) at d_i420 + k * in_stride ->
 * d_rgba + k * out_stride; asynchronous on `hip_stream` (NULL: null stream) */
int  h264mi_yuv2rgba_device(const void *d_i420, void *d_rgba, int width, int height, int npics,
                            size_t in_stride, size_t out_stride, void *hip_stream);
int  h264mi_engine_sync(h264mi_engine *e);
/* number of (launch, picture) slots flagged since the last call: residual
 * range errors (reference transform.c:181) or a bounded wait that expired;
 * flags accumulate over every launch and are collected by h264mi_engine_sync */
uint32_t h264mi_engine_errors(h264mi_engine *e);
/* average duration (us) of the last batch's kernels: [0] k_mb, [1] k_rows */
int  h264mi_engine_last_timing(h264mi_engine *e, float *us2);
/* per-batch kernel timing with HIP events on the engine's stream:
 * record up to max_batches batches (0 disables); the report syncs and returns
 * the summed durations of k_mb and of k_rows, in microseconds */
int  h264mi_engine_set_timing(h264mi_engine *e, int max_batches);
/* time only every stride-th launch (the event markers between launches cost
 * the stream a few us each; default 1) */
int  h264mi_engine_set_timing_stride(h264mi_engine *e, int stride);
int  h264mi_engine_timing_report(h264mi_engine *e, double *inter_us, double *wave_us, int *nbatches);
/* frame-pipelined batches: one launch reconstructs `depth` consecutive
 * pictures of each of `nstreams` streams, and a picture's motion
 * compensation starts as soon as the reference samples it reads are final
 * (per-MB dependency tracking on the GPU).  set_pipeline sizes the
 * per-picture buffers (nstreams x depth).  d_pics: nstreams*depth PicDesc,
 * picture-major (k*nstreams + s).  Frame slots form a ring: picture k of
 * the launch writes slot (base_pic + k) mod nslots of its stream and record
 * ref[] fields name ring slots, so no picture of a launch overwrites a slot
 * another picture of the launch reads (nslots >= depth + reference span).
 * lag_rows: row k+1 of the launch's picture order trails by this many MB
 * rows; it must exceed every MV's reference reach in MB rows by 2 (the
 * caller computes it from the records; <= 0 = whole pictures in sequence). */
int  h264mi_engine_set_pipeline(h264mi_engine *e, int depth);
/* stream groups: decode_device batches are split into `ngroups` groups of
 * pictures, each reconstructed on its own HIP stream (k_mb then k_rows), so
 * one group's motion compensation overlaps the other groups' row kernels.
 * The groups are offset once (a short delay kernel) so that, with equal
 * per-picture cost, their k_mb phases stay apart.  The caller keeps
 * d_recs / d_coef / d_pics unchanged until h264mi_engine_sync.  1 = off. */
#define H264MI_MAX_GROUPS 8
int  h264mi_engine_set_groups(h264mi_engine *e, int ngroups);
int  h264mi_engine_decode_pipelined(h264mi_engine *e, int nstreams, int depth, const void *d_recs,
                                    const int16_t *d_coef, const void *d_pics, int base_pic, int lag_rows);
/* diagnostics: per k_rows workgroup (row r of batch picture p at index
 * r * npics + p) 16 u64: wall-clock start/end (100 MHz) and shader-clock sums
 * of its phases, then 4 u64 per MB (hand-off timestamps); enable != 0 allocates, out != NULL copies the last launch */
int  h264mi_engine_profile(h264mi_engine *e, int enable, unsigned long long *out, size_t n);
void *h264mi_engine_frame_ptr(h264mi_engine *e, int stream, int slot);          /* device pointer */
/* diagnostics: name of the last batch's reconstruction kernel ("k_wgpp",
 * "k_wg", "k_mb+k_rows", ...; "" before the first batch) */
const char *h264mi_engine_kernel(h264mi_engine *e);
size_t h264mi_engine_frame_bytes(h264mi_engine *e);

/* MB-record capture: run the host parser over a whole Annex-B stream and keep
 * every picture's record batch (the §8d "pre-parsed MB-record batches"). */
typedef struct h264mi_capture h264mi_capture;
h264mi_capture *h264mi_capture_stream(const uint8_t *buf, size_t len, int no_reorder);
int  h264mi_capture_info(const h264mi_capture *c, int *w_mbs, int *h_mbs, int *nslots, int *npics, int *errors);
int  h264mi_capture_picture(const h264mi_capture *c, int i, const void **rec, const int16_t **coef,
                            uint32_t *ncoef, int *cur_slot, uint64_t *alg_ref_bytes);
int  h264mi_capture_stats(const h264mi_capture *c, int i, uint32_t *n_inter, uint32_t *n_intra, uint32_t *n_coded);
void h264mi_capture_free(h264mi_capture *c);

/* Device memory helpers for the device-resident path (HIP device pointers) */
void *h264mi_device_alloc(size_t bytes);
int   h264mi_device_free(void *p);
int   h264mi_copy_h2d(void *dst, const void *src, size_t bytes);

#ifdef __cplusplus
}
#endif

#endif
