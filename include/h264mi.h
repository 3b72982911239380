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
H264SwDecApiVersion H264SwDecGetAPIVersion(void);

/* Application hooks (reference inc/H264SwDecApi.h:160-173).  The library
 * allocates / frees each instance through H264SwDecMalloc / H264SwDecFree
 * (H264SwDecApi.c:147, :301) and calls H264SwDecTrace with the API trace when
 * built with -DH264DEC_TRACE.  libh264mi.so carries the reference's default
 * definitions (malloc / free / memcpy / memset, H264SwDecApi.c:78-96); an
 * application defining its own (DecTestBench.c:678-760) overrides them. */
void  H264SwDecTrace(char *string);
void *H264SwDecMalloc(u32 size);
void  H264SwDecFree(void *ptr);
void  H264SwDecMemcpy(void *dest, void *src, u32 count);
void  H264SwDecMemset(void *ptr, i32 value, u32 count);                                /* :487 */
/* NextPicture, the picture converted to RGBA on the GPU: what Decoder.js
 * delivers with `rgb: true` (templates/DecoderPost.js:82-97, the asm.js
 * converter :322-560, per pixel yuv2rgbcalc :514-560).  rgba: picWidth *
 * picHeight * 4 bytes; pOutput->pOutputPicture = rgba.  No reference C
 * counterpart: the reference converts in JavaScript. */
H264SwDecRet H264SwDecNextPictureRGBA(H264SwDecInst decInst, H264SwDecPicture *pOutput, u32 flushBuffer, u8 *rgba);
/* Extension (no reference counterpart): where an instance's time went, in
 * seconds since H264SwDecInit -- host parse (NAL extraction, headers, CAVLC /
 * MB layer, DPB, concealment), record upload + kernel launch, waiting for the
 * device in NextPicture, and the output copy -- plus pictures output.  Any
 * pointer may be NULL. */
H264SwDecRet H264SwDecGetTiming(H264SwDecInst decInst, double *parse_s, double *submit_s, double *wait_s,
                                double *copy_s, u32 *pictures);
/* Extension: per-GPU shared engine for concurrent instances (threads) of one
 * process.  With lanes >= 2 (or H264MI_SHARE=lanes in the environment), the
 * instances decoding pictures of the same size on one device share one
 * engine of `lanes` streams (one such engine per picture size): each H264SwDecDecode hands its picture to the
 * batch being collected and returns once a launch took it; a batch launches
 * when every attached instance has submitted or 1 ms (H264MI_SHARE_WAIT_US)
 * after its first picture, as one k_prep + k_wgpp launch.  Set before the instances are
 * configured (their first picture); 0 turns it off.  Outputs, order and
 * error reporting per instance are unchanged.  The reference's model is N
 * independent instances (TestBenchMultipleInstance.c:134-305). */
int h264mi_set_share(int lanes);
/* batches / pictures launched by device's shared engine; returns the
 * instances attached (0: none) */
int h264mi_share_stats(int device, unsigned long long *batches, unsigned long long *pictures);
/* diagnostics, host CPU attribution of this process: the CPU seconds of the
 * speculative-parse worker threads that have exited (threads named
 * "h264mi-spec"), and how many were started */
int h264mi_host_thread_stats(double *spec_worker_cpu_s, unsigned long long *workers_started);

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

/* Engine C-ABI revision, bumped whenever a function or a record field keeps
 * its name but changes meaning, so that an integration built against an
 * older revision can refuse to run (compare H264MI_ENGINE_ABI at build time
 * with h264mi_engine_abi() at run time):
 *   5  h264mi_engine_frame_bytes returns the packed I420 size of one picture;
 *      slots are h264mi_engine_slot_bytes apart and their chroma rows
 *      h264mi_engine_chroma_pitch (H264MI_CPITCH) apart -- before, it was the
 *      slot stride of unpadded I420 slots
 *   6  PicDesc.flags bit 3 (PD_NO_DEBLOCK) for device-resident callers */
#define H264MI_ENGINE_ABI 6
int h264mi_engine_abi(void);

/* Reconstruction engine for `nstreams` independent streams of one size
 * (w_mbs x h_mbs macroblocks), each with `nslots` frame slots in HBM. */
h264mi_engine *h264mi_engine_create(int device, int w_mbs, int h_mbs, int nstreams, int nslots);
void h264mi_engine_destroy(h264mi_engine *e);

/* Reconstruct one picture per listed stream (host-resident record batches):
 * recs[i] -> w*h MbRec (96 B each), coefs[i] -> ncoef[i] int16x16 blocks. */
int h264mi_engine_decode(h264mi_engine *e, int npics, const int *stream, const int *cur_slot,
                         const void *const *recs, const int16_t *const *coefs, const uint32_t *ncoef);

/* Shape hint for the next launch of a device-resident batch (the host path,
 * h264mi_engine_decode, derives it from the records itself): 1 if some picture
 * of the batch has more than half its MBs intra, 0 if none.  P-picture
 * launches then run 4-wave row workgroups (2 MC waves, every MB row resident
 * at once), intra-heavy ones 5-wave workgroups (3 MC waves); without a hint
 * the launch uses 3.  A hint covers one launch.  Returns 0, or -1 on a bad
 * argument. */
int h264mi_engine_hint_intra(h264mi_engine *e, int intra_heavy);
/* MC waves per row workgroup of the last launch: 2 or 3, or 6 for an
 * intra-heavy launch whose rows all fit two workgroups per CU (diagnostics) */
int h264mi_engine_last_mc_waves(h264mi_engine *e);
/* the next frame-pipelined launch's dependency mode: 1 whole MB rows of the
 * earlier steps' pictures (MbRec.i4 rows from h264mi_capture), 2 (MB row, MB
 * column) cells (geometry in the kernel), 0 the engine's default
 * (H264MI_DEP_MODE=rows|cols, default rows); last_deps: the mode the last
 * launch ran (0: one step, no dependency) */
int h264mi_engine_hint_deps(h264mi_engine *e, int mode);
int h264mi_engine_last_deps(h264mi_engine *e);

/* Neighbour-based error concealment on the device (ConcealMb's intra branch,
 * h264bsd_conceal.c:337-579, replaces the host pass over a copy of the
 * picture): the MBs order[0..n) of stream `stream`'s slot `slot` -- which holds
 * the picture's decoded MBs reconstructed with the loop filter off -- are
 * concealed in place in that order, behind the work already queued;
 * decoded[0..w*h) flags the decoded MBs.  Inputs are copied before return.
 * 0, or -1 on a bad argument / HIP error.  The H264SwDec* path uses it for I
 * pictures with lost MBs (H264MI_HOST_CONCEAL=1: the host path instead). */
int h264mi_engine_conceal(h264mi_engine *e, int stream, int slot, const int *order, int n,
                          const uint8_t *decoded);
/* diagnostics: k_conceal launches in this process */
unsigned long long h264mi_conceal_launches(void);
/* diagnostics: engines of H264SwDec* instances taken from the pool of
 * released ones (H264MI_ENGINE_POOL) / newly created, in this process */
void h264mi_engine_pool_stats(unsigned long long *reused, unsigned long long *created);
/* frees every released engine and pinned output frame the pools hold (what
 * instances still use is not touched; the library also drains at unload);
 * returns the engines freed.  The pinned-frame pool keeps at most
 * H264MI_HOST_POOL_MB (default 256) MB. */
int  h264mi_pool_drain(void);
/* pooled engines / pinned bytes held now */
void h264mi_pool_held(int *engines, size_t *pinned_bytes);

/* Device-resident variant (records already in HBM; kernel-only timing):
 * d_recs = npics*w*h MbRec in batch order with coefficient offsets relative
 * to d_coef, d_pics = npics PicDesc. */
int h264mi_engine_decode_device(h264mi_engine *e, int npics, const void *d_recs, const int16_t *d_coef,
                                const void *d_pics);
/* Same, with the NEXT batch named (device pointers as above; it must be the
 * batch of the following decode_device* call): this launch's tail
 * workgroups compute the next batch's deblocking records and residuals as its
 * own MB rows drain, so that batch needs no k_prep launch of its own. */
int h264mi_engine_decode_device_next(h264mi_engine *e, int npics, const void *d_recs, const int16_t *d_coef,
                                     const void *d_pics, const void *next_recs, const int16_t *next_coef,
                                     const void *next_pics);
/* Frame-pipelined batch: P consecutive pictures of each of S streams in one
 * launch, descriptors step-major (j * S + s), every PicDesc.rec_base relative
 * to d_recs.  A picture reading a slot that an earlier picture of the batch
 * reconstructs waits, per 128-B line of its reference windows, for those rows
 * to be final (device row tags), so the later picture's top rows overlap the
 * earlier one's bottom rows.  The caller guarantees that no picture of the
 * batch writes a slot an earlier picture of the batch reads or writes.
 * P <= the engine's steps (h264mi_engine_set_steps, 1..H264MI_MAX_STEPS;
 * default 1; more than 1 needs at most 32 frame slots per stream). */
int h264mi_engine_decode_device_steps(h264mi_engine *e, int S, int P, const void *d_recs, const int16_t *d_coef,
                                      const void *d_pics, const void *next_recs, const int16_t *next_coef,
                                      const void *next_pics);
/* The same, naming the next batch's step count next_P (1 .. steps) when it
 * differs from P: the next batch's k_prep runs in this launch's tail over its
 * S * next_P pictures (a plan mixing one- and two-step launches). */
int h264mi_engine_decode_device_steps_next(h264mi_engine *e, int S, int P, const void *d_recs,
                                           const int16_t *d_coef, const void *d_pics, const void *next_recs,
                                           const int16_t *next_coef, const void *next_pics, int next_P);
#define H264MI_MAX_STEPS 4
int h264mi_engine_set_steps(h264mi_engine *e, int steps);

int  h264mi_engine_read(h264mi_engine *e, int stream, int slot, uint8_t *dst);   /* D2H I420 */
/* D2H of a slot as RGBA (w*16 * h*16 * 4 bytes), converted on the GPU
 * (DecoderPost.js yuv2rgbcalc :514-560 per pixel) */
int  h264mi_engine_read_rgba(h264mi_engine *e, int stream, int slot, uint8_t *dst);
/* the conversion kernel on device buffers: npics MB-aligned I420 pictures
 * of width x height (multiples of 16) at d_i420 + k * in_stride ->
 * d_rgba + k * out_stride; asynchronous on `hip_stream` (NULL: null stream) */
int  h264mi_yuv2rgba_device(const void *d_i420, void *d_rgba, int width, int height, int npics,
                            size_t in_stride, size_t out_stride, void *hip_stream);
/* the same with the chroma rows cpitch bytes apart (an engine slot:
 * h264mi_engine_chroma_pitch; the packed form above is cpitch = width / 2) */
int  h264mi_yuv2rgba_device_pitch(const void *d_i420, void *d_rgba, int width, int height, int cpitch, int npics,
                                  size_t in_stride, size_t out_stride, void *hip_stream);
int  h264mi_engine_sync(h264mi_engine *e);
/* number of (launch, picture) slots flagged since the last call: residual
 * range errors (reference transform.c:181) or a bounded wait that expired;
 * flags accumulate over every launch and are collected by h264mi_engine_sync */
uint32_t h264mi_engine_errors(h264mi_engine *e);
/* the OR of the device flag words of every picture synced since the last
 * call (1 residual range, 2 / 16 / 32 bounded waits expired; with
 * H264MI_CHECK=1 the dependency checker's 64 ring data, 128 ring overwrite,
 * 256 partner region, 512 intra progress, 1024 reference rows not final) */
uint32_t h264mi_engine_error_bits(h264mi_engine *e);
/* MB rows per k_wgpp workgroup the engine launches for a batch of npics
 * pictures (1..3: by batch size, H264MI_RPW, the LDS budget) */
int  h264mi_engine_rows_per_workgroup(h264mi_engine *e, int npics);
/* duration (us) of the last batch's k_wgpp launch: us2[1] (us2[0] = 0);
 * needs H264MI_TIMING in the environment */
int  h264mi_engine_last_timing(h264mi_engine *e, float *us2);
/* per-batch kernel timing with HIP events carried by k_wgpp's dispatch
 * packet: record up to max_batches launches (0 disables); the report syncs
 * and returns the summed k_wgpp durations in *wave_us (*inter_us = 0), in
 * microseconds */
int  h264mi_engine_set_timing(h264mi_engine *e, int max_batches);
/* time only every stride-th launch (default 1) */
int  h264mi_engine_set_timing_stride(h264mi_engine *e, int stride);
int  h264mi_engine_timing_report(h264mi_engine *e, double *inter_us, double *wave_us, int *nbatches);
/* the recorded launches' k_wgpp durations one by one (us[i], in recording
 * order, at most cap); returns how many (call before timing_report, which
 * resets the record) */
int  h264mi_engine_timing_list(h264mi_engine *e, double *us, int cap);
/* diagnostics: per k_wgpp workgroup (row r of batch picture p at index
 * r * npics + p) 16 u64: wall-clock start/end (100 MHz) and shader-clock sums
 * of its phases, then 4 u64 per MB (chain stamps); enable != 0 allocates and
 * switches to the profiling kernel, out != NULL copies the last launch */
int  h264mi_engine_profile(h264mi_engine *e, int enable, unsigned long long *out, size_t n);
/* device pointer of a frame slot: I420 with the chroma rows padded to
 * h264mi_engine_chroma_pitch bytes (H264MI_CPITCH, include/h264mi_records.h),
 * slots h264mi_engine_slot_bytes apart */
void *h264mi_engine_frame_ptr(h264mi_engine *e, int stream, int slot);
/* diagnostics: name of the last batch's reconstruction kernel ("k_wgpp";
 * "" before the first batch) */
const char *h264mi_engine_kernel(h264mi_engine *e);
/* packed I420 bytes of one picture (h264mi_engine_read's output) */
size_t h264mi_engine_frame_bytes(h264mi_engine *e);
size_t h264mi_engine_slot_bytes(h264mi_engine *e);
int    h264mi_engine_chroma_pitch(h264mi_engine *e);

/* MB-record capture: run the host parser over a whole Annex-B stream and keep
 * every picture's record batch (the §8d "pre-parsed MB-record batches"). */
typedef struct h264mi_capture h264mi_capture;
h264mi_capture *h264mi_capture_stream(const uint8_t *buf, size_t len, int no_reorder);
int  h264mi_capture_info(const h264mi_capture *c, int *w_mbs, int *h_mbs, int *nslots, int *npics, int *errors);
int  h264mi_capture_picture(const h264mi_capture *c, int i, const void **rec, const int16_t **coef,
                            uint32_t *ncoef, int *cur_slot, uint64_t *alg_ref_bytes);
int  h264mi_capture_stats(const h264mi_capture *c, int i, uint32_t *n_inter, uint32_t *n_intra, uint32_t *n_coded);
/* picture i's reference footprint in whole 128-B lines (distinct lines of
 * each reference slot the k_wgpp MC windows touch, x 128): the line-granular
 * reference traffic beside alg_ref_bytes' bytes used (measurement helper; no
 * reference counterpart) */
int  h264mi_capture_ref_lines(const h264mi_capture *c, int i, uint64_t *ref_line_bytes);
void h264mi_capture_free(h264mi_capture *c);

/* Device memory helpers for the device-resident path (HIP device pointers).
 * h264mi_device_alloc allocates on the calling thread's CURRENT HIP device;
 * a multi-GPU caller uses the engine-scoped forms below instead. */
void *h264mi_device_alloc(size_t bytes);
int   h264mi_device_free(void *p);
int   h264mi_copy_h2d(void *dst, const void *src, size_t bytes);
/* Engine-scoped: memory on the engine's own GPU whatever the caller's current
 * device (one process per GPU, TestBenchMultipleInstance.c:134-305 style
 * independent instances); copy_h2d refuses a destination on another GPU. */
int   h264mi_engine_device(const h264mi_engine *e);
void *h264mi_engine_alloc(h264mi_engine *e, size_t bytes);
int   h264mi_engine_free(h264mi_engine *e, void *p);
int   h264mi_engine_copy_h2d(h264mi_engine *e, void *dst, const void *src, size_t bytes);
/* HIP device ordinal a device pointer lives on, -1 for host / unknown memory */
int   h264mi_pointer_device(const void *p);

#ifdef __cplusplus
}
#endif

#endif
