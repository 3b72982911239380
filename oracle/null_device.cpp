// ORACLE -- TEST INFRASTRUCTURE ONLY.  A CPU stand-in for the GPU under the
// product's H264Backend adapter (broadway_amd/csrc/host/hipback.cpp), so that
// the adapter's own threading -- per-GPU shared engines (h264mi_set_share:
// batch collection, the 1 ms launch timeout, per-instance completion events,
// the per-batch result ring), the pool of released engines and the pinned
// output-frame pool, the blocking waits -- runs under ThreadSanitizer and
// AddressSanitizer + UBSan on a machine without a GPU (the
// round-3 verdict's "sanitize the product's own threading").
//
// Two layers, linked in place of the HIP runtime and of engine.hip:
//  - the HIP runtime calls the adapter makes, on host memory: "device"
//    allocations are malloc'd, copies and memsets run at once on the calling
//    thread (a stream is in-order and every queued item here has already
//    completed, so events and synchronisation are no-ops that still check
//    their arguments);
//  - the engine core's interface (engine_int.h and the h264mi_engine_* calls
//    of include/h264mi.h the adapter uses): an engine is one oracle context
//    per stream lane (recon_cpu.c, the CPU restatement of the reconstruction),
//    so every picture decoded through the product C-ABI on this build is the
//    reference's picture and the tests compare MD5s as well as sanitizer
//    reports.
// Device-side concealment (k_conceal) runs the product's host restatement of
// the same neighbour path (conceal.c) on the slot, in the given order.
#include <hip/hip_runtime_api.h>
#include <atomic>
#include <mutex>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../broadway_amd/csrc/hip/engine_int.h"
#include "recon_cpu.h"
#include "../broadway_amd/csrc/host/decoder.h"

// ------------------------------------------------------------ HIP runtime
struct NullEvent { unsigned flags; std::atomic<int> recorded; };
static std::atomic<long> g_live_events{0}, g_live_host{0}, g_live_dev{0};

extern "C" {
hipError_t hipGetDeviceCount(int *count) { *count = 1; return hipSuccess; }
hipError_t hipSetDevice(int device) { return device == 0 ? hipSuccess : hipErrorInvalidDevice; }
const char *hipGetErrorString(hipError_t e) { return e == hipSuccess ? "hipSuccess" : "null-device error"; }
hipError_t hipMalloc(void **ptr, size_t size)
{
    *ptr = calloc(1, size ? size : 1);
    if (!*ptr) return hipErrorOutOfMemory;
    g_live_dev++;
    return hipSuccess;
}
hipError_t hipFree(void *ptr) { if (ptr) { g_live_dev--; free(ptr); } return hipSuccess; }
hipError_t hipHostMalloc(void **ptr, size_t size, unsigned int flags)
{
    *ptr = malloc(size ? size : 1);
    if (!*ptr) return hipErrorOutOfMemory;
    g_live_host++;
    return hipSuccess;
}
hipError_t hipHostFree(void *ptr) { if (ptr) { g_live_host--; free(ptr); } return hipSuccess; }
hipError_t hipMemcpy(void *dst, const void *src, size_t n, hipMemcpyKind kind) { memmove(dst, src, n); return hipSuccess; }
hipError_t hipMemcpyAsync(void *dst, const void *src, size_t n, hipMemcpyKind kind, hipStream_t stream)
{
    memmove(dst, src, n);
    return hipSuccess;
}
hipError_t hipMemsetAsync(void *dst, int value, size_t n, hipStream_t stream) { memset(dst, value, n); return hipSuccess; }
hipError_t hipEventCreateWithFlags(hipEvent_t *event, unsigned flags)
{
    NullEvent *e = new NullEvent();
    e->flags = flags;
    e->recorded = 0;
    *event = (hipEvent_t)e;
    g_live_events++;
    return hipSuccess;
}
hipError_t hipEventRecord(hipEvent_t event, hipStream_t stream)
{
    if (!event) return hipErrorInvalidHandle;
    ((NullEvent *)event)->recorded = 1;
    return hipSuccess;
}
hipError_t hipEventSynchronize(hipEvent_t event) { return event ? hipSuccess : hipErrorInvalidHandle; }
hipError_t hipEventDestroy(hipEvent_t event)
{
    if (!event) return hipErrorInvalidHandle;
    delete (NullEvent *)event;
    g_live_events--;
    return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t stream) { return hipSuccess; }
}

// live allocations and events (tests: the pools give everything back)
extern "C" void null_device_live(long *events, long *host_blocks, long *dev_blocks)
{
    *events = g_live_events.load(); *host_blocks = g_live_host.load(); *dev_blocks = g_live_dev.load();
}

// ------------------------------------------------------------ the engine
struct h264mi_engine {
    int w, h, nstreams, nslots, blocking;
    void **lane;            // oracle context per stream lane (nslots frames each)
    unsigned *err;          // "device" flag words, one per batch picture
    hipStream_t st;         // a distinct non-null handle per engine
    std::mutex mu;          // one engine's stream is in order: one launch at a time
};

extern "C" h264mi_engine *h264mi_engine_create(int device, int w_mbs, int h_mbs, int nstreams, int nslots)
{
    if (device != 0 || w_mbs < 1 || h_mbs < 1 || nstreams < 1 || nslots < 1) return NULL;
    h264mi_engine *e = new h264mi_engine();
    e->w = w_mbs; e->h = h_mbs; e->nstreams = nstreams; e->nslots = nslots;
    e->blocking = getenv("H264MI_BLOCKING_SYNC") && atoi(getenv("H264MI_BLOCKING_SYNC"));
    e->lane = (void **)calloc((size_t)nstreams, sizeof(void *));
    (void)hipMalloc((void **)&e->err, sizeof(unsigned) * nstreams);
    for (int i = 0; i < nstreams; i++) e->lane[i] = oracle_ctx_create(w_mbs, h_mbs, nslots);
    e->st = (hipStream_t)e;
    return e;
}

extern "C" void h264mi_engine_destroy(h264mi_engine *e)
{
    if (!e) return;
    for (int i = 0; i < e->nstreams; i++) oracle_ctx_destroy(e->lane[i]);
    free(e->lane);
    (void)hipFree(e->err);
    delete e;
}

extern "C" int h264mi_engine_device(const h264mi_engine *e) { return e ? 0 : -1; }
extern "C" void *h264mi_engine_frame_ptr(h264mi_engine *e, int stream, int slot)
{
    if (!e || stream < 0 || stream >= e->nstreams || slot < 0 || slot >= e->nslots) return NULL;
    return oracle_ctx_frame(e->lane[stream], slot);
}
extern "C" size_t h264mi_engine_frame_bytes(h264mi_engine *e) { return e ? (size_t)e->w * e->h * 384 : 0; }
// the null device keeps its slots packed (chroma pitch = w * 8)
extern "C" int h264mi_engine_chroma_pitch(h264mi_engine *e) { return e ? e->w * 8 : 0; }
size_t engine_slot_bytes(const h264mi_engine *e) { return (size_t)e->w * e->h * 384; }
int engine_copy_out(h264mi_engine *e, int stream, int slot, uint8_t *dst, hipStream_t st)
{
    void *p = h264mi_engine_frame_ptr(e, stream, slot);
    if (!p) return -1;
    memcpy(dst, p, h264mi_engine_frame_bytes(e));
    return 0;
}
extern "C" int h264mi_engine_sync(h264mi_engine *e) { return e ? 0 : -1; }
extern "C" int h264mi_engine_read(h264mi_engine *e, int stream, int slot, uint8_t *dst)
{
    void *p = h264mi_engine_frame_ptr(e, stream, slot);
    if (!p) return -1;
    memcpy(dst, p, h264mi_engine_frame_bytes(e));
    return 0;
}
extern "C" int h264mi_engine_read_rgba(h264mi_engine *e, int stream, int slot, uint8_t *dst) { return -1; }
extern "C" int h264mi_yuv2rgba_device(const void *d_i420, void *d_rgba, int width, int height, int npics,
                                      size_t in_stride, size_t out_stride, void *stream)
{
    return -1;
}
extern "C" int h264mi_yuv2rgba_device_pitch(const void *d_i420, void *d_rgba, int width, int height, int cpitch,
                                            int npics, size_t in_stride, size_t out_stride, void *stream)
{
    return -1;
}
extern "C" int h264mi_engine_conceal(h264mi_engine *e, int stream, int slot, const int *order, int n,
                                     const uint8_t *decoded)
{
    uint8_t *img = (uint8_t *)h264mi_engine_frame_ptr(e, stream, slot);
    if (!img || n < 0 || n > e->w * e->h || (n && (!order || !decoded))) return -1;
    std::lock_guard<std::mutex> g(e->mu);
    uint8_t *dec = (uint8_t *)malloc((size_t)e->w * e->h);
    memcpy(dec, decoded, (size_t)e->w * e->h);
    for (int k = 0; k < n; k++) {
        if (order[k] < 0 || order[k] >= e->w * e->h) { free(dec); return -1; }
        h264dec_conceal_mb_intra(img, e->w, e->h, order[k] / e->w, order[k] % e->w, dec);
        dec[order[k]] = 1;
    }
    free(dec);
    return 0;
}

int engine_decode_host(h264mi_engine *e, int npics, const int *stream, const int *cur_slot,
                       const void *const *recs, const int16_t *const *coefs, const uint32_t *ncoef,
                       int intra_heavy)
{
    if (!e || npics < 1 || npics > e->nstreams) return -1;
    std::lock_guard<std::mutex> g(e->mu);
    for (int i = 0; i < npics; i++) {
        if (stream[i] < 0 || stream[i] >= e->nstreams || cur_slot[i] < 0 || cur_slot[i] >= e->nslots) return -1;
        // a flag the caller forced onto the picture's word stays there (the
        // device ORs its own into it)
        if (oracle_recon_picture(e->lane[stream[i]], (const MbRec *)recs[i], coefs[i], e->w, e->h, cur_slot[i]))
            e->err[i] |= 1u;
    }
    return 0;
}
int engine_decode_direct(h264mi_engine *e, int stream, int cur_slot, const void *rec, const int16_t *coef,
                         uint32_t ncoef, int intra_heavy)
{
    const void *recs[1] = {rec};
    const int16_t *coefs[1] = {coef};
    return engine_decode_host(e, 1, &stream, &cur_slot, recs, coefs, &ncoef, intra_heavy);
}
int engine_records_wait(h264mi_engine *e) { return e ? 0 : -1; }
int engine_wait(h264mi_engine *e) { return e ? 0 : -1; }
hipStream_t engine_stream(h264mi_engine *e) { return e->st; }
unsigned *engine_err_words(h264mi_engine *e) { return e->err; }
void engine_shape(const h264mi_engine *e, int *w_mbs, int *h_mbs, int *nstreams, int *nslots, int *blocking)
{
    *w_mbs = e->w; *h_mbs = e->h; *nstreams = e->nstreams; *nslots = e->nslots; *blocking = e->blocking;
}
int engine_poolable(const h264mi_engine *e) { return 1; }
int engine_conceal_fits(const h264mi_engine *e) { return 1; }
int engine_reuse(h264mi_engine *e)
{
    for (int i = 0; i < e->nstreams; i++)
        for (int s = 0; s < e->nslots; s++) memset(oracle_ctx_frame(e->lane[i], s), 0, h264mi_engine_frame_bytes(e));
    memset(e->err, 0, sizeof(unsigned) * e->nstreams);
    return 0;
}
