// H264Backend adapter of the HIP reconstruction engine (engine.hip) for the
// single-stream host decoder (decoder.c): per decoder instance a private
// engine, or a lane of the device's shared engine (h264mi_set_share); the
// pool of released engines and pinned output frames.  Plain host C++ over
// the HIP runtime API and the engine's internal interface (engine_int.h): no
// device code here, so that tests/null_device can build this file against a
// CPU stand-in of both and run its threading under TSan / ASan + UBSan.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <atomic>
#include <chrono>
#include <mutex>
#include <pthread.h>
#include <time.h>
#include "../hip/engine_int.h"
#include "decoder.h"

#define HIPCHECK(x)                                                                    \
    do {                                                                               \
        hipError_t err_ = (x);                                                         \
        if (err_ != hipSuccess) {                                                      \
            fprintf(stderr, "h264mi: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(err_), \
                    __FILE__, __LINE__);                                               \
            return -1;                                                                 \
        }                                                                              \
    } while (0)

// H264MI_BLOCKING_SYNC=1: an engine created now waits by sleeping
static int env_blocking()
{
    const char *v = getenv("H264MI_BLOCKING_SYNC");
    return v && atoi(v) ? 1 : 0;
}

// Released private engines, kept for the next decoder instance of the same
// shape: DecTestBench-style callers create one H264SwDec instance per stream
// (H264SwDecInit ... H264SwDecRelease), and a fresh engine costs ~20 device
// and pinned allocations, a stream, events and a frame clear.  A pooled
// engine is idle (its stream drained) and is handed out as a fresh one would
// be: frames cleared, no batch prepped, settings re-read.  H264MI_ENGINE_POOL=0
// turns it off; h264mi_pool_drain() frees what the pools hold (also run at
// process exit).
// at process exit the pools are drained by an atexit handler registered
// when something is first pooled -- after the HIP runtime initialised, so
// it runs before the runtime's own teardown (a library destructor would run
// too late in a process that loaded the runtime first, e.g. through torch)
extern "C" int h264mi_pool_drain(void);
static void pool_drain_at_exit() { (void)h264mi_pool_drain(); }
static void register_drain_once()
{
    static std::once_flag once;
    std::call_once(once, [] { atexit(pool_drain_at_exit); });
}

#define ENGINE_POOL_MAX 4
static std::mutex g_pool_mu;
static h264mi_engine *g_pool[ENGINE_POOL_MAX];
static std::atomic<unsigned long long> g_pool_reused, g_pool_created;

extern "C" void h264mi_engine_pool_stats(unsigned long long *reused, unsigned long long *created)
{
    if (reused) *reused = g_pool_reused.load();
    if (created) *created = g_pool_created.load();
}

static bool engine_pool_on()
{
    const char *v = getenv("H264MI_ENGINE_POOL");
    return !v || atoi(v) != 0;
}

static h264mi_engine *engine_get(int device, int w_mbs, int h_mbs, int nstreams, int nslots)
{
    h264mi_engine *e = NULL;
    const int blocking = env_blocking();
    if (engine_pool_on()) {
        std::lock_guard<std::mutex> g(g_pool_mu);
        for (int i = 0; i < ENGINE_POOL_MAX && !e; i++) {
            h264mi_engine *x = g_pool[i];
            int xw = 0, xh = 0, xs = 0, xn = 0, xb = 0;
            if (x) engine_shape(x, &xw, &xh, &xs, &xn, &xb);
            // the waits' kind (H264MI_BLOCKING_SYNC) is fixed when an engine is
            // created: it is part of the key
            if (x && h264mi_engine_device(x) == device && xw == w_mbs && xh == h_mbs && xs == nstreams &&
                xn == nslots && xb == blocking) {
                e = x;
                g_pool[i] = NULL;
            }
        }
    }
    if (!e) {
        g_pool_created++;
        return h264mi_engine_create(device, w_mbs, h_mbs, nstreams, nslots);
    }
    g_pool_reused++;
    if (engine_reuse(e)) { h264mi_engine_destroy(e); return NULL; }
    return e;
}

static void engine_put(h264mi_engine *e)
{
    if (!e) return;
    // engines with diagnostics state (timing events, profiling buffers) are not kept
    if (engine_pool_on() && engine_poolable(e) && hipSetDevice(h264mi_engine_device(e)) == hipSuccess &&
        hipStreamSynchronize(engine_stream(e)) == hipSuccess) {
        std::lock_guard<std::mutex> g(g_pool_mu);
        for (int i = 0; i < ENGINE_POOL_MAX; i++)
            if (!g_pool[i]) { g_pool[i] = e; register_drain_once(); return; }
    }
    h264mi_engine_destroy(e);
}

// -------- H264Backend adapter for the single-stream host decoder ----------

// Per-GPU shared engines (H264MI_SHARE=N, or h264mi_set_share): the decoder
// instances of a process that decode pictures of the same size on the same
// device share one engine of N lanes (one engine per picture size) (a lane = a stream index of the frame
// pool).  Each instance's H264SwDecDecode hands its picture's records to the
// batch being collected and returns once a launch has taken it: the batch
// launches when every attached instance has submitted, or SHARE_WAIT_US
// after its first picture -- one k_prep + k_wgpp launch for the pictures of
// up to N concurrent instances (threads) instead of one launch each.  The
// reference's multi-instance model is N independent instances
// (TestBenchMultipleInstance.c:134-305); each instance here still sees only
// its own pictures, in its own order.
#define SHARE_MAX 32
#define SHARE_SLOTS 17                    // MaxDpbFrames (16) + the current picture
#define SHARE_WAIT_US 1000                // default batch wait (H264MI_SHARE_WAIT_US)

struct HipBackendCtx;
struct SharedEng {
    std::mutex mu;
    // batch launched: a pthread condition on CLOCK_MONOTONIC, waited on with
    // pthread_cond_timedwait (std::condition_variable::wait_for waits through
    // pthread_cond_clockwait, which ThreadSanitizer builds of this toolchain
    // do not see release the mutex)
    pthread_cond_t cv;
    SharedEng()
    {
        pthread_condattr_t at;
        pthread_condattr_init(&at);
        pthread_condattr_setclock(&at, CLOCK_MONOTONIC);
        pthread_cond_init(&cv, &at);
        pthread_condattr_destroy(&at);
    }
    ~SharedEng() { pthread_cond_destroy(&cv); }
    int device, w, h, lanes;
    h264mi_engine *e;
    uint32_t used;                        // attached lanes
    int active;
    // the batch being collected
    int np;
    int stream[SHARE_MAX], slot[SHARE_MAX];
    const void *recs[SHARE_MAX];
    const int16_t *coefs[SHARE_MAX];
    uint32_t nc[SHARE_MAX];
    HipBackendCtx *who[SHARE_MAX];
    bool force[SHARE_MAX];                // test hook: start this picture with a device flag set
    bool heavy[SHARE_MAX];                // more than half the picture's MBs intra (launch_nmc)
    unsigned long long collecting, launched;   // batch ids: collecting > launched while np > 0
    // result of each launch, by batch id: a waiter whose batch was launched
    // by another thread reads its own batch's entry, however many batches
    // launched before it got the lock back
#define SHARE_RC_RING 64
    int rc_ring[SHARE_RC_RING];
};
static std::mutex g_share_mu;
#define SHARE_SIZES 4                     // shared engines per device, one per picture size
static SharedEng *g_share[16][SHARE_SIZES];
// totals per device; atomics, since share_launch runs under an engine's
// lock and the lock order is g_share_mu before SharedEng::mu
static std::atomic<unsigned long long> g_share_batches[16], g_share_pictures[16];
static int g_share_lanes = -1;            // -1: H264MI_SHARE from the environment
static int g_share_wait_us = SHARE_WAIT_US;

struct HipBackendCtx {
    int device;
    h264mi_engine *e;   // private engine, or the shared one's
    SharedEng *sh;      // shared engine (NULL: private)
    int lane;           // stream index in e
    hipEvent_t ev_last; // shared: after this instance's latest work on the engine stream
    uint8_t *d_rgba;    // shared: RGBA staging
    uint8_t **pref;     // per slot: host buffer a D2H copy of the slot's current picture was queued into
    // pinned, per frame slot: the device flags (ReconArgs::err: residual range,
    // expired bounded waits) of the picture reconstructed into the slot, copied
    // behind its launch -- a read reports the flags of the picture it reads,
    // whatever order pictures are output in and whatever else was read before
    unsigned *h_slot_err;
    // test hook (H264MI_DEBUG_FLAG_PICTURE=k): the k-th reconstruction of this
    // instance (1-based) starts with a forced device flag, to check that the
    // flag reaches exactly that picture's output whatever the output order
    unsigned ndecodes, force_flag_at;
    int nslots;
    unsigned enq, synced;   // work items queued on the engine's stream / of those, waited for by hb_sync
};

extern "C" int h264mi_set_share(int lanes)
{
    if (lanes < 0 || lanes > SHARE_MAX) return -1;
    std::lock_guard<std::mutex> g(g_share_mu);
    g_share_lanes = lanes;
    return 0;
}

static int share_lanes()
{
    std::lock_guard<std::mutex> g(g_share_mu);
    if (g_share_lanes < 0) {
        const char *v = getenv("H264MI_SHARE");
        const int n = v ? atoi(v) : 0;
        g_share_lanes = n > 1 && n <= SHARE_MAX ? n : 0;
        const char *w = getenv("H264MI_SHARE_WAIT_US");
        if (w && atoi(w) > 0) g_share_wait_us = atoi(w);
    }
    return g_share_lanes;
}

// caller holds sh->mu
static void share_launch(SharedEng *sh)
{
    if (sh->np == 0) return;
    h264mi_engine *e = sh->e;
    for (int i = 0; i < sh->np; i++)
        if (sh->force[i]) (void)hipMemsetAsync(engine_err_words(e) + i, 0x01, sizeof(unsigned), engine_stream(e));
    bool heavy = false;
    for (int i = 0; i < sh->np; i++) heavy |= sh->heavy[i];
    int rc = engine_decode_host(e, sh->np, sh->stream, sh->slot, sh->recs, sh->coefs, sh->nc, heavy ? 1 : 0);
    // each picture's device flags (ReconArgs::err, one word per batch
    // picture) into its instance's word for the slot it was reconstructed
    // into, then cleared for the next batch
    for (int i = 0; i < sh->np && rc == 0; i++)
        if (hipMemcpyAsync(sh->who[i]->h_slot_err + sh->slot[i], engine_err_words(e) + i, sizeof(unsigned),
                           hipMemcpyDeviceToHost, engine_stream(e)) != hipSuccess)
            rc = -1;
    if (hipMemsetAsync(engine_err_words(e), 0, sizeof(unsigned) * sh->np, engine_stream(e)) != hipSuccess) rc = -1;
    sh->rc_ring[sh->collecting % SHARE_RC_RING] = rc;
    for (int i = 0; i < sh->np; i++) (void)hipEventRecord(sh->who[i]->ev_last, engine_stream(e));
    g_share_batches[sh->device] += 1;
    g_share_pictures[sh->device] += (unsigned long long)sh->np;
    sh->np = 0;
    sh->launched = sh->collecting;
    sh->collecting++;
    pthread_cond_broadcast(&sh->cv);
}

static void share_detach(HipBackendCtx *c)
{
    SharedEng *sh = c->sh;
    if (!sh) return;
    std::lock_guard<std::mutex> g(g_share_mu);
    bool last;
    {
        std::unique_lock<std::mutex> l(sh->mu);
        sh->used &= ~(1u << c->lane);
        sh->active--;
        if (sh->np > 0 && sh->np >= sh->active) share_launch(sh);      // the others need not wait for us
        last = sh->active == 0;
        if (last) (void)hipStreamSynchronize(engine_stream(sh->e));
    }
    (void)hipEventDestroy(c->ev_last);
    (void)hipFree(c->d_rgba);
    c->ev_last = NULL; c->d_rgba = NULL;
    if (last) {
        for (int k = 0; k < SHARE_SIZES; k++)
            if (g_share[sh->device][k] == sh) g_share[sh->device][k] = NULL;
        h264mi_engine_destroy(sh->e);
        delete sh;
    }
    c->sh = NULL; c->e = NULL;
}

// attach to the device's shared engine for a w x h stream; 0 = attached
static int share_attach(HipBackendCtx *c, int w_mbs, int h_mbs, int nslots)
{
    const int lanes = share_lanes();
    if (lanes < 2 || nslots > SHARE_SLOTS || c->device < 0 || c->device >= 16) return -1;
    std::lock_guard<std::mutex> g(g_share_mu);
    SharedEng *sh = NULL;
    int free_k = -1;
    for (int k = 0; k < SHARE_SIZES; k++) {
        SharedEng *x = g_share[c->device][k];
        if (x && x->w == w_mbs && x->h == h_mbs) sh = x;
        else if (!x && free_k < 0) free_k = k;
    }
    if (!sh) {
        if (free_k < 0) return -1;                          // SHARE_SIZES sizes in use: a private engine
        h264mi_engine *e = h264mi_engine_create(c->device, w_mbs, h_mbs, lanes, SHARE_SLOTS);
        if (!e) return -1;
        sh = new SharedEng();
        sh->device = c->device; sh->w = w_mbs; sh->h = h_mbs; sh->lanes = lanes; sh->e = e;
        sh->used = 0; sh->active = 0; sh->np = 0; sh->collecting = 1; sh->launched = 0;
        g_share[c->device][free_k] = sh;
    }
    std::lock_guard<std::mutex> l(sh->mu);
    int lane = -1;
    for (int i = 0; i < sh->lanes; i++)
        if (!(sh->used & (1u << i))) { lane = i; break; }
    if (lane < 0) return -1;                                // all lanes taken: a private engine
    // a waiting instance sleeps (its core parses for another instance)
    if (hipEventCreateWithFlags(&c->ev_last, hipEventDisableTiming | hipEventBlockingSync) != hipSuccess) return -1;
    (void)hipEventRecord(c->ev_last, engine_stream(sh->e));
    sh->used |= 1u << lane;
    sh->active++;
    c->sh = sh; c->lane = lane; c->e = sh->e;
    return 0;
}

// caller holds sh->mu: wait until batch `mine` was launched, at most the
// share wait; false on timeout
static bool wait_launched(SharedEng *sh, unsigned long long mine)
{
    struct timespec dl;
    clock_gettime(CLOCK_MONOTONIC, &dl);
    dl.tv_nsec += (long)g_share_wait_us * 1000;
    dl.tv_sec += dl.tv_nsec / 1000000000;
    dl.tv_nsec %= 1000000000;
    while (sh->launched < mine)
        if (pthread_cond_timedwait(&sh->cv, sh->mu.native_handle(), &dl) != 0 && sh->launched < mine) return false;
    return true;
}

static int hb_configure(void *vctx, int w_mbs, int h_mbs, int nslots)
{
    HipBackendCtx *c = (HipBackendCtx *)vctx;
    if (c->sh) share_detach(c);
    else if (c->e) engine_put(c->e);
    c->e = NULL;
    free(c->pref);
    (void)hipHostFree(c->h_slot_err);
    c->h_slot_err = NULL;
    c->pref = (uint8_t **)calloc((size_t)nslots, sizeof(uint8_t *));
    c->nslots = c->pref ? nslots : 0;
    if (hipSetDevice(c->device) != hipSuccess ||
        hipHostMalloc(&c->h_slot_err, sizeof(unsigned) * (nslots > 0 ? nslots : 1), hipHostMallocDefault) != hipSuccess) {
        c->h_slot_err = NULL;
        return -1;
    }
    memset(c->h_slot_err, 0, sizeof(unsigned) * (nslots > 0 ? nslots : 1));
    if (share_attach(c, w_mbs, h_mbs, nslots) != 0) {
        c->lane = 0;
        c->e = engine_get(c->device, w_mbs, h_mbs, 1, nslots);
    }
    return c->e && c->pref ? 0 : -1;
}

static int hb_decode(void *vctx, const PicBuild *pb, int cur_slot)
{
    HipBackendCtx *c = (HipBackendCtx *)vctx;
    if (cur_slot >= 0 && cur_slot < c->nslots) c->pref[cur_slot] = NULL;
    c->enq++;
    const bool force = ++c->ndecodes == c->force_flag_at;
    if (!c->sh) {
        // (the slot is checked before anything is queued: a failed call
        // leaves no flag behind for the next picture)
        if (cur_slot < 0 || cur_slot >= c->nslots) return -1;
        h264mi_engine *e = c->e;
        hipStream_t st = engine_stream(e);
        if (force) HIPCHECK(hipMemsetAsync(engine_err_words(e), 0x01, sizeof(unsigned), st));
        int stream = 0;
        const void *recs[1] = {pb->rec};
        const int16_t *coefs[1] = {pb->coef};
        uint32_t nc[1] = {pb->ncoef};
        const int heavy = 2 * (int)pb->n_intra > pb->nmbs;
        // the decoder's own picture is in pinned memory (hb_host_alloc): uploaded
        // straight from it, the decoder waits (hb_records_wait) before reusing it
        if (pb->pinned ? engine_decode_direct(e, stream, cur_slot, pb->rec, pb->coef, pb->ncoef, heavy)
                       : engine_decode_host(e, 1, &stream, &cur_slot, recs, coefs, nc, heavy)) {
            (void)hipMemsetAsync(engine_err_words(e), 0, sizeof(unsigned), st);
            return -1;
        }
        // the picture's device flags into the slot's word, behind its launch
        HIPCHECK(hipMemcpyAsync(c->h_slot_err + cur_slot, engine_err_words(e), sizeof(unsigned), hipMemcpyDeviceToHost, st));
        HIPCHECK(hipMemsetAsync(engine_err_words(e), 0, sizeof(unsigned), st));
        return 0;
    }
    SharedEng *sh = c->sh;
    std::unique_lock<std::mutex> l(sh->mu);
    const int i = sh->np++;
    sh->stream[i] = c->lane; sh->slot[i] = cur_slot;
    sh->recs[i] = pb->rec; sh->coefs[i] = pb->coef; sh->nc[i] = pb->ncoef;
    sh->who[i] = c;
    sh->force[i] = force;
    sh->heavy[i] = 2 * (int)pb->n_intra > pb->nmbs;
    const unsigned long long mine = sh->collecting;
    if (sh->np >= sh->active) {
        share_launch(sh);
    } else if (!wait_launched(sh, mine)) {
        share_launch(sh);                 // the others are late: launch what is there
    }
    // (a waiter gets the lock back long before SHARE_RC_RING more batches
    // launch: each later batch takes a picture or a 1 ms wait of another instance)
    return sh->rc_ring[mine % SHARE_RC_RING];
}

static int hb_records_wait(void *vctx)
{
    HipBackendCtx *c = (HipBackendCtx *)vctx;
    // a shared engine's decode returns after its batch consumed the records
    if (c->sh || !c->e) return 0;
    return engine_records_wait(c->e);
}

static int hb_prefetch(void *vctx, int slot, uint8_t *dst)
{
    HipBackendCtx *c = (HipBackendCtx *)vctx;
    if (slot < 0 || slot >= c->nslots) return -1;
    h264mi_engine *e = c->e;
    HIPCHECK(hipSetDevice(h264mi_engine_device(e)));
    std::unique_lock<std::mutex> l;
    if (c->sh) l = std::unique_lock<std::mutex>(c->sh->mu);
    if (engine_copy_out(e, c->lane, slot, dst, engine_stream(e))) return -1;
    if (c->sh) HIPCHECK(hipEventRecord(c->ev_last, engine_stream(e)));
    c->pref[slot] = dst;
    c->enq++;
    return 0;
}

// the device flags of the picture in `slot` (ReconArgs::err: residual range,
// expired bounded waits), copied behind its launch into the slot's word,
// reach the caller as return 1; wait: sync first (the copy is stream-ordered)
static int slot_flagged(HipBackendCtx *c, int slot, bool wait = true)
{
    if (wait) {
        if (c->sh) HIPCHECK(hipEventSynchronize(c->ev_last));
        else if (engine_wait(c->e)) return -1;      // (flags: copied into h_slot_err behind each decode)
    }
    if (slot < 0 || slot >= c->nslots) return -1;
    const unsigned f = c->h_slot_err[slot];
    if (f) fprintf(stderr, "h264mi: device flagged the picture in slot %d (flags %#x)\n", slot, f);
    return f ? 1 : 0;
}

static int hb_sync(void *vctx)
{
    HipBackendCtx *c = (HipBackendCtx *)vctx;
    const unsigned n = c->enq;
    if (c->sh) {
        HIPCHECK(hipEventSynchronize(c->ev_last));
    } else if (engine_wait(c->e)) {
        return -1;
    }
    c->synced = n;
    return 0;
}

static int hb_read(void *vctx, int slot, uint8_t *dst)
{
    HipBackendCtx *c = (HipBackendCtx *)vctx;
    if (c->sh) {
        if (slot < 0 || slot >= c->nslots) return -1;
        if (c->pref[slot] != dst) {
            std::lock_guard<std::mutex> l(c->sh->mu);
            if (engine_copy_out(c->e, c->lane, slot, dst, engine_stream(c->e))) return -1;
            HIPCHECK(hipEventRecord(c->ev_last, engine_stream(c->e)));
        }
        return slot_flagged(c, slot);
    }
    // copied there already (hb_prefetch): only wait for it
    if (slot >= 0 && slot < c->nslots && c->pref[slot] == dst) return slot_flagged(c, slot, c->synced != c->enq);
    if (h264mi_engine_read(c->e, 0, slot, dst)) return -1;
    return slot_flagged(c, slot, false);
}

static int hb_read_rgba(void *vctx, int slot, uint8_t *dst)
{
    HipBackendCtx *c = (HipBackendCtx *)vctx;
    if (c->sh) {
        h264mi_engine *e = c->e;
        int w = 0, h = 0, ns = 0, nsl = 0, bl = 0;
        engine_shape(e, &w, &h, &ns, &nsl, &bl);
        const size_t bytes = (size_t)w * h * 256 * 4;
        if (slot < 0 || slot >= c->nslots) return -1;
        if (!c->d_rgba) HIPCHECK(hipMalloc(&c->d_rgba, bytes));
        {
            std::lock_guard<std::mutex> l(c->sh->mu);
            if (h264mi_yuv2rgba_device_pitch(h264mi_engine_frame_ptr(e, c->lane, slot), c->d_rgba, w * 16, h * 16,
                                             h264mi_engine_chroma_pitch(e), 1, 0, 0, engine_stream(e)))
                return -1;
            HIPCHECK(hipMemcpyAsync(dst, c->d_rgba, bytes, hipMemcpyDeviceToHost, engine_stream(e)));
            HIPCHECK(hipEventRecord(c->ev_last, engine_stream(e)));
        }
        return slot_flagged(c, slot);
    }
    if (h264mi_engine_read_rgba(c->e, 0, slot, dst)) return -1;
    return slot_flagged(c, slot, false);
}

// Pinned host blocks (decoder output frames) kept after free for the next
// decoder instance: pinning tens of MB per instance is a large share of a
// short stream's host time.  Exact-size reuse, at most H264MI_HOST_POOL_MB
// (default 256: ten 1080p output frames and their headroom) kept per process;
// h264mi_pool_drain() returns them.
#define HOST_POOL_N 16
static size_t host_pool_cap()
{
    const char *v = getenv("H264MI_HOST_POOL_MB");
    const long mb = v ? atol(v) : 256;
    return mb > 0 ? (size_t)mb << 20 : 0;
}
static std::mutex g_hpool_mu;
static struct { void *p; size_t bytes; } g_hpool[HOST_POOL_N], g_hlive[4 * HOST_POOL_N];

static void *hb_host_alloc(void *vctx, size_t bytes)
{
    void *p = NULL;
    {
        std::lock_guard<std::mutex> g(g_hpool_mu);
        for (int i = 0; i < HOST_POOL_N && !p; i++)
            if (g_hpool[i].p && g_hpool[i].bytes == bytes) { p = g_hpool[i].p; g_hpool[i].p = NULL; }
    }
    if (!p && hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) return NULL;
    std::lock_guard<std::mutex> g(g_hpool_mu);
    for (int i = 0; i < 4 * HOST_POOL_N; i++)
        if (!g_hlive[i].p) { g_hlive[i].p = p; g_hlive[i].bytes = bytes; break; }
    return p;
}

static void hb_host_free(void *vctx, void *p)
{
    if (!p) return;
    {
        std::lock_guard<std::mutex> g(g_hpool_mu);
        size_t bytes = 0;
        for (int i = 0; i < 4 * HOST_POOL_N; i++)
            if (g_hlive[i].p == p) { bytes = g_hlive[i].bytes; g_hlive[i].p = NULL; break; }
        size_t kept = 0;
        for (int i = 0; i < HOST_POOL_N; i++) kept += g_hpool[i].p ? g_hpool[i].bytes : 0;
        if (bytes && engine_pool_on() && kept + bytes <= host_pool_cap())
            for (int i = 0; i < HOST_POOL_N; i++)
                if (!g_hpool[i].p) { g_hpool[i].p = p; g_hpool[i].bytes = bytes; register_drain_once(); return; }
    }
    (void)hipHostFree(p);
}

static int hb_conceal(void *vctx, int slot, const int *order, int n, const uint8_t *decoded)
{
    HipBackendCtx *c = (HipBackendCtx *)vctx;
    if (slot >= 0 && slot < c->nslots) c->pref[slot] = NULL;
    if (c->sh) {
        std::lock_guard<std::mutex> l(c->sh->mu);
        if (h264mi_engine_conceal(c->e, c->lane, slot, order, n, decoded)) return -1;
        HIPCHECK(hipEventRecord(c->ev_last, engine_stream(c->e)));
        return 0;
    }
    return h264mi_engine_conceal(c->e, c->lane, slot, order, n, decoded);
}

static int hb_conceal_ok(void *vctx)
{
    const HipBackendCtx *c = (const HipBackendCtx *)vctx;
    return c->e && engine_conceal_fits(c->e);
}

static int hb_copy(void *vctx, int dst, int src)
{
    HipBackendCtx *c = (HipBackendCtx *)vctx;
    if (dst >= 0 && dst < c->nslots) c->pref[dst] = NULL;
    if (c->sh) {
        std::lock_guard<std::mutex> l(c->sh->mu);
        HIPCHECK(hipMemcpyAsync(h264mi_engine_frame_ptr(c->e, c->lane, dst), h264mi_engine_frame_ptr(c->e, c->lane, src),
                                engine_slot_bytes(c->e), hipMemcpyDeviceToDevice, engine_stream(c->e)));
        HIPCHECK(hipEventRecord(c->ev_last, engine_stream(c->e)));
        return 0;
    }
    if (h264mi_engine_sync(c->e)) return -1;
    HIPCHECK(hipMemcpy(h264mi_engine_frame_ptr(c->e, 0, dst), h264mi_engine_frame_ptr(c->e, 0, src),
                       engine_slot_bytes(c->e), hipMemcpyDeviceToDevice));
    return 0;
}

static void hb_destroy(void *vctx)
{
    HipBackendCtx *c = (HipBackendCtx *)vctx;
    if (c->sh) share_detach(c);
    else if (c->e) engine_put(c->e);
    free(c->pref);
    (void)hipHostFree(c->h_slot_err);
    free(c);
}

// batches / pictures the device's shared engines launched since the process
// started; returns the instances attached now
extern "C" int h264mi_share_stats(int device, unsigned long long *batches, unsigned long long *pictures)
{
    if (device < 0 || device >= 16) return -1;
    std::lock_guard<std::mutex> g(g_share_mu);
    if (batches) *batches = g_share_batches[device].load();
    if (pictures) *pictures = g_share_pictures[device].load();
    int n = 0;
    for (int k = 0; k < SHARE_SIZES; k++) {
        SharedEng *sh = g_share[device][k];
        if (!sh) continue;
        std::lock_guard<std::mutex> l(sh->mu);
        n += sh->active;
    }
    return n;
}

extern "C" H264Backend h264mi_hip_backend_create(int device)
{
    H264Backend be;
    memset(&be, 0, sizeof(be));
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
        fprintf(stderr, "h264mi: no HIP device %d: the reconstruction path needs an MI355X\n", device);
        return be;                                  /* ctx == NULL: H264SwDecInit fails */
    }
    HipBackendCtx *c = (HipBackendCtx *)calloc(1, sizeof(HipBackendCtx));
    c->device = device;
    const char *ff = h264mi_test_hooks() ? getenv("H264MI_DEBUG_FLAG_PICTURE") : NULL;
    c->force_flag_at = ff && atoi(ff) > 0 ? (unsigned)atoi(ff) : 0;
    be.ctx = c;
    be.configure = hb_configure;
    be.decode = hb_decode;
    be.read = hb_read;
    be.read_rgba = hb_read_rgba;
    be.host_alloc = hb_host_alloc;
    be.host_free = hb_host_free;
    be.records_wait = hb_records_wait;
    be.copy = hb_copy;
    // H264MI_HOST_CONCEAL=1: conceal on the host (a copy of the picture, conceal.c)
    be.conceal = getenv("H264MI_HOST_CONCEAL") && atoi(getenv("H264MI_HOST_CONCEAL")) ? NULL : hb_conceal;
    be.conceal_ok = hb_conceal_ok;
    be.sync = hb_sync;
    be.prefetch = hb_prefetch;
    be.destroy = hb_destroy;
    return be;
}

// Frees every engine and pinned frame the pools hold (engines and frames in
// use are not touched); returns how many engines were freed.  Also run at
// process exit (register_drain_once).
extern "C" int h264mi_pool_drain(void)
{
    h264mi_engine *eng[ENGINE_POOL_MAX];
    int n = 0;
    {
        std::lock_guard<std::mutex> g(g_pool_mu);
        for (int i = 0; i < ENGINE_POOL_MAX; i++)
            if (g_pool[i]) { eng[n++] = g_pool[i]; g_pool[i] = NULL; }
    }
    for (int i = 0; i < n; i++) h264mi_engine_destroy(eng[i]);
    void *blk[HOST_POOL_N];
    int m = 0;
    {
        std::lock_guard<std::mutex> g(g_hpool_mu);
        for (int i = 0; i < HOST_POOL_N; i++)
            if (g_hpool[i].p) { blk[m++] = g_hpool[i].p; g_hpool[i].p = NULL; g_hpool[i].bytes = 0; }
    }
    for (int i = 0; i < m; i++) (void)hipHostFree(blk[i]);
    return n;
}

// pooled engines and pinned bytes held right now (diagnostics, tests)
extern "C" void h264mi_pool_held(int *engines, size_t *pinned_bytes)
{
    int n = 0;
    size_t b = 0;
    {
        std::lock_guard<std::mutex> g(g_pool_mu);
        for (int i = 0; i < ENGINE_POOL_MAX; i++) n += g_pool[i] != NULL;
    }
    {
        std::lock_guard<std::mutex> g(g_hpool_mu);
        for (int i = 0; i < HOST_POOL_N; i++) b += g_hpool[i].p ? g_hpool[i].bytes : 0;
    }
    if (engines) *engines = n;
    if (pinned_bytes) *pinned_bytes = b;
}

