// h264mi engine: HBM-resident frame slots, record upload, kernel launches.
// One engine serves `nstreams` independent bitstreams of one picture size
// (streams shard across GPUs with no collective; within a GPU
// one launch reconstructs one picture from each stream of the batch).
#include "recon_kernels.hip"
#include "color.hip"
#include "conceal.hip"
#include <hip/hip_ext.h>

#include <stdio.h>
#include <atomic>
#include <stdlib.h>
#include <string.h>
#include "../../../include/h264mi.h"

#define HIPCHECK(x)                                                                    \
    do {                                                                               \
        hipError_t err_ = (x);                                                         \
        if (err_ != hipSuccess) {                                                      \
            fprintf(stderr, "h264mi: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(err_), \
                    __FILE__, __LINE__);                                               \
            return -1;                                                                 \
        }                                                                              \
    } while (0)

struct h264mi_engine {
    int dev;
    int w, h, nmbs, nstreams, nslots;
    size_t frame_bytes;
    uint8_t *d_frames;
    unsigned long long *d_mbx;    // row mailboxes: 32 granules (256 B) per batch MB
    unsigned epoch;
    unsigned long long *d_prof;   // optional per-MB chain stamps (profiling k_wgpp)
    size_t prof_cap;
    int pipe_cap;                 // pictures per launch the per-picture buffers hold
    unsigned long long *d_gjunk;  // 64 KiB store sink (ReconArgs::gjunk)
    const char *last_kernel;      // name of the last batch's reconstruction kernel (diagnostics)
    uint8_t *d_dbrec;         // 64 B per batch MB (x2: k_prep double buffer)
    int16_t *d_res;           // 384 x int16 per batch MB (x2)
    // k_prep (deblocking records + residuals) writes buffer half prep_parity;
    // a batch prepped by the previous launch's tail workgroups is `prepped`
    int prep_parity;
    const void *prepped_rec, *prepped_pics;
    unsigned long long *d_rows_done;   // row workgroups finished, all launches (tail-prep trigger)
    // k_conceal inputs (order + decoded flags): pinned staging, device copy,
    // and an event after the upload (the staging's reuse waits for it)
    uint8_t *h_conceal, *d_conceal;
    hipEvent_t ev_conceal;
    int prep_wgs;                      // tail workgroups per launch (H264MI_PREP_WGS, default 2048)
    unsigned long long rows_launched;
    int prep_at_pct;                   // tail prep waits for this % of the launch's rows (H264MI_PREP_AT; 0: no wait)
    int mc_waves;                      // MC waves per row workgroup: 0 = per launch (below), 2 or 3 forced (H264MI_MC_WAVES)
    int launch_intra;                  // next launch: 1 = has an intra-heavy picture, 0 = none, -1 = unknown
    int rpw_max;                       // MB rows per k_wgpp workgroup allowed by LDS, 1..3
    int rpw_env;                       // H264MI_RPW: fixed rows per workgroup (0: by batch size)
    int ncu;
    MbRec *d_rec;
    int16_t *d_coef;
    size_t coef_cap;          // blocks
    PicDesc *d_pics;
    unsigned *d_err;
    MbRec *h_rec;             // pinned staging
    int16_t *h_coef;
    size_t h_coef_cap;
    PicDesc *h_pics;
    unsigned *h_err;
    hipStream_t st;
    hipEvent_t ev_staged, ev0, ev1, ev2;
    hipEvent_t ev_block;      // H264MI_BLOCKING_SYNC: h264mi_engine_sync sleeps on this event
    uint32_t err_accum;
    int timing;
    // per-batch kernel timing (h264mi_engine_set_timing): event triples
    hipEvent_t *tev;
    int tev_cap, tev_n;
    int tev_stride, tev_seq;  // record every tev_stride-th launch (h264mi_engine_set_timing_stride)
    uint8_t *d_rgba;          // h264mi_engine_read_rgba staging (w*h*4 B, allocated on first use)
    int steps;                // pictures per stream per launch (h264mi_engine_set_steps)
    unsigned *d_done;         // per picture row of a launch: epoch tag once the row is final in its slot
};

// per-picture buffers of one launch (deblocking records, residuals, row
// mailboxes, error flags), for `cap` pictures
static void free_pic_buffers(h264mi_engine *e)
{
    (void)hipFree(e->d_mbx); (void)hipFree(e->d_dbrec); (void)hipFree(e->d_res); (void)hipFree(e->d_err);
    (void)hipFree(e->d_done);
    (void)hipHostFree(e->h_err);
    e->d_mbx = NULL; e->d_dbrec = NULL; e->d_res = NULL; e->d_err = NULL; e->d_done = NULL;
    e->h_err = NULL;
    e->pipe_cap = 0;
}

static int alloc_pic_buffers(h264mi_engine *e, int cap)
{
    const size_t np = (size_t)cap, mbs = np * e->nmbs;
    bool ok = hipMalloc(&e->d_mbx, mbs * 256) == hipSuccess &&
              hipMalloc(&e->d_dbrec, 2 * mbs * 64) == hipSuccess &&
              hipMalloc(&e->d_res, 2 * mbs * 768) == hipSuccess &&
              hipMalloc(&e->d_err, sizeof(unsigned) * np) == hipSuccess &&
              hipMalloc(&e->d_done, sizeof(unsigned) * np * e->h) == hipSuccess &&
              hipHostMalloc(&e->h_err, sizeof(unsigned) * np, hipHostMallocDefault) == hipSuccess;
    if (!ok) { free_pic_buffers(e); return -1; }
    // cleared granules carry epoch 0, which no launch uses
    (void)hipMemsetAsync(e->d_mbx, 0, mbs * 256, e->st);
    (void)hipMemsetAsync(e->d_err, 0, sizeof(unsigned) * np, e->st);
    (void)hipMemsetAsync(e->d_done, 0, sizeof(unsigned) * np * e->h, e->st);
    memset(e->h_err, 0, sizeof(unsigned) * np);
    e->pipe_cap = cap;
    return 0;
}

// settings read from the environment at engine creation (and again when a
// pooled engine is taken for a new decoder instance)
static void engine_config(h264mi_engine *e)
{
    e->timing = getenv("H264MI_TIMING") != NULL;
    const char *pw = getenv("H264MI_PREP_WGS");
    e->prep_wgs = pw && atoi(pw) > 0 ? atoi(pw) : 2048;
    const char *pa = getenv("H264MI_PREP_AT");
    e->prep_at_pct = pa ? atoi(pa) : 0;
    const char *mw = getenv("H264MI_MC_WAVES");
    e->mc_waves = mw && (atoi(mw) == 2 || atoi(mw) == 3) ? atoi(mw) : 0;
    e->launch_intra = -1;
    const char *rp = getenv("H264MI_RPW");
    e->rpw_env = rp ? atoi(rp) : 0;
    if (e->rpw_env < 0 || e->rpw_env > 3) e->rpw_env = 0;
    // the group's LDS mailboxes (w * 256 B per inner row boundary) beside
    // the static LDS of its rows (regions, MC scratch, a RINGG-slot ring)
    // within the CU's 160 KB
    // k_wgpp's LDS is dynamic (WgppLds): allow every variant the CU's 160 KB
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_wgpp<3, false, true, 1>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_wgpp<3, true, true, 1>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_wgpp<3, false, true, 2>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_wgpp<3, true, true, 2>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_wgpp<3, false, true, 3>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_wgpp<3, true, true, 3>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_wgpp<2, false, true, 1>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_wgpp<2, false, true, 2>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_wgpp<2, true, true, 1>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    const size_t row_lds = sizeof(PPLds) + (size_t)(e->mc_waves == 2 ? 2 : 3) * sizeof(McScratch) + sizeof(MbRing<RINGG>);
    e->rpw_max = e->mc_waves == 2 ? 2 : 3;
    while (e->rpw_max > 1 && (size_t)(e->rpw_max - 1) * e->w * 256 + (size_t)e->rpw_max * row_lds > 156 * 1024)
        e->rpw_max--;
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, e->dev) != hipSuccess || ncu < 1) ncu = 256;
    e->ncu = ncu;
}

extern "C" h264mi_engine *h264mi_engine_create(int device, int w_mbs, int h_mbs, int nstreams, int nslots)
{
    if (w_mbs < 1 || h_mbs < 1 || h_mbs > 1024 || nstreams < 1 || nslots < 1) return NULL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device >= ndev) {
        fprintf(stderr, "h264mi: no HIP device %d (count %d)\n", device, ndev);
        return NULL;
    }
    if (hipSetDevice(device) != hipSuccess) return NULL;
    // H264MI_BLOCKING_SYNC=1: a thread waiting for the GPU sleeps instead of
    // spinning (many decoder processes with parse threads on few host cores)
    const bool blocking = getenv("H264MI_BLOCKING_SYNC") && atoi(getenv("H264MI_BLOCKING_SYNC"));
    if (blocking) (void)hipSetDeviceFlags(hipDeviceScheduleBlockingSync);
    h264mi_engine *e = (h264mi_engine *)calloc(1, sizeof(h264mi_engine));
    if (!e) return NULL;
    e->dev = device;
    e->w = w_mbs; e->h = h_mbs; e->nmbs = w_mbs * h_mbs;
    e->nstreams = nstreams; e->nslots = nslots;
    e->steps = 1;
    e->frame_bytes = (size_t)e->nmbs * 384;
    e->coef_cap = (size_t)nstreams * e->nmbs * 8 + 1024;
    e->h_coef_cap = e->coef_cap;
    bool ok = hipMalloc(&e->d_frames, e->frame_bytes * nslots * nstreams) == hipSuccess &&

              hipMalloc(&e->d_rec, sizeof(MbRec) * nstreams * e->nmbs) == hipSuccess &&
              hipMalloc(&e->d_coef, e->coef_cap * 32) == hipSuccess &&
              hipMalloc(&e->d_pics, sizeof(PicDesc) * nstreams) == hipSuccess &&
              hipMalloc(&e->d_gjunk, 65536) == hipSuccess &&

              hipHostMalloc(&e->h_rec, sizeof(MbRec) * nstreams * e->nmbs, hipHostMallocDefault) == hipSuccess &&
              hipHostMalloc(&e->h_coef, e->h_coef_cap * 32, hipHostMallocDefault) == hipSuccess &&
              hipHostMalloc(&e->h_pics, sizeof(PicDesc) * nstreams, hipHostMallocDefault) == hipSuccess &&

              hipStreamCreateWithFlags(&e->st, hipStreamNonBlocking) == hipSuccess &&
              hipEventCreateWithFlags(&e->ev_staged, hipEventDisableTiming | (blocking ? hipEventBlockingSync : 0)) == hipSuccess &&
              hipEventCreate(&e->ev0) == hipSuccess && hipEventCreate(&e->ev1) == hipSuccess &&
              hipEventCreate(&e->ev2) == hipSuccess &&
              (!blocking || hipEventCreateWithFlags(&e->ev_block, hipEventDisableTiming | hipEventBlockingSync) == hipSuccess) &&
              hipMalloc(&e->d_rows_done, sizeof(unsigned long long)) == hipSuccess;
    ok = ok && alloc_pic_buffers(e, nstreams) == 0;
    if (!ok) {
        fprintf(stderr, "h264mi: engine allocation failed\n");
        h264mi_engine_destroy(e);
        return NULL;
    }
    (void)hipMemsetAsync(e->d_frames, 0, e->frame_bytes * nslots * nstreams, e->st);
    (void)hipMemsetAsync(e->d_rows_done, 0, sizeof(unsigned long long), e->st);
    engine_config(e);
    e->epoch = 0;
    (void)hipEventRecord(e->ev_staged, e->st);
    (void)hipStreamSynchronize(e->st);
    return e;
}

extern "C" void h264mi_engine_destroy(h264mi_engine *e)
{
    if (!e) return;
    if (e->st) (void)hipStreamSynchronize(e->st);
    free_pic_buffers(e);
    (void)hipFree(e->d_rgba);
    (void)hipFree(e->d_frames); (void)hipFree(e->d_prof); (void)hipFree(e->d_rec); (void)hipFree(e->d_coef);
    (void)hipFree(e->d_pics); (void)hipFree(e->d_gjunk);
    (void)hipHostFree(e->h_rec); (void)hipHostFree(e->h_coef); (void)hipHostFree(e->h_pics);
    if (e->ev_staged) (void)hipEventDestroy(e->ev_staged);
    if (e->ev0) (void)hipEventDestroy(e->ev0);
    if (e->ev1) (void)hipEventDestroy(e->ev1);
    if (e->ev2) (void)hipEventDestroy(e->ev2);
    if (e->ev_block) (void)hipEventDestroy(e->ev_block);
    (void)hipFree(e->d_rows_done);
    if (e->h_conceal) (void)hipHostFree(e->h_conceal);
    if (e->d_conceal) (void)hipFree(e->d_conceal);
    if (e->ev_conceal) (void)hipEventDestroy(e->ev_conceal);
    h264mi_engine_set_timing(e, 0);
    if (e->st) (void)hipStreamDestroy(e->st);
    free(e);
}

// Released private engines, kept for the next decoder instance of the same
// shape: DecTestBench-style callers create one H264SwDec instance per stream
// (H264SwDecInit ... H264SwDecRelease), and a fresh engine costs ~20 device
// and pinned allocations, a stream, events and a frame clear.  A pooled
// engine is idle (its stream drained) and is handed out as a fresh one would
// be: frames cleared, no batch prepped, settings re-read.  H264MI_ENGINE_POOL=0
// turns it off.
#include <mutex>
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
    if (engine_pool_on()) {
        std::lock_guard<std::mutex> g(g_pool_mu);
        for (int i = 0; i < ENGINE_POOL_MAX && !e; i++) {
            h264mi_engine *x = g_pool[i];
            if (x && x->dev == device && x->w == w_mbs && x->h == h_mbs && x->nstreams == nstreams && x->nslots == nslots) {
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
    if (hipSetDevice(device) != hipSuccess) { h264mi_engine_destroy(e); return NULL; }
    engine_config(e);
    e->prepped_rec = e->prepped_pics = NULL;
    e->err_accum = 0;
    e->steps = 1;
    e->last_kernel = NULL;
    // the epoch keeps counting: the mailboxes hold tags of earlier launches only
    (void)hipMemsetAsync(e->d_frames, 0, e->frame_bytes * e->nslots * e->nstreams, e->st);
    return e;
}

static void engine_put(h264mi_engine *e)
{
    if (!e) return;
    // engines with diagnostics state (timing events, profiling buffers) are not kept
    if (engine_pool_on() && !e->tev && !e->d_prof && hipSetDevice(e->dev) == hipSuccess &&
        hipStreamSynchronize(e->st) == hipSuccess) {
        std::lock_guard<std::mutex> g(g_pool_mu);
        for (int i = 0; i < ENGINE_POOL_MAX; i++)
            if (!g_pool[i]) { g_pool[i] = e; return; }
    }
    h264mi_engine_destroy(e);
}

// k_prep of a batch as its own launch (the batch was not prepped by the
// previous launch's tail): deblocking records + residuals into buffer half hb
static int launch_prep(h264mi_engine *e, int npics, const MbRec *d_rec, const int16_t *d_coef,
                       const PicDesc *d_pics, int hb)
{
    const size_t mbs = (size_t)e->pipe_cap * e->nmbs;
    PrepArgs pa;
    pa.rec = d_rec; pa.coef = d_coef; pa.pics = d_pics;
    pa.dbrec = e->d_dbrec + hb * mbs * 64;
    pa.res = e->d_res + hb * mbs * 384;
    pa.nmbs_total = npics * e->nmbs;
    pa.w = e->w; pa.h = e->h;
    hipLaunchKernelGGL(k_prep, dim3((pa.nmbs_total + 3) / 4), dim3(256), 0, e->st, pa);
    HIPCHECK(hipGetLastError());
    return 0;
}

// One reconstruction step for a batch of npics pictures (one per stream), all
// on the engine's stream: k_prep unless the previous launch's tail already
// prepped this batch, then k_wgpp -- one workgroup per (picture, MB row): MC
// waves + ping-pong deblocking row waves -- plus, when the next batch is
// known (next_rec != NULL), tail workgroups that run the next batch's k_prep
// as this launch's rows drain.  k_prep outputs alternate between two buffer
// halves; stream order separates writer and reader.
// rows per workgroup: while the batch's rows fit the chip as single-row
// workgroups (three per CU), one row each -- a picture's latency is the
// bound and three chains on one CU contend; beyond that, three rows per
// workgroup with LDS hand-offs inside (measured, 1080p: S = 8 410 vs 440 us
// per launch; S = 32 1368 vs 1113 us).  H264MI_RPW fixes it; the LDS budget
// (rpw_max) and the 2-MC-wave builds cap it.
static int rows_per_wg(const h264mi_engine *e, int S)
{
    int rpw = e->rpw_env ? e->rpw_env : (S * e->h > 3 * e->ncu ? 3 : 1);
    if (rpw > e->rpw_max) rpw = e->rpw_max;
    if (e->mc_waves == 2 && rpw > 2) rpw = 2;
    return rpw;
}

// MC waves per single-row workgroup, per launch.  Three MC waves make a
// 5-wave workgroup, admitted 2 per CU (tools/ubench/census.hip): a 1080p
// picture's rows 64..67 then wait ~180 us for a slot, but intra pictures,
// whose MC is the critical path, need the third wave.  Two make a 4-wave
// workgroup, 3 per CU, every row resident from the start; with the MC
// urgency priority (recon_kernels.hip mc_row) P pictures gain (measured,
// configs[3] P-only: 350 vs 355 us per launch; a launch with an I picture:
// ~40 us slower).  So: 2 unless the launch holds an intra-heavy picture
// (more than half its MBs intra) or its content is unknown.
static int launch_nmc(const h264mi_engine *e, int rpw)
{
    if (e->mc_waves) return e->mc_waves;
    if (rpw > 1) return 3;
    return e->launch_intra == 0 ? 2 : 3;
}

static int launch_batch(h264mi_engine *e, int S, int P, const MbRec *d_rec, const int16_t *d_coef,
                        const PicDesc *d_pics, const MbRec *next_rec, const int16_t *next_coef,
                        const PicDesc *next_pics)
{
    const int npics = S * P;
    const size_t mbs = (size_t)e->pipe_cap * e->nmbs;
    const int hb = e->prep_parity;
    // study knob (H264MI_NO_TAIL_PREP=1): every batch's k_prep as its own
    // launch in front of k_wgpp, none in the tail -- k_wgpp's time without
    // the next batch's prep work beside the chain
    static const bool no_tail = getenv("H264MI_NO_TAIL_PREP") && atoi(getenv("H264MI_NO_TAIL_PREP"));
    if (no_tail) next_rec = nullptr, next_coef = nullptr, next_pics = nullptr;
    if (!(e->prepped_rec && e->prepped_rec == (const void *)d_rec && e->prepped_pics == (const void *)d_pics))
        if (launch_prep(e, npics, d_rec, d_coef, d_pics, hb)) return -1;
    ReconArgs a;
    memset(&a, 0, sizeof(a));
    a.frames = e->d_frames;
    a.frame_bytes = e->frame_bytes;
    a.rec = d_rec;
    a.coef = d_coef;
    a.mbx = e->d_mbx;
    a.gjunk = e->d_gjunk;
    if (++e->epoch >= (1u << 20)) {           // granule tags: epoch in the high dword
        if (h264mi_engine_sync(e)) return -1;
        HIPCHECK(hipMemsetAsync(e->d_mbx, 0, mbs * 256, e->st));
        HIPCHECK(hipMemsetAsync(e->d_done, 0, sizeof(unsigned) * e->pipe_cap * e->h, e->st));
        e->epoch = 1;
    }
    a.epoch = e->epoch;
    a.prof = e->d_prof;
    a.prof_mode = e->d_prof && getenv("H264MI_PROF_MODE") ? atoi(getenv("H264MI_PROF_MODE")) : 0;
    // study knobs: MC lead over the row's deblocking (MBs; 0 / unset = the
    // ring depth), before the chain has begun (LEAD0, at least 4) and after
    static const int mc_lead0 = getenv("H264MI_MC_LEAD0") ? std::max(4, atoi(getenv("H264MI_MC_LEAD0"))) : 0;
    static const int mc_lead = getenv("H264MI_MC_LEAD") ? std::max(4, atoi(getenv("H264MI_MC_LEAD"))) : 0;
    a.mc_lead0 = mc_lead0;
    a.mc_lead = mc_lead;
    static const int row_prio = getenv("H264MI_ROW_PRIO") ? atoi(getenv("H264MI_ROW_PRIO")) : 0;
    a.row_prio_split = row_prio;
    a.pics = d_pics;
    a.npics = npics;
    a.w = e->w; a.h = e->h;
    a.err = e->d_err;
    a.S = S;
    a.P = P;
    a.done = e->d_done;
    a.dbrec = e->d_dbrec + hb * mbs * 64;
    a.res = e->d_res + hb * mbs * 384;
    const int rows = npics * e->h;
    if (next_rec) {
        a.prep_wgs = e->prep_wgs;
        a.rows_done = e->d_rows_done;
        a.prep_target = e->rows_launched + (unsigned long long)((long long)rows * e->prep_at_pct / 100);
        a.n_rec = next_rec; a.n_coef = next_coef; a.n_pics = next_pics;
        a.n_dbrec = e->d_dbrec + (hb ^ 1) * mbs * 64;
        a.n_res = e->d_res + (hb ^ 1) * mbs * 384;
        a.n_nmbs_total = npics * e->nmbs;
    } else {
        a.rows_done = e->d_rows_done;
    }
    hipEvent_t t0 = e->ev0, t2 = e->ev2;
    bool rec_tev = false;
    if (e->tev && e->tev_n < e->tev_cap && e->tev_seq++ % (e->tev_stride > 0 ? e->tev_stride : 1) == 0) {
        t0 = e->tev[3 * e->tev_n]; t2 = e->tev[3 * e->tev_n + 2];
        e->tev_n++;
        rec_tev = true;
    }
    const bool rec = e->timing || rec_tev;
    e->last_kernel = "k_wgpp";
    const int rpw = rows_per_wg(e, S);
    const dim3 grid(npics * ((e->h + rpw - 1) / rpw) + a.prep_wgs);
    const int nmc = launch_nmc(e, rpw);
    e->launch_intra = -1;                     // a hint covers one launch
    const size_t lmbx = nmc == 2 && (!a.prof || rpw == 1) ? (rpw == 2 ? WgppLds<2, 2>::bytes(e->w) : WgppLds<2, 1>::bytes(e->w))
                        : rpw == 3 ? WgppLds<3, 3>::bytes(e->w) : rpw == 2 ? WgppLds<3, 2>::bytes(e->w)
                        : WgppLds<3, 1>::bytes(e->w);
    if (a.prof) {
        if (rec) (void)hipEventRecord(t0, e->st);
        if (rpw == 3) hipLaunchKernelGGL((k_wgpp<3, true, true, 3>), grid, dim3(960), lmbx, e->st, a);
        else if (rpw == 2) hipLaunchKernelGGL((k_wgpp<3, true, true, 2>), grid, dim3(640), lmbx, e->st, a);
        else if (nmc == 2) hipLaunchKernelGGL((k_wgpp<2, true, true, 1>), grid, dim3(256), lmbx, e->st, a);
        else hipLaunchKernelGGL((k_wgpp<3, true, true, 1>), grid, dim3(320), lmbx, e->st, a);
        if (rec) (void)hipEventRecord(t2, e->st);
    } else if (nmc == 2) {
        // sizing study (H264MI_MC_WAVES=2): two MC waves per row workgroup
        if (rpw == 2)
            hipExtLaunchKernelGGL((k_wgpp<2, false, true, 2>), grid, dim3(512), lmbx, e->st, rec ? t0 : nullptr,
                                  rec ? t2 : nullptr, 0, a);
        else
            hipExtLaunchKernelGGL((k_wgpp<2, false, true, 1>), grid, dim3(256), lmbx, e->st, rec ? t0 : nullptr,
                                  rec ? t2 : nullptr, 0, a);
    } else if (rpw == 3) {
        // the timing events ride on the kernel's own dispatch packet
        // (hipExtLaunchKernelGGL): no marker packets between launches
        hipExtLaunchKernelGGL((k_wgpp<3, false, true, 3>), grid, dim3(960), lmbx, e->st, rec ? t0 : nullptr,
                              rec ? t2 : nullptr, 0, a);
    } else if (rpw == 2) {
        hipExtLaunchKernelGGL((k_wgpp<3, false, true, 2>), grid, dim3(640), lmbx, e->st, rec ? t0 : nullptr,
                              rec ? t2 : nullptr, 0, a);
    } else {
        hipExtLaunchKernelGGL((k_wgpp<3, false, true, 1>), grid, dim3(320), lmbx, e->st, rec ? t0 : nullptr,
                              rec ? t2 : nullptr, 0, a);
    }
    HIPCHECK(hipGetLastError());
    e->rows_launched += rows;
    e->prepped_rec = next_rec;
    e->prepped_pics = next_pics;
    e->prep_parity = hb ^ 1;                  // the half the next batch was (or will be) prepped into
    return 0;
}

// intra_heavy: the batch's launch shape hint when the caller knows it (the
// host path counts intra MBs while parsing); -1: derive it from the records
static int engine_decode_host(h264mi_engine *e, int npics, const int *stream, const int *cur_slot,
                              const void *const *recs, const int16_t *const *coefs, const uint32_t *ncoef,
                              int intra_heavy);

extern "C" int h264mi_engine_decode(h264mi_engine *e, int npics, const int *stream, const int *cur_slot,
                                    const void *const *recs, const int16_t *const *coefs, const uint32_t *ncoef)
{
    return engine_decode_host(e, npics, stream, cur_slot, recs, coefs, ncoef, -1);
}

static int engine_decode_host(h264mi_engine *e, int npics, const int *stream, const int *cur_slot,
                              const void *const *recs, const int16_t *const *coefs, const uint32_t *ncoef,
                              int intra_heavy)
{
    if (!e || npics < 1 || npics > e->nstreams) return -1;
    HIPCHECK(hipSetDevice(e->dev));
    // staging buffers are reused: wait until the previous upload consumed them
    HIPCHECK(hipEventSynchronize(e->ev_staged));
    size_t total = 0;
    for (int i = 0; i < npics; i++) total += ncoef[i];
    if (total + 16 > e->coef_cap) {
        HIPCHECK(hipStreamSynchronize(e->st));
        (void)hipFree(e->d_coef);
        (void)hipHostFree(e->h_coef);
        e->coef_cap = e->h_coef_cap = total + total / 2 + 1024;
        HIPCHECK(hipMalloc(&e->d_coef, e->coef_cap * 32));
        HIPCHECK(hipHostMalloc(&e->h_coef, e->h_coef_cap * 32, hipHostMallocDefault));
    }
    size_t cbase = 0;
    for (int i = 0; i < npics; i++) {
        if (stream[i] < 0 || stream[i] >= e->nstreams || cur_slot[i] < 0 || cur_slot[i] >= e->nslots) return -1;
        memcpy(e->h_rec + (size_t)i * e->nmbs, recs[i], sizeof(MbRec) * e->nmbs);
        if (ncoef[i]) memcpy(e->h_coef + cbase * 16, coefs[i], (size_t)ncoef[i] * 32);
        PicDesc &pd = e->h_pics[i];
        pd.rec_base = (uint32_t)(i * e->nmbs);
        pd.frame_base = (uint32_t)(stream[i] * e->nslots);
        pd.cur_slot = (uint32_t)cur_slot[i];
        pd.flags = 0;
        pd.coef_base = (uint32_t)cbase;
        pd.rsv[0] = pd.rsv[1] = pd.rsv[2] = 0;
        cbase += ncoef[i];
    }
    HIPCHECK(hipMemcpyAsync(e->d_rec, e->h_rec, sizeof(MbRec) * e->nmbs * npics, hipMemcpyHostToDevice, e->st));
    if (cbase) HIPCHECK(hipMemcpyAsync(e->d_coef, e->h_coef, cbase * 32, hipMemcpyHostToDevice, e->st));
    HIPCHECK(hipMemcpyAsync(e->d_pics, e->h_pics, sizeof(PicDesc) * npics, hipMemcpyHostToDevice, e->st));
    HIPCHECK(hipEventRecord(e->ev_staged, e->st));
    // the batch's shape hint from its records (launch_nmc)
    int heavy = intra_heavy > 0;
    for (int i = 0; i < npics && !heavy && intra_heavy < 0; i++) {
        const MbRec *r = (const MbRec *)recs[i];
        int n = 0;
        for (int m = 0; m < e->nmbs; m++) n += r[m].type >= MBT_I4x4;
        heavy = 2 * n > e->nmbs;
    }
    e->launch_intra = heavy;
    return launch_batch(e, npics, 1, e->d_rec, e->d_coef, e->d_pics, NULL, NULL, NULL);
}

// the next launch's content, for callers holding their records on the device
// (launch_nmc): 1 = some picture has more than half its MBs intra, 0 = none
extern "C" int h264mi_engine_hint_intra(h264mi_engine *e, int intra_heavy)
{
    if (!e || intra_heavy < 0 || intra_heavy > 1) return -1;
    e->launch_intra = intra_heavy;
    return 0;
}

extern "C" int h264mi_engine_decode_device(h264mi_engine *e, int npics, const void *d_recs, const int16_t *d_coef,
                                           const void *d_pics)
{
    return h264mi_engine_decode_device_next(e, npics, d_recs, d_coef, d_pics, NULL, NULL, NULL);
}

extern "C" int h264mi_engine_decode_device_next(h264mi_engine *e, int npics, const void *d_recs,
                                                const int16_t *d_coef, const void *d_pics, const void *next_recs,
                                                const int16_t *next_coef, const void *next_pics)
{
    if (!e || npics < 1 || npics > e->nstreams || !d_recs || !d_pics) return -1;
    if (next_recs && !next_pics) return -1;
    HIPCHECK(hipSetDevice(e->dev));
    return launch_batch(e, npics, 1, (const MbRec *)d_recs, d_coef, (const PicDesc *)d_pics, (const MbRec *)next_recs,
                        next_coef, (const PicDesc *)next_pics);
}

// frame-pipelined batches: P (<= the engine's steps) consecutive pictures of
// each of S streams in one launch, step-major (descriptor j * S + s), every
// PicDesc.rec_base relative to d_recs; the caller guarantees that no picture
// of the batch writes a slot an earlier picture of the batch reads or writes
extern "C" int h264mi_engine_decode_device_steps(h264mi_engine *e, int S, int P, const void *d_recs,
                                                 const int16_t *d_coef, const void *d_pics, const void *next_recs,
                                                 const int16_t *next_coef, const void *next_pics)
{
    if (!e || S < 1 || S > e->nstreams || P < 1 || P > e->steps || !d_recs || !d_pics) return -1;
    if (next_recs && !next_pics) return -1;
    HIPCHECK(hipSetDevice(e->dev));
    return launch_batch(e, S, P, (const MbRec *)d_recs, d_coef, (const PicDesc *)d_pics, (const MbRec *)next_recs,
                        next_coef, (const PicDesc *)next_pics);
}

// diagnostics: resident k_wgpp workgroups per CU the runtime computes for
// the main single-row kernel (rpw 1), and its kernel attributes
extern "C" int h264mi_kernel_occupancy(int *blocks_per_cu, int *lds_bytes, int *vgprs, int *sgprs)
{
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(&k_wgpp<3, false, true, 1>)) != hipSuccess) return -1;
    int n = 0;
    const size_t lds = WgppLds<3, 1>::bytes(120);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_wgpp<3, false, true, 1>, 320, lds) != hipSuccess) return -1;
    if (blocks_per_cu) *blocks_per_cu = n;
    if (lds_bytes) *lds_bytes = (int)(fa.sharedSizeBytes + lds);
    if (vgprs) *vgprs = fa.numRegs;
    if (sgprs) *sgprs = 0;
    return 0;
}

extern "C" int h264mi_engine_set_steps(h264mi_engine *e, int steps)
{
    if (!e || steps < 1 || steps > 2) return -1;
    if (steps == e->steps) return 0;
    if (h264mi_engine_sync(e)) return -1;
    free_pic_buffers(e);
    if (alloc_pic_buffers(e, e->nstreams * steps)) return -1;
    e->steps = steps;
    e->prepped_rec = NULL; e->prepped_pics = NULL;
    e->prep_parity = 0;
    HIPCHECK(hipStreamSynchronize(e->st));
    return 0;
}

extern "C" const char *h264mi_engine_kernel(h264mi_engine *e)
{
    return e && e->last_kernel ? e->last_kernel : "";
}

// wait for everything queued on the engine's stream (sleeping under
// H264MI_BLOCKING_SYNC); no flag accounting
static int engine_wait(h264mi_engine *e)
{
    HIPCHECK(hipSetDevice(e->dev));
    if (e->ev_block) {
        HIPCHECK(hipEventRecord(e->ev_block, e->st));
        HIPCHECK(hipEventSynchronize(e->ev_block));
    } else {
        HIPCHECK(hipStreamSynchronize(e->st));
    }
    return 0;
}

extern "C" int h264mi_engine_sync(h264mi_engine *e)
{
    if (!e) return -1;
    HIPCHECK(hipSetDevice(e->dev));
    // per-picture error flags OR-accumulate over every launch since the last
    // sync (no per-launch reset): fetch them into pinned memory and clear
    // them behind the launches, one wait for all, then count the flagged
    // picture slots
    HIPCHECK(hipMemcpyAsync(e->h_err, e->d_err, sizeof(unsigned) * e->pipe_cap, hipMemcpyDeviceToHost, e->st));
    HIPCHECK(hipMemsetAsync(e->d_err, 0, sizeof(unsigned) * e->pipe_cap, e->st));
    // a blocking-sync event: the waiting thread sleeps whatever the device's
    // scheduling flags (which take effect only before the first context)
    if (engine_wait(e)) return -1;
    for (int i = 0; i < e->pipe_cap; i++) e->err_accum += e->h_err[i] ? 1 : 0;
    return 0;
}

extern "C" int h264mi_engine_rows_per_workgroup(h264mi_engine *e, int npics)
{
    return e && npics > 0 ? rows_per_wg(e, npics) : 0;
}

extern "C" uint32_t h264mi_engine_errors(h264mi_engine *e)
{
    if (!e) return 0;
    uint32_t v = e->err_accum;
    e->err_accum = 0;
    return v;
}

extern "C" int h264mi_engine_last_timing(h264mi_engine *e, float *us2)
{
    if (!e || !e->timing) return -1;
    float ms0 = 0, ms1 = 0;
    HIPCHECK(hipEventSynchronize(e->ev2));
    HIPCHECK(hipEventElapsedTime(&ms1, e->ev0, e->ev2));
    us2[0] = ms0 * 1000.f;
    us2[1] = ms1 * 1000.f;
    return 0;
}

extern "C" int h264mi_engine_set_timing(h264mi_engine *e, int max_batches)
{
    if (!e) return -1;
    if (e->tev) {
        for (int i = 0; i < 3 * e->tev_cap; i++) (void)hipEventDestroy(e->tev[i]);
        free(e->tev);
        e->tev = NULL;
    }
    e->tev_cap = e->tev_n = 0;
    e->tev_seq = 0;
    if (max_batches <= 0) return 0;
    e->tev = (hipEvent_t *)calloc((size_t)max_batches * 3, sizeof(hipEvent_t));
    if (!e->tev) return -1;
    for (int i = 0; i < 3 * max_batches; i++) HIPCHECK(hipEventCreate(&e->tev[i]));
    e->tev_cap = max_batches;
    return 0;
}

extern "C" int h264mi_engine_set_timing_stride(h264mi_engine *e, int stride)
{
    if (!e || stride < 1) return -1;
    e->tev_stride = stride;
    e->tev_seq = 0;
    return 0;
}

extern "C" int h264mi_engine_timing_report(h264mi_engine *e, double *inter_us, double *wave_us, int *nbatches)
{
    if (!e || !e->tev) return -1;
    if (h264mi_engine_sync(e)) return -1;
    double a = 0, b = 0;
    for (int i = 0; i < e->tev_n; i++) {
        float m0 = 0, m1 = 0;
        HIPCHECK(hipEventElapsedTime(&m1, e->tev[3 * i], e->tev[3 * i + 2]));
        a += m0 * 1000.0;
        b += m1 * 1000.0;
    }
    *inter_us = a;
    *wave_us = b;
    *nbatches = e->tev_n;
    e->tev_n = 0;
    return 0;
}

extern "C" int h264mi_engine_profile(h264mi_engine *e, int enable, unsigned long long *out, size_t n)
{
    if (!e) return -1;
    HIPCHECK(hipSetDevice(e->dev));
    if (out && e->d_prof) {
        HIPCHECK(hipStreamSynchronize(e->st));
        HIPCHECK(hipMemcpy(out, e->d_prof, sizeof(unsigned long long) * (n < e->prof_cap ? n : e->prof_cap),
                           hipMemcpyDeviceToHost));
    }
    if (enable && !e->d_prof) {
        e->prof_cap = (size_t)e->pipe_cap * e->h * 16 + (size_t)e->pipe_cap * e->nmbs * PROF_MB;
        HIPCHECK(hipMalloc(&e->d_prof, sizeof(unsigned long long) * e->prof_cap));
        HIPCHECK(hipMemset(e->d_prof, 0, sizeof(unsigned long long) * e->prof_cap));
    } else if (!enable && e->d_prof) {
        HIPCHECK(hipStreamSynchronize(e->st));
        (void)hipFree(e->d_prof);
        e->d_prof = NULL;
        e->prof_cap = 0;
    }
    return 0;
}

extern "C" int h264mi_engine_read(h264mi_engine *e, int stream, int slot, uint8_t *dst)
{
    if (!e || stream < 0 || stream >= e->nstreams || slot < 0 || slot >= e->nslots) return -1;
    if (h264mi_engine_sync(e)) return -1;
    HIPCHECK(hipMemcpy(dst, e->d_frames + e->frame_bytes * ((size_t)stream * e->nslots + slot), e->frame_bytes,
                       hipMemcpyDeviceToHost));
    return 0;
}

// I420 -> RGBA (DecoderPost.js `rgb: true`, color.hip) for `npics` pictures
// of width x height pixels at in + k * in_stride -> out + k * out_stride,
// device pointers, on `stream` (NULL: the null stream); asynchronous
extern "C" int h264mi_yuv2rgba_device(const void *d_i420, void *d_rgba, int width, int height, int npics,
                                      size_t in_stride, size_t out_stride, void *stream)
{
    if (!d_i420 || !d_rgba || width <= 0 || height <= 0 || (width & 15) || (height & 15) || npics < 1) return -1;
    const int nblk = ((height >> 1) * (width >> 2) + 127) >> 7;
    hipLaunchKernelGGL(k_yuv2rgba, dim3(nblk, npics), dim3(64), 0, (hipStream_t)stream,
                       (const uint8_t *)d_i420, (uint8_t *)d_rgba, width, height, in_stride, out_stride);
    HIPCHECK(hipGetLastError());
    return 0;
}

extern "C" int h264mi_engine_read_rgba(h264mi_engine *e, int stream, int slot, uint8_t *dst)
{
    if (!e || stream < 0 || stream >= e->nstreams || slot < 0 || slot >= e->nslots) return -1;
    const size_t bytes = (size_t)e->nmbs * 256 * 4;
    if (!e->d_rgba) HIPCHECK(hipMalloc(&e->d_rgba, bytes));
    if (h264mi_yuv2rgba_device(e->d_frames + e->frame_bytes * ((size_t)stream * e->nslots + slot), e->d_rgba,
                               e->w * 16, e->h * 16, 1, 0, 0, e->st))
        return -1;
    HIPCHECK(hipMemcpyAsync(dst, e->d_rgba, bytes, hipMemcpyDeviceToHost, e->st));
    HIPCHECK(hipStreamSynchronize(e->st));
    return 0;
}

extern "C" void *h264mi_engine_frame_ptr(h264mi_engine *e, int stream, int slot)
{
    if (!e) return NULL;
    return e->d_frames + e->frame_bytes * ((size_t)stream * e->nslots + slot);
}

extern "C" size_t h264mi_engine_frame_bytes(h264mi_engine *e) { return e ? e->frame_bytes : 0; }

// neighbour-based concealment of a picture's missing MBs on the device
// (k_conceal, conceal.hip), behind the work already on the engine's stream:
// slot `slot` of stream `stream` holds the decoded MBs reconstructed with the
// loop filter off; order[0..n) are the MBs to conceal in h264bsdConceal's
// order, decoded[0..w*h) the MBs decoded (1) or missing (0).  The inputs are
// copied before returning.
static std::atomic<unsigned long long> g_conceal_launches{0};
// diagnostics: k_conceal launches in this process (tests: the device path ran)
extern "C" unsigned long long h264mi_conceal_launches(void) { return g_conceal_launches.load(); }

extern "C" int h264mi_engine_conceal(h264mi_engine *e, int stream, int slot, const int *order, int n,
                                     const uint8_t *decoded)
{
    if (!e || stream < 0 || stream >= e->nstreams || slot < 0 || slot >= e->nslots || n < 0 || n > e->nmbs ||
        (n && (!order || !decoded)))
        return -1;
    if (!n) return 0;
    for (int i = 0; i < n; i++) if (order[i] < 0 || order[i] >= e->nmbs) return -1;
    HIPCHECK(hipSetDevice(e->dev));
    const size_t bytes = (size_t)e->nmbs * (sizeof(int) + 1);
    if (!e->d_conceal) {
        HIPCHECK(hipMalloc(&e->d_conceal, bytes));
        HIPCHECK(hipHostMalloc(&e->h_conceal, bytes, hipHostMallocDefault));
        HIPCHECK(hipEventCreateWithFlags(&e->ev_conceal, hipEventDisableTiming));
    } else {
        HIPCHECK(hipEventSynchronize(e->ev_conceal));
    }
    memcpy(e->h_conceal, order, sizeof(int) * (size_t)n);
    memcpy(e->h_conceal + sizeof(int) * (size_t)e->nmbs, decoded, (size_t)e->nmbs);
    HIPCHECK(hipMemcpyAsync(e->d_conceal, e->h_conceal, bytes, hipMemcpyHostToDevice, e->st));
    HIPCHECK(hipEventRecord(e->ev_conceal, e->st));
    hipLaunchKernelGGL(k_conceal, dim3(1), dim3(64), (size_t)e->nmbs, e->st, (uint8_t *)h264mi_engine_frame_ptr(e, stream, slot),
                       e->w, e->h, (const int *)e->d_conceal, n, (const uint8_t *)(e->d_conceal + sizeof(int) * (size_t)e->nmbs));
    HIPCHECK(hipGetLastError());
    g_conceal_launches++;
    return 0;
}

extern "C" void *h264mi_device_alloc(size_t bytes)
{
    void *p = NULL;
    if (hipMalloc(&p, bytes) != hipSuccess) return NULL;
    return p;
}

extern "C" int h264mi_device_free(void *p) { return hipFree(p) == hipSuccess ? 0 : -1; }

extern "C" int h264mi_copy_h2d(void *dst, const void *src, size_t bytes)
{
    return hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
}

// engine-scoped device memory: on the engine's GPU whatever the calling
// thread's current device is (one process per GPU: rank r's record batches
// must live on GPU r, next to its frame slots and launches)
extern "C" int h264mi_engine_device(const h264mi_engine *e) { return e ? e->dev : -1; }

extern "C" void *h264mi_engine_alloc(h264mi_engine *e, size_t bytes)
{
    if (!e || !bytes || hipSetDevice(e->dev) != hipSuccess) return NULL;
    void *p = NULL;
    if (hipMalloc(&p, bytes) != hipSuccess) return NULL;
    return p;
}

extern "C" int h264mi_engine_free(h264mi_engine *e, void *p)
{
    if (!e || hipSetDevice(e->dev) != hipSuccess) return -1;
    return hipFree(p) == hipSuccess ? 0 : -1;
}

extern "C" int h264mi_engine_copy_h2d(h264mi_engine *e, void *dst, const void *src, size_t bytes)
{
    if (!e || h264mi_pointer_device(dst) != e->dev) return -1;
    HIPCHECK(hipSetDevice(e->dev));
    HIPCHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, e->st));
    HIPCHECK(hipStreamSynchronize(e->st));
    return 0;
}

extern "C" int h264mi_pointer_device(const void *p)
{
    if (!p) return -1;
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    if (at.type != hipMemoryTypeDevice) return -1;
    return at.device;
}

// -------- H264Backend adapter for the single-stream host decoder ----------
#include "../host/decoder.h"
#include <mutex>
#include <condition_variable>
#include <chrono>
#include <atomic>

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
    std::condition_variable cv;
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
        if (sh->force[i]) (void)hipMemsetAsync(e->d_err + i, 0x01, sizeof(unsigned), e->st);
    bool heavy = false;
    for (int i = 0; i < sh->np; i++) heavy |= sh->heavy[i];
    int rc = engine_decode_host(e, sh->np, sh->stream, sh->slot, sh->recs, sh->coefs, sh->nc, heavy ? 1 : 0);
    // each picture's device flags (ReconArgs::err, one word per batch
    // picture) into its instance's word for the slot it was reconstructed
    // into, then cleared for the next batch
    for (int i = 0; i < sh->np && rc == 0; i++)
        if (hipMemcpyAsync(sh->who[i]->h_slot_err + sh->slot[i], e->d_err + i, sizeof(unsigned),
                           hipMemcpyDeviceToHost, e->st) != hipSuccess)
            rc = -1;
    if (hipMemsetAsync(e->d_err, 0, sizeof(unsigned) * sh->np, e->st) != hipSuccess) rc = -1;
    sh->rc_ring[sh->collecting % SHARE_RC_RING] = rc;
    for (int i = 0; i < sh->np; i++) (void)hipEventRecord(sh->who[i]->ev_last, e->st);
    g_share_batches[sh->device] += 1;
    g_share_pictures[sh->device] += (unsigned long long)sh->np;
    sh->np = 0;
    sh->launched = sh->collecting;
    sh->collecting++;
    sh->cv.notify_all();
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
        if (last) (void)hipStreamSynchronize(sh->e->st);
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
    (void)hipEventRecord(c->ev_last, sh->e->st);
    sh->used |= 1u << lane;
    sh->active++;
    c->sh = sh; c->lane = lane; c->e = sh->e;
    return 0;
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
        if (force) HIPCHECK(hipMemsetAsync(c->e->d_err, 0x01, sizeof(unsigned), c->e->st));
        int stream = 0;
        const void *recs[1] = {pb->rec};
        const int16_t *coefs[1] = {pb->coef};
        uint32_t nc[1] = {pb->ncoef};
        h264mi_engine *e = c->e;
        if (engine_decode_host(e, 1, &stream, &cur_slot, recs, coefs, nc, 2 * (int)pb->n_intra > pb->nmbs)) return -1;
        // the picture's device flags into the slot's word, behind its launch
        if (cur_slot < 0 || cur_slot >= c->nslots) return -1;
        HIPCHECK(hipMemcpyAsync(c->h_slot_err + cur_slot, e->d_err, sizeof(unsigned), hipMemcpyDeviceToHost, e->st));
        HIPCHECK(hipMemsetAsync(e->d_err, 0, sizeof(unsigned), e->st));
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
    } else if (!sh->cv.wait_for(l, std::chrono::microseconds(g_share_wait_us), [&] { return sh->launched >= mine; })) {
        share_launch(sh);                 // the others are late: launch what is there
    }
    // (a waiter gets the lock back long before SHARE_RC_RING more batches
    // launch: each later batch takes a picture or a 1 ms wait of another instance)
    return sh->rc_ring[mine % SHARE_RC_RING];
}

static int hb_prefetch(void *vctx, int slot, uint8_t *dst)
{
    HipBackendCtx *c = (HipBackendCtx *)vctx;
    if (slot < 0 || slot >= c->nslots) return -1;
    h264mi_engine *e = c->e;
    HIPCHECK(hipSetDevice(e->dev));
    std::unique_lock<std::mutex> l;
    if (c->sh) l = std::unique_lock<std::mutex>(c->sh->mu);
    HIPCHECK(hipMemcpyAsync(dst, h264mi_engine_frame_ptr(e, c->lane, slot), e->frame_bytes, hipMemcpyDeviceToHost, e->st));
    if (c->sh) HIPCHECK(hipEventRecord(c->ev_last, e->st));
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
            HIPCHECK(hipMemcpyAsync(dst, h264mi_engine_frame_ptr(c->e, c->lane, slot), c->e->frame_bytes,
                                    hipMemcpyDeviceToHost, c->e->st));
            HIPCHECK(hipEventRecord(c->ev_last, c->e->st));
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
        const size_t bytes = (size_t)e->nmbs * 256 * 4;
        if (slot < 0 || slot >= c->nslots) return -1;
        if (!c->d_rgba) HIPCHECK(hipMalloc(&c->d_rgba, bytes));
        {
            std::lock_guard<std::mutex> l(c->sh->mu);
            if (h264mi_yuv2rgba_device(h264mi_engine_frame_ptr(e, c->lane, slot), c->d_rgba, e->w * 16, e->h * 16, 1, 0,
                                       0, e->st))
                return -1;
            HIPCHECK(hipMemcpyAsync(dst, c->d_rgba, bytes, hipMemcpyDeviceToHost, e->st));
            HIPCHECK(hipEventRecord(c->ev_last, e->st));
        }
        return slot_flagged(c, slot);
    }
    if (h264mi_engine_read_rgba(c->e, 0, slot, dst)) return -1;
    return slot_flagged(c, slot, false);
}

// Pinned host blocks (decoder output frames) kept after free for the next
// decoder instance: pinning tens of MB per instance is a large share of a
// short stream's host time.  Exact-size reuse, at most HOST_POOL_BYTES kept.
#define HOST_POOL_N 16
#define HOST_POOL_BYTES (1ull << 30)
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
        if (bytes && engine_pool_on() && kept + bytes <= HOST_POOL_BYTES)
            for (int i = 0; i < HOST_POOL_N; i++)
                if (!g_hpool[i].p) { g_hpool[i].p = p; g_hpool[i].bytes = bytes; return; }
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
        HIPCHECK(hipEventRecord(c->ev_last, c->e->st));
        return 0;
    }
    return h264mi_engine_conceal(c->e, c->lane, slot, order, n, decoded);
}

static int hb_copy(void *vctx, int dst, int src)
{
    HipBackendCtx *c = (HipBackendCtx *)vctx;
    if (dst >= 0 && dst < c->nslots) c->pref[dst] = NULL;
    if (c->sh) {
        std::lock_guard<std::mutex> l(c->sh->mu);
        HIPCHECK(hipMemcpyAsync(h264mi_engine_frame_ptr(c->e, c->lane, dst), h264mi_engine_frame_ptr(c->e, c->lane, src),
                                c->e->frame_bytes, hipMemcpyDeviceToDevice, c->e->st));
        HIPCHECK(hipEventRecord(c->ev_last, c->e->st));
        return 0;
    }
    if (h264mi_engine_sync(c->e)) return -1;
    HIPCHECK(hipMemcpy(h264mi_engine_frame_ptr(c->e, 0, dst), h264mi_engine_frame_ptr(c->e, 0, src),
                       h264mi_engine_frame_bytes(c->e), hipMemcpyDeviceToDevice));
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
    const char *ff = getenv("H264MI_DEBUG_FLAG_PICTURE");
    c->force_flag_at = ff && atoi(ff) > 0 ? (unsigned)atoi(ff) : 0;
    be.ctx = c;
    be.configure = hb_configure;
    be.decode = hb_decode;
    be.read = hb_read;
    be.read_rgba = hb_read_rgba;
    be.host_alloc = hb_host_alloc;
    be.host_free = hb_host_free;
    be.copy = hb_copy;
    // H264MI_HOST_CONCEAL=1: conceal on the host (a copy of the picture, conceal.c)
    be.conceal = getenv("H264MI_HOST_CONCEAL") && atoi(getenv("H264MI_HOST_CONCEAL")) ? NULL : hb_conceal;
    be.sync = hb_sync;
    be.prefetch = hb_prefetch;
    be.destroy = hb_destroy;
    return be;
}
