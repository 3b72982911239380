// h264mi engine: HBM-resident frame slots, record upload, kernel launches.
// One engine serves `nstreams` independent bitstreams of one picture size
// (streams shard across GPUs with no collective; within a GPU
// one launch reconstructs one picture from each stream of the batch).
#include "recon_kernels.hip"
#include "color.hip"
#include <hip/hip_ext.h>

#include <stdio.h>
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
    unsigned long long *d_mbx;    // k_rows row mailboxes: 32 granules (256 B) per batch MB
    unsigned epoch;
    unsigned long long *d_prof;   // optional k_rows phase clocks
    size_t prof_cap;
    int pipe_cap;                 // pictures per launch the per-picture buffers hold
    uint32_t *d_progress;         // k_wg<PIPE>: per picture row drained-store progress
    uint32_t *d_order, *h_order;  // k_wg: (picture, row) dispatch order
    unsigned long long *d_gjunk;  // 64 KiB store sink (ReconArgs::gjunk)
    int classic;                  // single-picture launches: k_wg (default) or k_mb + k_rows (H264MI_KERNEL=classic)
    int wg_nmc;                   // MC waves per k_wg workgroup (H264MI_WG_NMC: 2, 3 or 4)
    const char *last_kernel;      // name of the last batch's reconstruction kernel (diagnostics)
    int wg_pp;                    // single-picture k_wg launches: two ping-pong row units (k_wgpp, default; H264MI_WG_PP=0: one)
    // stream groups (h264mi_engine_set_groups): the pictures of a device-input
    // batch split into G groups, each on its own HIP stream, so one group's
    // k_mb overlaps the other groups' latency-bound k_rows
    int ngroups;
    hipStream_t gst[H264MI_MAX_GROUPS];
    int stagger_pending;
    int order_depth, order_lag;
    uint8_t *d_dbrec;         // 64 B per batch MB (x2: k_prep double buffer)
    int16_t *d_res;           // 384 x int16 per batch MB (x2)
    // k_prep (deblocking records + residuals one batch ahead, on its own
    // stream): buffer half prep_parity, ordered by events
    int prep;                 // H264MI_PREP (default 1)
    int prep_parity;
    int prep_serial;
    double prep_delay_us;     // H264MI_PREP_DELAY_US: k_prep starts this long after it could (< 0: default)          // H264MI_PREP_SERIAL: k_prep waits for the previous k_wgpp (diagnostics)
    hipStream_t st2;
    hipEvent_t ev_in, ev_prep, ev_wgdone[2];
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
    uint32_t err_accum;
    int timing;
    // per-batch kernel timing (h264mi_engine_set_timing): event triples
    hipEvent_t *tev;
    int tev_cap, tev_n;
    int tev_stride, tev_seq;  // record every tev_stride-th launch (h264mi_engine_set_timing_stride)
    bool tev_single;        // single-kernel launches: t0 .. t2 only (one marker fewer between launches)
    uint8_t *d_rgba;          // h264mi_engine_read_rgba staging (w*h*4 B, allocated on first use)
};

// per-picture buffers of one launch (deblocking records, intra residuals,
// row mailboxes, error flags, pipeline progress/counters), for `cap` pictures
static void free_pic_buffers(h264mi_engine *e)
{
    (void)hipFree(e->d_mbx); (void)hipFree(e->d_dbrec); (void)hipFree(e->d_res); (void)hipFree(e->d_err);
    (void)hipFree(e->d_progress);
    (void)hipHostFree(e->h_err);
    (void)hipFree(e->d_order); (void)hipHostFree(e->h_order);
    e->d_order = NULL; e->h_order = NULL; e->order_depth = e->order_lag = 0;
    e->d_mbx = NULL; e->d_dbrec = NULL; e->d_res = NULL; e->d_err = NULL;
    e->d_progress = NULL; e->h_err = NULL;
    e->pipe_cap = 0;
}

static int alloc_pic_buffers(h264mi_engine *e, int cap)
{
    const size_t np = (size_t)cap, mbs = np * e->nmbs, rows = np * e->h;
    bool ok = hipMalloc(&e->d_mbx, mbs * 256) == hipSuccess &&
              hipMalloc(&e->d_dbrec, 2 * mbs * 64) == hipSuccess &&
              hipMalloc(&e->d_res, 2 * mbs * 768) == hipSuccess &&
              hipMalloc(&e->d_err, sizeof(unsigned) * np) == hipSuccess &&
              hipMalloc(&e->d_progress, rows * 4) == hipSuccess &&
              hipHostMalloc(&e->h_err, sizeof(unsigned) * np, hipHostMallocDefault) == hipSuccess &&
              hipMalloc(&e->d_order, sizeof(uint32_t) * rows) == hipSuccess &&
              hipHostMalloc(&e->h_order, sizeof(uint32_t) * rows, hipHostMallocDefault) == hipSuccess;
    if (!ok) { free_pic_buffers(e); return -1; }
    // cleared granules / progress carry epoch 0, which no launch uses
    (void)hipMemsetAsync(e->d_mbx, 0, mbs * 256, e->st);
    (void)hipMemsetAsync(e->d_progress, 0, rows * 4, e->st);
    (void)hipMemsetAsync(e->d_err, 0, sizeof(unsigned) * np, e->st);
    memset(e->h_err, 0, sizeof(unsigned) * np);
    e->pipe_cap = cap;
    return 0;
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
    h264mi_engine *e = (h264mi_engine *)calloc(1, sizeof(h264mi_engine));
    if (!e) return NULL;
    e->dev = device;
    e->w = w_mbs; e->h = h_mbs; e->nmbs = w_mbs * h_mbs;
    e->nstreams = nstreams; e->nslots = nslots;
    e->frame_bytes = (size_t)e->nmbs * 384;
    e->coef_cap = (size_t)nstreams * e->nmbs * 8 + 1024;
    e->h_coef_cap = e->coef_cap;
    e->timing = getenv("H264MI_TIMING") != NULL;
    e->ngroups = 1;
    {
        const char *km = getenv("H264MI_KERNEL");
        e->classic = km && !strcmp(km, "classic");
        const char *nm = getenv("H264MI_WG_NMC");
        const char *pp = getenv("H264MI_WG_PP");
        e->wg_pp = pp ? atoi(pp) : 1;
        // MC waves per workgroup (default 3: with the ping-pong row waves a
        // 5-wave workgroup at <= 128 VGPRs, three per CU keep every row of
        // 8 1080p pictures resident)
        e->wg_nmc = nm ? atoi(nm) : 3;
        e->prep_serial = getenv("H264MI_PREP_SERIAL") != NULL;
        const char *pd = getenv("H264MI_PREP_DELAY_US");
        e->prep_delay_us = pd ? atof(pd) : -1.0;
        const char *pr = getenv("H264MI_PREP");
        e->prep = pr ? atoi(pr) : 1;
    }
    bool ok = hipMalloc(&e->d_frames, e->frame_bytes * nslots * nstreams) == hipSuccess &&

              hipMalloc(&e->d_rec, sizeof(MbRec) * nstreams * e->nmbs) == hipSuccess &&
              hipMalloc(&e->d_coef, e->coef_cap * 32) == hipSuccess &&
              hipMalloc(&e->d_pics, sizeof(PicDesc) * nstreams) == hipSuccess &&
              hipMalloc(&e->d_gjunk, 65536) == hipSuccess &&

              hipHostMalloc(&e->h_rec, sizeof(MbRec) * nstreams * e->nmbs, hipHostMallocDefault) == hipSuccess &&
              hipHostMalloc(&e->h_coef, e->h_coef_cap * 32, hipHostMallocDefault) == hipSuccess &&
              hipHostMalloc(&e->h_pics, sizeof(PicDesc) * nstreams, hipHostMallocDefault) == hipSuccess &&

              hipStreamCreateWithFlags(&e->st, hipStreamNonBlocking) == hipSuccess &&
              hipEventCreateWithFlags(&e->ev_staged, hipEventDisableTiming) == hipSuccess &&
              hipEventCreate(&e->ev0) == hipSuccess && hipEventCreate(&e->ev1) == hipSuccess &&
              hipEventCreate(&e->ev2) == hipSuccess &&
              hipStreamCreateWithFlags(&e->st2, hipStreamNonBlocking) == hipSuccess &&
              hipEventCreateWithFlags(&e->ev_in, hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&e->ev_prep, hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&e->ev_wgdone[0], hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&e->ev_wgdone[1], hipEventDisableTiming) == hipSuccess;
    ok = ok && alloc_pic_buffers(e, nstreams) == 0;
    if (!ok) {
        fprintf(stderr, "h264mi: engine allocation failed\n");
        h264mi_engine_destroy(e);
        return NULL;
    }
    (void)hipMemsetAsync(e->d_frames, 0, e->frame_bytes * nslots * nstreams, e->st);
    e->epoch = 0;
    (void)hipEventRecord(e->ev_staged, e->st);
    (void)hipStreamSynchronize(e->st);
    return e;
}

extern "C" void h264mi_engine_destroy(h264mi_engine *e)
{
    if (!e) return;
    if (e->st) (void)hipStreamSynchronize(e->st);
    if (e->st2) (void)hipStreamSynchronize(e->st2);
    free_pic_buffers(e);
    (void)hipFree(e->d_rgba);
    (void)hipFree(e->d_frames); (void)hipFree(e->d_prof); (void)hipFree(e->d_rec); (void)hipFree(e->d_coef);
    (void)hipFree(e->d_pics); (void)hipFree(e->d_gjunk);
    (void)hipHostFree(e->h_rec); (void)hipHostFree(e->h_coef); (void)hipHostFree(e->h_pics);
    if (e->ev_staged) (void)hipEventDestroy(e->ev_staged);
    if (e->ev0) (void)hipEventDestroy(e->ev0);
    if (e->ev1) (void)hipEventDestroy(e->ev1);
    if (e->ev2) (void)hipEventDestroy(e->ev2);
    if (e->ev_in) (void)hipEventDestroy(e->ev_in);
    if (e->ev_prep) (void)hipEventDestroy(e->ev_prep);
    for (int i = 0; i < 2; i++)
        if (e->ev_wgdone[i]) (void)hipEventDestroy(e->ev_wgdone[i]);
    if (e->st2) (void)hipStreamDestroy(e->st2);
    h264mi_engine_set_timing(e, 0);
    for (int g = 0; g < H264MI_MAX_GROUPS; g++)
        if (e->gst[g]) { (void)hipStreamSynchronize(e->gst[g]); (void)hipStreamDestroy(e->gst[g]); }
    if (e->st) (void)hipStreamDestroy(e->st);
    free(e);
}

// (picture k, row r) pairs by r + lag*k, then k: with lag > every reference
// reach in rows + 1, each unit's dependencies come earlier in the order
static int pipe_order(h264mi_engine *e, int depth, int lag)
{
    if (e->order_depth == depth && e->order_lag == lag) return 0;
    int n = 0;
    for (int key = 0; key <= e->h - 1 + lag * (depth - 1); key++)
        for (int k = 0; k < depth; k++) {
            const int r = key - lag * k;
            if (r >= 0 && r < e->h) e->h_order[n++] = ((uint32_t)k << 16) | (uint32_t)r;
        }
    HIPCHECK(hipMemcpyAsync(e->d_order, e->h_order, sizeof(uint32_t) * n, hipMemcpyHostToDevice, e->st));
    e->order_depth = depth;
    e->order_lag = lag;
    return 0;
}

// one-off offset of a group stream (stagger): spin on the wall clock (100 MHz)
__global__ void k_delay(unsigned long long ticks)
{
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

static int launch_groups(h264mi_engine *e, int npics, ReconArgs a);

static int launch_batch(h264mi_engine *e, int npics, const MbRec *d_rec, const int16_t *d_coef,
                        const PicDesc *d_pics, bool pipe = false, int depth = 1, int base_pic = 0, int lag = 0,
                        bool grouped = false)
{
    ReconArgs a;
    memset(&a, 0, sizeof(a));
    a.frames = e->d_frames;
    a.frame_bytes = e->frame_bytes;
    a.rec = d_rec;
    a.coef = d_coef;
    a.mbx = e->d_mbx;
    a.gjunk = e->d_gjunk;
    if (++e->epoch >= (1u << 20)) {           // tags: granules epoch, progress (epoch << 12) | count
        if (h264mi_engine_sync(e)) return -1; // group streams may still read the mailboxes
        HIPCHECK(hipMemsetAsync(e->d_mbx, 0, (size_t)e->pipe_cap * e->nmbs * 256, e->st));
        HIPCHECK(hipMemsetAsync(e->d_progress, 0, (size_t)e->pipe_cap * e->h * 4, e->st));
        e->epoch = 1;
    }
    a.epoch = e->epoch;
    a.prof = e->d_prof;
    a.pics = d_pics;
    a.npics = npics;
    a.w = e->w; a.h = e->h;
    a.dbrec = e->d_dbrec;
    a.res = e->d_res;
    a.err = e->d_err;
    a.progress = e->d_progress;
    a.S = npics / depth;
    a.ring = e->nslots;
    a.base_pic = base_pic % e->nslots;
    if (grouped && !pipe && e->classic && e->ngroups > 1 && npics >= e->ngroups) {
        e->tev_single = false;
        return launch_groups(e, npics, a);
    }
    const bool wg = pipe || !e->classic;
    if (wg) {
        if (pipe) a.prof = NULL;
        if (pipe_order(e, depth, lag < 1 ? e->h : lag)) return -1;
        a.order = e->d_order;
    }
    // k_prep: this batch's deblocking records and residuals on st2, into the
    // buffer half the launch before last read (ev_wgdone); device-resident
    // input (bench) lets it overlap the previous batch's k_wg
    const bool prep = wg && !pipe && e->prep;
    const int pbuf = e->prep_parity;
    if (prep) {
        e->prep_parity ^= 1;
        const size_t mbs = (size_t)e->pipe_cap * e->nmbs;
        a.dbrec = e->d_dbrec + pbuf * mbs * 64;
        a.res = e->d_res + pbuf * mbs * 384;
        if (!grouped) {     // host-staged input: the upload is on st
            HIPCHECK(hipEventRecord(e->ev_in, e->st));
            HIPCHECK(hipStreamWaitEvent(e->st2, e->ev_in, 0));
        }
        HIPCHECK(hipStreamWaitEvent(e->st2, e->ev_wgdone[pbuf], 0));
        if (e->prep_serial) HIPCHECK(hipStreamWaitEvent(e->st2, e->ev_wgdone[pbuf ^ 1], 0));   // experiment: no overlap
        // start k_prep in the row kernel's tail, when the top rows have
        // finished and their CUs are idle: its memory traffic beside live row
        // chains lengthens their L2 hand-offs (k_wgpp 449 us with k_prep
        // 120 us in, 404 at 50 us, 385 at 250-300 us; 8 x 1080p).  Default:
        // 65 % of the picture's chain estimate W * 1.6 + H * 2.8 us (248 us
        // at 1080p); H264MI_PREP_DELAY_US overrides.  Only for device-
        // resident batches queued back to back (decode_device): a host-staged
        // batch (the H264SwDec path, one picture per host parse) finds the
        // GPU idle, and its k_prep must not wait at all.
        const double dly = e->prep_delay_us >= 0 ? e->prep_delay_us
                           : grouped ? 0.65 * (e->w * 1.6 + e->h * 2.8) : 0.0;
        if (dly > 0.5) hipLaunchKernelGGL(k_delay, dim3(1), dim3(64), 0, e->st2, (unsigned long long)(dly * 100.0));
        hipLaunchKernelGGL(k_prep, dim3((npics * e->nmbs + 3) / 4), dim3(256), 0, e->st2, a);
        HIPCHECK(hipGetLastError());
        HIPCHECK(hipEventRecord(e->ev_prep, e->st2));
        HIPCHECK(hipStreamWaitEvent(e->st, e->ev_prep, 0));
    }
    hipEvent_t t0 = e->ev0, t1 = e->ev1, t2 = e->ev2;
    bool rec_tev = false;
    if (e->tev && e->tev_n < e->tev_cap && e->tev_seq++ % (e->tev_stride > 0 ? e->tev_stride : 1) == 0) {
        t0 = e->tev[3 * e->tev_n]; t1 = e->tev[3 * e->tev_n + 1]; t2 = e->tev[3 * e->tev_n + 2];
        e->tev_n++;
        rec_tev = true;
    }
    const bool rec = e->timing || rec_tev;
    // k_wgpp (the default path): the timing events ride on the kernel's own
    // dispatch packet (hipExtLaunchKernelGGL), no marker packets around it
    const bool pp_fast = wg && !pipe && e->wg_pp && prep && !a.prof;
    if (rec && !pp_fast) (void)hipEventRecord(t0, e->st);
    e->last_kernel = !wg ? "k_mb+k_rows" : pipe ? "k_wg" : (e->wg_pp && prep) ? "k_wgpp" : "k_wg";
    e->tev_single = wg;
    if (!wg) {
        hipLaunchKernelGGL(k_mb, dim3(((npics * e->nmbs + 7) / 8) * 8), dim3(64), 0, e->st, a);
        HIPCHECK(hipGetLastError());
        if (rec) (void)hipEventRecord(t1, e->st);
        if (a.prof) hipLaunchKernelGGL(k_rows<true>, dim3(npics * e->h), dim3(64), 0, e->st, a);
        else hipLaunchKernelGGL(k_rows<false>, dim3(npics * e->h), dim3(64), 0, e->st, a);
        HIPCHECK(hipGetLastError());
    } else {
        // one launch: row workgroups with in-workgroup MC (k_wg); the k_mb
        // slot of the timing is empty
        const dim3 grid(a.S * e->h * depth);
        const int nmc = e->wg_nmc;
        if (pipe) {
            if (nmc == 2) hipLaunchKernelGGL((k_wg<true, 2, false>), grid, dim3(192), 0, e->st, a);
            else if (nmc == 4) hipLaunchKernelGGL((k_wg<true, 4, false>), grid, dim3(320), 0, e->st, a);
            else hipLaunchKernelGGL((k_wg<true, 3, false>), grid, dim3(256), 0, e->st, a);
        } else if (e->wg_pp && prep) {
            if (a.prof) {
                if (nmc == 2) hipLaunchKernelGGL((k_wgpp<2, true, true>), grid, dim3(256), 0, e->st, a);
                else hipLaunchKernelGGL((k_wgpp<3, true, true>), grid, dim3(320), 0, e->st, a);
            } else if (nmc == 2) {
                hipExtLaunchKernelGGL((k_wgpp<2, false, true>), grid, dim3(256), 0, e->st, rec ? t0 : nullptr,
                                      rec ? t2 : nullptr, 0, a);
            } else {
                hipExtLaunchKernelGGL((k_wgpp<3, false, true>), grid, dim3(320), 0, e->st, rec ? t0 : nullptr,
                                      rec ? t2 : nullptr, 0, a);
            }
        } else if (prep) {
            if (a.prof) hipLaunchKernelGGL((k_wg<false, 3, true, true>), grid, dim3(256), 0, e->st, a);
            else if (nmc == 2) hipLaunchKernelGGL((k_wg<false, 2, false, true>), grid, dim3(192), 0, e->st, a);
            else hipLaunchKernelGGL((k_wg<false, 3, false, true>), grid, dim3(256), 0, e->st, a);
        } else if (a.prof) {
            hipLaunchKernelGGL((k_wg<false, 3, true>), grid, dim3(256), 0, e->st, a);
        } else {
            if (nmc == 2) hipLaunchKernelGGL((k_wg<false, 2, false>), grid, dim3(192), 0, e->st, a);
            else if (nmc == 4) hipLaunchKernelGGL((k_wg<false, 4, false>), grid, dim3(320), 0, e->st, a);
            else hipLaunchKernelGGL((k_wg<false, 3, false>), grid, dim3(256), 0, e->st, a);
        }
        HIPCHECK(hipGetLastError());
    }
    if (rec && !pp_fast) (void)hipEventRecord(t2, e->st);
    if (prep) HIPCHECK(hipEventRecord(e->ev_wgdone[pbuf], e->st));
    return 0;
}

// k_mb + k_rows per group of pictures, each group on its own stream.  Groups
// use disjoint mailbox / error ranges (picture index p0.. of the batch);
// deblocking records and residuals are per batch MB already.
static int launch_groups(h264mi_engine *e, int npics, ReconArgs a)
{
    const int G = e->ngroups;
    for (int g = 0; g < G; g++) {
        const int p0 = g * npics / G, n = (g + 1) * npics / G - p0;
        hipStream_t gs = e->gst[g];
        if (e->stagger_pending && g > 0) {
            // offset group g by g/G of an estimated picture latency, once:
            // equal-length group cycles then keep the groups' k_mb apart
            const double est_us = (e->w + 3.0 * e->h) * 2.8;
            hipLaunchKernelGGL(k_delay, dim3(1), dim3(64), 0, gs, (unsigned long long)(est_us * 100.0 * g / G));
        }
        ReconArgs ag = a;
        ag.pics = a.pics + p0;
        ag.npics = n;
        ag.mbx = e->d_mbx + (size_t)p0 * e->nmbs * 32;
        ag.err = e->d_err + p0;
        ag.prof = NULL;
        const bool rec = g == 0 && e->tev && e->tev_n < e->tev_cap;
        hipEvent_t t0 = rec ? e->tev[3 * e->tev_n] : NULL, t1 = rec ? e->tev[3 * e->tev_n + 1] : NULL,
                   t2 = rec ? e->tev[3 * e->tev_n + 2] : NULL;
        if (rec) (void)hipEventRecord(t0, gs);
        hipLaunchKernelGGL(k_mb, dim3(((n * e->nmbs + 7) / 8) * 8), dim3(64), 0, gs, ag);
        HIPCHECK(hipGetLastError());
        if (rec) (void)hipEventRecord(t1, gs);
        hipLaunchKernelGGL(k_rows<false>, dim3(n * e->h), dim3(64), 0, gs, ag);
        HIPCHECK(hipGetLastError());
        if (rec) { (void)hipEventRecord(t2, gs); e->tev_n++; }
    }
    e->stagger_pending = 0;
    return 0;
}

extern "C" int h264mi_engine_set_groups(h264mi_engine *e, int ngroups)
{
    if (!e || ngroups < 1 || ngroups > H264MI_MAX_GROUPS || ngroups > e->nstreams) return -1;
    HIPCHECK(hipSetDevice(e->dev));
    if (h264mi_engine_sync(e)) return -1;
    for (int g = 0; g < ngroups; g++)
        if (!e->gst[g]) HIPCHECK(hipStreamCreateWithFlags(&e->gst[g], hipStreamNonBlocking));
    e->ngroups = ngroups;
    e->stagger_pending = ngroups > 1;
    return 0;
}

extern "C" int h264mi_engine_decode(h264mi_engine *e, int npics, const int *stream, const int *cur_slot,
                                    const void *const *recs, const int16_t *const *coefs, const uint32_t *ncoef)
{
    if (!e || npics < 1 || npics > e->nstreams) return -1;
    HIPCHECK(hipSetDevice(e->dev));
    // staging buffers are reused: wait until the previous upload consumed them
    HIPCHECK(hipEventSynchronize(e->ev_staged));
    for (int i = 0; i < npics; i++) e->err_accum += 0;
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
    return launch_batch(e, npics, e->d_rec, e->d_coef, e->d_pics);
}

extern "C" int h264mi_engine_decode_device(h264mi_engine *e, int npics, const void *d_recs, const int16_t *d_coef,
                                           const void *d_pics)
{
    if (!e || npics < 1 || npics > e->nstreams) return -1;
    HIPCHECK(hipSetDevice(e->dev));
    return launch_batch(e, npics, (const MbRec *)d_recs, d_coef, (const PicDesc *)d_pics, false, 1, 0, 0, true);
}

extern "C" int h264mi_engine_set_pipeline(h264mi_engine *e, int depth)
{
    if (!e || depth < 1) return -1;
    HIPCHECK(hipSetDevice(e->dev));
    HIPCHECK(hipStreamSynchronize(e->st));
    HIPCHECK(hipStreamSynchronize(e->st2));
    const int cap = e->nstreams * depth;
    if (cap == e->pipe_cap) return 0;
    free_pic_buffers(e);
    if (alloc_pic_buffers(e, cap)) return -1;
    HIPCHECK(hipStreamSynchronize(e->st));
    return 0;
}

extern "C" int h264mi_engine_decode_pipelined(h264mi_engine *e, int nstreams, int depth, const void *d_recs,
                                              const int16_t *d_coef, const void *d_pics, int base_pic, int lag_rows)
{
    if (!e || nstreams < 1 || nstreams > e->nstreams || depth < 1 || nstreams * depth > e->pipe_cap) return -1;
    if (base_pic < 0 || depth > e->nslots) return -1;
    HIPCHECK(hipSetDevice(e->dev));
    return launch_batch(e, nstreams * depth, (const MbRec *)d_recs, d_coef, (const PicDesc *)d_pics, true, depth,
                        base_pic, lag_rows);
}

extern "C" const char *h264mi_engine_kernel(h264mi_engine *e)
{
    return e && e->last_kernel ? e->last_kernel : "";
}

extern "C" int h264mi_engine_sync(h264mi_engine *e)
{
    if (!e) return -1;
    HIPCHECK(hipSetDevice(e->dev));
    HIPCHECK(hipStreamSynchronize(e->st));
    HIPCHECK(hipStreamSynchronize(e->st2));
    for (int g = 0; g < H264MI_MAX_GROUPS; g++)
        if (e->gst[g]) HIPCHECK(hipStreamSynchronize(e->gst[g]));
    // per-picture error flags OR-accumulate over every launch since the last
    // sync (no per-launch reset): count the flagged picture slots, then clear
    HIPCHECK(hipMemcpy(e->h_err, e->d_err, sizeof(unsigned) * e->pipe_cap, hipMemcpyDeviceToHost));
    for (int i = 0; i < e->pipe_cap; i++) e->err_accum += e->h_err[i] ? 1 : 0;
    HIPCHECK(hipMemset(e->d_err, 0, sizeof(unsigned) * e->pipe_cap));
    return 0;
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
    if (e->tev_single) {
        HIPCHECK(hipEventElapsedTime(&ms1, e->ev0, e->ev2));
    } else {
        HIPCHECK(hipEventElapsedTime(&ms0, e->ev0, e->ev1));
        HIPCHECK(hipEventElapsedTime(&ms1, e->ev1, e->ev2));
    }
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
        if (e->tev_single) {
            HIPCHECK(hipEventElapsedTime(&m1, e->tev[3 * i], e->tev[3 * i + 2]));
        } else {
            HIPCHECK(hipEventElapsedTime(&m0, e->tev[3 * i], e->tev[3 * i + 1]));
            HIPCHECK(hipEventElapsedTime(&m1, e->tev[3 * i + 1], e->tev[3 * i + 2]));
        }
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
        e->prof_cap = (size_t)e->nstreams * e->h * 16 + (size_t)e->nstreams * e->nmbs * 4;
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

// -------- H264Backend adapter for the single-stream host decoder ----------
#include "../host/decoder.h"

struct HipBackendCtx {
    int device;
    h264mi_engine *e;
};

static int hb_configure(void *vctx, int w_mbs, int h_mbs, int nslots)
{
    HipBackendCtx *c = (HipBackendCtx *)vctx;
    if (c->e) h264mi_engine_destroy(c->e);
    c->e = h264mi_engine_create(c->device, w_mbs, h_mbs, 1, nslots);
    return c->e ? 0 : -1;
}

static int hb_decode(void *vctx, const PicBuild *pb, int cur_slot)
{
    HipBackendCtx *c = (HipBackendCtx *)vctx;
    int stream = 0;
    const void *recs[1] = {pb->rec};
    const int16_t *coefs[1] = {pb->coef};
    uint32_t nc[1] = {pb->ncoef};
    return h264mi_engine_decode(c->e, 1, &stream, &cur_slot, recs, coefs, nc);
}

static int hb_read(void *vctx, int slot, uint8_t *dst)
{
    HipBackendCtx *c = (HipBackendCtx *)vctx;
    return h264mi_engine_read(c->e, 0, slot, dst);
}

static int hb_read_rgba(void *vctx, int slot, uint8_t *dst)
{
    HipBackendCtx *c = (HipBackendCtx *)vctx;
    return h264mi_engine_read_rgba(c->e, 0, slot, dst);
}

static void *hb_host_alloc(void *vctx, size_t bytes)
{
    void *p = NULL;
    return hipHostMalloc(&p, bytes, hipHostMallocDefault) == hipSuccess ? p : NULL;
}

static void hb_host_free(void *vctx, void *p) { (void)hipHostFree(p); }

static int hb_copy(void *vctx, int dst, int src)
{
    HipBackendCtx *c = (HipBackendCtx *)vctx;
    if (h264mi_engine_sync(c->e)) return -1;
    HIPCHECK(hipMemcpy(h264mi_engine_frame_ptr(c->e, 0, dst), h264mi_engine_frame_ptr(c->e, 0, src),
                       h264mi_engine_frame_bytes(c->e), hipMemcpyDeviceToDevice));
    return 0;
}

static void hb_destroy(void *vctx)
{
    HipBackendCtx *c = (HipBackendCtx *)vctx;
    if (c->e) h264mi_engine_destroy(c->e);
    free(c);
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
    be.ctx = c;
    be.configure = hb_configure;
    be.decode = hb_decode;
    be.read = hb_read;
    be.read_rgba = hb_read_rgba;
    be.host_alloc = hb_host_alloc;
    be.host_free = hb_host_free;
    be.copy = hb_copy;
    be.destroy = hb_destroy;
    return be;
}
