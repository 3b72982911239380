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
#include "engine_int.h"

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
    size_t frame_bytes;           // device slot stride (H264MI_SLOT_BYTES: chroma rows padded to 128 B)
    size_t pic_bytes;             // packed I420 picture (what leaves the device)
    int cpitch;                   // chroma row pitch in a slot (H264MI_CPITCH)
    uint8_t *d_frames;
    unsigned long long *d_mbx;    // row mailboxes: 32 granules (256 B) per batch MB
    unsigned epoch;
    unsigned long long *d_prof;   // optional per-MB chain stamps (profiling k_wgpp)
    size_t prof_cap;
    int pipe_cap;                 // pictures per launch the per-picture buffers hold
    unsigned long long *d_gjunk;  // 64 KiB store sink (ReconArgs::gjunk)
    const char *last_kernel;      // name of the last batch's reconstruction kernel (diagnostics)
    int last_dep;                 // the last batch's dependency mode (DEP_NONE / DEP_ROWS / DEP_COLS)
    int last_nmc;                 // the last batch's MC waves per row workgroup
    uint8_t *d_dbrec;         // 64 B per batch MB (x2: k_prep double buffer)
    int16_t *d_res;           // 384 x int16 per batch MB (x2)
    // k_prep (deblocking records + residuals) writes buffer half prep_parity;
    // a batch prepped by the previous launch's tail workgroups is `prepped`
    int prep_parity;
    int conceal_fits;                         // k_conceal's per-MB flags fit its LDS
    const void *prepped_rec, *prepped_pics;
    int prepped_n;                            // pictures the tail prepped
    unsigned long long *d_rows_done;   // row workgroups finished, all launches (tail-prep trigger)
    // k_conceal inputs (order + decoded flags): pinned staging, device copy,
    // and an event after the upload (the staging's reuse waits for it)
    uint8_t *h_conceal, *d_conceal;
    hipEvent_t ev_conceal;
    int prep_wgs;                      // tail workgroups per launch (H264MI_PREP_WGS, default 2048)
    unsigned long long rows_launched;
    int prep_at_pct;                   // tail prep waits for this % of the launch's rows (H264MI_PREP_AT; 0: no wait)
    int mc_waves;                      // MC waves per row workgroup: 0 = per launch (below), 2, 3 or 6 forced (H264MI_MC_WAVES)
    int intra_mc6;                     // intra-heavy launches may take 6 MC waves (launch_nmc; H264MI_INTRA_MC6=0: 3)
    int launch_intra;                  // next launch: 1 = has an intra-heavy picture, 0 = none, -1 = unknown
    int dep_mode;                      // frame-pipelined launches: DEP_ROWS / DEP_COLS (H264MI_DEP_MODE; default rows)
    int launch_dep;                    // next launch's mode (h264mi_engine_hint_deps), 0 = dep_mode
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
    unsigned long long *d_prog;   // per picture row of a launch, per row wave: {MBs stored, epoch} (frame-pipelined launches)
    unsigned *d_done;             // per picture row of a launch: epoch once the row is stored
    int check;                // H264MI_CHECK=1: the dependency-checker kernels (recon_kernels.hip CHK_*)
    int check_inject;         // H264MI_CHECK_INJECT: test hook (ReconArgs::chk_inject)
    int check_short_cols, check_short_rows;   // H264MI_CHECK_INJECT_REFCOLS / _REFROWS: test hooks
    uint32_t err_bits;        // OR of every picture's device flags since the last h264mi_engine_error_bits
};

// per-picture buffers of one launch (deblocking records, residuals, row
// mailboxes, error flags), for `cap` pictures
static void free_pic_buffers(h264mi_engine *e)
{
    (void)hipFree(e->d_mbx); (void)hipFree(e->d_dbrec); (void)hipFree(e->d_res); (void)hipFree(e->d_err);
    (void)hipFree(e->d_prog);
    (void)hipFree(e->d_done);
    (void)hipHostFree(e->h_err);
    e->d_mbx = NULL; e->d_dbrec = NULL; e->d_res = NULL; e->d_err = NULL; e->d_prog = NULL; e->d_done = NULL;
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
              hipMalloc(&e->d_prog, sizeof(unsigned long long) * 2 * PROG_STRIDE * np * e->h) == hipSuccess &&
              hipMalloc(&e->d_done, sizeof(unsigned) * np * e->h) == hipSuccess &&
              hipHostMalloc(&e->h_err, sizeof(unsigned) * np, hipHostMallocDefault) == hipSuccess;
    if (!ok) { free_pic_buffers(e); return -1; }
    // cleared granules carry epoch 0, which no launch uses
    (void)hipMemsetAsync(e->d_mbx, 0, mbs * 256, e->st);
    (void)hipMemsetAsync(e->d_err, 0, sizeof(unsigned) * np, e->st);
    (void)hipMemsetAsync(e->d_prog, 0, sizeof(unsigned long long) * 2 * PROG_STRIDE * np * e->h, e->st);
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
    e->mc_waves = mw && (atoi(mw) == 2 || atoi(mw) == 3 || atoi(mw) == 6) ? atoi(mw) : 0;
    const char *m6 = getenv("H264MI_INTRA_MC6");
    e->intra_mc6 = m6 ? atoi(m6) != 0 : 1;
    e->launch_intra = -1;
    {
        const char *dm = getenv("H264MI_DEP_MODE");
        e->dep_mode = dm && (!strcmp(dm, "cols") || atoi(dm) == DEP_COLS) ? DEP_COLS : DEP_ROWS;
        e->launch_dep = 0;
    }
    e->check = getenv("H264MI_CHECK") && atoi(getenv("H264MI_CHECK"));
    e->check_inject = h264mi_test_hooks() && getenv("H264MI_CHECK_INJECT") ? atoi(getenv("H264MI_CHECK_INJECT")) : 0;
    e->check_short_cols = h264mi_test_hooks() && getenv("H264MI_CHECK_INJECT_REFCOLS") ? atoi(getenv("H264MI_CHECK_INJECT_REFCOLS")) : 0;
    e->check_short_rows = h264mi_test_hooks() && getenv("H264MI_CHECK_INJECT_REFROWS") ? atoi(getenv("H264MI_CHECK_INJECT_REFROWS")) : 0;
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
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_wgpp<6, true, true, 1>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_wgpp<6, false, true, 1>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_wgpp<6, false, true, 1, true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_wgpp<2, false, true, 2>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_wgpp<2, true, true, 1>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_wgpp<3, false, true, 1, true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_wgpp<2, false, true, 1, true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_wgpp<3, false, true, 2, true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_wgpp<2, false, true, 2, true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_wgpp<3, false, true, 3, true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_wgpp<2, false, true, 1, false, DEP_ROWS>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_wgpp<2, false, true, 1, true, DEP_ROWS>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_wgpp<2, true, true, 1, false, DEP_ROWS>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_wgpp<2, false, true, 1, false, DEP_COLS>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_wgpp<2, false, true, 1, true, DEP_COLS>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_wgpp<2, true, true, 1, false, DEP_COLS>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    const size_t row_lds = sizeof(PPLds) + (size_t)(e->mc_waves == 2 ? 2 : e->mc_waves == 6 ? 6 : 3) * sizeof(McScratch) + sizeof(MbRing<RINGG>);
    e->rpw_max = e->mc_waves == 2 ? 2 : 3;
    while (e->rpw_max > 1 && (size_t)(e->rpw_max - 1) * e->w * 256 + (size_t)e->rpw_max * row_lds > 156 * 1024)
        e->rpw_max--;
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, e->dev) != hipSuccess || ncu < 1) ncu = 256;
    e->ncu = ncu;
    // k_conceal keeps one decoded flag per MB in dynamic LDS: up to the CU's
    // 160 KB less its static part; larger pictures conceal on the host
    // (engine_conceal_fits -> the backend's conceal_ok)
    // (one byte per MB; the attribute is raised only for pictures above the
    // default 64 KB limit (less k_conceal's static sums and headroom), so a
    // device that refuses it still conceals
    // the sizes that fit)
    e->conceal_fits = (size_t)e->nmbs <= 60 * 1024 ||
                      ((size_t)e->nmbs <= CONCEAL_LDS_MAX &&
                       hipFuncSetAttribute(reinterpret_cast<const void *>(&k_conceal),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, CONCEAL_LDS_MAX) == hipSuccess);
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
    e->frame_bytes = H264MI_SLOT_BYTES(w_mbs, h_mbs);
    e->pic_bytes = (size_t)e->nmbs * 384;
    e->cpitch = H264MI_CPITCH(w_mbs);
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
    if (e->mc_waves == 6) rpw = 1;
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
// (more than half its MBs intra) or its content is unknown.  A launch of
// two steps per stream always takes 2: twice the rows compete for workgroup
// slots, and 768 of them beat the third wave even with an IDR among the
// pictures (configs[3] GOP mix: launches holding an IDR 671 vs 754 us,
// profiles/r75_ab_idr_second.txt).  An intra-heavy launch whose rows all fit
// two 8-wave workgroups per CU takes six MC waves: an intra row's pace is its
// MC waves' throughput (each wave holds an MB through the left-neighbour
// waits of its 4x4 blocks), 720p I pictures 341.6 / 324.0 / 320.2 / 316.7 us
// with 3 / 4 / 5 / 6 (profiles/r162_*, r163_*); above that the rows would
// wait for slots.
static int launch_nmc(const h264mi_engine *e, int rpw, int P, int npics)
{
    if (e->mc_waves) return e->mc_waves;
    if (rpw > 1) return 3;
    if (P > 1) return 2;
    if (e->launch_intra == 0) return 2;
    return e->launch_intra > 0 && e->intra_mc6 && npics * e->h <= 2 * e->ncu ? 6 : 3;
}

static int launch_batch(h264mi_engine *e, int S, int P, const MbRec *d_rec, const int16_t *d_coef,
                        const PicDesc *d_pics, const MbRec *next_rec, const int16_t *next_coef,
                        const PicDesc *next_pics, int next_npics = -1)
{
    const int npics = S * P;
    const size_t mbs = (size_t)e->pipe_cap * e->nmbs;
    const int hb = e->prep_parity;
    // study knob (H264MI_NO_TAIL_PREP=1): every batch's k_prep as its own
    // launch in front of k_wgpp, none in the tail -- k_wgpp's time without
    // the next batch's prep work beside the chain
    static const bool no_tail = getenv("H264MI_NO_TAIL_PREP") && atoi(getenv("H264MI_NO_TAIL_PREP"));
    if (no_tail) next_rec = nullptr, next_coef = nullptr, next_pics = nullptr;
    if (next_npics < 0) next_npics = npics;
    if (!(e->prepped_rec && e->prepped_rec == (const void *)d_rec && e->prepped_pics == (const void *)d_pics &&
          e->prepped_n == npics))
        if (launch_prep(e, npics, d_rec, d_coef, d_pics, hb)) return -1;
    ReconArgs a;
    memset(&a, 0, sizeof(a));
    a.frames = e->d_frames;
    a.frame_bytes = e->frame_bytes;
    a.cpitch = e->cpitch;
    a.rec = d_rec;
    a.coef = d_coef;
    a.mbx = e->d_mbx;
    a.gjunk = e->d_gjunk;
    if (++e->epoch >= (1u << 20)) {           // granule tags: epoch in the high dword
        if (h264mi_engine_sync(e)) return -1;
        HIPCHECK(hipMemsetAsync(e->d_mbx, 0, mbs * 256, e->st));
        HIPCHECK(hipMemsetAsync(e->d_prog, 0, sizeof(unsigned long long) * 2 * PROG_STRIDE * e->pipe_cap * e->h, e->st));
        HIPCHECK(hipMemsetAsync(e->d_done, 0, sizeof(unsigned) * e->pipe_cap * e->h, e->st));
        e->epoch = 1;
    }
    a.epoch = e->epoch;
    // (a launch of more pictures than the stamp buffer holds runs unstamped)
    a.prof = e->d_prof && (size_t)npics * ((size_t)e->h * 16 + (size_t)e->nmbs * PROF_MB) <= e->prof_cap ? e->d_prof : nullptr;
    a.prof_mode = e->d_prof && getenv("H264MI_PROF_MODE") ? atoi(getenv("H264MI_PROF_MODE")) : 0;
    // study knobs: MC lead over the row's deblocking (MBs; 0 / unset = the
    // ring depth), before the chain has begun (LEAD0, at least 4) and after
    static const int mc_lead0 = getenv("H264MI_MC_LEAD0") ? std::max(4, atoi(getenv("H264MI_MC_LEAD0"))) : 0;
    static const int mc_lead = getenv("H264MI_MC_LEAD") ? std::max(4, atoi(getenv("H264MI_MC_LEAD"))) : 0;
    a.mc_lead0 = mc_lead0;
    a.mc_lead = mc_lead;
    // row waves at s_setprio 1 off the chain (slot waits, copy-in, frame
    // stores) and 3 on it: on by default since the 4-workgroups-per-CU shape
    // (profiles/r85_ab_row_prio.txt: 305.3 vs 307.3 us per step, 6 of 6
    // rounds); H264MI_ROW_PRIO=0 turns it off
    static const int row_prio = getenv("H264MI_ROW_PRIO") ? atoi(getenv("H264MI_ROW_PRIO")) : 1;
    a.row_prio_split = row_prio;
    // the 2-MC-wave urgency distance (MBs; H264MI_MC_URGENCY): 8, and 12 in
    // launches of three or more steps (profiles/r93_ab_knobs_pipe3.txt: 303.0
    // vs 303.9 us per step, 4 of 4 rounds)
    static const int mc_urg = getenv("H264MI_MC_URGENCY") ? atoi(getenv("H264MI_MC_URGENCY")) : 0;
    a.mc_urgency = mc_urg > 0 ? mc_urg : P > 2 ? 12 : 8;
    // study knob: the top MB rows' urgent MC waves at the row waves' priority
    // (H264MI_MC_TOP rows; 0 = off)
    static const int mc_top = getenv("H264MI_MC_TOP") ? atoi(getenv("H264MI_MC_TOP")) : 0;
    a.mc_top = mc_top;
    a.chk_inject = e->check ? e->check_inject : 0;
    a.chk_short_cols = e->check ? e->check_short_cols : 0;
    a.chk_short_rows = e->check ? e->check_short_rows : 0;

    a.pics = d_pics;
    a.npics = npics;
    a.w = e->w; a.h = e->h;
    a.err = e->d_err;
    a.S = S;
    // study build only (-DSTUDY_NODEP; output NOT valid): the steps of a
    // launch wait on nothing -- the overlap an exact finer-grained dependency
    // could reach at most.  A compile-time switch, like
    // STUDY_NEAR: no environment variable changes what the library computes
#ifdef STUDY_NODEP
    a.P = 1;
#else
    a.P = P;
#endif
    a.prog = e->d_prog;
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
        a.n_nmbs_total = next_npics * e->nmbs;
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
    // frame-pipelined launches: the DEP_ROWS / DEP_COLS instances (single-row,
    // 2 MC waves).  The mode is the caller's hint for this launch or the
    // engine's default; whole rows need every slot below 32 (a bit mask)
    const bool dep3 = P > 1;
    int dmode = e->launch_dep ? e->launch_dep : e->dep_mode;
    if (e->nslots > 32) dmode = DEP_COLS;
    e->launch_dep = 0;                        // a hint covers one launch
    e->last_dep = dep3 ? dmode : DEP_NONE;
    const int rpw = dep3 ? 1 : rows_per_wg(e, S);
    const dim3 grid(npics * ((e->h + rpw - 1) / rpw) + a.prep_wgs);
    const int nmc = dep3 ? 2 : launch_nmc(e, rpw, P, npics);
    e->last_nmc = nmc;
    e->launch_intra = -1;                     // a hint covers one launch
    const size_t lmbx = nmc == 2 && (!a.prof || rpw == 1) ? (rpw == 2 ? WgppLds<2, 2>::bytes(e->w)
                                                                      : WgppLds<2, 1>::bytes(e->w, dep3 && dmode == DEP_COLS))
                        : rpw == 3 ? WgppLds<3, 3>::bytes(e->w) : rpw == 2 ? WgppLds<3, 2>::bytes(e->w)
                        : nmc == 6 ? WgppLds<6, 1>::bytes(e->w) : WgppLds<3, 1>::bytes(e->w);
    if (dep3) {
        e->last_kernel = e->check ? "k_wgpp_check" : a.prof ? "k_wgpp_prof" : "k_wgpp";
#define DEP_LAUNCH(M)                                                                                          \
        do {                                                                                                   \
            if (a.prof && !e->check)                                                                           \
                hipExtLaunchKernelGGL((k_wgpp<2, true, true, 1, false, M>), grid, dim3(256), lmbx, e->st,      \
                                      rec ? t0 : nullptr, rec ? t2 : nullptr, 0, a);                          \
            else if (e->check)                                                                                 \
                hipExtLaunchKernelGGL((k_wgpp<2, false, true, 1, true, M>), grid, dim3(256), lmbx, e->st,      \
                                      rec ? t0 : nullptr, rec ? t2 : nullptr, 0, a);                          \
            else                                                                                               \
                hipExtLaunchKernelGGL((k_wgpp<2, false, true, 1, false, M>), grid, dim3(256), lmbx, e->st,     \
                                      rec ? t0 : nullptr, rec ? t2 : nullptr, 0, a);                          \
        } while (0)
        if (dmode == DEP_COLS) DEP_LAUNCH(DEP_COLS);
        else DEP_LAUNCH(DEP_ROWS);
#undef DEP_LAUNCH
    } else if (a.prof) {
        if (rec) (void)hipEventRecord(t0, e->st);
        if (rpw == 3) hipLaunchKernelGGL((k_wgpp<3, true, true, 3>), grid, dim3(960), lmbx, e->st, a);
        else if (rpw == 2) hipLaunchKernelGGL((k_wgpp<3, true, true, 2>), grid, dim3(640), lmbx, e->st, a);
        else if (nmc == 2) hipLaunchKernelGGL((k_wgpp<2, true, true, 1>), grid, dim3(256), lmbx, e->st, a);
        else if (nmc == 6) hipLaunchKernelGGL((k_wgpp<6, true, true, 1>), grid, dim3(512), lmbx, e->st, a);
        else hipLaunchKernelGGL((k_wgpp<3, true, true, 1>), grid, dim3(320), lmbx, e->st, a);
        if (rec) (void)hipEventRecord(t2, e->st);
    } else if (e->check) {
        // dependency checker (H264MI_CHECK=1): every hand-off verified at
        // its consumer, violations in the pictures' error words
        e->last_kernel = "k_wgpp_check";
        if (rec) (void)hipEventRecord(t0, e->st);
        if (rpw == 3) hipLaunchKernelGGL((k_wgpp<3, false, true, 3, true>), grid, dim3(960), lmbx, e->st, a);
        else if (rpw == 2 && nmc == 2) hipLaunchKernelGGL((k_wgpp<2, false, true, 2, true>), grid, dim3(512), lmbx, e->st, a);
        else if (rpw == 2) hipLaunchKernelGGL((k_wgpp<3, false, true, 2, true>), grid, dim3(640), lmbx, e->st, a);
        else if (nmc == 2) hipLaunchKernelGGL((k_wgpp<2, false, true, 1, true>), grid, dim3(256), lmbx, e->st, a);
        else if (nmc == 6) hipLaunchKernelGGL((k_wgpp<6, false, true, 1, true>), grid, dim3(512), lmbx, e->st, a);
        else hipLaunchKernelGGL((k_wgpp<3, false, true, 1, true>), grid, dim3(320), lmbx, e->st, a);
        if (rec) (void)hipEventRecord(t2, e->st);
    } else if (nmc == 2) {
        // sizing study (H264MI_MC_WAVES=2): two MC waves per row workgroup
        if (rpw == 2)
            hipExtLaunchKernelGGL((k_wgpp<2, false, true, 2>), grid, dim3(512), lmbx, e->st, rec ? t0 : nullptr,
                                  rec ? t2 : nullptr, 0, a);
        else
            hipExtLaunchKernelGGL((k_wgpp<2, false, true, 1>), grid, dim3(256), lmbx, e->st, rec ? t0 : nullptr,
                                  rec ? t2 : nullptr, 0, a);
    } else if (nmc == 6) {
        hipExtLaunchKernelGGL((k_wgpp<6, false, true, 1>), grid, dim3(512), lmbx, e->st, rec ? t0 : nullptr,
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
    e->prepped_n = next_npics;
    e->prep_parity = hb ^ 1;                  // the half the next batch was (or will be) prepped into
    return 0;
}

// intra_heavy: the batch's launch shape hint when the caller knows it (the
// host path counts intra MBs while parsing); -1: derive it from the records

extern "C" int h264mi_engine_decode(h264mi_engine *e, int npics, const int *stream, const int *cur_slot,
                                    const void *const *recs, const int16_t *const *coefs, const uint32_t *ncoef)
{
    return engine_decode_host(e, npics, stream, cur_slot, recs, coefs, ncoef, -1);
}

int engine_decode_host(h264mi_engine *e, int npics, const int *stream, const int *cur_slot,
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
        {
            const MbRec *r = (const MbRec *)recs[i];
            int n = 0, db = 0;
            for (int m = 0; m < e->nmbs; m++) { n += r[m].type >= MBT_I4x4; db |= r[m].avail & DB_INNER; }
            pd.flags = (2 * n > e->nmbs ? PD_INTRA_HEAVY : 0) | (db ? 0 : PD_NO_DEBLOCK);
        }
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
    for (int i = 0; i < npics && !heavy && intra_heavy < 0; i++) heavy = (e->h_pics[i].flags & PD_INTRA_HEAVY) != 0;
    e->launch_intra = heavy;
    return launch_batch(e, npics, 1, e->d_rec, e->d_coef, e->d_pics, NULL, NULL, NULL);
}

int engine_decode_direct(h264mi_engine *e, int stream, int cur_slot, const void *rec, const int16_t *coef,
                         uint32_t ncoef, int intra_heavy)
{
    if (!e || stream < 0 || stream >= e->nstreams || cur_slot < 0 || cur_slot >= e->nslots) return -1;
    HIPCHECK(hipSetDevice(e->dev));
    // the descriptor staging is reused: wait until the previous upload consumed it
    HIPCHECK(hipEventSynchronize(e->ev_staged));
    if ((size_t)ncoef + 16 > e->coef_cap) {
        HIPCHECK(hipStreamSynchronize(e->st));
        (void)hipFree(e->d_coef);
        (void)hipHostFree(e->h_coef);
        e->coef_cap = e->h_coef_cap = ncoef + ncoef / 2 + 1024;
        HIPCHECK(hipMalloc(&e->d_coef, e->coef_cap * 32));
        HIPCHECK(hipHostMalloc(&e->h_coef, e->h_coef_cap * 32, hipHostMallocDefault));
    }
    PicDesc &pd = e->h_pics[0];
    pd.rec_base = 0;
    pd.frame_base = (uint32_t)(stream * e->nslots);
    pd.cur_slot = (uint32_t)cur_slot;
    {
        const MbRec *r = (const MbRec *)rec;
        int n = 0, db = 0;
        for (int m = 0; m < e->nmbs; m++) { n += r[m].type >= MBT_I4x4; db |= r[m].avail & DB_INNER; }
        pd.flags = (2 * n > e->nmbs ? PD_INTRA_HEAVY : 0) | (db ? 0 : PD_NO_DEBLOCK);
    }
    pd.coef_base = 0;
    pd.rsv[0] = pd.rsv[1] = pd.rsv[2] = 0;
    HIPCHECK(hipMemcpyAsync(e->d_rec, rec, sizeof(MbRec) * e->nmbs, hipMemcpyHostToDevice, e->st));
    if (ncoef) HIPCHECK(hipMemcpyAsync(e->d_coef, coef, (size_t)ncoef * 32, hipMemcpyHostToDevice, e->st));
    HIPCHECK(hipMemcpyAsync(e->d_pics, e->h_pics, sizeof(PicDesc), hipMemcpyHostToDevice, e->st));
    HIPCHECK(hipEventRecord(e->ev_staged, e->st));
    e->launch_intra = intra_heavy >= 0 ? intra_heavy : (pd.flags & PD_INTRA_HEAVY) != 0;
    return launch_batch(e, 1, 1, e->d_rec, e->d_coef, e->d_pics, NULL, NULL, NULL);
}

int engine_records_wait(h264mi_engine *e)
{
    if (!e) return -1;
    HIPCHECK(hipSetDevice(e->dev));
    HIPCHECK(hipEventSynchronize(e->ev_staged));
    return 0;
}

// the next launch's content, for callers holding their records on the device
// (launch_nmc): 1 = some picture has more than half its MBs intra, 0 = none
extern "C" int h264mi_engine_hint_intra(h264mi_engine *e, int intra_heavy)
{
    if (!e || intra_heavy < 0 || intra_heavy > 1) return -1;
    e->launch_intra = intra_heavy;
    return 0;
}

// the next frame-pipelined launch's dependency mode: 1 whole MB rows, 2 (MB
// row, MB column) cells, 0 the engine's default (H264MI_DEP_MODE)
extern "C" int h264mi_engine_hint_deps(h264mi_engine *e, int mode)
{
    if (!e || mode < 0 || mode > DEP_COLS) return -1;
    e->launch_dep = mode;
    return 0;
}
extern "C" int h264mi_engine_last_deps(h264mi_engine *e) { return e ? e->last_dep : -1; }
extern "C" int h264mi_engine_last_mc_waves(h264mi_engine *e) { return e ? e->last_nmc : -1; }

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

// the same, naming the next batch's steps (1 .. the engine's steps) when it
// has a different count: its k_prep in this launch's tail covers S * next_P
// pictures (a plan mixing one- and two-step launches keeps its tail preps)
extern "C" int h264mi_engine_decode_device_steps_next(h264mi_engine *e, int S, int P, const void *d_recs,
                                                      const int16_t *d_coef, const void *d_pics,
                                                      const void *next_recs, const int16_t *next_coef,
                                                      const void *next_pics, int next_P)
{
    if (!e || S < 1 || S > e->nstreams || P < 1 || P > e->steps || !d_recs || !d_pics) return -1;
    if (!next_recs || !next_pics || next_P < 1 || next_P > e->steps) return -1;
    HIPCHECK(hipSetDevice(e->dev));
    return launch_batch(e, S, P, (const MbRec *)d_recs, d_coef, (const PicDesc *)d_pics, (const MbRec *)next_recs,
                        next_coef, (const PicDesc *)next_pics, S * next_P);
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

// the profiling kernels' stamp buffer, sized for the engine's current
// picture capacity (every picture of a launch: per-row and per-MB stamps)
static int prof_alloc(h264mi_engine *e)
{
    (void)hipFree(e->d_prof);
    e->d_prof = NULL;
    e->prof_cap = (size_t)e->pipe_cap * e->h * 16 + (size_t)e->pipe_cap * e->nmbs * PROF_MB;
    HIPCHECK(hipMalloc(&e->d_prof, sizeof(unsigned long long) * e->prof_cap));
    HIPCHECK(hipMemset(e->d_prof, 0, sizeof(unsigned long long) * e->prof_cap));
    return 0;
}

extern "C" int h264mi_engine_set_steps(h264mi_engine *e, int steps)
{
    // (frame-pipelined launches name the earlier steps' target slots in a
    // 32-bit mask: recon_kernels.hip dep_wait)
    // (a later step's producers: by slot equality, 8-bit slots (DEP_COLS), or
    // a 32-bit slot mask (DEP_ROWS; engines of more slots run DEP_COLS))
    if (!e || steps < 1 || steps > H264MI_MAX_STEPS || (steps > 1 && e->nslots > 255)) return -1;
    if (steps == e->steps) return 0;
    if (h264mi_engine_sync(e)) return -1;
    free_pic_buffers(e);
    if (alloc_pic_buffers(e, e->nstreams * steps)) return -1;
    e->steps = steps;
    e->prepped_rec = NULL; e->prepped_pics = NULL;
    e->prep_parity = 0;
    // a profiling buffer allocated for the old capacity would be overrun by
    // the stamps of a launch of more pictures: resize it with the capacity
    if (e->d_prof && prof_alloc(e)) return -1;
    HIPCHECK(hipStreamSynchronize(e->st));
    return 0;
}

extern "C" const char *h264mi_engine_kernel(h264mi_engine *e)
{
    return e && e->last_kernel ? e->last_kernel : "";
}

// wait for everything queued on the engine's stream (sleeping under
// H264MI_BLOCKING_SYNC); no flag accounting
int engine_wait(h264mi_engine *e)
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
    for (int i = 0; i < e->pipe_cap; i++) {
        e->err_accum += e->h_err[i] ? 1 : 0;
        e->err_bits |= e->h_err[i];
    }
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

extern "C" uint32_t h264mi_engine_error_bits(h264mi_engine *e)
{
    if (!e) return 0;
    const uint32_t v = e->err_bits;
    e->err_bits = 0;
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

extern "C" int h264mi_engine_timing_list(h264mi_engine *e, double *us, int cap)
{
    if (!e || !e->tev || !us || cap < 0) return -1;
    if (h264mi_engine_sync(e)) return -1;
    const int n = e->tev_n < cap ? e->tev_n : cap;
    for (int i = 0; i < n; i++) {
        float m = 0;
        HIPCHECK(hipEventElapsedTime(&m, e->tev[3 * i], e->tev[3 * i + 2]));
        us[i] = m * 1000.0;
    }
    return n;
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
        if (prof_alloc(e)) return -1;
    } else if (!enable && e->d_prof) {
        HIPCHECK(hipStreamSynchronize(e->st));
        (void)hipFree(e->d_prof);
        e->d_prof = NULL;
        e->prof_cap = 0;
    }
    return 0;
}

// D2H of a slot as packed I420 on `st`, asynchronous: the luma plane and the
// padded chroma rows (H264MI_CPITCH) as one strided copy of 2 * h * 8 rows
int engine_copy_out(h264mi_engine *e, int stream, int slot, uint8_t *dst, hipStream_t st)
{
    const uint8_t *src = e->d_frames + e->frame_bytes * ((size_t)stream * e->nslots + slot);
    const size_t ysz = (size_t)e->nmbs * 256, cw = (size_t)e->w * 8;
    if ((size_t)e->cpitch == cw) {
        HIPCHECK(hipMemcpyAsync(dst, src, e->pic_bytes, hipMemcpyDeviceToHost, st));
        return 0;
    }
    HIPCHECK(hipMemcpyAsync(dst, src, ysz, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipMemcpy2DAsync(dst + ysz, cw, src + ysz, (size_t)e->cpitch, cw, (size_t)e->h * 16, hipMemcpyDeviceToHost, st));
    return 0;
}
size_t engine_slot_bytes(const h264mi_engine *e) { return e->frame_bytes; }

extern "C" int h264mi_engine_read(h264mi_engine *e, int stream, int slot, uint8_t *dst)
{
    if (!e || stream < 0 || stream >= e->nstreams || slot < 0 || slot >= e->nslots) return -1;
    if (h264mi_engine_sync(e)) return -1;
    if (engine_copy_out(e, stream, slot, dst, e->st)) return -1;
    HIPCHECK(hipStreamSynchronize(e->st));
    return 0;
}

// I420 -> RGBA (DecoderPost.js `rgb: true`, color.hip) for `npics` pictures
// of width x height pixels at in + k * in_stride -> out + k * out_stride,
// device pointers, on `stream` (NULL: the null stream); asynchronous
extern "C" int h264mi_yuv2rgba_device_pitch(const void *d_i420, void *d_rgba, int width, int height, int cpitch,
                                            int npics, size_t in_stride, size_t out_stride, void *stream)
{
    if (!d_i420 || !d_rgba || width <= 0 || height <= 0 || (width & 15) || (height & 15) || npics < 1 ||
        cpitch < width / 2)
        return -1;
    const int nblk = ((height >> 1) * (width >> 2) + 127) >> 7;
    hipLaunchKernelGGL(k_yuv2rgba, dim3(nblk, npics), dim3(64), 0, (hipStream_t)stream,
                       (const uint8_t *)d_i420, (uint8_t *)d_rgba, width, height, cpitch, in_stride, out_stride);
    HIPCHECK(hipGetLastError());
    return 0;
}

extern "C" int h264mi_yuv2rgba_device(const void *d_i420, void *d_rgba, int width, int height, int npics,
                                      size_t in_stride, size_t out_stride, void *stream)
{
    return h264mi_yuv2rgba_device_pitch(d_i420, d_rgba, width, height, width / 2, npics, in_stride, out_stride, stream);
}

extern "C" int h264mi_engine_read_rgba(h264mi_engine *e, int stream, int slot, uint8_t *dst)
{
    if (!e || stream < 0 || stream >= e->nstreams || slot < 0 || slot >= e->nslots) return -1;
    const size_t bytes = (size_t)e->nmbs * 256 * 4;
    if (!e->d_rgba) HIPCHECK(hipMalloc(&e->d_rgba, bytes));
    if (h264mi_yuv2rgba_device_pitch(e->d_frames + e->frame_bytes * ((size_t)stream * e->nslots + slot), e->d_rgba,
                                     e->w * 16, e->h * 16, e->cpitch, 1, 0, 0, e->st))
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

extern "C" int h264mi_engine_abi(void) { return H264MI_ENGINE_ABI; }
extern "C" size_t h264mi_engine_frame_bytes(h264mi_engine *e) { return e ? e->pic_bytes : 0; }
extern "C" size_t h264mi_engine_slot_bytes(h264mi_engine *e) { return e ? e->frame_bytes : 0; }
extern "C" int h264mi_engine_chroma_pitch(h264mi_engine *e) { return e ? e->cpitch : 0; }

// neighbour-based concealment of a picture's missing MBs on the device
// (k_conceal, conceal.hip), behind the work already on the engine's stream:
// slot `slot` of stream `stream` holds the decoded MBs reconstructed with the
// loop filter off; order[0..n) are the MBs to conceal in h264bsdConceal's
// order, decoded[0..w*h) the MBs decoded (1) or missing (0).  The inputs are
// copied before returning.
static std::atomic<unsigned long long> g_conceal_launches{0};
// diagnostics: k_conceal launches in this process (tests: the device path ran)
extern "C" unsigned long long h264mi_conceal_launches(void) { return g_conceal_launches.load(); }
int engine_conceal_fits(const h264mi_engine *e) { return e && e->conceal_fits; }

extern "C" int h264mi_engine_conceal(h264mi_engine *e, int stream, int slot, const int *order, int n,
                                     const uint8_t *decoded)
{
    if (!e || stream < 0 || stream >= e->nstreams || slot < 0 || slot >= e->nslots || n < 0 || n > e->nmbs ||
        (n && (!order || !decoded)))
        return -1;
    if (!n) return 0;
    if (!e->conceal_fits) return -2;          // picture too large for k_conceal's LDS
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
                       e->w, e->h, e->cpitch, (const int *)e->d_conceal, n, (const uint8_t *)(e->d_conceal + sizeof(int) * (size_t)e->nmbs));
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

// -------- internal interface of the H264Backend adapter (engine_int.h) ----
hipStream_t engine_stream(h264mi_engine *e) { return e->st; }
unsigned *engine_err_words(h264mi_engine *e) { return e->d_err; }

void engine_shape(const h264mi_engine *e, int *w_mbs, int *h_mbs, int *nstreams, int *nslots, int *blocking)
{
    *w_mbs = e->w; *h_mbs = e->h; *nstreams = e->nstreams; *nslots = e->nslots;
    *blocking = e->ev_block != NULL;
}

int engine_poolable(const h264mi_engine *e) { return !e->tev && !e->d_prof; }

int engine_reuse(h264mi_engine *e)
{
    HIPCHECK(hipSetDevice(e->dev));
    engine_config(e);
    e->prepped_rec = e->prepped_pics = NULL;
    e->prepped_n = 0;
    e->err_accum = 0;
    e->err_bits = 0;          // the previous owner's device / checker flags
    e->steps = 1;
    e->last_kernel = NULL;
    // the epoch keeps counting: the mailboxes hold tags of earlier launches only
    HIPCHECK(hipMemsetAsync(e->d_frames, 0, e->frame_bytes * e->nslots * e->nstreams, e->st));
    return 0;
}
