#define _GNU_SOURCE
/* Speculative parallel slice-data parsing (host throughput of the end-to-end
 * path; no reference counterpart -- the reference parses one NAL per call).
 *
 * The C API is sequential: every call decodes the next NAL unit.  When a
 * picture's first slice is decoded and the caller's buffer already holds the
 * picture's next slice NAL units (a byte stream handed over whole, as
 * DecTestBench does), worker threads parse those slices ahead -- header,
 * RefPicList0 from a snapshot of the DPB, and the whole slice_data() into a
 * private PicBuild -- while the calling thread parses the first slice.
 * Slices are independent in slice_data() (neighbours in other slices are
 * unavailable, H.264 §6.4.x), so a private parse sees exactly what the
 * sequential one sees.
 *
 * The sequential path stays the authority: when the calling thread reaches
 * such a NAL it parses the slice header itself and takes the worker's result
 * only if the NAL bytes, the slice header, the parameter sets and the
 * reference list are identical and the slice parsed without error and
 * overlaps no decoded MB; otherwise it parses the slice itself.  Results are
 * therefore the sequential decoder's, bit for bit. */
#include "decoder.h"

#include <pthread.h>
#include <stdio.h>
#include <time.h>
#include <stdlib.h>
#include <string.h>

#define SPEC_MAX_JOBS 16

typedef struct SpecJob {
    /* set by the caller */
    const uint8_t *nal_ptr;    /* caller's buffer position of the NAL unit */
    uint32_t read_bytes;       /* bytes the NAL consumes (nal_scan) */
    uint8_t *raw;              /* private copy of those bytes */
    uint32_t raw_cap;
    uint8_t *rbsp;
    uint32_t rbsp_cap;
    int      is_first;         /* the picture's first slice (launched ahead) */
    int      started;          /* claimed by a worker or by the calling thread */
    /* worker results */
    int      done, ok;
    SliceHdr sh;
    int      ref_slot[MAX_REFS];
    PicBuild pb;
    int      pb_ready;
} SpecJob;

struct SpecPool {
    pthread_t       *th;
    int              nth;
    pthread_mutex_t  mu;
    pthread_cond_t   cv_work, cv_done;
    int              stop;
    SpecJob          jobs[SPEC_MAX_JOBS];
    int              njobs, next;   /* jobs[order[next..njobs)] wait for a worker */
    int              order[SPEC_MAX_JOBS];
    int              running;
    unsigned long    taken, declined;   /* statistics (H264MI_SPEC_STATS) */
    int              stats;
    double           w_cpu, c_cpu, m_cpu;   /* thread CPU: worker jobs, commits, the caller's own slices */
    double           a_cpu;                 /* the caller's whole decode calls */
    unsigned long    w_mbs, m_mbs;
    /* snapshot of the picture the jobs belong to */
    Sps              sps;
    Pps              pps;
    Dpb              dpb;
    SliceHdr         first;         /* the picture's first slice header */
    const uint8_t   *pic_ptr;       /* buffer position of the picture's first slice NAL */
    NalHdr           nh;
    int              w, h, cip, cur_slot;
};

static double thread_cpu(void)
{
    struct timespec t;
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static void run_job(SpecPool *sp, SpecJob *j)
{
    j->ok = 0;
    uint32_t init, size, rb;
    int emul;
    /* j->read_bytes is the caller's (spec_take matches jobs by it under the
     * lock): scan into a local, never write the shared field here */
    if (nal_scan(j->raw, j->read_bytes, &init, &size, &rb, &emul) || rb != j->read_bytes) return;
    if (j->rbsp_cap < size + 8) {
        free(j->rbsp);
        j->rbsp_cap = size + 64 + size / 2;
        j->rbsp = (uint8_t *)malloc(j->rbsp_cap);
        if (!j->rbsp) { j->rbsp_cap = 0; return; }
    }
    const int n = nal_unescape(j->raw + init, size, emul, j->rbsp);
    if (n < 2 || (j->rbsp[0] & 0x80)) return;
    const NalHdr nh = {(j->rbsp[0] >> 5) & 3, j->rbsp[0] & 31};
    if (nh.type != sp->nh.type || (nh.ref_idc != 0) != (sp->nh.ref_idc != 0)) return;
    BitReader br;
    br_init(&br, j->rbsp + 1, (size_t)n - 1);
    if (parse_slice_header(&br, &nh, &sp->sps, &sp->pps, &j->sh)) return;
    const SliceHdr *f = &sp->first;
    if (j->sh.pps_id != f->pps_id || j->sh.frame_num != f->frame_num || j->sh.idr_pic_id != f->idr_pic_id ||
        j->sh.poc_lsb != f->poc_lsb || j->sh.delta_poc_bottom != f->delta_poc_bottom ||
        (j->is_first ? j->sh.first_mb != f->first_mb : j->sh.first_mb <= f->first_mb))
        return;                                   /* not a slice of this picture */
    Dpb dpb = sp->dpb;                            /* dpb_build_list updates list / PicNums */
    if (dpb_build_list(&dpb, &j->sh, j->ref_slot)) return;
    if (!j->pb_ready || j->pb.w != sp->w || j->pb.h != sp->h) {
        if (j->pb_ready) picbuild_free(&j->pb);
        j->pb_ready = 0;
        if (picbuild_init(&j->pb, sp->w, sp->h)) return;
        picbuild_reset(&j->pb, sp->cip);
        j->pb_ready = 1;
    }
    picbuild_reuse(&j->pb, sp->cip);
    j->pb.cur_slot = sp->cur_slot;
    if (parse_slice_data(&j->pb, &br, &j->sh, &sp->pps, j->ref_slot)) return;
    j->ok = 1;
}

/* host CPU attribution (h264mi_host_thread_stats): the speculative-parse
 * workers' whole-thread CPU, added when each worker exits */
static unsigned long long g_worker_cpu_ns, g_workers_started;

int h264mi_host_thread_stats(double *spec_worker_cpu_s, unsigned long long *workers_started)
{
    if (spec_worker_cpu_s) *spec_worker_cpu_s = 1e-9 * (double)__atomic_load_n(&g_worker_cpu_ns, __ATOMIC_RELAXED);
    if (workers_started) *workers_started = __atomic_load_n(&g_workers_started, __ATOMIC_RELAXED);
    return 0;
}

static void *worker(void *arg)
{
    SpecPool *sp = (SpecPool *)arg;
    pthread_setname_np(pthread_self(), "h264mi-spec");
    __atomic_add_fetch(&g_workers_started, 1, __ATOMIC_RELAXED);
    pthread_mutex_lock(&sp->mu);
    for (;;) {
        while (!sp->stop && sp->next < sp->njobs && sp->jobs[sp->order[sp->next]].started) sp->next++;
        if (sp->stop) break;
        if (sp->next >= sp->njobs) { pthread_cond_wait(&sp->cv_work, &sp->mu); continue; }
        SpecJob *j = &sp->jobs[sp->order[sp->next++]];
        j->started = 1;
        sp->running++;
        pthread_mutex_unlock(&sp->mu);
        const double t0 = sp->stats ? thread_cpu() : 0.0;
        run_job(sp, j);
        pthread_mutex_lock(&sp->mu);
        if (sp->stats) {
            sp->w_cpu += thread_cpu() - t0;
            if (j->ok) sp->w_mbs += (unsigned long)j->pb.ndecoded;
        }
        j->done = 1;
        sp->running--;
        pthread_cond_broadcast(&sp->cv_done);
    }
    pthread_mutex_unlock(&sp->mu);
    __atomic_add_fetch(&g_worker_cpu_ns, (unsigned long long)(thread_cpu() * 1e9), __ATOMIC_RELAXED);
    return NULL;
}

SpecPool *spec_create(int nthreads)
{
    if (nthreads < 0) return NULL;
    SpecPool *sp = (SpecPool *)calloc(1, sizeof(SpecPool));
    if (!sp) return NULL;
    sp->stats = getenv("H264MI_SPEC_STATS") != NULL;
    pthread_mutex_init(&sp->mu, NULL);
    pthread_cond_init(&sp->cv_work, NULL);
    pthread_cond_init(&sp->cv_done, NULL);
    sp->th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int i = 0; sp->th && i < nthreads; i++)
        if (pthread_create(&sp->th[i], NULL, worker, sp) == 0) sp->nth++;
    if (!sp->nth && nthreads) { spec_destroy(sp); return NULL; }
    return sp;
}

/* the calling thread as a worker: run every queued job nobody has started */
void spec_help(SpecPool *sp)
{
    if (!sp) return;
    pthread_mutex_lock(&sp->mu);
    for (;;) {
        while (sp->next < sp->njobs && sp->jobs[sp->order[sp->next]].started) sp->next++;
        if (sp->next >= sp->njobs) break;
        SpecJob *j = &sp->jobs[sp->order[sp->next++]];
        j->started = 1;
        sp->running++;
        pthread_mutex_unlock(&sp->mu);
        const double t0 = sp->stats ? thread_cpu() : 0.0;
        run_job(sp, j);
        pthread_mutex_lock(&sp->mu);
        if (sp->stats) {
            sp->w_cpu += thread_cpu() - t0;
            if (j->ok) sp->w_mbs += (unsigned long)j->pb.ndecoded;
        }
        j->done = 1;
        sp->running--;
        pthread_cond_broadcast(&sp->cv_done);
    }
    pthread_mutex_unlock(&sp->mu);
}

/* wait for the workers, then forget every job */
void spec_drain(SpecPool *sp)
{
    if (!sp) return;
    pthread_mutex_lock(&sp->mu);
    sp->next = sp->njobs;                         /* nothing more starts */
    while (sp->running) pthread_cond_wait(&sp->cv_done, &sp->mu);
    sp->njobs = sp->next = 0;
    pthread_mutex_unlock(&sp->mu);
}

void spec_destroy(SpecPool *sp)
{
    if (!sp) return;
    if (sp->stats)
        fprintf(stderr, "h264mi: speculative slices taken %lu, parsed again %lu; thread CPU per MB: workers %.3f us "
                "(%lu MBs), caller %.3f us (%lu MBs), commits %.3f us per taken MB; caller decode calls %.3f s "
                "(own slices %.3f, commits %.3f, rest %.3f)\n", sp->taken, sp->declined,
                1e6 * sp->w_cpu / (double)(sp->w_mbs ? sp->w_mbs : 1), sp->w_mbs,
                1e6 * sp->m_cpu / (double)(sp->m_mbs ? sp->m_mbs : 1), sp->m_mbs,
                1e6 * sp->c_cpu / (double)(sp->w_mbs ? sp->w_mbs : 1), sp->a_cpu, sp->m_cpu, sp->c_cpu,
                sp->a_cpu - sp->m_cpu - sp->c_cpu);
    pthread_mutex_lock(&sp->mu);
    sp->stop = 1;
    pthread_cond_broadcast(&sp->cv_work);
    pthread_mutex_unlock(&sp->mu);
    for (int i = 0; i < sp->nth; i++) pthread_join(sp->th[i], NULL);
    for (int i = 0; i < SPEC_MAX_JOBS; i++) {
        free(sp->jobs[i].raw);
        free(sp->jobs[i].rbsp);
        if (sp->jobs[i].pb_ready) picbuild_free(&sp->jobs[i].pb);
    }
    free(sp->th);
    pthread_mutex_destroy(&sp->mu);
    pthread_cond_destroy(&sp->cv_work);
    pthread_cond_destroy(&sp->cv_done);
    free(sp);
}

static void queue_slices(SpecPool *sp, const uint8_t *buf, uint32_t pos, uint32_t len, int first_is_first);

/* Start of a picture: its first slice (header sh, NAL header nh) was just
 * read from buf[0..first_bytes); queue the slice NAL units that follow it in
 * buf[first_bytes..len). */
void spec_launch(SpecPool *sp, const H264Dec *d, const Sps *sps, const Pps *pps, const NalHdr *nh,
                 const SliceHdr *sh, const uint8_t *buf, uint32_t first_bytes, uint32_t len)
{
    if (!sp) return;
    spec_drain(sp);
    pthread_mutex_lock(&sp->mu);
    sp->sps = *sps;
    sp->pps = *pps;
    sp->dpb = d->dpb;
    sp->first = *sh;
    sp->nh = *nh;
    sp->w = d->pb.w; sp->h = d->pb.h; sp->cip = pps->cip; sp->cur_slot = d->cur_slot;
    sp->pic_ptr = buf;
    queue_slices(sp, buf, first_bytes, len, 0);
    pthread_cond_broadcast(&sp->cv_work);
    pthread_mutex_unlock(&sp->mu);
}

/* queue the slice NAL units of buf[pos..len) up to the first non-slice NAL
 * (caller holds the lock) */
static void queue_slices(SpecPool *sp, const uint8_t *buf, uint32_t pos, uint32_t len, int first_is_first)
{
    while (sp->njobs < SPEC_MAX_JOBS && pos < len) {
        uint32_t init, size, rb;
        int emul;
        if (nal_scan(buf + pos, len - pos, &init, &size, &rb, &emul) || size < 2 || rb == 0) break;
        const uint8_t t = buf[pos + init] & 31;
        if (t != NAL_SLICE && t != NAL_IDR) break;     /* a non-slice NAL ends the access unit */
        /* so does a slice with first_mb_in_slice 0 (ue(v) '1': the top bit of
         * the byte after the NAL header, never an emulation-prevention byte)
         * after the first job: the next picture.  Its slices would only be
         * scanned, copied, unescaped and declined by run_job (their header is
         * not this picture's); with arbitrary slice order a later slice of
         * this picture may start at MB 0 too, and is then parsed by the
         * calling thread instead */
        if (sp->njobs > 0 && size > 1 && (buf[pos + init + 1] & 0x80)) break;
        SpecJob *j = &sp->jobs[sp->njobs];
        if (j->raw_cap < rb) {
            free(j->raw);
            j->raw_cap = rb + rb / 2 + 64;
            j->raw = (uint8_t *)malloc(j->raw_cap);
            if (!j->raw) { j->raw_cap = 0; break; }
        }
        memcpy(j->raw, buf + pos, rb);           /* the caller may reuse its buffer */
        j->nal_ptr = buf + pos;
        j->read_bytes = rb;
        j->is_first = first_is_first && sp->njobs == 0;
        j->done = j->ok = j->started = 0;
        sp->order[sp->njobs] = sp->njobs;
        sp->njobs++;
        pos += rb;
    }
    /* workers take the picture's first slice last: the calling thread, when
     * it gets there before any worker, parses that one itself */
    if (first_is_first && sp->njobs > 1) {
        for (int i = 0; i + 1 < sp->njobs; i++) sp->order[i] = i + 1;
        sp->order[sp->njobs - 1] = 0;
    }
}

/* A picture was just finished and buf[0..len) continues the stream: when it
 * starts with the next picture's first slice, parse that picture's slices
 * ahead -- all of them -- against the DPB as the finished picture left it
 * and the frame slot the next picture will take (dpb_alloc_current).  A gap
 * in frame_num or new parameter sets make the results differ; spec_take then
 * declines them. */
void spec_launch_ahead(SpecPool *sp, const H264Dec *d, const uint8_t *buf, uint32_t len)
{
    if (!sp || !len || d->active_sps < 0 || d->active_sps >= MAX_SPS) return;
    spec_drain(sp);
    uint32_t init, size, rb;
    int emul;
    if (nal_scan(buf, len, &init, &size, &rb, &emul) || size < 2) return;
    const uint8_t t = buf[init] & 31;
    if (t != NAL_SLICE && t != NAL_IDR) return;
    /* the first slice's header, from its first bytes */
    uint8_t hdr[256];
    const uint32_t hs = size < 200 ? size : 200;
    uint32_t k = 0;
    int zc = 0;
    for (uint32_t i = 0; i < hs; i++) {             /* emulation-prevention removal, prefix only */
        const uint8_t b = buf[init + i];
        if (zc == 2 && b == 3 && emul) { zc = 0; continue; }
        zc = b == 0 ? zc + 1 : 0;
        hdr[k++] = b;
    }
    if (hdr[0] & 0x80) return;
    const NalHdr nh = {(hdr[0] >> 5) & 3, hdr[0] & 31};
    BitReader br;
    br_init(&br, hdr + 1, k - 1);
    int pps_id;
    if (peek_slice_pps_id(&br, &pps_id) || !d->pps[pps_id].valid || d->pps[pps_id].sps_id != d->active_sps) return;
    const Sps *sps = &d->sps[d->active_sps];
    const Pps *pps = &d->pps[pps_id];
    SliceHdr sh;
    if (parse_slice_header(&br, &nh, sps, pps, &sh)) return;
    pthread_mutex_lock(&sp->mu);
    sp->sps = *sps;
    sp->pps = *pps;
    sp->dpb = d->dpb;
    sp->first = sh;
    sp->nh = nh;
    sp->w = d->pb.w; sp->h = d->pb.h; sp->cip = pps->cip;
    sp->cur_slot = d->dpb.pic[d->dpb.size].slot;     /* what dpb_alloc_current will return */
    sp->pic_ptr = buf;
    queue_slices(sp, buf, 0, len, 1);
    pthread_cond_broadcast(&sp->cv_work);
    pthread_mutex_unlock(&sp->mu);
}

/* slices of the picture starting at buf are being parsed ahead */
int spec_active_for(const SpecPool *sp, const uint8_t *buf)
{
    return sp && sp->njobs && sp->pic_ptr == buf;
}

static int commit(SpecPool *sp, SpecJob *j, H264Dec *d, const uint8_t *buf, uint32_t read_bytes, const SliceHdr *sh,
                  const Pps *pps, const int *ref_slot);

/* The calling thread reached the slice NAL at buf (read_bytes long) whose
 * header it parsed into sh, with reference list ref_slot: take a matching
 * worker result into d->pb.  1: taken (the slice is decoded), 0: parse it. */
int spec_take(SpecPool *sp, H264Dec *d, const uint8_t *buf, uint32_t read_bytes, const SliceHdr *sh,
              const Pps *pps, const int *ref_slot)
{
    if (!sp) return 0;
    pthread_mutex_lock(&sp->mu);
    SpecJob *j = NULL;
    for (int i = 0; i < sp->njobs; i++)
        if (sp->jobs[i].nal_ptr == buf && sp->jobs[i].read_bytes == read_bytes) { j = &sp->jobs[i]; break; }
    if (j) {
        if (!j->started) {                        /* not started: parse it here instead */
            j->started = 1;
            pthread_mutex_unlock(&sp->mu);
            return 0;
        }
        while (!j->done) pthread_cond_wait(&sp->cv_done, &sp->mu);
    }
    pthread_mutex_unlock(&sp->mu);
    const double t0 = sp->stats ? thread_cpu() : 0.0;
    const int r = j && j->ok && commit(sp, j, d, buf, read_bytes, sh, pps, ref_slot);
    if (sp->stats) sp->c_cpu += thread_cpu() - t0;
    if (j) { if (r) sp->taken++; else sp->declined++; }
    return r;
}

static int commit(SpecPool *sp, SpecJob *j, H264Dec *d, const uint8_t *buf, uint32_t read_bytes, const SliceHdr *sh,
                  const Pps *pps, const int *ref_slot)
{
    PicBuild *pb = &d->pb, *q = &j->pb;
    if (memcmp(j->raw, buf, read_bytes) || memcmp(&j->sh, sh, sizeof(*sh)) ||
        memcmp(j->ref_slot, ref_slot, sizeof(j->ref_slot)) || memcmp(&sp->pps, pps, sizeof(*pps)) ||
        pb->cur_slot != sp->cur_slot || pb->pc.cip != sp->cip)
        return 0;
    const int first = sh->first_mb, count = q->ndecoded;
    if (first + count > pb->nmbs || pb->ndecoded + count > pb->nmbs) return 0;
    for (int i = first; i < first + count; i++) if (pb->decoded[i]) return 0;
    const uint32_t off = pb->ncoef;
    int16_t *dst = picbuild_coef_alloc(pb, q->ncoef);
    if (!dst && q->ncoef) return 0;
    if (q->ncoef) memcpy(dst, q->coef, (size_t)q->ncoef * 32);
    const uint16_t tag = (uint16_t)++pb->nslices;
    /* of the neighbour state (MbInfo) later code reads only the slice id of
     * MBs in other slices: neighbours across a slice boundary are unavailable
     * (mbctx_neighbour), and un-marking / concealment look at ids and
     * decoded flags */
    for (int i = first; i < first + count; i++) {
        pb->rec[i] = q->rec[i];
        pb->rec[i].coef += off;
        pb->rec[i].slice = tag;
        pb->pc.slice[i] = tag;
        pb->decoded[i] = 1;
    }
    pb->ndecoded += count;
    pb->last_mb_addr = q->last_mb_addr;
    pb->is_p |= q->is_p;
    pb->alg_ref_bytes += q->alg_ref_bytes;
    pb->n_inter += q->n_inter;
    pb->n_intra += q->n_intra;
    pb->n_coded_blocks += q->n_coded_blocks;
    return 1;
}

/* statistics: the calling thread parsed a slice itself */
int spec_stats_on(const SpecPool *sp) { return sp && sp->stats; }
double spec_thread_cpu(void) { return thread_cpu(); }
void spec_account_caller(SpecPool *sp, double cpu)
{
    if (sp) sp->a_cpu += cpu;
}
void spec_account_main(SpecPool *sp, double cpu, int mbs)
{
    if (!sp) return;
    sp->m_cpu += cpu;
    sp->m_mbs += (unsigned long)mbs;
}
