/* h264mi_dec -- DecTestBench-style command line decoder over the product
 * C-ABI (libh264mi.so: host parser + HIP reconstruction), the end-to-end
 * path of SURVEY.md §8d: host CAVLC parse + H2D of the MB records + kernels +
 * D2H of every output picture.  Call protocol of the reference testbench
 * (Decoder/src/DecTestBench.c:230-410): decode, drain NextPicture after each
 * PIC_RDY, flush at end of stream.
 *   h264mi_dec [-R] [-Oout.yuv|-Onone] [-rN] [-T] [-SN] [-Acpus] in.h264 [in2.h264 ...]
 * -rN decodes the stream N times (one instance each; HIP start-up is paid
 * once, before the timed loop); -T prints the wall time of the decode loops.
 * Several inputs: one thread per input, each with its own instances
 * (TestBenchMultipleInstance.c's N instances, concurrently); -SN lets them
 * share one N-lane engine per GPU (h264mi_set_share); -O applies to the
 * first input.  -Acpus (a cpulist: "0-7,16,18") pins the process and every
 * thread it starts (parse workers included) to those host cores before
 * anything else runs -- one GPU's decoder processes on cores of that GPU's
 * NUMA node (bench.py end_to_end); the GPU is H264MI_DEVICE (default 0).
 * -G (start gate): after its HIP warm-up the process prints "ready" and
 * waits for one byte on stdin before its timed loop, so that a driver can
 * start several processes' loops together; -T then also prints the loop's
 * CLOCK_MONOTONIC start / end (comparable across the host's processes) and
 * the host CPU of the loop by thread: the decoding threads, the
 * speculative-parse workers, and every other thread of the process (HIP
 * runtime threads) from /proc/self/task. */
#define _GNU_SOURCE
#include "../../../include/h264mi.h"

#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <dirent.h>
#include <unistd.h>
#include <sys/resource.h>

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* "0-3,8,10-11" -> cpu set; 0 on success */
static int parse_cpulist(const char *s, cpu_set_t *set)
{
    CPU_ZERO(set);
    int n = 0;
    while (*s) {
        char *e;
        long a = strtol(s, &e, 10), b = a;
        if (e == s || a < 0 || a >= CPU_SETSIZE) return -1;
        if (*e == '-') {
            s = e + 1;
            b = strtol(s, &e, 10);
            if (e == s || b < a || b >= CPU_SETSIZE) return -1;
        }
        for (long c = a; c <= b; c++) { CPU_SET((int)c, set); n++; }
        if (*e == ',') e++;
        else if (*e) return -1;
        s = e;
    }
    return n ? 0 : -1;
}

/* CPU seconds (user + system) of every live thread of this process but
 * `skip` (whose CPU is counted elsewhere), from /proc/self/task/<tid>/stat;
 * *n: how many */
static double other_threads_cpu(pid_t skip, int *n)
{
    DIR *d = opendir("/proc/self/task");
    if (!d) return -1.0;
    const double tick = 1.0 / (double)sysconf(_SC_CLK_TCK);
    double sum = 0.0;
    int k = 0;
    struct dirent *de;
    while ((de = readdir(d)) != NULL) {
        if (de->d_name[0] < '0' || de->d_name[0] > '9') continue;
        const pid_t tid = (pid_t)atoi(de->d_name);
        if (tid == skip) continue;
        char path[64], buf[1024];
        snprintf(path, sizeof(path), "/proc/self/task/%d/stat", (int)tid);
        FILE *f = fopen(path, "r");
        if (!f) continue;
        const size_t m = fread(buf, 1, sizeof(buf) - 1, f);
        fclose(f);
        buf[m] = 0;
        const char *p = strrchr(buf, ')');      /* comm may hold spaces */
        if (!p) continue;
        unsigned long ut = 0, st = 0;
        /* fields after comm: state(3) ... utime(14) stime(15) */
        if (sscanf(p + 2, "%*c %*d %*d %*d %*d %*d %*u %*u %*u %*u %*u %lu %lu", &ut, &st) == 2) {
            sum += (double)(ut + st) * tick;
            k++;
        }
    }
    closedir(d);
    if (n) *n = k;
    return sum;
}

static double g_t[4];   /* parse, submit, wait, copy (H264SwDecGetTiming), summed over instances */
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;

static int decode_once(const uint8_t *stream, uint32_t len, uint8_t *work, int no_reorder, FILE *fo, int *errs)
{
    H264SwDecInst inst;
    if (H264SwDecInit(&inst, (u32)no_reorder) != H264SWDEC_OK) return -1;
    memcpy(work, stream, len);          /* the decoder edits its input in place */
    H264SwDecInput in;
    H264SwDecOutput out;
    H264SwDecPicture pic;
    H264SwDecInfo info;
    memset(&in, 0, sizeof(in));
    in.pStream = work;
    in.dataLen = len;
    size_t size = 0;
    int pics = 0;
    u32 pic_id = 0;
    while (in.dataLen > 0) {
        in.picId = pic_id;
        H264SwDecRet r = H264SwDecDecode(inst, &in, &out);
        if (r == H264SWDEC_HDRS_RDY_BUFF_NOT_EMPTY) {
            if (H264SwDecGetInfo(inst, &info) != H264SWDEC_OK) break;
            size = (size_t)info.picWidth * info.picHeight * 3 / 2;
        } else if (r == H264SWDEC_PIC_RDY || r == H264SWDEC_PIC_RDY_BUFF_NOT_EMPTY) {
            pic_id++;
            while (H264SwDecNextPicture(inst, &pic, 0) == H264SWDEC_PIC_RDY) {
                pics++;
                *errs += (int)pic.nbrOfErrMBs;
                if (fo) fwrite(pic.pOutputPicture, 1, size, fo);
            }
        } else if (r < 0) {
            (*errs)++;
        }
        u32 used = (u32)(out.pStrmCurrPos - in.pStream);
        if (used == 0 && r < 0) break;
        in.dataLen -= used;
        in.pStream = out.pStrmCurrPos;
    }
    while (H264SwDecNextPicture(inst, &pic, 1) == H264SWDEC_PIC_RDY) {
        pics++;
        *errs += (int)pic.nbrOfErrMBs;
        if (fo) fwrite(pic.pOutputPicture, 1, size, fo);
    }
    double t[4];
    if (H264SwDecGetTiming(inst, &t[0], &t[1], &t[2], &t[3], NULL) == H264SWDEC_OK) {
        pthread_mutex_lock(&g_mu);
        for (int i = 0; i < 4; i++) g_t[i] += t[i];
        pthread_mutex_unlock(&g_mu);
    }
    H264SwDecRelease(inst);
    return pics;
}

typedef struct Job {
    uint8_t *buf, *work;
    uint32_t len;
    int reps, no_reorder, pics, errs, fail;
    FILE *fo;
} Job;

static double g_job_cpu;   /* CPU of the decoding threads themselves (the rest: parse workers, HIP runtime) */

static void *run_job(void *arg)
{
    Job *j = (Job *)arg;
    struct timespec c0, c1;
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &c0);
    for (int k = 0; k < j->reps; k++) {
        const int n = decode_once(j->buf, j->len, j->work, j->no_reorder, k == 0 ? j->fo : NULL, &j->errs);
        if (n < 0) { j->fail = 1; break; }
        j->pics += n;
    }
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &c1);
    pthread_mutex_lock(&g_mu);
    g_job_cpu += (double)(c1.tv_sec - c0.tv_sec) + 1e-9 * (double)(c1.tv_nsec - c0.tv_nsec);
    pthread_mutex_unlock(&g_mu);
    return NULL;
}

static int load(const char *path, Job *j)
{
    FILE *f = fopen(path, "rb");
    if (!f) { perror(path); return -1; }
    fseek(f, 0, SEEK_END);
    long len = ftell(f);
    rewind(f);
    j->buf = (uint8_t *)malloc((size_t)len);
    j->work = (uint8_t *)malloc((size_t)len);
    if (!j->buf || !j->work || fread(j->buf, 1, (size_t)len, f) != (size_t)len) { fclose(f); return -1; }
    fclose(f);
    j->len = (uint32_t)len;
    return 0;
}

int main(int argc, char **argv)
{
    const char *out = NULL;
    const char *ins[256];
    int nin = 0, no_reorder = 0, timing = 0, reps = 1, share = 0, gate = 0;
    const char *cpus = NULL;
    for (int i = 1; i < argc; i++) {
        if (!strncmp(argv[i], "-O", 2)) out = argv[i] + 2;
        else if (!strcmp(argv[i], "-R")) no_reorder = 1;
        else if (!strcmp(argv[i], "-T")) timing = 1;
        else if (!strncmp(argv[i], "-r", 2)) reps = atoi(argv[i] + 2);
        else if (!strncmp(argv[i], "-S", 2)) share = atoi(argv[i] + 2);
        else if (!strncmp(argv[i], "-A", 2)) cpus = argv[i] + 2;
        else if (!strcmp(argv[i], "-G")) gate = 1;
        else if (nin < 256) ins[nin++] = argv[i];
    }
    if (!nin || reps < 1) {
        fprintf(stderr, "usage: h264mi_dec [-R] [-Oout] [-rN] [-T] [-SN] [-Acpus] [-G] in.h264 [in2.h264 ...]\n");
        return 2;
    }
    if (cpus) {
        /* before any thread or GPU context exists: everything started later inherits it */
        cpu_set_t set;
        if (parse_cpulist(cpus, &set) || sched_setaffinity(0, sizeof(set), &set)) {
            fprintf(stderr, "bad -A cpu list '%s'\n", cpus);
            return 2;
        }
    }
    Job *jobs = (Job *)calloc((size_t)nin, sizeof(Job));
    for (int i = 0; i < nin; i++) {
        if (load(ins[i], &jobs[i])) return 2;
        jobs[i].reps = reps;
        jobs[i].no_reorder = no_reorder;
    }
    FILE *fo = (out && strcmp(out, "none")) ? fopen(out, "wb") : NULL;
    jobs[0].fo = fo;
    if (share && h264mi_set_share(share)) { fprintf(stderr, "bad -S\n"); return 2; }
    /* HIP start-up (device, code objects) outside the timed loop */
    {
        H264SwDecInst warm;
        if (H264SwDecInit(&warm, 0) != H264SWDEC_OK) { fprintf(stderr, "DECODER INITIALIZATION FAILED\n"); return 1; }
        H264SwDecRelease(warm);
    }
    if (gate) {
        /* start gate: every process of the run warmed up, released together */
        printf("ready\n");
        fflush(stdout);
        if (getchar() == EOF) { fprintf(stderr, "start gate closed\n"); return 2; }
    }
    int pics = 0, errs = 0;
    struct rusage ru0, ru1;
    double w0 = 0.0, w1 = 0.0;
    h264mi_host_thread_stats(&w0, NULL);
    const pid_t main_tid = (pid_t)getpid();
    int nother0 = 0, nother1 = 0;
    const double oth0 = other_threads_cpu(main_tid, &nother0);
    struct timespec mc0, mc1;
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &mc0);
    getrusage(RUSAGE_SELF, &ru0);
    const double t0 = now_s();
    if (nin == 1) {
        run_job(&jobs[0]);
    } else {
        pthread_t *th = (pthread_t *)calloc((size_t)nin, sizeof(pthread_t));
        for (int i = 0; i < nin; i++) pthread_create(&th[i], NULL, run_job, &jobs[i]);
        for (int i = 0; i < nin; i++) pthread_join(th[i], NULL);
        free(th);
    }
    const double t1 = now_s();
    getrusage(RUSAGE_SELF, &ru1);
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &mc1);
    const double oth1 = other_threads_cpu(main_tid, &nother1);
    h264mi_host_thread_stats(&w1, NULL);
    if (fo) fclose(fo);
    for (int i = 0; i < nin; i++) {
        if (jobs[i].fail) { fprintf(stderr, "DECODER INITIALIZATION FAILED\n"); return 1; }
        pics += jobs[i].pics;
        errs += jobs[i].errs;
    }
    printf("pictures %d errors %d\n", pics, errs);
    if (timing) {
        printf("decode_seconds %.6f fps %.2f\n", t1 - t0, pics / (t1 - t0));
        printf("t_parse %.6f\nt_submit %.6f\nt_wait %.6f\nt_copy %.6f\n", g_t[0], g_t[1], g_t[2], g_t[3]);
        /* host CPU time of the whole process over the timed loop (all threads) */
        const double cpu = (ru1.ru_utime.tv_sec - ru0.ru_utime.tv_sec) + 1e-6 * (ru1.ru_utime.tv_usec - ru0.ru_utime.tv_usec) +
                           (ru1.ru_stime.tv_sec - ru0.ru_stime.tv_sec) + 1e-6 * (ru1.ru_stime.tv_usec - ru0.ru_stime.tv_usec);
        printf("cpu_seconds %.6f\n", cpu);
        printf("cpu_decode_threads_seconds %.6f\n", g_job_cpu);
        /* by thread: the spec workers (exited ones, library counter), the
         * main thread when it is not a decoding thread, the threads alive
         * at the end of the loop other than main (HIP runtime threads, live
         * spec workers of shared instances) -- their CPU over the loop */
        const double main_cpu = (double)(mc1.tv_sec - mc0.tv_sec) + 1e-9 * (double)(mc1.tv_nsec - mc0.tv_nsec);
        printf("cpu_spec_workers_seconds %.6f\n", w1 - w0);
        printf("cpu_main_thread_seconds %.6f\n", main_cpu);
        if (oth0 >= 0 && oth1 >= 0)
            printf("cpu_other_live_threads_seconds %.6f\nother_live_threads %d\n", oth1 - oth0, nother1);
        printf("t_start_mono %.6f\nt_end_mono %.6f\n", t0, t1);
        printf("cpu_sys_seconds %.6f\n", (ru1.ru_stime.tv_sec - ru0.ru_stime.tv_sec) + 1e-6 * (ru1.ru_stime.tv_usec - ru0.ru_stime.tv_usec));
        unsigned long long nb = 0, np = 0;
        h264mi_share_stats(0, &nb, &np);
        if (share) printf("share_batches %llu\nshare_pictures %llu\n", nb, np);
        cpu_set_t now;
        if (!sched_getaffinity(0, sizeof(now), &now)) printf("cpus_allowed %d\n", CPU_COUNT(&now));
    }
    for (int i = 0; i < nin; i++) { free(jobs[i].buf); free(jobs[i].work); }
    free(jobs);
    return errs ? 1 : 0;
}
