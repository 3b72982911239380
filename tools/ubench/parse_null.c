/* Host cost of the drop-in decode loop without reconstruction: the product
 * decoder core (h264dec_decode: NAL scan, slice headers, CAVLC / MB layer
 * into records, DPB, speculative slice workers) over a backend whose decode
 * does nothing.  Prints wall and process CPU seconds per picture, so the
 * speculative workers' share of the CPU shows next to the sequential parse.
 *   gcc -O3 -Ibroadway_amd/csrc tools/ubench/parse_null.c <common + host
 *       sources except api.c / capture.c> -lpthread
 *   H264MI_PARSE_THREADS=0|3 ./parse_null in.h264 [passes] */
#include "host/decoder.h"

#include <stdio.h>
#include <stdlib.h>
#include <time.h>

typedef struct { uint8_t *frame; size_t bytes; } NullCtx;

static int n_configure(void *ctx, int w, int h, int nslots)
{
    NullCtx *c = (NullCtx *)ctx;
    free(c->frame);
    c->bytes = (size_t)w * h * 384;
    c->frame = (uint8_t *)calloc(1, c->bytes);
    return c->frame ? 0 : -1;
}
/* PN_COPY=1: the decode copies the picture's records and coefficient blocks
 * into a staging buffer with memcpy (what the HIP backend does into pinned
 * memory), PN_COPY=2: with non-temporal stores -- the host cost of the copy
 * and of the caches it evicts */
#include <immintrin.h>
static uint8_t *g_stage;
static size_t g_stage_cap;
static void copy_nt(void *dst, const void *src, size_t n)
{
    uint8_t *d = (uint8_t *)dst;
    const uint8_t *s = (const uint8_t *)src;
    while (n && ((uintptr_t)d & 31)) { *d++ = *s++; n--; }
    for (; n >= 128; n -= 128, d += 128, s += 128) {
        const __m256i a = _mm256_loadu_si256((const __m256i *)s), b = _mm256_loadu_si256((const __m256i *)(s + 32));
        const __m256i c = _mm256_loadu_si256((const __m256i *)(s + 64)), e = _mm256_loadu_si256((const __m256i *)(s + 96));
        _mm256_stream_si256((__m256i *)d, a); _mm256_stream_si256((__m256i *)(d + 32), b);
        _mm256_stream_si256((__m256i *)(d + 64), c); _mm256_stream_si256((__m256i *)(d + 96), e);
    }
    memcpy(d, s, n);
    _mm_sfence();
}
static int n_decode(void *ctx, const PicBuild *pb, int slot)
{
    static int mode = -1;
    if (mode < 0) mode = getenv("PN_COPY") ? atoi(getenv("PN_COPY")) : 0;
    if (!mode) return 0;
    const size_t rb = (size_t)pb->nmbs * sizeof(MbRec), cb = (size_t)pb->ncoef * 32;
    if (rb + cb > g_stage_cap) { free(g_stage); g_stage_cap = 2 * (rb + cb); g_stage = (uint8_t *)aligned_alloc(64, g_stage_cap); }
    if (mode == 1) { memcpy(g_stage, pb->rec, rb); memcpy(g_stage + rb, pb->coef, cb); }
    else { copy_nt(g_stage, pb->rec, rb); copy_nt(g_stage + rb, pb->coef, cb); }
    return 0;
}
static int n_read(void *ctx, int slot, uint8_t *dst) { return 0; }
static int n_copy(void *ctx, int d, int s) { return 0; }
static void n_destroy(void *ctx) { free(((NullCtx *)ctx)->frame); free(ctx); }

static double now(clockid_t id)
{
    struct timespec t;
    clock_gettime(id, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

int main(int argc, char **argv)
{
    if (argc < 2) { fprintf(stderr, "usage: parse_null in.h264 [passes]\n"); return 2; }
    FILE *f = fopen(argv[1], "rb");
    if (!f) { perror(argv[1]); return 2; }
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t *buf = (uint8_t *)malloc((size_t)n);
    if (fread(buf, 1, (size_t)n, f) != (size_t)n) return 2;
    fclose(f);
    const int passes = argc > 2 ? atoi(argv[2]) : 1;
    long pics = 0;
    double best = 1e30;
    const double w0 = now(CLOCK_MONOTONIC), c0 = now(CLOCK_PROCESS_CPUTIME_ID), m0 = now(CLOCK_THREAD_CPUTIME_ID);
    for (int pass = 0; pass < passes; pass++) {
        const double pc0 = now(CLOCK_PROCESS_CPUTIME_ID);
        const long pics0 = pics;
        H264Backend be = {0};
        be.ctx = calloc(1, sizeof(NullCtx));
        be.configure = n_configure; be.decode = n_decode; be.read = n_read;
        be.copy = n_copy; be.destroy = n_destroy;
        static H264Dec dec;
        h264dec_init(&dec, 0, be);
        const uint8_t *p = buf;
        uint32_t left = (uint32_t)n, id = 0;
        while (left > 0) {
            uint32_t rb = 0;
            const int r = h264dec_decode(&dec, p, left, id, &rb);
            if (r == DEC_PIC_RDY) id++;
            if (r == DEC_PIC_RDY || r == DEC_HDRS_RDY) {
                uint32_t pid, idr, em;
                while (h264dec_next_output(&dec, &pid, &idr, &em)) pics++;
            }
            if (rb > left) rb = left;
            p += rb;
            left -= rb;
        }
        h264dec_flush(&dec);
        {
            uint32_t pid, idr, em;
            while (h264dec_next_output(&dec, &pid, &idr, &em)) pics++;
        }
        h264dec_release(&dec);
        const double t = (now(CLOCK_PROCESS_CPUTIME_ID) - pc0) / (double)(pics - pics0);
        if (t < best) best = t;
    }
    const double w1 = now(CLOCK_MONOTONIC), c1 = now(CLOCK_PROCESS_CPUTIME_ID), m1 = now(CLOCK_THREAD_CPUTIME_ID);
    printf("pictures %ld  wall %.3f ms/picture  cpu %.3f ms/picture (calling thread %.3f; best pass %.3f)\n", pics,
           1e3 * (w1 - w0) / pics, 1e3 * (c1 - c0) / pics, 1e3 * (m1 - m0) / pics, 1e3 * best);
    return 0;
}
