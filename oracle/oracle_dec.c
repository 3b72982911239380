/* ORACLE -- TEST INFRASTRUCTURE ONLY.
 * CLI: decode an Annex-B file with the product host parser + the CPU oracle
 * reconstruction, mirroring the reference testbench loop
 * (Decoder/src/DecTestBench.c:230-410: decode, drain NextPicture after every
 * PIC_RDY, flush at end of stream).  Writes raw I420 (MB-aligned, no crop).
 *   oracle_dec [-R] [-Oout.yuv|-Onone] [-T] in.h264
 * -T prints wall time of the decode loop (CPU baseline). */
#include "recon_cpu.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

int main(int argc, char **argv)
{
    const char *out = NULL, *in = NULL;
    int no_reorder = 0, timing = 0;
    for (int i = 1; i < argc; i++) {
        if (!strncmp(argv[i], "-O", 2)) out = argv[i] + 2;
        else if (!strcmp(argv[i], "-R")) no_reorder = 1;
        else if (!strcmp(argv[i], "-T")) timing = 1;
        else in = argv[i];
    }
    if (!in) { fprintf(stderr, "usage: oracle_dec [-R] [-Oout] [-T] in.h264\n"); return 2; }
    FILE *f = fopen(in, "rb");
    if (!f) { perror(in); return 2; }
    fseek(f, 0, SEEK_END);
    long len = ftell(f);
    rewind(f);
    uint8_t *buf = (uint8_t *)malloc((size_t)len);
    if (fread(buf, 1, (size_t)len, f) != (size_t)len) { fclose(f); return 2; }
    fclose(f);
    FILE *fo = (out && strcmp(out, "none")) ? fopen(out, "wb") : NULL;

    static H264Dec dec;
    h264dec_init(&dec, no_reorder, oracle_backend_create());
    const uint8_t *p = buf;
    uint32_t left = (uint32_t)len;
    int pics = 0, errs = 0;
    double t0 = now_s();
    uint32_t pic_id = 0;
    while (left > 0) {
        uint32_t rb = 0;
        int r = h264dec_decode(&dec, p, left, pic_id, &rb);
        if (r == DEC_PIC_RDY) pic_id++;
        if (r == DEC_ERROR || r == DEC_PARAM_SET_ERROR) { errs++; if (getenv("ORACLE_DEBUG")) fprintf(stderr, "nal at %ld: ret %d\n", (long)(p - buf), r); }
        if (r == DEC_PIC_RDY || r == DEC_HDRS_RDY) {
            const uint8_t *pic;
            uint32_t id, idr, em;
            while ((pic = h264dec_next_output(&dec, &id, &idr, &em)) != NULL) {
                pics++;
                errs += (int)em;
                if (fo) fwrite(pic, 1, dec.frame_bytes, fo);
            }
        }
        if (rb > left) rb = left;
        p += rb;
        left -= rb;
    }
    h264dec_flush(&dec);
    {
        const uint8_t *pic;
        uint32_t id, idr, em;
        while ((pic = h264dec_next_output(&dec, &id, &idr, &em)) != NULL) {
            pics++;
            errs += (int)em;
            if (fo) fwrite(pic, 1, dec.frame_bytes, fo);
        }
    }
    double t1 = now_s();
    if (fo) fclose(fo);
    printf("pictures %d errors %d\n", pics, errs);
    if (timing) printf("decode_seconds %.6f fps %.2f\n", t1 - t0, pics / (t1 - t0));
    h264dec_release(&dec);
    free(buf);
    return errs ? 1 : 0;
}
