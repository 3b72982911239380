/* Host parse cost: CPU seconds (process CPU clock, best of 5) to turn an
 * Annex-B stream into MB records with the product parser (h264mi_capture_stream,
 * csrc/host; H264MI_PARSE_THREADS sets the speculative slice workers).
 *   gcc -O3 -Ibroadway_amd/csrc tools/ubench/parse_cpu.c <host + common sources> -lpthread */
#include <stdio.h>
#include <stdlib.h>
#include <time.h>
void *h264mi_capture_stream(const void *buf, size_t n, int no_reorder);
void h264mi_capture_free(void *c);
int main(int argc, char **argv) {
    FILE *f = fopen(argv[1], "rb"); fseek(f, 0, SEEK_END); long n = ftell(f); fseek(f, 0, SEEK_SET);
    unsigned char *b = malloc(n); if (fread(b, 1, n, f) != (size_t)n) return 1; fclose(f);
    double best = 1e9;
    for (int r = 0; r < 5; r++) {
        struct timespec t0, t1; clock_gettime(CLOCK_PROCESS_CPUTIME_ID, &t0);
        void *h = h264mi_capture_stream(b, n, 0);
        clock_gettime(CLOCK_PROCESS_CPUTIME_ID, &t1);
        double s = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
        if (s < best) best = s;
        h264mi_capture_free(h);
    }
    printf("best cpu %.3f s\n", best);
    return 0;
}
