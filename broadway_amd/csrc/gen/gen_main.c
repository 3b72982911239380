/* h264gen CLI: write a seeded synthetic Baseline stream to a file.
 *   h264gen -c CONFIG -s SEED [-n FRAMES] [-w W_MBS -h H_MBS] [-o out.h264]
 *           [key=value ...]   (any GenParams field, e.g. slices=4 cip=1) */
#include "h264gen.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define FIELD(name) {#name, offsetof(GenParams, name)}
static const struct { const char *n; size_t off; } kFields[] = {
    FIELD(w_mbs), FIELD(h_mbs), FIELD(crop_right), FIELD(crop_bottom), FIELD(nframes),
    FIELD(gop), FIELD(slices), FIELD(pm_skip), FIELD(pm_16x16), FIELD(pm_16x8),
    FIELD(pm_8x16), FIELD(pm_8x8), FIELD(pm_intra), FIELD(p8x8_ref0_pct), FIELD(im_i4),
    FIELD(im_i16), FIELD(im_pcm), FIELD(i4_rem_pct), FIELD(qp_min), FIELD(qp_max),
    FIELD(qp_delta), FIELD(dbf_idc1_pct), FIELD(dbf_idc2_pct), FIELD(dbf_off),
    FIELD(num_ref_frames), FIELD(cip), FIELD(chroma_qp_offset), FIELD(poc_type),
    FIELD(coef_pct), FIELD(level_tail_pct), FIELD(mv_jitter), FIELD(offpic_pct),
    FIELD(log2_max_frame_num)};

int main(int argc, char **argv)
{
    int config = 2;
    unsigned long long seed = 1;
    const char *out = "out.h264";
    GenParams p;
    int have = 0;
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "-c") && i + 1 < argc) config = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-s") && i + 1 < argc) seed = strtoull(argv[++i], 0, 10);
        else if (!strcmp(argv[i], "-o") && i + 1 < argc) out = argv[++i];
    }
    if (h264gen_preset(&p, config, seed)) { fprintf(stderr, "bad config\n"); return 2; }
    have = 1;
    for (int i = 1; i < argc; i++) {
        char *eq = strchr(argv[i], '=');
        if (!eq) continue;
        size_t kl = (size_t)(eq - argv[i]);
        int found = 0;
        for (size_t f = 0; f < sizeof(kFields) / sizeof(kFields[0]); f++)
            if (strlen(kFields[f].n) == kl && !strncmp(kFields[f].n, argv[i], kl)) {
                *(int *)((char *)&p + kFields[f].off) = atoi(eq + 1);
                found = 1;
            }
        if (!found) { fprintf(stderr, "unknown field %s\n", argv[i]); return 2; }
    }
    (void)have;
    uint8_t *buf; size_t len;
    if (h264gen_generate(&p, &buf, &len)) { fprintf(stderr, "generation failed\n"); return 1; }
    FILE *f = fopen(out, "wb");
    if (!f) { perror(out); return 1; }
    fwrite(buf, 1, len, f);
    fclose(f);
    h264gen_free(buf);
    return 0;
}
