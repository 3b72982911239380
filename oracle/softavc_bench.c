/* ORACLE HARNESS -- TEST INFRASTRUCTURE ONLY (build container).
 *
 * Drives the REFERENCE decoder's H264SwDec* API the way the SoftAVC OMX
 * component does (Decoder/SoftAVC.cpp:289-400): one input buffer per NAL unit
 * (start code included), picId incremented per input buffer,
 * intraConcealmentMethod = 1 (SoftAVC.cpp:335), the buffer re-fed while the
 * decoder returns *_BUFF_NOT_EMPTY, NextPicture(…, 0) drained after every
 * buffer and NextPicture(…, 1) at end of stream (drainAllOutputBuffers).
 * DecTestBench.c hardcodes intraConcealmentMethod = 0 (:211); this harness is
 * how the SoftAVC setting gets pinned (oracle/Makefile.ref builds it from the
 * reference sources into oracle/_ref/refdec_softavc; nothing is shipped).
 *
 *   refdec_softavc [-Mmethod] in.h264 out.yuv
 * prints "PIC <picId> <isIdr> <nbrOfErrMBs>" per output picture and
 * "SIZE <w> <h>"; writes the MB-aligned I420 frames to out.yuv. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "H264SwDecApi.h"

static long next_start(const unsigned char *b, long n, long from)
{
    for (long i = from; i + 3 < n; i++)
        if (b[i] == 0 && b[i + 1] == 0 && b[i + 2] == 1) return i > 0 && b[i - 1] == 0 ? i - 1 : i;
    return n;
}

int main(int argc, char **argv)
{
    unsigned method = 1;
    const char *in = NULL, *out = NULL;
    for (int i = 1; i < argc; i++) {
        if (!strncmp(argv[i], "-M", 2)) method = (unsigned)atoi(argv[i] + 2);
        else if (!in) in = argv[i];
        else out = argv[i];
    }
    if (!in || !out) { fprintf(stderr, "usage: refdec_softavc [-Mmethod] in.h264 out.yuv\n"); return 2; }
    FILE *f = fopen(in, "rb");
    if (!f) return 2;
    fseek(f, 0, SEEK_END);
    const long n = ftell(f);
    rewind(f);
    unsigned char *buf = malloc((size_t)n + 16);
    if (fread(buf, 1, (size_t)n, f) != (size_t)n) return 2;
    fclose(f);
    FILE *fo = fopen(out, "wb");
    H264SwDecInst inst;
    if (H264SwDecInit(&inst, 0) != H264SWDEC_OK) return 3;
    u32 pic_size = 0, pic_id = 0;
    H264SwDecPicture pic;
    H264SwDecInfo info;
    long pos = next_start(buf, n, 0);
    while (pos < n) {
        const long end = next_start(buf, n, pos + 3);
        H264SwDecInput ip;
        H264SwDecOutput op;
        memset(&ip, 0, sizeof(ip));
        ip.pStream = buf + pos;
        ip.dataLen = (u32)(end - pos);
        ip.picId = ++pic_id;
        ip.intraConcealmentMethod = method;
        while (ip.dataLen > 0) {
            const H264SwDecRet ret = H264SwDecDecode(inst, &ip, &op);
            if (ret == H264SWDEC_HDRS_RDY_BUFF_NOT_EMPTY || ret == H264SWDEC_PIC_RDY_BUFF_NOT_EMPTY) {
                ip.dataLen -= (u32)(op.pStrmCurrPos - ip.pStream);
                ip.pStream = op.pStrmCurrPos;
                if (ret == H264SWDEC_HDRS_RDY_BUFF_NOT_EMPTY && H264SwDecGetInfo(inst, &info) == H264SWDEC_OK) {
                    pic_size = info.picWidth * info.picHeight * 3 / 2;
                    printf("SIZE %u %u\n", info.picWidth, info.picHeight);
                }
            } else {
                ip.dataLen = 0;
            }
        }
        while (pic_size && H264SwDecNextPicture(inst, &pic, 0) == H264SWDEC_PIC_RDY) {
            printf("PIC %u %u %u\n", pic.picId, pic.isIdrPicture, pic.nbrOfErrMBs);
            fwrite(pic.pOutputPicture, 1, pic_size, fo);
        }
        pos = end;
    }
    while (pic_size && H264SwDecNextPicture(inst, &pic, 1) == H264SWDEC_PIC_RDY) {
        printf("PIC %u %u %u\n", pic.picId, pic.isIdrPicture, pic.nbrOfErrMBs);
        fwrite(pic.pOutputPicture, 1, pic_size, fo);
    }
    H264SwDecRelease(inst);
    fclose(fo);
    free(buf);
    return 0;
}
