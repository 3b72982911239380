/* Per-picture MB-record batch built by the host parser (the caller side of
 * the reconstruction hot path).  One PicBuild holds every MbRec of one
 * picture plus its compacted coefficient blocks; it is handed to a backend
 * (HIP kernels in the product, the CPU oracle in tests) once the picture is
 * complete.  Mirrors what the reference accumulates in storage_t.mb[] while
 * h264bsdDecodeSliceData runs (slice_data.c:85-235). */
#ifndef H264MI_PICBUILD_H
#define H264MI_PICBUILD_H

#include <stdint.h>
#include "../common/mbrec.h"
#include "../common/mbctx.h"
#include "syntax.h"

typedef struct PicBuild {
    int w, h, nmbs;
    MbRec   *rec;          /* nmbs */
    int16_t *coef;         /* coefficient blocks, 16 x int16 each */
    uint32_t ncoef, cap;   /* in blocks */
    PicCtx   pc;           /* neighbour state (MbInfo per MB) */
    int      ndecoded;
    int      nslices;
    int      is_p;         /* any P slice in the picture */
    uint64_t alg_ref_bytes;    /* algorithmic MC footprint bytes */
    uint32_t n_inter, n_intra, n_coded_blocks;
} PicBuild;

int  picbuild_init(PicBuild *pb, int w_mbs, int h_mbs);
void picbuild_free(PicBuild *pb);
void picbuild_reset(PicBuild *pb, int cip);      /* start of a new picture */

/* Parse the slice_data() of one slice (reader positioned after the header).
 * ref_slot[i] = DPB slot of RefPicList0[i] (-1 if absent).
 * Returns 0 on success, -1 on a syntax/semantic error. */
int parse_slice_data(PicBuild *pb, BitReader *br, const SliceHdr *sh, const Pps *pps,
                     const int *ref_slot, uint16_t slice_tag);

#endif
