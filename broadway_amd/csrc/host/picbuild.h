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
    uint8_t *decoded;      /* per MB: mbStorage_t.decoded (successfully decoded, not un-marked) */
    int      ndecoded;     /* MBs of completed slices (slice_t.numDecodedMbs) */
    int      nslices;      /* slices started; the current slice's id (slice_t.sliceId) */
    int      last_mb_addr; /* I slices: last MB decoded without error (slice_t.lastMbAddr) */
    int      mb_decode_err;    /* current MB parsed but fails reconstruction (see slicedata.c) */
    int      cur_slot;         /* frame slot of the picture (a failed MB keeps its old samples) */
    int      is_p;         /* any P slice in the picture */
    uint64_t alg_ref_bytes;    /* algorithmic MC footprint bytes */
    uint32_t n_inter, n_intra, n_coded_blocks;
    /* optional allocator of rec / coef (picbuild_init_alloc): the HIP
     * backend's pinned host memory, which it uploads from directly (no staging
     * copy); `pinned` = rec and coef came from it */
    void  *(*halloc)(void *ctx, size_t bytes);
    void   (*hfree)(void *ctx, void *p);
    void    *hctx;
    int      pinned;
} PicBuild;

int  picbuild_init(PicBuild *pb, int w_mbs, int h_mbs);
int  picbuild_init_alloc(PicBuild *pb, int w_mbs, int h_mbs, void *(*halloc)(void *, size_t),
                         void (*hfree)(void *, void *), void *hctx);
void picbuild_free(PicBuild *pb);
void picbuild_reset(PicBuild *pb, int cip);      /* start of a new picture */
void picbuild_reuse(PicBuild *pb, int cip);      /* the next slice into a private PicBuild (slice ids count on) */

/* Parse the slice_data() of one slice (reader positioned after the header).
 * ref_slot[i] = DPB slot of RefPicList0[i] (-1 if absent).  The slice gets
 * the next slice id (1, 2, ... as slice_data.c:120).  Returns 0 on success,
 * -1 on a syntax or semantic error, a missing reference picture or a
 * residual out of range; the caller then un-marks the slice
 * (picbuild_mark_slice_corrupted). */
int parse_slice_data(PicBuild *pb, BitReader *br, const SliceHdr *sh, const Pps *pps,
                     const int *ref_slot);
/* h264bsdMarkSliceCorrupted (slice_data.c:302-358) for the current slice */
void picbuild_mark_slice_corrupted(PicBuild *pb, int first_mb);
/* n coefficient blocks at the end of the pool (NULL on allocation failure) */
int16_t *picbuild_coef_alloc(PicBuild *pb, uint32_t nblk);

#endif
