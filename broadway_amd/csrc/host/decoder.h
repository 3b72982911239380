/* Host decoder control: one instance per bitstream.  Per NAL unit it does
 * what the reference's h264bsdDecode (h264bsd_decoder.c:162-560) does --
 * NAL extraction, parameter-set storage/activation, access-unit boundary
 * detection, slice header + slice data parse into an MB-record batch, DPB
 * bookkeeping -- but instead of reconstructing on the CPU it hands each
 * complete picture to a reconstruction backend (HIP kernels in the product
 * library; the CPU oracle only in tests). */
#ifndef H264MI_DECODER_H
#define H264MI_DECODER_H

#include <stddef.h>
#include <stdint.h>
#include "syntax.h"
#include "dpb.h"
#include "picbuild.h"

#ifdef __cplusplus
extern "C" {
#endif

/* 1 when H264MI_TEST=1: the test hooks are honoured (capture.c) */
int h264mi_test_hooks(void);

/* Reconstruction backend interface (the device boundary). */
typedef struct H264Backend {
    void *ctx;
    /* (re)allocate frame slots for a w x h (MBs) stream with nslots frames */
    int  (*configure)(void *ctx, int w_mbs, int h_mbs, int nslots);
    /* reconstruct + deblock the picture described by pb into slot cur_slot
     * (may run asynchronously; records are consumed before returning, except
     * from a PicBuild allocated with host_alloc when records_wait is set) */
    int  (*decode)(void *ctx, const PicBuild *pb, int cur_slot);
    /* optional: the decoder then allocates its picture's records and
     * coefficients with host_alloc (pinned), decode uploads straight from
     * them, and the decoder calls this before it writes that PicBuild again
     * (the upload of the last picture has completed on return) */
    int  (*records_wait)(void *ctx);
    /* copy slot as planar I420 (w*16 * h*16 * 3/2 bytes) to host memory;
     * 0 ok, -1 failure, 1 copied but the device flagged an error in a
     * reconstruction since the last read */
    int  (*read)(void *ctx, int slot, uint8_t *dst);
    /* copy slot converted to RGBA (w*16 * h*16 * 4 bytes, DecoderPost.js
     * rgb output; same returns); NULL when the backend has no conversion */
    int  (*read_rgba)(void *ctx, int slot, uint8_t *dst);
    /* optional: host memory for the output frames (pinned by the HIP
     * backend, so each picture's D2H copy runs at DMA speed); NULL: malloc */
    void *(*host_alloc)(void *ctx, size_t bytes);
    void (*host_free)(void *ctx, void *p);
    /* copy one slot into another (error concealment of lost pictures) */
    int  (*copy)(void *ctx, int dst_slot, int src_slot);
    /* optional: neighbour-based concealment on the backend, in place on slot
     * (holding the decoded MBs reconstructed with the loop filter off), of
     * the MBs order[0..n) in that order; decoded = the w*h decoded flags.
     * NULL: the host conceals a copy of the picture (conceal.c) */
    int  (*conceal)(void *ctx, int slot, const int *order, int n, const uint8_t *decoded);
    /* optional: whether conceal serves the configured picture size (NULL: it does) */
    int  (*conceal_ok)(void *ctx);
    /* optional: wait for the reconstructions issued so far (timing split of
     * the output path into device wait and copy) */
    int  (*sync)(void *ctx);
    /* optional: start copying slot to dst (host memory) behind the
     * reconstructions issued so far; a later read of the same slot into the
     * same dst then only waits for that copy (the D2H overlaps host work) */
    int  (*prefetch)(void *ctx, int slot, uint8_t *dst);
    void (*destroy)(void *ctx);
} H264Backend;

enum {
    DEC_RDY = 0, DEC_PIC_RDY = 1, DEC_HDRS_RDY = 2, DEC_ERROR = 3,
    DEC_PARAM_SET_ERROR = 4, DEC_MEMALLOC_ERROR = 5,
};

typedef struct SpecPool SpecPool;

typedef struct PocState {
    int prev_msb, prev_lsb;
    int prev_frame_num_offset, prev_frame_num;
    int prev_mmco5;
} PocState;

typedef struct H264Dec {
    Sps  sps[MAX_SPS];
    Pps  pps[MAX_PPS];
    int  active_sps, active_pps;   /* -1: none; MAX+1: forced re-activation */
    int  pending_activation;
    int  old_sps_id;
    int  no_reorder_app;
    Dpb  dpb;
    PicBuild pb;
    int  pb_ready;
    H264Backend be;
    /* picture state */
    int  pic_started, valid_slice_in_au, skip_redundant;
    SliceHdr sh;                   /* header of the last decoded slice */
    NalHdr   prev_nal;             /* prevNalUnit: NAL of the last valid slice header */
    NalHdr   aub_prev_nal;         /* aub->nuPrev: last slice NAL seen by the boundary check */
    int  cur_pic_id;
    int  cur_slot;
    int  num_concealed;
    PocState poc;
    /* access-unit boundary state (reference storage_t.aub) */
    int  aub_first_call;
    int  aub_prev_frame_num, aub_prev_idr_id, aub_prev_poc_lsb, aub_prev_dpoc_bottom;
    int  aub_prev_dpoc[2];
    /* re-entry on an unfinished buffer (decoder.c:184-206) */
    int  prev_buf_not_finished;
    const uint8_t *prev_buf_ptr;
    uint32_t prev_bytes;
    uint8_t *rbsp;
    size_t   rbsp_cap;
    int  intra_conceal;
    /* host-side output frames (one per slot), filled by backend->read */
    uint8_t *out_frames;
    size_t   frame_bytes;
    int      nslots;
    /* statistics */
    uint64_t pics_decoded, alg_ref_bytes, coded_blocks;
    /* speculative parallel slice parsing (specparse.c); NULL: off */
    SpecPool *spec;
    int spec_help;              /* the caller parses ahead instead of waiting (H264MI_PARSE_HELP) */
    /* end-to-end time split (seconds): host parse, record upload + launch,
     * wait for the device, output copy; pictures output */
    double   t_parse, t_submit, t_wait, t_copy;
    uint64_t n_output;
} H264Dec;

double h264dec_now(void);

int  h264dec_init(H264Dec *d, int no_output_reordering, H264Backend be);
void h264dec_release(H264Dec *d);
/* decode the next NAL unit found at buf[0..len); *read_bytes = consumed */
int  h264dec_decode(H264Dec *d, const uint8_t *buf, uint32_t len, uint32_t pic_id,
                    uint32_t *read_bytes);
/* flush for end of stream */
void h264dec_flush(H264Dec *d);
/* next output picture; returns host pointer to I420 data or NULL */
const uint8_t *h264dec_next_output(H264Dec *d, uint32_t *pic_id, uint32_t *is_idr,
                                   uint32_t *err_mbs);
const uint8_t *h264dec_next_output_rgba(H264Dec *d, uint32_t *pic_id, uint32_t *is_idr, uint32_t *err_mbs,
                                        uint8_t *rgba);
int  h264dec_valid_param_sets(const H264Dec *d);
/* conceal the current picture's missing MBs (conceal.c); returns their
 * number or -1 */
int  h264dec_conceal(H264Dec *d, int is_i);
/* wait until the backend no longer reads d->pb (H264Backend.records_wait) */
void h264dec_pb_writable(H264Dec *d);
/* ConcealMb's neighbour path for the MB at (row, col) of an I420 picture of
 * w x h MBs in host memory, reading the MBs flagged in dec (the host
 * restatement of k_conceal; conceal.c) */
void h264dec_conceal_mb_intra(uint8_t *img, int w, int h, int row, int col, const uint8_t *dec);

/* Annex-B NAL unit location and emulation-prevention removal (decoder.c) */
int  nal_scan(const uint8_t *bs, uint32_t len, uint32_t *init, uint32_t *size, uint32_t *read_bytes, int *emul);
int  nal_unescape(const uint8_t *src, uint32_t size, int emul, uint8_t *dst);

/* speculative parallel slice parsing (specparse.c) */
SpecPool *spec_create(int nthreads);
void spec_destroy(SpecPool *sp);
void spec_drain(SpecPool *sp);
void spec_launch(SpecPool *sp, const H264Dec *d, const Sps *sps, const Pps *pps, const NalHdr *nh,
                 const SliceHdr *sh, const uint8_t *buf, uint32_t first_bytes, uint32_t len);
int  spec_take(SpecPool *sp, H264Dec *d, const uint8_t *buf, uint32_t read_bytes, const SliceHdr *sh,
               const Pps *pps, const int *ref_slot);
void spec_launch_ahead(SpecPool *sp, const H264Dec *d, const uint8_t *buf, uint32_t len);
/* the calling thread runs the queued jobs no worker has started */
void spec_help(SpecPool *sp);
/* H264MI_SPEC_STATS: thread CPU per MB of worker and caller parses */
int  spec_stats_on(const SpecPool *sp);
double spec_thread_cpu(void);
void spec_account_main(SpecPool *sp, double cpu, int mbs);
void spec_account_caller(SpecPool *sp, double cpu);
int  spec_active_for(const SpecPool *sp, const uint8_t *buf);
const Sps *h264dec_active_sps(const H264Dec *d);

#ifdef __cplusplus
}
#endif

#endif
