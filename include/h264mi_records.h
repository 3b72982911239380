/* h264mi_records.h -- packed per-macroblock reconstruction record: the
 * host->device data contract of the C-ABI (include/h264mi.h).
 *
 * One MbRec per macroblock, 96 bytes, produced by the host parser (CAVLC +
 * MB-layer parse, MV prediction, intra-mode derivation) and consumed by the
 * HIP reconstruction kernels and by the CPU oracle.  It is the device-side
 * restatement of what the reference keeps in mbStorage_t / macroblockLayer_t
 * (h264bsd_macroblock_layer.h:141-188) after h264bsdDecodeMacroblockLayer and
 * the MV/mode derivation have run:
 *   - mv[16]        <- mbStorage_t.mv[16] (z-scan order, quarter-pel)
 *   - ref[4]        <- mbStorage_t.refAddr[4] as a DPB *slot* index
 *   - i4[8]         <- mbStorage_t.intra4x4PredMode[16] (4 bits each)
 *   - cbits/coef    <- residual_t.level/totalCoeff: only coded blocks travel,
 *                      each as 16 int16 levels in scan order
 *   - qp            <- mbStorage_t.qpY (0 for I_PCM, macroblock_layer.c:1003)
 *   - dbf/offA/offB <- mbStorage_t.disableDeblockingFilterIdc/filterOffsetA/B
 *   - slice         <- mbStorage_t.sliceId
 *
 * Coefficient blocks (int16[16] each) referenced by a record are stored
 * contiguously starting at block index `coef`, one block per set bit of
 * `cbits` in increasing bit order:
 *   bits  0..15  luma 4x4 blocks (z-scan); for I16x16 these are AC blocks
 *                (scan position 0 unused); a bit is set iff TotalCoeff > 0
 *   bits 16..19  Cb AC 4x4 blocks, bits 20..23 Cr AC (scan pos 0 unused)
 *   bit  24      I16x16 luma DC (16 levels, scan order)
 *   bit  25      Cb DC (levels 0..3), bit 26 Cr DC (levels 0..3)
 * I_PCM: cbits = 0 and 12 blocks at `coef` hold the 384 raw samples
 * (256 luma raster, 64 Cb, 64 Cr) as bytes.
 */
#ifndef H264MI_RECORDS_H
#define H264MI_RECORDS_H

#include <stdint.h>

enum {
    MBT_INTER = 0,      /* P_L0_* and P_8x8 (any partitioning) */
    MBT_SKIP  = 1,      /* P_Skip */
    MBT_I4x4  = 2,
    MBT_I16   = 3,
    MBT_IPCM  = 4,
};

/* avail bits: intra-prediction availability of neighbour MBs (slice +
 * constrained_intra_pred applied, h264bsdIsNeighbourAvailable +
 * intra_prediction.c:643-654) */
enum {
    AV_A = 1, AV_B = 2, AV_C = 4, AV_D = 8,
    /* deblocking: filterLeftMbEdgeFlag / filterTopMbEdgeFlag
     * (deblocking.c:288-319) */
    DB_LEFT = 16, DB_TOP = 32, DB_INNER = 64,
};

/* dbf bits */
enum {
    /* the MB counts as intra in the bS derivation although its samples are
     * an inter copy: a concealed MB is set to I_4x4 "to perform filtering"
     * (h264bsd_conceal.c:300-308) while P concealment copies the co-located
     * MB of a reference picture (:310-332) */
    DBF_INTRA = 1,
};

typedef struct MbRec {
    uint8_t  type;      /* MBT_* */
    uint8_t  qp;        /* QPY (I_PCM: 0) */
    uint8_t  qpc;       /* QPc = QpChroma[clip3(0,51,QPY+chroma_qp_index_offset)] */
    uint8_t  avail;     /* AV_* | DB_* */
    uint8_t  pred;      /* I16: mode (bits 0-1); chroma mode bits 4-5 */
    uint8_t  dbf;       /* DBF_* */
    int8_t   offA;      /* FilterOffsetA = slice_alpha_c0_offset_div2 << 1 */
    int8_t   offB;      /* FilterOffsetB */
    uint32_t cbits;     /* coded-block mask, see above */
    uint32_t coef;      /* first coefficient block index */
    uint8_t  i4[8];     /* I_4x4: Intra4x4PredMode, 4 bits per block, z-scan.
                           Inter (MBT_INTER / MBT_SKIP) in frame-pipelined batches with
                           whole-row waits: four uint16 (little endian), per 8x8
                           partition the last MB row of its reference slot that a 128-B
                           line read by its motion compensation touches (h264mi_capture
                           fills it) */
    uint8_t  ref[4];    /* DPB slot per 8x8 partition (inter only) */
    int16_t  mv[16][2]; /* per 4x4 block, z-scan, quarter-pel (x, y) */
    uint16_t slice;     /* slice id within the picture */
    uint16_t refidx;    /* RefPicList0 index per 8x8 partition, 4 bits each (inter only).
                           Informational: bS compares the pictures (ref slots), not the
                           indices (deblocking.c:348, 402); two indices can name one picture */
} MbRec;

#ifdef __cplusplus
static_assert(sizeof(MbRec) == 96, "MbRec must stay 96 bytes");
#else
_Static_assert(sizeof(MbRec) == 96, "MbRec must stay 96 bytes");
#endif

/* Per-picture descriptor, one per picture in a launch batch */
typedef struct PicDesc {
    uint32_t rec_base;      /* first MbRec index of this picture, relative to the launch's record
                               pointer (any offset: the pictures of a launch need not be
                               contiguous; k_prep outputs are indexed by batch position) */
    uint32_t frame_base;    /* index of this stream's slot 0 in the frame pool */
    uint32_t cur_slot;      /* slot being reconstructed */
    uint32_t flags;         /* bit2 (PD_INTRA_HEAVY): more than half the picture's MBs are intra
                               (a scheduling hint: intra MC waves first); bit3 (PD_NO_DEBLOCK): no
                               MB of the picture filters any edge (no record has DB_INNER: every
                               slice disable_deblocking_filter_idc 1) -- the MC output is final and
                               is stored without the deblocking row chain.  Set only when true: a
                               picture with filtering flagged so would come out unfiltered (the
                               dependency checker flags that, CHK_NODB).  Bits 0, 1 unused */
    uint32_t coef_base;     /* added to MbRec.coef (records are picture-relative) */
    uint32_t rsv[3];
} PicDesc;

enum { PD_INTRA_HEAVY = 4, PD_NO_DEBLOCK = 8 };

/* Device frame-slot layout (the engine's HBM frame pool): I420, luma rows
 * w*16 bytes apart, then the Cb and Cr planes with their rows padded to a
 * multiple of 128 bytes (the L2 line), so that no 128-B line holds bytes of
 * two chroma rows -- the frame-pipelined launches hand reference samples
 * from one picture to the next at (MB row, MB column) granularity and read a
 * line only once every byte of it is final (recon_kernels.hip dep_wait).
 * 1080p: 1024-byte chroma rows for 960 samples; 720p and 2160p: no padding.
 * What leaves the device (h264mi_engine_read, the H264SwDec output) is packed
 * I420, w*16 * h*16 * 3/2 bytes. */
#define H264MI_CPITCH(w_mbs) ((((w_mbs) * 8) + 127) & ~127)
#define H264MI_SLOT_BYTES(w_mbs, h_mbs) \
    ((size_t)(w_mbs) * 16 * (h_mbs) * 16 + 2 * (size_t)H264MI_CPITCH(w_mbs) * (h_mbs) * 8)

#endif
