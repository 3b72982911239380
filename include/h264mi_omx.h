/* h264mi OpenMAX DL surface -- the omxVCM4P10_* primitives the reference
 * decoder calls in its -DH264DEC_OMXDL configuration ("OMX-DL
 * names"), with the reference prototypes of
 * Decoder/omxdl/reference/vc/api/omxVC.h (line cited per function), argument
 * checks and results.  Every call runs its computation on the GPU (one small
 * launch on the calling thread's own HIP stream, synchronous): these are
 * drop-in names for code written against OpenMAX DL; the decoder's own path
 * is the fused k_prep / k_wgpp kernels (include/h264mi.h).
 *
 * The two CAVLC parsers (omxVCM4P10_DecodeCoeffsToPairCAVLC /
 * DecodeChromaDcCoeffsToPairCAVLC) run on the host (csrc/host/omx_cavlc.c):
 * bitstream parsing stays on the CPU in this design.  Not provided: the
 * encoder-side primitives (motion estimation, SAD/SATD, forward transforms)
 * and MPEG-4 part 2.
 *
 * Argument errors: every check of the reference is made before any output
 * is written (the reference's deblocking filters check bS / thresholds per
 * line while filtering, so on an error they may have filtered some lines). */
#ifndef H264MI_OMX_H
#define H264MI_OMX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#ifndef _OMXTYPES_H_            /* omxtypes.h:40-208 */
typedef uint8_t  OMX_U8;
typedef int8_t   OMX_S8;
typedef uint16_t OMX_U16;
typedef int16_t  OMX_S16;
typedef uint32_t OMX_U32;
typedef int32_t  OMX_S32;
typedef int      OMX_INT;
typedef int      OMXResult;
typedef struct { OMX_INT width; OMX_INT height; } OMXSize;
#endif

enum {                           /* omxtypes.h:51-67 */
    H264MI_OMX_Sts_NoErr = 0,
    H264MI_OMX_Sts_Err = -2,
    H264MI_OMX_Sts_BadArgErr = -5,
};

enum {                           /* omxVC.h:516-525 availability bits */
    H264MI_OMX_VC_UPPER = 1, H264MI_OMX_VC_LEFT = 2,
    H264MI_OMX_VC_UPPER_LEFT = 32, H264MI_OMX_VC_UPPER_RIGHT = 64,
};

/* omxVC.h:3101 -- CAVLC ChromaDCLevel (2x2) -> packed position-coefficient
 * pairs at *ppPosCoefbuf (advanced past them; untouched for an empty block) */
OMXResult omxVCM4P10_DecodeChromaDcCoeffsToPairCAVLC(const OMX_U8 **ppBitStream, OMX_S32 *pOffset, OMX_U8 *pNumCoeff,
                                                     OMX_U8 **ppPosCoefbuf);
/* omxVC.h:3160 -- CAVLC 4x4 block (sMaxNumCoeff 15 or 16; sVLCSelect = nC >= 0) */
OMXResult omxVCM4P10_DecodeCoeffsToPairCAVLC(const OMX_U8 **ppBitStream, OMX_S32 *pOffset, OMX_U8 *pNumCoeff,
                                             OMX_U8 **ppPosCoefbuf, OMX_INT sVLCSelect, OMX_INT sMaxNumCoeff);
/* diagnostic: 1 if this thread's last CAVLC call above returned
 * H264MI_OMX_Sts_Err for a bit pattern the reference decodes by reading its
 * tables out of range (TotalCoeff > sMaxNumCoeff, TotalCoeff + total_zeros >
 * sMaxNumCoeff, run_before > zerosLeft: undefined behaviour there), else 0 */
int h264mi_omx_cavlc_divergent(void);
/* omxVC.h:2426 -- predMode OMXVCM4P10Intra4x4PredMode 0..8 (VERT, HOR, DC,
 * DIAG_DL, DIAG_DR, VR, HD, VL, HU) */
OMXResult omxVCM4P10_PredictIntra_4x4(const OMX_U8 *pSrcLeft, const OMX_U8 *pSrcAbove, const OMX_U8 *pSrcAboveLeft,
                                      OMX_U8 *pDst, OMX_INT leftStep, OMX_INT dstStep, int predMode,
                                      OMX_S32 availability);
/* omxVC.h:2494 -- predMode 0..3 (VERT, HOR, DC, PLANE) */
OMXResult omxVCM4P10_PredictIntra_16x16(const OMX_U8 *pSrcLeft, const OMX_U8 *pSrcAbove, const OMX_U8 *pSrcAboveLeft,
                                        OMX_U8 *pDst, OMX_INT leftStep, OMX_INT dstStep, int predMode,
                                        OMX_S32 availability);
/* omxVC.h:2559 -- predMode 0..3 (DC, HOR, VERT, PLANE) */
OMXResult omxVCM4P10_PredictIntraChroma_8x8(const OMX_U8 *pSrcLeft, const OMX_U8 *pSrcAbove,
                                            const OMX_U8 *pSrcAboveLeft, OMX_U8 *pDst, OMX_INT leftStep,
                                            OMX_INT dstStep, int predMode, OMX_S32 availability);
/* omxVC.h:2612 -- quarter-sample luma; reads pSrc[-2 .. roi + 3] both ways */
OMXResult omxVCM4P10_InterpolateLuma(const OMX_U8 *pSrc, OMX_S32 srcStep, OMX_U8 *pDst, OMX_S32 dstStep, OMX_S32 dx,
                                     OMX_S32 dy, OMXSize roi);
/* omxVC.h:2664 -- eighth-sample chroma; reads pSrc[0 .. roi] both ways */
OMXResult omxVCM4P10_InterpolateChroma(const OMX_U8 *pSrc, OMX_S32 srcStep, OMX_U8 *pDst, OMX_S32 dstStep, OMX_S32 dx,
                                       OMX_S32 dy, OMXSize roi);
/* omxVC.h:2726, 2788, 2853, 2919 -- the four edges of one MB (plane) */
OMXResult omxVCM4P10_FilterDeblockingLuma_VerEdge_I(OMX_U8 *pSrcDst, OMX_S32 srcdstStep, const OMX_U8 *pAlpha,
                                                    const OMX_U8 *pBeta, const OMX_U8 *pThresholds,
                                                    const OMX_U8 *pBS);
OMXResult omxVCM4P10_FilterDeblockingLuma_HorEdge_I(OMX_U8 *pSrcDst, OMX_S32 srcdstStep, const OMX_U8 *pAlpha,
                                                    const OMX_U8 *pBeta, const OMX_U8 *pThresholds,
                                                    const OMX_U8 *pBS);
OMXResult omxVCM4P10_FilterDeblockingChroma_VerEdge_I(OMX_U8 *pSrcDst, OMX_S32 srcdstStep, const OMX_U8 *pAlpha,
                                                      const OMX_U8 *pBeta, const OMX_U8 *pThresholds,
                                                      const OMX_U8 *pBS);
OMXResult omxVCM4P10_FilterDeblockingChroma_HorEdge_I(OMX_U8 *pSrcDst, OMX_S32 srcdstStep, const OMX_U8 *pAlpha,
                                                      const OMX_U8 *pBeta, const OMX_U8 *pThresholds,
                                                      const OMX_U8 *pBS);
/* omxVC.h:3200 -- unpacks one 4x4 pair block (advances *ppSrc) */
OMXResult omxVCM4P10_TransformDequantLumaDCFromPair(const OMX_U8 **ppSrc, OMX_S16 *pDst, OMX_INT QP);
/* omxVC.h:3237 -- unpacks one 2x2 pair block (advances *ppSrc) */
OMXResult omxVCM4P10_TransformDequantChromaDCFromPair(const OMX_U8 **ppSrc, OMX_S16 *pDst, OMX_INT QP);
/* omxVC.h:3287 */
OMXResult omxVCM4P10_DequantTransformResidualFromPairAndAdd(const OMX_U8 **ppSrc, const OMX_U8 *pPred,
                                                            const OMX_S16 *pDC, OMX_U8 *pDst, OMX_INT predStep,
                                                            OMX_INT dstStep, OMX_INT QP, OMX_INT AC);

#ifdef __cplusplus
}
#endif
#endif
