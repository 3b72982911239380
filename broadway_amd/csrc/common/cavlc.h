/* CAVLC residual block coding (H.264 §9.2).
 * Decoder side replaces the reference's h264bsdDecodeResidualBlockCavlc
 * (h264bsd_cavlc.c:748-915); the encoder side exists for the synthetic
 * stream generator. */
#ifndef H264MI_CAVLC_H
#define H264MI_CAVLC_H

#include <stdint.h>
#include "bits.h"

/* Decode one residual block; coef[0..maxcoef-1] receives levels in scan
 * order (coef[0] is the first coded scan position of the block).  Returns
 * TotalCoeff (>= 0) or -1 on a syntax error. */
int cavlc_decode_block(BitReader *br, int nC, int maxcoef, int16_t *coef);
/* same, also returning the sum of |level| (the host residual range bound) */
int cavlc_decode_block_sum(BitReader *br, int nC, int maxcoef, int16_t *coef, uint32_t *abs_sum);

/* Encode one residual block (levels in scan order); returns TotalCoeff or -1
 * if a level cannot be represented in Baseline (level_prefix > 15). */
int cavlc_encode_block(BitWriter *bw, int nC, int maxcoef, const int16_t *coef);

#endif
