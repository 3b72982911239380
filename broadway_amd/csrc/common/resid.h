/* Residual range check of one macroblock, on the host at parse time.
 *
 * The reference rejects a macroblock whose inverse-transformed residual
 * leaves [-512, 511] in any 4x4 block (h264bsdProcessBlock,
 * h264bsd_transform.c:181-185, 196-197, 221-225, called from ProcessResidual,
 * h264bsd_macroblock_layer.c:1366-1421); the slice is then corrupted
 * (slice_data.c:186-193 -> decoder.c:462-467) and its MBs concealed.  The
 * GPU computes the residual later, so the host decides this here, where the
 * slice-level consequences (stop the slice, un-mark its MBs) are applied.
 * A magnitude bound settles almost every block without transforming it. */
#ifndef H264MI_RESID_H
#define H264MI_RESID_H

#include <stdint.h>

/* blk: the parser's coefficient blocks in scan order -- [0..15] luma (I16:
 * position 0 unused), [16..23] Cb/Cr AC (position 0 unused), [24] I16 luma
 * DC, [25]/[26] Cb/Cr DC (4 levels); only blocks whose cbits bit is set are
 * read.  bsum[b]: sum of |level| of block b (from the CAVLC decode).
 * Returns 1 if every processed block stays in range. */
int mb_residual_in_range(const int16_t *const *blk, const uint32_t *bsum, uint32_t cbits, int is_i16,
                         int qp, int qpc);

#endif
