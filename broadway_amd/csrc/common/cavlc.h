/* CAVLC residual block coding (H.264 §9.2).
 * Decoder side replaces the reference's h264bsdDecodeResidualBlockCavlc
 * (h264bsd_cavlc.c:748-915); the encoder side exists for the synthetic
 * stream generator. */
#ifndef H264MI_CAVLC_H
#define H264MI_CAVLC_H

#include <stdint.h>
#include "bits.h"
#include "tables.h"

#include <string.h>

/* Decode one residual block; coef[0..maxcoef-1] receives levels in scan
 * order (coef[0] is the first coded scan position of the block).  Returns
 * TotalCoeff (>= 0) or -1 on a syntax error. */
int cavlc_decode_block(BitReader *br, int nC, int maxcoef, int16_t *coef);
/* same, also returning the sum of |level| (the host residual range bound);
 * inline: the parser's call sites pass constant maxcoef (16, 15, 4), which
 * the compiler folds into the clear, the range checks and the table choice */
static inline int cavlc_decode_block_sum(BitReader *br, int nC, int maxcoef, int16_t *coef, uint32_t *abs_sum)
{
    int len;
    *abs_sum = 0;
    /* constant sizes: inlined stores instead of a library call per block */
    if (maxcoef == 16) memset(coef, 0, 32);
    else if (maxcoef == 15) memset(coef, 0, 30);
    else memset(coef, 0, sizeof(int16_t) * (size_t)maxcoef);
    int sym = vlc_decode(&gCoeffTokenDec[coeff_token_class(nC)], br_peek(br, 16), &len);
    if (sym < 0) return -1;
    br_skip(br, len);
    int tc = sym >> 2, t1 = sym & 3;
    if (tc == 0) return 0;
    if (tc > maxcoef) return -1;

    int level[16];
    int suffix_len = (tc > 10 && t1 < 3) ? 1 : 0;
    int i = 0;
    if (t1) {                                    /* trailing_ones_sign_flags, one read */
        const uint32_t sg = br_u(br, t1);
        for (; i < t1; i++) level[i] = ((sg >> (t1 - 1 - i)) & 1) ? -1 : 1;
        *abs_sum += (uint32_t)t1;
    }
    for (; i < tc; i++) {
        /* level_prefix (leading zero bits then a one, §9.2.2.1) and
         * level_suffix from one 32-bit window: prefix <= 15, suffix <= 12 */
        const uint32_t w = br_peek(br, 32);
        if ((w >> 16) == 0) return -1;           /* level_prefix > 15 */
        const int prefix = __builtin_clz(w);
        int ssize = suffix_len;
        if (prefix == 14 && suffix_len == 0) ssize = 4;
        if (prefix == 15) ssize = 12;
        int code = prefix << suffix_len;
        if (ssize > 0) code += (int)((w << (prefix + 1)) >> (32 - ssize));
        br_skip(br, prefix + 1 + ssize);
        if (prefix == 15 && suffix_len == 0) code += 15;
        if (i == t1 && t1 < 3) code += 2;
        int lv = (code & 1) ? (-code - 1) >> 1 : (code + 2) >> 1;
        level[i] = lv;
        if (suffix_len == 0) suffix_len = 1;
        int alv = lv < 0 ? -lv : lv;
        *abs_sum += (uint32_t)alv;
        if (alv > (3 << (suffix_len - 1)) && suffix_len < 6) suffix_len++;
    }

    int total_zeros = 0;
    if (tc < maxcoef) {
        const VlcTable *t = (maxcoef == 4) ? &gTotalZerosDcDec[tc - 1] : &gTotalZerosDec[tc - 1];
        total_zeros = vlc_decode(t, br_peek(br, 16), &len);
        if (total_zeros < 0) return -1;
        br_skip(br, len);
        if (tc + total_zeros > maxcoef) return -1;
    }

    int zeros_left = total_zeros;
    int pos = tc + total_zeros - 1;              /* scan index of highest coefficient */
    for (int i = 0; i < tc; i++) {
        coef[pos] = (int16_t)level[i];
        int run = 0;
        if (i < tc - 1 && zeros_left > 0) {
            int k = zeros_left < 7 ? zeros_left : 7;
            run = vlc_decode(&gRunBeforeDec[k - 1], br_peek(br, 16), &len);
            if (run < 0) return -1;
            br_skip(br, len);
            if (run > zeros_left) return -1;
        } else if (i == tc - 1) {
            run = zeros_left;
        }
        zeros_left -= run;
        pos -= 1 + run;
    }
    if (br->err) return -1;
    return tc;
}


/* Encode one residual block (levels in scan order); returns TotalCoeff or -1
 * if a level cannot be represented in Baseline (level_prefix > 15). */
int cavlc_encode_block(BitWriter *bw, int nC, int maxcoef, const int16_t *coef);

#endif
