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
/* One block through the BitReader (any position, end of buffer included):
 * the path for blocks that start within CAVLC_SLACK bytes of the end. */
static inline int cavlc_block_checked_(BitReader *br, int nC, int maxcoef, int16_t *coef, uint32_t *abs_sum)
{
    int len;
    *abs_sum = 0;
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
    if (t1) {
        const uint32_t sg = br_u(br, t1);
        for (; i < t1; i++) level[i] = ((sg >> (t1 - 1 - i)) & 1) ? -1 : 1;
        *abs_sum += (uint32_t)t1;
    }
    for (; i < tc; i++) {
        const uint32_t w = br_peek(br, 32);
        if ((w >> 16) == 0) return -1;
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
    int pos = tc + total_zeros - 1;
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

/* the longest residual block is 641 bits (coeff_token 16 + 3 sign bits + 15
 * levels of 28 bits + ... + total_zeros 9 + 14 run_before of 11 bits); a
 * block starting CAVLC_SLACK bytes or more before the end cannot read past it
 * even with the 8-byte window below */
#define CAVLC_SLACK 96

/* 64 stream bits at bit position pos, MSB first, the low (pos & 7) of them
 * zero (8 readable bytes at pos / 8) */
static inline uint64_t cavlc_load64_(const uint8_t *buf, size_t pos)
{
    uint64_t v;
    memcpy(&v, buf + (pos >> 3), 8);
    return __builtin_bswap64(v) << (pos & 7);
}

/* same, also returning the sum of |level| (the host residual range bound);
 * inline: the parser's call sites pass constant maxcoef (16, 15, 4), which
 * the compiler folds into the clear, the range checks and the table choice.
 * Away from the end of the buffer the block is read through a 64-bit
 * register cache refilled with unchecked 8-byte loads (a field costs a table
 * load and a shift on the dependency chain, no per-field bounds checks),
 * packed one-load VLC tables and a branch-free suffixLength / run_before;
 * the stream position on every return, error returns included, is the one
 * the checked path leaves. */
static inline int cavlc_decode_block_sum(BitReader *br, int nC, int maxcoef, int16_t *coef, uint32_t *abs_sum)
{
    if (__builtin_expect((br->pos >> 3) + CAVLC_SLACK > br->size, 0))
        return cavlc_block_checked_(br, nC, maxcoef, coef, abs_sum);
    const uint8_t *const buf = br->buf;
    size_t pos = br->pos;                        /* position of the cache's first bit */
    uint64_t c = cavlc_load64_(buf, pos);
    int avail = 64 - (int)(pos & 7);             /* valid bits in c (>= 32 before every field) */
#define CV_NEED(n) do { if (avail < (n)) { c = cavlc_load64_(buf, pos); avail = 64 - (int)(pos & 7); } } while (0)
#define CV_SKIP(n) do { const int n_ = (n); c <<= n_; avail -= n_; pos += (size_t)n_; } while (0)
    /* nC -1 .. 16 -> coeff_token table (Table 9-5 columns) */
    static const uint8_t kClass[18] = {4, 0, 0, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 3, 3, 3, 3, 3};
    const uint32_t e = vlc_pk(&gCoeffTokenPk[kClass[nC + 1]], (uint32_t)(c >> 48));
    if (maxcoef == 16) memset(coef, 0, 32);
    else if (maxcoef == 15) memset(coef, 0, 30);
    else memset(coef, 0, sizeof(int16_t) * (size_t)maxcoef);
    if (!e) return -1;
    CV_SKIP((int)(e & 31));
    const int tc = (int)(e >> 7), t1 = (int)(e >> 5) & 3;
    if (tc == 0) { br->pos = pos; *abs_sum = 0; return 0; }
    if (tc > maxcoef) { br->pos = pos; return -1; }

    int level[16];
    uint32_t sum = (uint32_t)t1;
    {                                            /* trailing_ones_sign_flags: up to 3 */
        level[0] = 1 - 2 * (int)(c >> 63);
        level[1] = 1 - 2 * (int)((c >> 62) & 1);
        level[2] = 1 - 2 * (int)((c >> 61) & 1);
        CV_SKIP(t1);
    }
    int i = t1;
    int suffix_len = (tc > 10 && t1 < 3) ? 1 : 0;
    for (; i < tc; i++) {
        CV_NEED(32);
        const uint32_t w = (uint32_t)(c >> 32);
        if (__builtin_expect((w >> 16) == 0, 0)) { br->pos = pos; return -1; }   /* level_prefix > 15 */
        const int prefix = __builtin_clz(w);
        int code, used;
        if (__builtin_expect(prefix < 14, 1)) {
            /* suffix of suffix_len bits (0: none) */
            code = (prefix << suffix_len) + (int)(((uint64_t)(w << prefix << 1)) >> (32 - suffix_len));
            used = prefix + 1 + suffix_len;
        } else {
            const int ssize = prefix == 15 ? 12 : (suffix_len ? suffix_len : 4);
            code = (prefix << suffix_len) + (int)((w << (prefix + 1)) >> (32 - ssize));
            if (prefix == 15 && suffix_len == 0) code += 15;
            used = prefix + 1 + ssize;
        }
        CV_SKIP(used);
        code += (i == t1 && t1 < 3) ? 2 : 0;
        const int mag = (code + 2) >> 1;
        const int neg = code & 1;
        level[i] = neg ? -mag : mag;
        sum += (uint32_t)mag;
        suffix_len += suffix_len == 0;
        suffix_len += (mag > (3 << (suffix_len - 1))) & (suffix_len < 6);
    }

    int total_zeros = 0;
    if (tc < maxcoef) {
        CV_NEED(16);
        const VlcPk *t = (maxcoef == 4) ? &gTotalZerosDcPk[tc - 1] : &gTotalZerosPk[tc - 1];
        const uint32_t z = vlc_pk(t, (uint32_t)(c >> 48));
        if (!z) { br->pos = pos; return -1; }
        CV_SKIP((int)(z & 31));
        total_zeros = (int)(z >> 5);
        if (tc + total_zeros > maxcoef) { br->pos = pos; return -1; }
    }

    /* levels from the highest scan position down, run_before between them
     * (Table 9-10): zerosLeft 1..6 codes are at most 3 bits (kRunSmall, row
     * 0 = zerosLeft 0: no code); above 6, 1..3-bit 'run = 7 - code' or
     * leading zeros then a one, 'run = zeros + 4' -- no branch per field */
    static const uint8_t kRunSmall[7][8] = {
        {0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00},
        {0x11, 0x11, 0x11, 0x11, 0x01, 0x01, 0x01, 0x01},   /* 1: 1 | 0 */
        {0x22, 0x22, 0x12, 0x12, 0x01, 0x01, 0x01, 0x01},   /* 2: 1 | 01 | 00 */
        {0x32, 0x32, 0x22, 0x22, 0x12, 0x12, 0x02, 0x02},   /* 3: 11 10 01 00 */
        {0x43, 0x33, 0x22, 0x22, 0x12, 0x12, 0x02, 0x02},   /* 4: 11 10 01 001 000 */
        {0x53, 0x43, 0x33, 0x23, 0x12, 0x12, 0x02, 0x02},   /* 5: 11 10 011 010 001 000 */
        {0x13, 0x23, 0x43, 0x33, 0x63, 0x53, 0x02, 0x02},   /* 6: 11 000 001 011 010 101 100 */
    };
    int zeros_left = total_zeros;
    int at = tc + total_zeros - 1;
    for (i = 0; i < tc - 1; i++) {
        coef[at] = (int16_t)level[i];
        CV_NEED(16);
        const uint32_t w = (uint32_t)(c >> 32);
        const uint32_t top3 = w >> 29;
        const int lz = __builtin_clz(w | 1);
        const int small = kRunSmall[zeros_left < 7 ? zeros_left : 0][top3];
        const int big = zeros_left > 6;
        const int run = big ? (top3 ? 7 - (int)top3 : lz + 4) : small >> 4;
        const int len = big ? (top3 ? 3 : lz + 1) : small & 15;
        if (__builtin_expect(run > zeros_left || (big & (lz > 10)), 0)) {
            br->pos = pos + (run > zeros_left && !(big & (lz > 10)) ? len : 0);
            return -1;
        }
        CV_SKIP(len);
        zeros_left -= run;
        at -= 1 + run;
    }
#undef CV_NEED
#undef CV_SKIP
    coef[at] = (int16_t)level[tc - 1];           /* the rest of the zeros lie below it */
    br->pos = pos;
    *abs_sum = sum;
    return tc;
}


/* Encode one residual block (levels in scan order); returns TotalCoeff or -1
 * if a level cannot be represented in Baseline (level_prefix > 15). */
int cavlc_encode_block(BitWriter *bw, int nC, int maxcoef, const int16_t *coef);

#endif
