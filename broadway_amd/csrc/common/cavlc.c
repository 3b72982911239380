/* CAVLC residual block coding, H.264 §9.2 (see cavlc.h). */
#include "cavlc.h"
#include "tables.h"

#include <string.h>

int cavlc_decode_block(BitReader *br, int nC, int maxcoef, int16_t *coef)
{
    uint32_t sum;
    return cavlc_decode_block_sum(br, nC, maxcoef, coef, &sum);
}

static void put_code(BitWriter *bw, VlcCode c) { bw_put(bw, c.code, c.len); }

int cavlc_encode_block(BitWriter *bw, int nC, int maxcoef, const int16_t *coef)
{
    int lev[16], posn[16];
    int tc = 0;
    for (int i = maxcoef - 1; i >= 0; i--)       /* highest frequency first */
        if (coef[i]) { lev[tc] = coef[i]; posn[tc] = i; tc++; }
    int t1 = 0;
    while (t1 < tc && t1 < 3 && (lev[t1] == 1 || lev[t1] == -1)) t1++;

    put_code(bw, gCoeffTokenEnc[coeff_token_class(nC)][tc][t1]);
    if (tc == 0) return 0;

    int suffix_len = (tc > 10 && t1 < 3) ? 1 : 0;
    for (int i = 0; i < tc; i++) {
        if (i < t1) { bw_put(bw, lev[i] < 0, 1); continue; }
        int lv = lev[i];
        int code = lv > 0 ? 2 * lv - 2 : -2 * lv - 1;
        if (i == t1 && t1 < 3) code -= 2;
        int prefix, suffix = 0, ssize = 0;
        if (suffix_len == 0) {
            if (code < 14) { prefix = code; }
            else if (code < 30) { prefix = 14; suffix = code - 14; ssize = 4; }
            else { prefix = 15; suffix = code - 30; ssize = 12; }
        } else {
            if (code < (15 << suffix_len)) {
                prefix = code >> suffix_len;
                suffix = code & ((1 << suffix_len) - 1);
                ssize = suffix_len;
            } else {
                prefix = 15; suffix = code - (15 << suffix_len); ssize = 12;
            }
        }
        if (ssize == 12 && suffix >= 4096) return -1;
        bw_put(bw, 0, prefix);
        bw_put(bw, 1, 1);
        if (ssize) bw_put(bw, (uint32_t)suffix, ssize);
        if (suffix_len == 0) suffix_len = 1;
        int alv = lv < 0 ? -lv : lv;
        if (alv > (3 << (suffix_len - 1)) && suffix_len < 6) suffix_len++;
    }

    int total_zeros = posn[0] + 1 - tc;
    if (tc < maxcoef) {
        if (maxcoef == 4) put_code(bw, gTotalZerosDcEnc[tc - 1][total_zeros]);
        else put_code(bw, gTotalZerosEnc[tc - 1][total_zeros]);
    }
    int zeros_left = total_zeros;
    for (int i = 0; i < tc - 1 && zeros_left > 0; i++) {
        int run = posn[i] - posn[i + 1] - 1;
        int k = zeros_left < 7 ? zeros_left : 7;
        put_code(bw, gRunBeforeEnc[k - 1][run]);
        zeros_left -= run;
    }
    return tc;
}
