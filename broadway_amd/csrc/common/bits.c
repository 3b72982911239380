/* BitWriter (generator side) -- see bits.h */
#include "bits.h"

#include <stdlib.h>

void bw_init(BitWriter *bw)
{
    bw->cap = 4096;
    bw->buf = (uint8_t *)malloc(bw->cap);
    bw->nbytes = 0;
    bw->acc = 0;
    bw->nacc = 0;
}

void bw_free(BitWriter *bw)
{
    free(bw->buf);
    bw->buf = NULL;
}

static void bw_byte(BitWriter *bw, uint8_t b)
{
    if (bw->nbytes == bw->cap) {
        bw->cap *= 2;
        bw->buf = (uint8_t *)realloc(bw->buf, bw->cap);
    }
    bw->buf[bw->nbytes++] = b;
}

void bw_put(BitWriter *bw, uint32_t val, int n)
{
    for (int i = n - 1; i >= 0; i--) {
        bw->acc = (bw->acc << 1) | ((val >> i) & 1u);
        if (++bw->nacc == 8) {
            bw_byte(bw, (uint8_t)bw->acc);
            bw->acc = 0;
            bw->nacc = 0;
        }
    }
}

void bw_ue(BitWriter *bw, uint32_t v)
{
    uint64_t x = (uint64_t)v + 1;
    int len = 63 - __builtin_clzll(x);      /* number of leading zeros */
    bw_put(bw, 0, len);
    if (len >= 32) {
        bw_put(bw, (uint32_t)(x >> 32), len + 1 - 32);
        bw_put(bw, (uint32_t)x, 32);
    } else {
        bw_put(bw, (uint32_t)x, len + 1);
    }
}

void bw_se(BitWriter *bw, int32_t v)
{
    uint32_t k = v > 0 ? (uint32_t)(2 * v - 1) : (uint32_t)(-2 * (int64_t)v);
    bw_ue(bw, k);
}

void bw_te(BitWriter *bw, uint32_t v, uint32_t cmax)
{
    if (cmax > 1) bw_ue(bw, v);
    else bw_put(bw, !v, 1);
}

void bw_trailing(BitWriter *bw)
{
    bw_put(bw, 1, 1);
    while (bw->nacc) bw_put(bw, 0, 1);
}

int bw_aligned(const BitWriter *bw) { return bw->nacc == 0; }

size_t bw_bits(const BitWriter *bw) { return bw->nbytes * 8 + (size_t)bw->nacc; }
