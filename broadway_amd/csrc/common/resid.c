/* Residual range check -- see resid.h. */
#include "resid.h"
#include "tables.h"

#include <string.h>

static int pos_class(int r)
{
    const int x = r & 3, y = r >> 2;
    return (!(x & 1) && !(y & 1)) ? 0 : ((x & 1) && (y & 1)) ? 1 : 2;
}

/* full 4x4 inverse transform of dequantized d (raster); 1 if every output
 * (x + 32) >> 6 is in [-512, 511].  The reference's DC-only and first-row
 * shortcuts (transform.c:188-226) compute the same values. */
static int idct_in_range(const int32_t *d)
{
    int32_t t[16];
    for (int i = 0; i < 4; i++) {
        const int32_t *r = d + 4 * i;
        const int32_t a = r[0] + r[2], b = r[0] - r[2];
        const int32_t c = (r[1] >> 1) - r[3], e = r[1] + (r[3] >> 1);
        t[4 * i] = a + e; t[4 * i + 1] = b + c; t[4 * i + 2] = b - c; t[4 * i + 3] = a - e;
    }
    for (int j = 0; j < 4; j++) {
        const int32_t a = t[j] + t[8 + j], b = t[j] - t[8 + j];
        const int32_t c = (t[4 + j] >> 1) - t[12 + j], e = t[4 + j] + (t[12 + j] >> 1);
        const int32_t o[4] = {a + e, b + c, b - c, a - e};
        for (int k = 0; k < 4; k++)
            if ((uint32_t)(((o[k] + 32) >> 6) + 512) > 1023u) return 0;
    }
    return 1;
}

/* one block: levels lv (scan order from `start`) whose |level| sum is sum,
 * DC value dc already dequantized (start == 1).  |output| <= sum |d| + 5
 * before the final rounding, so a sum below 32730 cannot leave the range. */
static int block_in_range(const int16_t *lv, uint32_t sum, int start, int32_t dc, int qp)
{
    const int q6 = qp / 6, m6 = qp % 6;
    if (!lv) sum = 0;
    const uint64_t bound = (uint64_t)sum * (uint64_t)(kLevelScale[m6][1] << q6) + (uint64_t)(dc < 0 ? -(int64_t)dc : dc);
    if (bound < 32000) return 1;
    int32_t d[16];
    memset(d, 0, sizeof(d));
    if (lv)
        for (int s = start; s < 16; s++) {
            const int r = kZigzag4x4[s];
            d[r] = (int32_t)lv[s] * (kLevelScale[m6][pos_class(r)] << q6);
        }
    if (start) d[0] = dc;
    return idct_in_range(d);
}

int mb_residual_in_range(const int16_t *const *blk, const uint32_t *bsum, uint32_t cbits, int is_i16,
                         int qp, int qpc)
{
    /* whole-MB bound first: every block's DC and AC magnitudes are at most
     * its component's level sum times that QP's largest scale (DC transforms
     * are sums of +-levels with the smaller position-0 scale), luma at qp,
     * chroma at qpc */
    {
        uint32_t tl = 0, tc = 0;
        for (uint32_t m = cbits & 0x100FFFFu; m; m &= m - 1) tl += bsum[__builtin_ctz(m)];
        for (uint32_t m = cbits & 0x6FF0000u; m; m &= m - 1) tc += bsum[__builtin_ctz(m)];
        const uint64_t bound = (uint64_t)tl * (uint64_t)(kLevelScale[qp % 6][1] << (qp / 6)) +
                               (uint64_t)tc * (uint64_t)(kLevelScale[qpc % 6][1] << (qpc / 6));
        if (bound < 32000) return 1;
    }
    /* luma: h264bsdProcessLumaDc (transform.c:252-335) for I16, then one
     * ProcessBlock per block that has a DC or coded AC levels */
    int32_t dcy[16];
    memset(dcy, 0, sizeof(dcy));
    if (is_i16 && (cbits & (1u << 24))) {
        int32_t m[16], t[16];
        for (int s = 0; s < 16; s++) m[kZigzag4x4[s]] = blk[24][s];
        for (int i = 0; i < 4; i++) {
            const int32_t *q = m + 4 * i;
            t[4 * i] = q[0] + q[1] + q[2] + q[3];
            t[4 * i + 1] = q[0] + q[1] - q[2] - q[3];
            t[4 * i + 2] = q[0] - q[1] - q[2] + q[3];
            t[4 * i + 3] = q[0] - q[1] + q[2] - q[3];
        }
        const int v = kLevelScale[qp % 6][0], q6 = qp / 6;
        for (int j = 0; j < 4; j++) {
            const int32_t a = t[j], b = t[4 + j], c = t[8 + j], e = t[12 + j];
            const int32_t f[4] = {a + b + c + e, a + b - c - e, a - b - c + e, a - b + c - e};
            for (int k = 0; k < 4; k++) {
                const int32_t x = f[k] * v;
                dcy[4 * k + j] = q6 >= 2 ? x << (q6 - 2) : ((x << q6) + 2) >> 2;
            }
        }
    }
    for (int b = 0; b < 16; b++) {
        const int16_t *lv = (cbits & (1u << b)) ? blk[b] : NULL;
        if (is_i16) {
            const int32_t dc = dcy[kBlkY[b] * 4 + kBlkX[b]];
            if ((lv || dc) && !block_in_range(lv, bsum[b], 1, dc, qp)) return 0;
        } else if (lv && !block_in_range(lv, bsum[b], 0, 0, qp)) {
            return 0;
        }
    }
    /* chroma: h264bsdProcessChromaDc (transform.c:356-398), then ProcessBlock
     * at QPc for every block with a DC or coded AC levels */
    const int v = kLevelScale[qpc % 6][0], q6 = qpc / 6;
    for (int comp = 0; comp < 2; comp++) {
        int32_t f[4] = {0, 0, 0, 0};
        if (cbits & (3u << 25)) {
            const int16_t *x = (cbits & (1u << (25 + comp))) ? blk[25 + comp] : NULL;
            const int32_t c0 = x ? x[0] : 0, c1 = x ? x[1] : 0, c2 = x ? x[2] : 0, c3 = x ? x[3] : 0;
            f[0] = c0 + c1 + c2 + c3; f[1] = c0 - c1 + c2 - c3;
            f[2] = c0 + c1 - c2 - c3; f[3] = c0 - c1 - c2 + c3;
            for (int k = 0; k < 4; k++) f[k] = ((f[k] * v) << q6) >> 1;
        }
        for (int b = 0; b < 4; b++) {
            const int bit = 16 + comp * 4 + b;
            const int16_t *lv = (cbits & (1u << bit)) ? blk[bit] : NULL;
            if ((lv || f[b]) && !block_in_range(lv, bsum[bit], 1, f[b], qpc)) return 0;
        }
    }
    return 1;
}
