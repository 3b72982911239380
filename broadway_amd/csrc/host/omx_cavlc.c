/* OpenMAX DL CAVLC parsers on the host: omxVCM4P10_DecodeCoeffsToPairCAVLC
 * and omxVCM4P10_DecodeChromaDcCoeffsToPairCAVLC (prototypes omxVC.h:3101,
 * 3160; behaviour armVCM4P10_DecodeCoeffsToPair.c:77-282), the two OMX-DL
 * calls of the reference's -DH264DEC_OMXDL build that parse bits
 * (h264bsd_macroblock_layer.c:535-1308).  They decode with the product's own
 * CAVLC tables (common/tables.c) and emit the reference's packed
 * position-coefficient pairs, which omxVCM4P10_TransformDequant*FromPair /
 * DequantTransformResidualFromPairAndAdd (hip/omx.hip) consume:
 *
 *   pairs in reverse scan order (highest-frequency coefficient first), each
 *   {flags, level low byte[, level high byte]}: flags bits 0..3 = raster
 *   position (4x4: inverse zig-zag of the scan index; chroma DC: the index),
 *   0x10 = level outside [-128, 127] (third byte follows), 0x20 = last pair.
 *
 * The bit reader reads the 5 bytes at the current position per field, as the
 * reference's armGetBits / armUnPackVLC32 do (armCOMM_Bitstream.c), so no
 * call reads further past the end of a buffer than the reference would.
 *
 * Error results (OMX_Sts_Err, -2) follow the reference: the stream position
 * stays at the start of the field that failed to decode (earlier fields
 * consumed), *pNumCoeff holds TotalCoeff once coeff_token has decoded, and
 * the pair buffer is untouched.  Three bit patterns the reference decodes
 * into out-of-range table reads (undefined behaviour there) are OMX_Sts_Err
 * here, at the field that exposes them: TotalCoeff > sMaxNumCoeff (15-coeff
 * blocks; after coeff_token), TotalCoeff + total_zeros > sMaxNumCoeff (after
 * total_zeros) and run_before > zerosLeft (after that run_before). */
#include <stddef.h>
#include <stdint.h>

#include "../../../include/h264mi_omx.h"
#include "../common/tables.h"

#define OMX_STS_ERR H264MI_OMX_Sts_Err

/* set per call: 1 when the result is OMX_Sts_Err for one of the three
 * patterns the reference reads out of range (h264mi_omx_cavlc_divergent) */
static __thread int t_divergent;

int h264mi_omx_cavlc_divergent(void) { return t_divergent; }

typedef struct {
    const uint8_t *p;
    int off;            /* bit 0..7 within *p */
} OmxBits;

/* the 32 bits at the position (5-byte window, MSB first) */
static inline uint32_t ob_peek32(const OmxBits *b)
{
    const uint8_t *s = b->p;
    uint32_t v = ((uint32_t)s[0] << 24) | ((uint32_t)s[1] << 16) | ((uint32_t)s[2] << 8) | s[3];
    return b->off ? (v << b->off) | (s[4] >> (8 - b->off)) : v;
}

static inline void ob_skip(OmxBits *b, int n)
{
    const int o = b->off + n;
    b->p += o >> 3;
    b->off = o & 7;
}

static inline uint32_t ob_get(OmxBits *b, int n)
{
    const uint32_t v = ob_peek32(b) >> (32 - n);
    ob_skip(b, n);
    return v;
}

static inline int ob_vlc(OmxBits *b, const VlcTable *t)
{
    int len;
    const int s = vlc_decode(t, ob_peek32(b) >> 16, &len);
    if (s >= 0) ob_skip(b, len);
    return s;
}

/* raster position of 4x4 scan index k (frame zig-zag, H.264 Table 8-12) */
static const uint8_t kScan4x4[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};

/* one block: cls = coeff_token table (0..3 by nC, 4 = chroma DC), maxc 4, 15
 * or 16.  On return the caller's stream position is updated to b. */
static OMXResult decode_pairs(OmxBits *b, OMX_U8 *pNumCoeff, OMX_U8 **ppPosCoefbuf, int cls, int maxc)
{
    h264_tables_init();
    const int tok = ob_vlc(b, &gCoeffTokenDec[cls]);
    if (tok < 0) return OMX_STS_ERR;
    const int tc = tok >> 2, t1 = tok & 3;
    *pNumCoeff = (OMX_U8)tc;
    if (tc == 0) return H264MI_OMX_Sts_NoErr;
    if (tc > maxc) { t_divergent = 1; return OMX_STS_ERR; }

    /* levels, index 0 = highest scan position (the order they are coded in) */
    int level[16];
    for (int i = 0; i < t1; i++) level[i] = ob_get(b, 1) ? -1 : 1;
    int suffix_len = (tc > 10 && t1 < 3) ? 1 : 0;
    for (int i = t1; i < tc; i++) {
        const uint32_t w = ob_peek32(b) >> 16;
        if (w == 0) return OMX_STS_ERR;          /* level_prefix > 15: not Baseline */
        const int prefix = __builtin_clz(w) - 16;
        ob_skip(b, prefix + 1);
        int ssize = suffix_len;
        if (prefix == 14 && suffix_len == 0) ssize = 4;
        if (prefix == 15) ssize = 12;
        int code = (prefix << suffix_len) + (ssize ? (int)ob_get(b, ssize) : 0);
        if (prefix == 15 && suffix_len == 0) code += 15;
        if (i == t1 && t1 < 3) code += 2;       /* the first non-trailing level is not +-1 */
        level[i] = (code & 1) ? -((code + 1) >> 1) : (code >> 1) + 1;
        if (suffix_len == 0) suffix_len = 1;
        if ((code >> 1) + 1 > (3 << (suffix_len - 1)) && suffix_len < 6) suffix_len++;
    }

    int zeros = 0;
    if (tc < maxc) {
        zeros = ob_vlc(b, maxc == 4 ? &gTotalZerosDcDec[tc - 1] : &gTotalZerosDec[tc - 1]);
        if (zeros < 0) return OMX_STS_ERR;
        if (tc + zeros > maxc) { t_divergent = 1; return OMX_STS_ERR; }
    }
    /* runs: run[i] zeros below coefficient i in scan order */
    int run[16];
    int left = zeros;
    for (int i = 0; i < tc - 1; i++) {
        int r = 0;
        if (left > 0) {
            r = ob_vlc(b, &gRunBeforeDec[(left < 7 ? left : 7) - 1]);
            if (r < 0) return OMX_STS_ERR;
            if (r > left) { t_divergent = 1; return OMX_STS_ERR; }
        }
        run[i] = r;
        left -= r;
    }
    run[tc - 1] = left;

    /* pairs, highest scan position first; a 15-coefficient block's scan
     * indices start at 1 (DC coded elsewhere) */
    OMX_U8 *o = *ppPosCoefbuf;
    int k = tc + zeros - 1 + (maxc == 15);
    for (int i = 0; i < tc; i++) {
        int flags = maxc == 4 ? k : kScan4x4[k];
        const int lv = level[i];
        if (i == tc - 1) flags |= 0x20;
        const int big = lv < -128 || lv > 127;
        if (big) flags |= 0x10;
        *o++ = (OMX_U8)flags;
        *o++ = (OMX_U8)(lv & 255);
        if (big) *o++ = (OMX_U8)((lv >> 8) & 255);
        k -= run[i] + 1;
    }
    *ppPosCoefbuf = o;
    return H264MI_OMX_Sts_NoErr;
}

static OMXResult run_block(const OMX_U8 **ppBitStream, OMX_S32 *pOffset, OMX_U8 *pNumCoeff, OMX_U8 **ppPosCoefbuf,
                           int cls, int maxc)
{
    OmxBits b = {*ppBitStream, (int)*pOffset};
    t_divergent = 0;
    const OMXResult r = decode_pairs(&b, pNumCoeff, ppPosCoefbuf, cls, maxc);
    *ppBitStream = b.p;
    *pOffset = b.off;
    return r;
}

/* omxVC.h:3160, omxVCM4P10_DecodeCoeffsToPairCAVLC.c:91-126 */
OMXResult omxVCM4P10_DecodeCoeffsToPairCAVLC(const OMX_U8 **ppBitStream, OMX_S32 *pOffset, OMX_U8 *pNumCoeff,
                                             OMX_U8 **ppPosCoefbuf, OMX_INT sVLCSelect, OMX_INT sMaxNumCoeff)
{
    if (!ppBitStream || !*ppBitStream || !pOffset || *pOffset < 0 || *pOffset > 7 || !pNumCoeff || !ppPosCoefbuf ||
        !*ppPosCoefbuf || sVLCSelect < 0 || sMaxNumCoeff < 15 || sMaxNumCoeff > 16)
        return H264MI_OMX_Sts_BadArgErr;
    return run_block(ppBitStream, pOffset, pNumCoeff, ppPosCoefbuf, coeff_token_class(sVLCSelect), sMaxNumCoeff);
}

/* omxVC.h:3101, omxVCM4P10_DecodeChromaDcCoeffsToPairCAVLC.c:75-93 */
OMXResult omxVCM4P10_DecodeChromaDcCoeffsToPairCAVLC(const OMX_U8 **ppBitStream, OMX_S32 *pOffset, OMX_U8 *pNumCoeff,
                                                     OMX_U8 **ppPosCoefbuf)
{
    if (!ppBitStream || !*ppBitStream || !pOffset || *pOffset < 0 || *pOffset > 7 || !pNumCoeff || !ppPosCoefbuf ||
        !*ppPosCoefbuf)
        return H264MI_OMX_Sts_BadArgErr;
    return run_block(ppBitStream, pOffset, pNumCoeff, ppPosCoefbuf, 4, 4);
}
