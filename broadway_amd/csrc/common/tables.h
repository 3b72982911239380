/* Constant tables of ITU-T H.264 (Baseline subset) used on the host side.
 *
 * The CAVLC code tables are written as bit strings straight from the
 * standard's tables 9-5 (coeff_token), 9-7/9-8/9-9a (total_zeros) and 9-10
 * (run_before); they are expanded at start-up into decode lookup tables and
 * encode (code,len) pairs.  The reference keeps the same tables in a packed
 * decoder-specific form in h264bsd_cavlc.c:80-390.
 */
#ifndef H264MI_TABLES_H
#define H264MI_TABLES_H

#include <stdint.h>

/* scan position -> raster position (frame zig-zag, Table 8-12) */
extern const uint8_t kZigzag4x4[16];
/* coded_block_pattern mapping (Table 9-4, chroma_format_idc = 1) */
extern const uint8_t kCbpIntra[48];
extern const uint8_t kCbpInter[48];
/* QPc as a function of qPI (Table 8-15) */
extern const uint8_t kQpChroma[52];
/* normAdjust v(m, class): class 0 = (even,even), 1 = (odd,odd), 2 = other */
extern const uint8_t kLevelScale[6][3];
/* deblocking (Table 8-16, 8-17) */
extern const uint8_t kAlpha[52];
extern const uint8_t kBeta[52];
extern const uint8_t kTc0[52][3];

/* z-order 4x4 block index -> (x,y) in 4x4 units and back */
extern const uint8_t kBlkX[16];
extern const uint8_t kBlkY[16];
static inline int blk_index(int x4, int y4)
{
    return ((y4 >> 1) * 2 + (x4 >> 1)) * 4 + (y4 & 1) * 2 + (x4 & 1);
}

/* ---- CAVLC VLC tables ---------------------------------------------------- */

typedef struct { uint32_t code; uint8_t len; } VlcCode;

/* two-level lookup table decoder */
typedef struct {
    int16_t sym[256];       /* >=0 symbol, -1 invalid, <= -2: subtable index -(s+2) */
    uint8_t len[256];
    int16_t (*sub_sym)[256];
    uint8_t (*sub_len)[256];
    int     nsub;
} VlcTable;

/* encode tables (filled by h264_tables_init) */
extern VlcCode gCoeffTokenEnc[5][17][4];   /* [nC class 0..3, 4 = chroma DC][TotalCoeff][T1] */
extern VlcCode gTotalZerosEnc[15][16];     /* [TotalCoeff-1][total_zeros] */
extern VlcCode gTotalZerosDcEnc[3][4];     /* chroma DC */
extern VlcCode gRunBeforeEnc[7][15];       /* [min(zerosLeft,7)-1][run_before] */

/* decode tables; symbol = (TotalCoeff << 2) | T1 for coeff_token */
extern VlcTable gCoeffTokenDec[5];
extern VlcTable gTotalZerosDec[15];
extern VlcTable gTotalZerosDcDec[3];
extern VlcTable gRunBeforeDec[7];

/* the same tables packed for the parser's fast path: one 16-bit entry per
 * 8-bit index, (sym << 5) | len (len 1..16), 0 = invalid, 0x8000 | k = the
 * k-th 256-entry subtable of the next 8 bits (contiguous in sub) */
typedef struct {
    uint16_t t[256];
    uint16_t *sub;
} VlcPk;
extern VlcPk gCoeffTokenPk[5];
extern VlcPk gTotalZerosPk[15];
extern VlcPk gTotalZerosDcPk[3];
extern VlcPk gRunBeforePk[7];

/* entry for a 16-bit window (MSB = next stream bit): len = e & 31, sym = e >> 5 */
static inline uint32_t vlc_pk(const VlcPk *t, uint32_t peek16)
{
    uint32_t e = t->t[peek16 >> 8];
    if (__builtin_expect(e & 0x8000, 0)) e = t->sub[((e & 0x7FFFu) << 8) | (peek16 & 0xFFu)];
    return e;
}

void h264_tables_init(void);   /* idempotent, thread-safe */
/* returns sym or -1; inline: the CAVLC decode calls it several times per
 * coded block */
static inline int vlc_decode(const VlcTable *t, uint32_t peek16, int *len)
{
    const uint32_t hi = (peek16 >> 8) & 0xFF;
    int s = t->sym[hi];
    if (s >= 0) { *len = t->len[hi]; return s; }
    if (s == -1) { *len = 0; return -1; }
    const int sub = -(s + 2);
    const uint32_t lo = peek16 & 0xFF;
    *len = t->sub_len[sub][lo];
    return t->sub_sym[sub][lo];
}

static inline int coeff_token_class(int nC)
{
    if (nC < 0) return 4;
    if (nC < 2) return 0;
    if (nC < 4) return 1;
    if (nC < 8) return 2;
    return 3;
}

#endif
