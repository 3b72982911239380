/* Bit-level I/O for H.264 RBSP payloads (host side).
 *
 * BitReader: big-endian MSB-first reader over an RBSP (emulation-prevention
 *   bytes already removed), with Exp-Golomb helpers (H.264 §9.1) and the
 *   more_rbsp_data() test (§7.2).  Replaces the reference's h264bsd_stream.c
 *   (h264bsdGetBits/ShowBits/FlushBits, stream.c:72-229) and
 *   h264bsd_vlc.c (ue/se/te, vlc.c:103-391) with a 64-bit cache design.
 * BitWriter: the inverse, used by the synthetic stream generator.
 */
#ifndef H264MI_BITS_H
#define H264MI_BITS_H

#include <stdint.h>
#include <stddef.h>
#include <string.h>

typedef struct {
    const uint8_t *buf;
    size_t   size;      /* bytes */
    size_t   pos;       /* bit position */
    size_t   end_bits;  /* position of rbsp_stop_one_bit (exclusive end of data) */
    int      err;       /* set when reading past the end */
    /* read cache: the 64 bits from bit cbase (a byte boundary), MSB first;
     * pos stays the reader's state, the cache only saves re-reading bytes */
    uint64_t cache;
    size_t   cbase;
} BitReader;

/* the 8 bytes at byte (zero past the end) into the cache */
static inline void br_refill_(BitReader *br)
{
    const size_t byte = br->pos >> 3;
    uint64_t v = 0;
    if (byte + 8 <= br->size) {
        memcpy(&v, br->buf + byte, 8);
        v = __builtin_bswap64(v);
    } else {
        for (int i = 0; i < 8; i++) {
            v <<= 8;
            if (byte + i < br->size) v |= br->buf[byte + i];
        }
    }
    br->cache = v;
    br->cbase = byte << 3;
}

static inline void br_init(BitReader *br, const uint8_t *buf, size_t size)
{
    br->buf = buf;
    br->size = size;
    br->pos = 0;
    br->err = 0;
    /* locate rbsp_stop_one_bit: the last set bit of the payload */
    size_t n = size;
    while (n > 0 && buf[n - 1] == 0) n--;
    if (n == 0) {
        br->end_bits = 0;
    } else {
        uint8_t b = buf[n - 1];
        int tz = __builtin_ctz(b);
        br->end_bits = (n - 1) * 8 + (7 - tz);
    }
    br_refill_(br);
}

/* peek up to 32 bits (zero-padded past the end).  The position does not
 * move, but the reader's cache may be refilled: the reader is written, so a
 * reader shared between threads (or a const one) must be copied first */
static inline uint32_t br_peek(BitReader *br, int n)
{
    if (n == 0) return 0;
    size_t off = br->pos - br->cbase;
    if (off + (size_t)n > 64) {        /* also pos < cbase: off wraps to a huge value */
        br_refill_(br);
        off = br->pos & 7;
    }
    return (uint32_t)((br->cache << off) >> (64 - n));
}

static inline void br_skip(BitReader *br, int n)
{
    br->pos += (size_t)n;
    if (br->pos > br->size * 8) br->err = 1;
}

static inline uint32_t br_u(BitReader *br, int n)
{
    uint32_t v = br_peek(br, n);
    br_skip(br, n);
    return v;
}

static inline uint32_t br_u1(BitReader *br) { return br_u(br, 1); }

/* ue(v): §9.1 */
static inline uint32_t br_ue(BitReader *br)
{
    uint32_t p = br_peek(br, 32);
    if (p == 0) {               /* >= 32 leading zeros: invalid in our profile */
        br->err = 1;
        br_skip(br, 32);
        return 0;
    }
    int lz = __builtin_clz(p);
    if (lz > 15) {              /* long codes: read in two steps */
        br_skip(br, lz + 1);
        uint32_t suf = br_u(br, lz);
        return (uint32_t)((1ull << lz) - 1 + suf);
    }
    br_skip(br, 2 * lz + 1);
    return (p >> (31 - 2 * lz)) - 1;
}

/* se(v): §9.1.1 */
static inline int32_t br_se(BitReader *br)
{
    uint32_t k = br_ue(br);
    if (k & 1) return (int32_t)((k + 1) >> 1);
    return -(int32_t)(k >> 1);
}

/* te(v) with range cMax (§9.1): cMax == 1 -> inverted single bit */
static inline uint32_t br_te(BitReader *br, uint32_t cmax)
{
    if (cmax > 1) return br_ue(br);
    return !br_u1(br);
}

/* more_rbsp_data(): the reference's test (h264bsdMoreRbspData,
 * h264bsd_util.c): data remain unless at most 8 bits are left and they are
 * exactly the rbsp_stop_one_bit pattern 1 0..0 -- which is what decides
 * where a damaged (truncated) slice stops */
static inline int br_more_rbsp_data(BitReader *br)
{
    if (br->pos >= br->size * 8) return br->pos > br->size * 8;   /* past the end: reference reads on */
    const size_t bits = br->size * 8 - br->pos;
    if (bits > 8) return 1;
    return br_peek(br, (int)bits) != (1u << (bits - 1));
}

static inline int br_byte_aligned(const BitReader *br) { return (br->pos & 7) == 0; }

/* ------------------------------------------------------------------------- */

typedef struct {
    uint8_t *buf;
    size_t   cap;
    size_t   nbytes;    /* completed bytes */
    uint32_t acc;       /* pending bits (MSB-first), count in nacc */
    int      nacc;
} BitWriter;

void bw_init(BitWriter *bw);
void bw_free(BitWriter *bw);
void bw_put(BitWriter *bw, uint32_t val, int n);   /* n <= 32 */
void bw_ue(BitWriter *bw, uint32_t v);
void bw_se(BitWriter *bw, int32_t v);
void bw_te(BitWriter *bw, uint32_t v, uint32_t cmax);
void bw_trailing(BitWriter *bw);                    /* rbsp_trailing_bits */
int  bw_aligned(const BitWriter *bw);
size_t bw_bits(const BitWriter *bw);

#endif
