// I420 -> RGBA for Decoder.js's `rgb: true` output:
// the same integer arithmetic as DecoderPost.js's asm.js converter
// (yuv2rgbcalc, templates/DecoderPost.js:514-560, driven per 2x2 block by
// doit, :420-505):
//   a0 = 1192 (Y - 16)
//   R = (a0 + 1634 (V - 128)) >> 10
//   G = (a0 - 832 (V - 128) - 400 (U - 128)) >> 10
//   B = (a0 + 2066 (U - 128)) >> 10          (arithmetic shifts)
// each clamped to [0, 255], stored as the little-endian word
// 0xFF << 24 | B << 16 | G << 8 | R, i.e. bytes R G B A, row-major over the
// MB-aligned picture (width * height * 4 bytes).  The reference's (Y, U, V)
// result cache never changes a value (every word has A = 255), so it has no
// counterpart here.
//
// HBM-bound elementwise kernel: 1.5 B read + 4 B written per pixel.  A
// thread converts two 4-column groups f and f + 64 of a 128-group chunk in
// two rows: each wave-wide load / store instruction then covers one
// contiguous span (64 x 4 B of Y, 64 x 2 B of U or V, 64 x 16 B of RGBA),
// two at a row end.

__device__ __forceinline__ uint32_t rgba_px(int y, int cr, int cg, int cb)
{
    const int a0 = 1192 * (y - 16);
    const int r = med3i((a0 + cr) >> 10, 0, 255);
    const int g = med3i((a0 + cg) >> 10, 0, 255);
    const int b = med3i((a0 + cb) >> 10, 0, 255);
    return 0xFF000000u | ((uint32_t)b << 16) | ((uint32_t)g << 8) | (uint32_t)r;
}

// one 4-column group (2 chroma samples) of two rows
__device__ __forceinline__ void rgba_group(const uint8_t *Y, const uint8_t *U, const uint8_t *V, uint8_t *O,
                                           int width, size_t yo, size_t co)
{
    const uint32_t y0 = *(const uint32_t *)(Y + yo), y1 = *(const uint32_t *)(Y + yo + width);
    const uint32_t u2 = *(const uint16_t *)(U + co), v2 = *(const uint16_t *)(V + co);
    uint32_t o0[4], o1[4];
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const int u = (int)((u2 >> (8 * k)) & 255) - 128, v = (int)((v2 >> (8 * k)) & 255) - 128;
        const int cr = 1634 * v, cg = -832 * v - 400 * u, cb = 2066 * u;
        o0[2 * k] = rgba_px((int)((y0 >> (16 * k)) & 255), cr, cg, cb);
        o0[2 * k + 1] = rgba_px((int)((y0 >> (16 * k + 8)) & 255), cr, cg, cb);
        o1[2 * k] = rgba_px((int)((y1 >> (16 * k)) & 255), cr, cg, cb);
        o1[2 * k + 1] = rgba_px((int)((y1 >> (16 * k + 8)) & 255), cr, cg, cb);
    }
    // streaming output (nothing here reads it back): non-temporal stores
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 w0 = {o0[0], o0[1], o0[2], o0[3]}, w1 = {o1[0], o1[1], o1[2], o1[3]};
    __builtin_nontemporal_store(w0, (u32x4 *)(O + yo * 4));
    __builtin_nontemporal_store(w1, (u32x4 *)(O + (yo + width) * 4));
}

// grid: (ceil(groups / 128) blocks of 64 threads, npics), groups = the
// picture's (row pair, 4-column group) pairs in raster order, so no lane
// idles at row ends; picture k at in + k * in_stride -> out + k * out_stride;
// chroma rows cpitch bytes apart (width / 2 packed, H264MI_CPITCH in a slot)
__global__ __launch_bounds__(64) void k_yuv2rgba(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, int width,
                                                 int height, int cpitch, size_t in_stride, size_t out_stride)
{
    const int ng = width >> 2;                      // 4-column groups per row
    const int nf = ng * (height >> 1);
    const uint8_t *Y = in + blockIdx.y * in_stride;
    const uint8_t *U = Y + (size_t)width * height;
    const uint8_t *V = U + (size_t)cpitch * (height >> 1);
    uint8_t *O = out + blockIdx.y * out_stride;
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const int f = blockIdx.x * 128 + h * 64 + (int)threadIdx.x;
        if (f < nf) {
            const int y2 = f / ng, g = f - y2 * ng;
            rgba_group(Y, U, V, O, width, (size_t)(2 * y2) * width + 4 * g, (size_t)y2 * cpitch + 2 * g);
        }
    }
}
