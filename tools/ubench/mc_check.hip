// Unit check (diagnostics): mc_issue + mc_finish of recon_kernels.hip on
// random reference frames, random MB positions (edges included), random
// per-block MVs (all 16 luma / 64 chroma fractional positions, windows
// reaching up to 40 samples off the picture) and random residuals, against
// a direct scalar restatement of 8.4.2.2 (luma 6-tap, 8-239 .. 8-261;
// chroma 8-266) with h264bsdFillBlock's clamp (reconstruct.c:2222-2314).
// Mode 0: every block its own MV; mode 1: one MV per MB (16x16); mode 2:
// one MV per 8x8.  Prints mismatch counts per mode; exit 1 on any.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 mc_check.hip -o mc_check
#include "../../broadway_amd/csrc/hip/recon_kernels.hip"
#include <stdio.h>
#include <stdlib.h>

#define WM 40
#define HM 23

__device__ int pix(const uint8_t *f, int W, int H, int pitch, int x, int y)
{
    x = min(max(x, 0), W - 1);
    y = min(max(y, 0), H - 1);
    return f[y * pitch + x];
}
__device__ int t6(int a, int b, int c, int d, int e, int f) { return a - 5 * b + 20 * c + 20 * d - 5 * e + f; }
__device__ int c255(int v) { return min(max(v, 0), 255); }
// luma sample at integer (X, Y) + fraction (fx, fy) (8.4.2.2.1)
__device__ int luma_ref(const uint8_t *f, int W, int H, int X, int Y, int fx, int fy)
{
    auto G = [&](int dx, int dy) { return pix(f, W, H, W, X + dx, Y + dy); };
    auto b1 = [&](int dy) { return t6(G(-2, dy), G(-1, dy), G(0, dy), G(1, dy), G(2, dy), G(3, dy)); };
    auto h1 = [&](int dx) { return t6(G(dx, -2), G(dx, -1), G(dx, 0), G(dx, 1), G(dx, 2), G(dx, 3)); };
    const int b = c255((b1(0) + 16) >> 5), h = c255((h1(0) + 16) >> 5);
    const int s = c255((b1(1) + 16) >> 5), m = c255((h1(1) + 16) >> 5);
    const int j1 = t6(b1(-2), b1(-1), b1(0), b1(1), b1(2), b1(3));
    const int j = c255((j1 + 512) >> 10);
    const int g = G(0, 0);
    switch (fy * 4 + fx) {
    case 0: return g;
    case 1: return (g + b + 1) >> 1;
    case 2: return b;
    case 3: return (b + G(1, 0) + 1) >> 1;
    case 4: return (g + h + 1) >> 1;
    case 5: return (b + h + 1) >> 1;
    case 6: return (b + j + 1) >> 1;
    case 7: return (b + m + 1) >> 1;
    case 8: return h;
    case 9: return (h + j + 1) >> 1;
    case 10: return j;
    case 11: return (j + m + 1) >> 1;
    case 12: return (h + G(0, 1) + 1) >> 1;
    case 13: return (h + s + 1) >> 1;
    case 14: return (j + s + 1) >> 1;
    default: return (s + m + 1) >> 1;
    }
}

__global__ __launch_bounds__(64) void k_check(const uint8_t *frame, int16_t *res, uint8_t *dbrec, unsigned *err,
                                              unsigned *bad, int iters, int mode, unsigned seed, int with_res)
{
    __shared__ McScratch M;
    __shared__ uint8_t px[384], db[64];
    const int lane = threadIdx.x;
    ReconArgs a;
    memset(&a, 0, sizeof(a));
    a.frames = (uint8_t *)frame; a.frame_bytes = H264MI_SLOT_BYTES(WM, HM); a.cpitch = H264MI_CPITCH(WM);
    a.w = WM; a.h = HM;
    a.dbrec = dbrec; a.res = res; a.err = err;
    PicDesc pd;
    memset(&pd, 0, sizeof(pd));
    const int W16 = WM * 16, H16 = HM * 16, CW = W16 / 2, CH = H16 / 2;
    unsigned rng = seed * 747796405u + 2891336453u;
    auto rnd = [&](unsigned n) { rng = (unsigned)__builtin_amdgcn_readfirstlane((int)(rng * 1664525u + 1013904223u)); return (rng >> 8) % n; };
    unsigned nbad = 0;
    for (int it = 0; it < iters; it++) {
        // the same random stream in every lane (uniform)
        const int mb = __builtin_amdgcn_readfirstlane((int)rnd(WM * HM));
        const int mbx = mb % WM, mby = mb / WM;
        int mvs[16][2];
        for (int k = 0; k < 16; k++) {
            const int src = mode == 0 ? k : mode == 1 ? 0 : (k >> 2) * 4;
            if (src != k) { mvs[k][0] = mvs[src][0]; mvs[k][1] = mvs[src][1]; continue; }
            const bool far = rnd(8) == 0;
            mvs[k][0] = far ? (int)rnd(4 * 200) - 400 : (int)rnd(64) - 32;
            mvs[k][1] = far ? (int)rnd(4 * 200) - 400 : (int)rnd(64) - 32;
        }
        uint32_t v0 = 0;
        if (lane == 0) v0 = MBT_INTER | (26u << 8) | (26u << 16) | ((uint32_t)(AV_A | AV_B) << 24);
        if (lane == 2) v0 = with_res ? 0x00FFFFFFu : 0u;
        if (lane >= 7 && lane < 23) v0 = (uint32_t)(uint16_t)mvs[lane - 7][0] | ((uint32_t)(uint16_t)mvs[lane - 7][1] << 16);
        McLoad L;
        mc_issue(a, pd, 0, mb, v0, lane, L);
        drain_vm();
        wave_sync();
        mc_finish(a, 0, v0, lane, L, M, px, M.res, db);
        wave_sync();
        const int16_t *rb = res + (size_t)mb * 384;
        for (int i = lane; i < 384; i += 64) {
            int want;
            int rv = 0;
            if (i < 256) {
                const int x = i & 15, y = i >> 4;
                const int b = blk_of(x >> 2, y >> 2);
                const int mvx = mvs[b][0], mvy = mvs[b][1];
                want = luma_ref(frame, W16, H16, mbx * 16 + x + (mvx >> 2), mby * 16 + y + (mvy >> 2), mvx & 3, mvy & 3);
                if (with_res) rv = rb[b * 16 + (y & 3) * 4 + (x & 3)];
            } else {
                const int comp = (i - 256) >> 6, k = (i - 256) & 63, x = k & 7, y = k >> 3;
                const int b = blk_of(x >> 1, y >> 1);
                const int mvx = mvs[b][0], mvy = mvs[b][1];
                const int fx = mvx & 7, fy = mvy & 7;
                const uint8_t *cf = frame + W16 * H16 + comp * a.cpitch * CH;
                const int X = mbx * 8 + x + (mvx >> 3), Y = mby * 8 + y + (mvy >> 3);
                const int A = pix(cf, CW, CH, a.cpitch, X, Y), B = pix(cf, CW, CH, a.cpitch, X + 1, Y);
                const int C = pix(cf, CW, CH, a.cpitch, X, Y + 1), D = pix(cf, CW, CH, a.cpitch, X + 1, Y + 1);
                want = ((8 - fx) * (8 - fy) * A + fx * (8 - fy) * B + (8 - fx) * fy * C + fx * fy * D + 32) >> 6;
                const int rbk = 16 + comp * 4 + (y >> 2) * 2 + (x >> 2);
                if (with_res) rv = rb[rbk * 16 + (y & 3) * 4 + (x & 3)];
            }
            want = c255(want + rv);
            if (px[i] != want) {
                // first mismatches: {it, mb, sample, got | want << 8}
                const unsigned slot = atomicAdd(&bad[1], 1u);
                if (slot < 8) { bad[2 + slot * 4] = it; bad[3 + slot * 4] = mb; bad[4 + slot * 4] = i; bad[5 + slot * 4] = px[i] | (want << 8); }
                nbad++;
            }
        }
        wave_sync();
    }
    atomicAdd(bad, nbad);
}

int main()
{
    const size_t fb = H264MI_SLOT_BYTES(WM, HM);
    uint8_t *h = (uint8_t *)malloc(fb);
    srand(7);
    for (size_t i = 0; i < fb; i++) h[i] = (uint8_t)(rand() & 255);
    int16_t *hr = (int16_t *)malloc((size_t)WM * HM * 384 * 2);
    for (size_t i = 0; i < (size_t)WM * HM * 384; i++) hr[i] = (int16_t)(rand() % 601 - 300);
    uint8_t *frame, *dbrec;
    int16_t *res;
    unsigned *err, *bad;
    (void)hipMalloc(&frame, fb);
    (void)hipMemcpy(frame, h, fb, hipMemcpyHostToDevice);
    (void)hipMalloc(&res, (size_t)WM * HM * 384 * 2);
    (void)hipMemcpy(res, hr, (size_t)WM * HM * 384 * 2, hipMemcpyHostToDevice);
    (void)hipMalloc(&dbrec, (size_t)WM * HM * 64);
    (void)hipMemset(dbrec, 0, (size_t)WM * HM * 64);
    (void)hipMalloc(&err, 64);
    (void)hipMalloc(&bad, 64 * 4);
    int fail = 0;
    for (int wr = 0; wr < 2; wr++)
        for (int mode = 0; mode < 3; mode++) {
            (void)hipMemset(bad, 0, 64 * 4);
            hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, 0, frame, res, dbrec, err, bad, 2000, mode, 11u + mode, wr);
            unsigned hb[64];
            (void)hipMemcpy(hb, bad, sizeof(hb), hipMemcpyDeviceToHost);
            const unsigned nb = hb[0];
            printf("mc_check mode %d residual %d: %u mismatching samples of %d\n", mode, wr, nb, 2000 * 384);
            for (unsigned k = 0; k < 8 && k < hb[1]; k++)
                printf("  it %u mb (%u,%u) sample %u: got %u want %u\n", hb[2 + k * 4], hb[3 + k * 4] % WM, hb[3 + k * 4] / WM,
                       hb[4 + k * 4], hb[5 + k * 4] & 255, hb[5 + k * 4] >> 8);
            fail |= nb != 0;
        }
    printf(fail ? "mc_check FAILED\n" : "mc_check OK\n");
    return fail;
}
