// Micro-benchmark (diagnostics only): shader cycles of one lone wave's
// deblocking passes, deblock_dir() of recon_kernels.hip on a PPRegion in LDS
// filled with pseudo-random samples, and of the bare filter arithmetic
// (filt_line on registers, 4 edges), per bS mode:
//   0: MB edge bS 2, internal edges 0      (skip-like P MBs)
//   1: every edge bS 2                     (coded P MBs)
//   2: MB edge bS 4, internal edges 3      (intra MBs)
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 ubench_deblock.hip -o ubench_deblock
#include "../../broadway_amd/csrc/hip/recon_kernels.hip"
#include <stdio.h>

__global__ __launch_bounds__(64) void k_ub(unsigned long long *out, int iters, int bsmode)
{
    __shared__ PPRegion G;
    __shared__ uint8_t junk[256];
    const int lane = threadIdx.x;
    for (int i = lane; i < (int)sizeof(PPRegion); i += 64) ((uint8_t *)&G)[i] = (uint8_t)(100 + ((i * 37) & 15));
    __syncthreads();
    if (lane < 8) {
        const uint16_t w = bsmode == 0 ? 0x0002 : bsmode == 1 ? 0x2222 : 0x3334;
        ((uint16_t *)G.db)[lane] = w;
    }
    if (lane < 6) {
        uint8_t *o = G.db + 16 + lane * 8;
        o[0] = 40; o[1] = 10; o[2] = 1; o[3] = 2; o[4] = 3; o[5] = 30; o[6] = o[7] = 0;
    }
    __syncthreads();
    const DbPar Pv = dbpar(0, G.db, lane, true), Ph = dbpar(1, G.db, lane, true);
    unsigned long long t0 = clock64();
    for (int it = 0; it < iters; it++) {
        deblock_dir(0, Pv, G.ry, G.ru, G.rv, junk, lane);
        wave_sync();
    }
    unsigned long long t1 = clock64();
    for (int it = 0; it < iters; it++) {
        deblock_dir(1, Ph, G.ry, G.ru, G.rv, junk, lane);
        wave_sync();
    }
    unsigned long long t2 = clock64();
    // the row hand-off patch's arithmetic: one MB-edge step of one line
    // (row_pp applies it to MB c's rows 12..15 before publishing them)
    int pv[20];
    for (int j = 0; j < 20; j++) pv[j] = 100 + ((lane * 5 + j * 11) & 15);
    const int pbS = bsmode == 2 ? 4 : 2;
    unsigned long long tp0 = clock64();
    for (int it = 0; it < iters; it++) filt_line<true>(pv, 0, pbS, 40, 10, 10, 0x03020100u);
    unsigned long long tp1 = clock64();
    // the filter arithmetic alone: 4 dependent edges on a register line
    int v[20];
    for (int j = 0; j < 20; j++) v[j] = 100 + ((lane * 7 + j * 13) & 15);
    const int bS0 = bsmode == 2 ? 4 : 2, bSi = bsmode == 0 ? 0 : bsmode == 1 ? 2 : 3;
    for (int it = 0; it < iters; it++) {
        filt_line<true>(v, 0, bS0, 40, 10, 10, 0x03020100u);
        for (int k = 1; k < 4; k++) filt_line<false>(v, k, bSi, 40, 10, 10, 0x03020100u);
    }
    unsigned long long t3 = clock64();
    int acc = 0;
    for (int j = 0; j < 20; j++) acc += v[j] + pv[j];
    if (lane == 0) {
        out[0] = (t1 - t0) / iters; out[1] = (t2 - t1) / iters; out[2] = (t3 - t2) / iters;
        out[3] = G.ry[100] + acc;
        out[4] = (tp1 - tp0) / iters;
    }
}

// intra_tile (the MC wave's intra MB) of a lone wave, no left neighbour
// (nothing to wait for): mbtype 2 = I4x4 with modes cycling 0..8, 3 = I16x16
// plane, chroma plane
__global__ __launch_bounds__(64) void k_intra(unsigned long long *out, int iters, int mbtype)
{
    __shared__ McScratch M;
    __shared__ uint32_t i4tab[I4TAB_N];
    __shared__ uint8_t px[384];
    __shared__ int prog[4];
    const int lane = threadIdx.x;
    for (int e = lane; e < I4TAB_N; e += 64) i4tab[e] = i4_entry((e >> 4) % 9, e & 3, (e >> 2) & 3, e >= 9 * 16);
    for (int i = lane; i < (int)sizeof(McScratch); i += 64) ((uint8_t *)&M)[i] = (uint8_t)(90 + ((i * 29) & 31));
    for (int i = lane; i < 384; i += 64) M.res[i] = (int16_t)((i * 7) % 9 - 4);
    if (lane < 4) prog[lane] = 0;
    __syncthreads();
    uint64_t i4 = 0;
    for (int b = 0; b < 16; b++) i4 |= (uint64_t)(b % 9) << (4 * b);
    LeftNb N;
    N.lp = nullptr; N.lprog = &prog[0]; N.cprog = &prog[1]; N.my_lprog = &prog[2]; N.my_cprog = &prog[3];
    N.ltag = 0; N.mytag = 0; N.perr = nullptr; N.chk = false;
    const int avail = AV_B | AV_C | AV_D;
    unsigned long long t0 = clock64();
    for (int it = 0; it < iters; it++) {
        intra_tile(mbtype, avail, mbtype == MBT_I16 ? 3 | (3 << 4) : (3 << 4), i4, M.res, true, M.ty, M.tu, M.tv,
                   i4tab, M.junk, px, lane, N);
        wave_sync();
    }
    unsigned long long t1 = clock64();
    if (lane == 0) { out[0] = (t1 - t0) / iters; out[1] = px[17]; }
}

// mc_finish (the MC wave's inter MB: window staging, 6-tap luma, bilinear
// chroma, residual add) of a lone wave, loads already landed; fx/fy
// fractional positions cycle over all 16 luma / 64 chroma cases (mode 3: one
// position per MB, as skip / 16x16 MBs, cycling)
__global__ __launch_bounds__(64) void k_mc(unsigned long long *out, int iters, const uint8_t *frame, uint8_t *dbrec,
                                           int16_t *res, unsigned *err, int fmode)
{
    __shared__ McScratch M;
    __shared__ uint8_t px[384], db[64];
    const int lane = threadIdx.x;
    ReconArgs a;
    memset(&a, 0, sizeof(a));
    a.frames = (uint8_t *)frame; a.frame_bytes = H264MI_SLOT_BYTES(120, 68); a.cpitch = H264MI_CPITCH(120);
    a.w = 120; a.h = 68;
    a.dbrec = dbrec; a.res = res; a.err = err;
    PicDesc pd;
    memset(&pd, 0, sizeof(pd));
    // MbRec as dwords: type inter, cbits = all luma + chroma AC, refs slot 0,
    // per 4x4 block a different fractional MV
    uint32_t v0 = 0;
    if (lane == 0) v0 = MBT_INTER | (26u << 8) | (26u << 16) | ((uint32_t)(AV_A | AV_B) << 24);
    if (lane == 2) v0 = 0x00FFFFFFu;
    if (lane >= 7 && lane < 23) {
        const int b = lane - 7;
        // fmode 0: all 16 positions; 1: full-sample only; 2: half-sample
        // b / h only (no centre j)
        const int fx = fmode == 1 ? 0 : fmode == 2 ? ((b & 1) ? 2 : 0) : (b & 3);
        const int fy = fmode == 1 ? 0 : fmode == 2 ? ((b & 1) ? 0 : 2) : ((b >> 2) & 3);
        const int mvx = 4 * (b - 8) + fx, mvy = 4 * (3 - b) + fy;
        v0 = (uint32_t)(uint16_t)mvx | ((uint32_t)(uint16_t)mvy << 16);
    }
    McLoad L;
    unsigned long long acc = 0;
    for (int it = 0; it < iters; it++) {
        if (fmode == 3 && lane >= 7 && lane < 23) {
            // one MV per MB (skip / 16x16), its position cycling over the 16
            const int fx = it & 3, fy = (it >> 2) & 3;
            v0 = (uint32_t)(uint16_t)(4 * 3 + fx) | ((uint32_t)(uint16_t)(4 * -2 + fy) << 16);
        }
        const int mb = 30 * 120 + 40 + (it & 15);
        mc_issue(a, pd, 0, mb, v0, lane, L);
        drain_vm();
        wave_sync();
        const unsigned long long t0 = clock64();
        mc_finish(a, 0, v0, lane, L, M, px, M.res, db);
        wave_sync();
        acc += clock64() - t0;
    }
    if (lane == 0) { out[0] = acc / iters; out[1] = px[5]; }
}

// the row-to-row hand-off (row_pp's mailbox granules): two workgroups pass
// a token back and forth through 8-byte sc1 granules {value, tag}, polled
// as row_pp polls the row above (sc1 load, s_sleep 1); one-way latency =
// round trip / 2 on the wall clock.  Blocks 0 and `other` (0 + 8: the same
// XCD under round-robin placement; 0 + 1: another one)
__global__ __launch_bounds__(64) void k_hop(unsigned long long *g, unsigned long long *out, int rounds, int other)
{
    const int b = blockIdx.x;
    if (b != 0 && b != other) return;
    const int lane = threadIdx.x;
    unsigned long long *mine = g + (b == 0 ? 0 : 16), *theirs = g + (b == 0 ? 16 : 0);
    const unsigned long long w0 = wall_clock64();
    unsigned spins = 0;         // bounded: a lost partner ends the loop
    for (int k = 1; k <= rounds && spins < (1u << 24); k++) {
        if (b == 0) {
            if (lane == 0) st_gran(mine, (uint32_t)k, 7u);
            while (__builtin_amdgcn_readfirstlane((uint32_t)ld_gran(theirs)) != (uint32_t)k && ++spins < (1u << 24))
                __builtin_amdgcn_s_sleep(1);
        } else {
            while (__builtin_amdgcn_readfirstlane((uint32_t)ld_gran(theirs)) != (uint32_t)k && ++spins < (1u << 24))
                __builtin_amdgcn_s_sleep(1);
            if (lane == 0) st_gran(mine, (uint32_t)k, 7u);
        }
    }
    if (b == 0 && lane == 0) out[0] = (wall_clock64() - w0);
}

// wall-clock (100 MHz) against shader clock over the same loop: the clock
// the passes ran at
__global__ void k_clk(unsigned long long *out)
{
    const unsigned long long w0 = wall_clock64(), c0 = clock64();
    unsigned long long w1;
    do { w1 = wall_clock64(); } while (w1 - w0 < 100000);
    const unsigned long long c1 = clock64();
    if (threadIdx.x == 0) { out[0] = w1 - w0; out[1] = c1 - c0; }
}

int main()
{
    unsigned long long *d, h[4];
    (void)hipMalloc(&d, 64);
    hipLaunchKernelGGL(k_clk, dim3(1), dim3(64), 0, 0, d);
    (void)hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    const double mhz = (double)h[1] / (double)h[0] * 100.0;
    printf("shader clock %.0f MHz\n", mhz);
    double vh_us = 0, patch_us = 0, hop_us[2] = {0, 0};
    for (int mode = 0; mode < 3; mode++) {
        unsigned long long hh[5];
        hipLaunchKernelGGL(k_ub, dim3(1), dim3(64), 0, 0, d, 2000, mode);
        (void)hipMemcpy(hh, d, 40, hipMemcpyDeviceToHost);
        printf("bsmode %d: V %llu cycles (%.3f us), H %llu cycles (%.3f us), filt x4 %llu cycles, patch edge %llu cycles\n", mode,
               hh[0], hh[0] / mhz, hh[1], hh[1] / mhz, hh[2], hh[4]);
        if (mode == 1) { vh_us = (hh[0] + hh[1]) / mhz; patch_us = hh[4] / mhz; }
    }
    {
        unsigned long long *g;
        (void)hipMalloc(&g, 256);
        const int rounds = 2000;
        for (int k = 0; k < 2; k++) {
            (void)hipMemset(g, 0, 256);
            const int other = k == 0 ? 8 : 1;
            hipLaunchKernelGGL(k_hop, dim3(16), dim3(64), 0, 0, g, d, rounds, other);
            unsigned long long w = 0;
            (void)hipMemcpy(&w, d, 8, hipMemcpyDeviceToHost);
            hop_us[k] = (double)w / 100.0 / (2.0 * rounds);
            printf("granule hand-off one way (%s XCD): %.3f us\n", k == 0 ? "same" : "other", hop_us[k]);
        }
        (void)hipFree(g);
    }
    for (int t = 2; t <= 3; t++) {
        hipLaunchKernelGGL(k_intra, dim3(1), dim3(64), 0, 0, d, 500, t);
        (void)hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
        printf("intra_tile %s: %llu cycles (%.3f us)\n", t == 2 ? "I4x4" : "I16x16 plane", h[0], h[0] / mhz);
    }
    {
        uint8_t *frame, *dbrec;
        int16_t *res;
        unsigned *err;
        (void)hipMalloc(&frame, H264MI_SLOT_BYTES(120, 68));
        (void)hipMemset(frame, 77, H264MI_SLOT_BYTES(120, 68));
        (void)hipMalloc(&dbrec, 120 * 68 * 64);
        (void)hipMemset(dbrec, 0, 120 * 68 * 64);
        (void)hipMalloc(&res, 120 * 68 * 768);
        (void)hipMemset(res, 0, 120 * 68 * 768);
        (void)hipMalloc(&err, 64);
        for (int fm = 0; fm < 4; fm++) {
            hipLaunchKernelGGL(k_mc, dim3(1), dim3(64), 0, 0, d, 500, frame, dbrec, res, err, fm);
            (void)hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
            printf("mc_finish inter MB (%s): %llu cycles (%.3f us)\n", fm == 0 ? "16 positions" : fm == 1 ? "full-sample" : fm == 2 ? "half b/h only" : "one MV per MB, all positions",
                   h[0], h[0] / mhz);
        }
    }
    // the inputs of the bench line's latency roofline (bench.py latency_floor,
    // profiles/ubench.json): lone-wave V + H of a coded P MB (bsmode 1), the
    // hand-off patch edge, the granule hop (the slower placement)
    printf("JSON {\"shader_mhz\": %.0f, \"vh_us\": %.4f, \"patch_us\": %.4f, \"hop_same_xcd_us\": %.4f, \"hop_other_xcd_us\": %.4f}\n",
           mhz, vh_us, patch_us, hop_us[0], hop_us[1]);
    return 0;
}
