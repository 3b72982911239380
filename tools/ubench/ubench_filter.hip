// Microbenchmark (diagnostics, not a test): what one deblocking step costs a
// single wave, as deblock_dir runs them.  Times with clock64 (shader clock):
//   filter: 3 serial internal edges per iteration, lanes 0..31 carry lines
//           (luma 0..15, chroma 16..31), lanes 32..63 mirror them or are
//           switched off (exec = lanes 0..31)
//   lds:    20 ds_read_u8 down a column + 18 ds_write_b8 back (the H pass's
//           transposition), full / half exec
// Variants of the filter body: 0 = filt_line (SGPR masks), 1 = VGPR masks.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -o
// tools/ubench/ubench_filter tools/ubench/ubench_filter.hip; run on the GPU box.
#include "../../broadway_amd/csrc/hip/recon_kernels.hip"
#include <cstdio>
#include <cstring>
#include <vector>

__device__ __forceinline__ void filt_line_vm(int (&v)[20], const int k, const int bS, const int alpha, const int beta,
                                             const int beta_ap, const uint32_t tcs)
{
    const int o = 4 * k;
    const int p2 = v[o + 1], p1 = v[o + 2], p0 = v[o + 3];
    const int q0 = v[o + 4], q1 = v[o + 5], q2 = v[o + 6];
    const int bnz = -min(bS, 1);                                      // 0 / -1
    const int m0 = (int)__builtin_amdgcn_sad_u8((uint32_t)p0, (uint32_t)q0, (uint32_t)(-alpha & bnz));
    const int m1 = (int)__builtin_amdgcn_sad_u8((uint32_t)p1, (uint32_t)p0, (uint32_t)-beta);
    const int m2 = (int)__builtin_amdgcn_sad_u8((uint32_t)q1, (uint32_t)q0, (uint32_t)-beta);
    const int fm = max(m0, max(m1, m2)) >> 31;                        // -1: filter
    const int apm = (int)__builtin_amdgcn_sad_u8((uint32_t)p2, (uint32_t)p0, (uint32_t)-beta_ap) >> 31;
    const int aqm = (int)__builtin_amdgcn_sad_u8((uint32_t)q2, (uint32_t)q0, (uint32_t)-beta_ap) >> 31;
    const int tc0 = (int)__builtin_amdgcn_ubfe(tcs, (uint32_t)bS << 3, 8);
    const int tc = tc0 - apm - aqm;
    const int d = med3i((((q0 - p0) << 2) + (p1 - q1) + 4) >> 3, -tc, tc);
    const int avg = (int)__builtin_amdgcn_lerp((uint32_t)p0, (uint32_t)q0, 1u);
    const int ntc0 = -tc0;
    const int dp1 = med3i((mad_m2(p1, p2) + avg) >> 1, ntc0, tc0) & apm & fm;
    const int dq1 = med3i((mad_m2(q1, q2) + avg) >> 1, ntc0, tc0) & aqm & fm;
    const int n_p0 = clip255(p0 + d), n_q0 = clip255(q0 - d);
    v[o + 2] = p1 + dp1;
    v[o + 5] = q1 + dq1;
    v[o + 3] = (n_p0 & fm) | (p0 & ~fm);
    v[o + 4] = (n_q0 & fm) | (q0 & ~fm);
}

template <int VAR, bool HALF>
__global__ __launch_bounds__(64) void k_filt(const uint32_t *in, uint32_t *out, unsigned long long *cyc, int iters)
{
    const int lane = threadIdx.x;
    int v[20];
    for (int j = 0; j < 20; j++) v[j] = in[(lane & 31) * 20 + j] & 255;
    const uint32_t bsw = in[64 * 20 + (lane & 31)];
    const int alpha = 40, beta = 12;
    const uint32_t tcs = 0x06040200u;
    const bool chroma = (lane & 31) >= 16;
    __syncthreads();
    unsigned long long t0 = clock64();
    if (!HALF || lane < 32) {
        for (int it = 0; it < iters; it++) {
#pragma unroll
            for (int k = 1; k < 4; k++) {
                const int b = (int)((bsw >> (4 * k)) & 15);
                if (__builtin_amdgcn_ballot_w64(b != 0) == 0) continue;
                if (VAR == 0) filt_line<false>(v, k, b, alpha, beta, chroma ? 0 : beta, tcs);
                else filt_line_vm(v, k, b, alpha, beta, chroma ? 0 : beta, tcs);
            }
        }
    }
    unsigned long long t1 = clock64();
    uint32_t h = 0;
    for (int j = 0; j < 20; j++) h = h * 31 + (uint32_t)v[j];
    out[lane] = h;
    if (lane == 0) cyc[0] = t1 - t0;
}

template <bool HALF>
__global__ __launch_bounds__(64) void k_lds(uint32_t *out, unsigned long long *cyc, int iters)
{
    __shared__ uint8_t reg[24 * 32 + 256];
    const int lane = threadIdx.x;
    for (int i = lane; i < (int)sizeof reg; i += 64) reg[i] = (uint8_t)(i * 7);
    __syncthreads();
    uint8_t *col = reg + (lane & 31);
    uint8_t *jk = reg + 24 * 32 + (lane & 63) * 4;
    uint32_t acc = 0;
    unsigned long long t0 = clock64();
    if (!HALF || lane < 32) {
        for (int it = 0; it < iters; it++) {
            int v[20];
#pragma unroll
            for (int j = 0; j < 20; j++) v[j] = col[j * 32];
#pragma unroll
            for (int j = 0; j < 20; j++) acc += (uint32_t)v[j];
#pragma unroll
            for (int j = 1; j < 19; j++) *((lane & 1) ? col + j * 32 : jk) = (uint8_t)(v[j] + 1);
            asm volatile("" ::: "memory");
        }
    }
    unsigned long long t1 = clock64();
    out[lane] = acc;
    if (lane == 0) cyc[0] = t1 - t0;
}

static double run_filt(int var, bool half, const uint32_t *din, uint32_t *dout, unsigned long long *dcyc, int iters,
                       uint32_t *host_out)
{
    if (var == 0 && !half) k_filt<0, false><<<1, 64>>>(din, dout, dcyc, iters);
    if (var == 0 && half) k_filt<0, true><<<1, 64>>>(din, dout, dcyc, iters);
    if (var == 1 && !half) k_filt<1, false><<<1, 64>>>(din, dout, dcyc, iters);
    if (var == 1 && half) k_filt<1, true><<<1, 64>>>(din, dout, dcyc, iters);
    unsigned long long cyc = 0;
    hipMemcpy(&cyc, dcyc, 8, hipMemcpyDeviceToHost);
    hipMemcpy(host_out, dout, 256, hipMemcpyDeviceToHost);
    return (double)cyc / iters / 3;
}

int main()
{
    const int iters = 4000;
    std::vector<uint32_t> hin(64 * 21);
    uint32_t s = 12345;
    for (auto &x : hin) { s = s * 1103515245u + 12345u; x = (s >> 8) & 0xFFFFFF; }
    // samples near each other (edges filter), bS 1..2 on the internal edges
    for (int l = 0; l < 64; l++)
        for (int j = 0; j < 20; j++) hin[l * 20 + j] = 100 + (hin[l * 20 + j] % 9);
    for (int l = 0; l < 64; l++) hin[64 * 20 + l] = 0x2120u | ((l & 1) << 12);
    uint32_t *din, *dout;
    unsigned long long *dcyc;
    hipMalloc(&din, hin.size() * 4);
    hipMalloc(&dout, 64 * 4);
    hipMalloc(&dcyc, 8);
    hipMemcpy(din, hin.data(), hin.size() * 4, hipMemcpyHostToDevice);
    uint32_t ref[64], got[64];
    for (int rep = 0; rep < 2; rep++) {
        const double a = run_filt(0, false, din, dout, dcyc, iters, ref);
        const double b = run_filt(0, true, din, dout, dcyc, iters, got);
        const bool same_half = !memcmp(ref, got, 128);
        const double c = run_filt(1, false, din, dout, dcyc, iters, got);
        const bool same_vm = !memcmp(ref, got, 256);
        const double d = run_filt(1, true, din, dout, dcyc, iters, got);
        printf("filter cycles per edge step: sgpr-mask full %.1f half %.1f | vgpr-mask full %.1f half %.1f"
               "  (half-exec results %s, vgpr-mask results %s)\n",
               a, b, c, d, same_half ? "same" : "DIFFER", same_vm ? "same" : "DIFFER");
        unsigned long long cyc = 0;
        k_lds<false><<<1, 64>>>(dout, dcyc, iters);
        hipMemcpy(&cyc, dcyc, 8, hipMemcpyDeviceToHost);
        const double lf = (double)cyc / iters;
        k_lds<true><<<1, 64>>>(dout, dcyc, iters);
        hipMemcpy(&cyc, dcyc, 8, hipMemcpyDeviceToHost);
        printf("H transposition (20 ds_read_u8 + 18 ds_write_b8): full exec %.0f cycles, half exec %.0f cycles\n", lf,
               (double)cyc / iters);
    }
    return 0;
}
