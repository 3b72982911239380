// Residency census: how many workgroups of a k_wgpp-shaped kernel (320
// threads = 5 waves, 46,608 B of LDS, 128 VGPRs) are resident per CU at once.
// Every workgroup arrives (one atomic add), then waits until all NWG have
// arrived or ~200 us pass; a workgroup that arrived before the deadline
// while the others were still resident counts as co-resident.  Printed: how
// many arrived within the first 100 us, and the per-CU histogram.
//   census [threads] [lds_bytes] [live floats per lane: 112 | 88 | 72]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <map>

__device__ __forceinline__ unsigned long long wclk() { return __builtin_amdgcn_s_memrealtime(); }

template <int T, int NV>
__global__ __launch_bounds__(T) __attribute__((amdgpu_waves_per_eu(4))) void census(unsigned *cnt, unsigned *info,
                                                                                   int total, float seed)
{
    extern __shared__ float lds[];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    // register pressure: ~120 live VGPRs per lane
    float v[NV];
#pragma unroll
    for (int i = 0; i < NV; i++) v[i] = seed * (float)(i + lane);
#pragma unroll
    for (int i = 0; i < NV; i++) asm volatile("" : "+v"(v[i]));
    lds[threadIdx.x] = v[0];
    __syncthreads();
    unsigned long long t0 = wclk();
    unsigned order = 0;
    if (threadIdx.x == 0) {
        order = atomicAdd(cnt, 1u);
        info[blockIdx.x * 4 + 0] = order;
        info[blockIdx.x * 4 + 1] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
        info[blockIdx.x * 4 + 2] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);
        info[blockIdx.x * 4 + 3] = (unsigned)t0;
    }
    // wait for everyone (bounded: 100 MHz clock, 20000 ticks = 200 us)
    if (wid == 0) {
        while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)total &&
               wclk() - t0 < 20000)
            __builtin_amdgcn_s_sleep(8);
    }
    __syncthreads();
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < NV; i++) acc += v[i];
    if (acc == 1234.5f) info[0] = 0;
}

int main(int argc, char **argv)
{
    const int T = argc > 1 ? atoi(argv[1]) : 320;
    const int lds = argc > 2 ? atoi(argv[2]) : 46608;
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess) return 1;
    const int total = 3 * ncu;
    unsigned *cnt, *info;
    if (hipMalloc(&cnt, 4) != hipSuccess || hipMalloc(&info, total * 16) != hipSuccess) return 1;
    if (hipMemset(cnt, 0, 4) != hipSuccess || hipMemset(info, 0, total * 16) != hipSuccess) return 1;
    const int nv = argc > 3 ? atoi(argv[3]) : 112;
    int occ = 0;
#define RUN(TT, NN)                                                                                      \
    if (T == TT && nv == NN) {                                                                           \
        hipLaunchKernelGGL((census<TT, NN>), dim3(total), dim3(TT), lds, 0, cnt, info, total, 1.0f);     \
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, census<TT, NN>, TT, lds);               \
    }
    RUN(320, 112) RUN(320, 88) RUN(320, 72) RUN(256, 112) RUN(384, 112) RUN(512, 112)
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    unsigned *h = (unsigned *)malloc(total * 16);
    if (hipMemcpy(h, info, total * 16, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    unsigned tmin = ~0u;
    for (int i = 0; i < total; i++) tmin = h[i * 4 + 3] < tmin ? h[i * 4 + 3] : tmin;
    int early = 0;
    std::map<unsigned, int> per_cu;
    for (int i = 0; i < total; i++) {
        if (h[i * 4 + 3] - tmin < 10000) {   // arrived within 100 us of the first
            early++;
            const unsigned hw = h[i * 4 + 1], xcc = h[i * 4 + 2] & 15;
            per_cu[(xcc << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15)]++;
        }
    }
    std::map<int, int> hist;
    for (auto &kv : per_cu) hist[kv.second]++;
    printf("threads %d lds %d nv %d: occupancy API %d/CU, %d of %d workgroups resident within 100 us, %zu CUs;",
           T, lds, nv, occ, early, total, per_cu.size());
    for (auto &kv : hist) printf(" %d CUs x %d", kv.second, kv.first);
    printf("\n");
    return 0;
}
