// H.264 Baseline macroblock reconstruction + in-loop deblocking for gfx950.
//
// Two kernels per picture batch (one picture from each of S streams):
//   k_prep  -- every MB of the batch, fully parallel (one wave per MB): the
//              work that reads no reconstructed sample -- the deblocking
//              record (bS of the 32 4x4 edge segments + alpha/beta/tc0/indexA
//              per edge class; GetBoundaryStrengths / thresholds,
//              deblocking.c:1134-1532) and the residual (dequant + 4x4 IDCT +
//              luma/chroma DC transforms, transform.c:94-398) with the
//              reference's [-512,511] range check.
//   k_wgpp  -- one workgroup per (picture, MB row): three MC waves walk the
//              row's MBs (6-tap luma / bilinear chroma MC from the
//              HBM-resident reference slots, reconstruct.c:1819-2314; intra
//              4x4 / 16x16 / chroma / I_PCM from unfiltered neighbours,
//              intra_prediction.c:475-988; clip-add) into an LDS ring; two
//              ping-pong row waves deblock the row in the reference's
//              raster-equivalent order (h264bsdFilterPicture,
//              deblocking.c:574-1736) and hand the final bottom rows to the
//              row below through tagged-granule mailboxes.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../../include/h264mi_records.h"

#define WAVE 64
// profiling build: u64 stamps per MB (row waves [0..2], MC [3], intra [4..5])
#define PROF_MB 8

struct ReconArgs {
    uint8_t *frames;          // frame pool (I420 per slot, chroma rows cpitch apart: H264MI_CPITCH)
    unsigned long long frame_bytes;     // slot stride (H264MI_SLOT_BYTES)
    int cpitch;               // chroma row pitch (bytes)
    const MbRec *rec;         // batch records (pictures back to back)
    const int16_t *coef;      // batch coefficient blocks
    const PicDesc *pics;
    int npics;
    int w, h;                 // picture size in MBs
    uint8_t *dbrec;           // 64 B deblocking record per MB of the batch
    int16_t *res;             // 384 residual samples per MB (intra MBs only)
    unsigned int *err;        // per picture: bit0 residual range error, bit1/2/4 bounded-wait timeouts
    unsigned long long *mbx;  // row mailboxes: 32 tagged granules per MB of the batch
    unsigned int epoch;       // launch counter != 0: granule tag (no reset between launches)
    unsigned long long *prof; // optional per-MB chain stamps (profiling k_wgpp)
    int S;                    // pictures (streams) of the batch
    unsigned long long *gjunk; // 64 KiB sink: 128 x 64 granules for lanes with nothing to store
    // tail workgroups (blockIdx >= S * h): k_prep of the NEXT batch, started
    // once *rows_done (row workgroups finished, all launches) >= prep_target
    int prep_wgs;
    unsigned long long *rows_done;
    unsigned long long prep_target;
    const MbRec *n_rec;
    const int16_t *n_coef;
    const PicDesc *n_pics;
    uint8_t *n_dbrec;
    int16_t *n_res;
    int n_nmbs_total;
    // frame-pipelined launches (P > 1): the launch holds P consecutive
    // pictures of each of the S streams, step-major (picture p = j * S + s);
    // step j's MC reads of a slot written by step j - k of the same launch
    // wait until the lines they read are final there: DEP_ROWS by whole MB
    // rows (done tags), DEP_COLS by (MB row, MB column) through the store
    // progress granules PROG_AT(prog, p - k * S, h, r, w) = {MBs of row wave
    // w's parity stored, epoch} (row_pp, dep_wait_cols)
    int P;
    unsigned long long *prog;
    // DEP_ROWS launches: one u32 per (picture, MB row), epoch once the row is
    // final in its slot (row workgroup r after its frame stores and an agent
    // release; chained: step j's row r only after step j - 1's)
    unsigned int *done;
    // profiling build only: 1 = the row waves only drain the MC ring (no
    // deblocking, no stores) -- SQ counters of such a launch minus those of
    // a normal one split the instruction counts by wave role (tools/sq_roles.py)
    int prof_mode;
    // how far (MBs) a row's MC waves may run ahead of its deblocking: lead0
    // until the row's chain has taken its first MB, lead after that; 0 = the
    // ring depth (H264MI_MC_LEAD0 / H264MI_MC_LEAD, engine.hip)
    int mc_lead0, mc_lead;
    // study knob (H264MI_ROW_PRIO=1): row waves at s_setprio 1 outside the
    // chain (slot waits, copy-in, frame stores) and 3 on it (hdone wait ..
    // publish); 0 = 3 throughout
    int row_prio_split;
    int mc_urgency;          // MBs ahead of the row's deblocking under which MC waves issue at prio 2 (2-MC shape)
    int mc_top;              // MB rows r < mc_top: urgent MC waves issue at prio 3 (the row waves' level)
    // dependency-checker builds (k_wgpp<..., CHK = true>): test hook that
    // deliberately breaks one hand-off so the tests can see the checker fire
    // (0: none; 1: MB 5 of every row hands the row waves a wrong ring tag)
    int chk_inject;
    // (frame-pipelined CHK launches) test hooks: dep_wait waits for this many
    // MB columns / rows less than the loads need, which CHK_REFROW must catch
    int chk_short_cols, chk_short_rows;

};

// Dependency checker (the reference's compile-time
// _ASSERT_USED / _RANGE_CHECK knobs, h264bsd_util.h:35-123): in the CHK
// instantiations of k_wgpp every hand-off is verified at the consumer, each
// kind of violation setting its own bit of the picture's error word:
//   CHK_RING    the MC ring slot the row waves read holds another MB's data
//   CHK_RING_WR an MC wave writes a slot the row waves have not released
//   CHK_REGION  the partner row wave's region holds another MB than the one
//               whose H pass its hdone announced
//   CHK_PROG    an intra progress word names another MB than the left one
//   CHK_REFROW  (frame-pipelined launches) a reference line is read from a
//               picture of the same launch before every (MB row, MB column)
//               holding a byte of it was published final -- checks the
//               host's set_ref_rows against the loads' own geometry
// The checker's MB tags ride in bytes 22..23 of the 64-B deblocking record
// (class 0's threshold entry {alpha, beta, tc0[3], indexA} leaves them
// unused): the MC wave writes MB c's index there with the record it puts in
// the ring slot; the row wave's copy-in carries it into its region.  No LDS
// layout changes for the normal kernels.
#define CHK_TAG_OFF 22
// frame-pipelined launches: store-progress granules, one 128-B line per
// (picture, MB row, row wave), so that a line is rewritten only by its own
// wave and polls between two publishes hit the L2 (a line the granules of
// eight rows shared was rewritten every ~0.3 us: every poll went to memory)
#ifndef PROG_STRIDE
#define PROG_STRIDE 16          // u64 per row wave
#endif
#define PROG_AT(base, pic, h, r, w) ((base) + (((size_t)(pic) * (h) + (r)) * 2 + (w)) * PROG_STRIDE)
// DEP_COLS finality rule, the one place it is stated (dep_rows_ok waits on
// it, chk_access checks the loads against it).  It follows row_pp's store
// map: MB x of row R is final once row R has stored MBs 0..x + DEPC_SAME_ROW - 1
// (MB x + 1 stores MB x's columns 12..15 after its left edge) and row R + 1
// MBs 0..x + DEPC_ROW_BELOW - 1 (MB (R + 1, x) stores row R's rows 12..15
// after its top edge).  Where row_pp stores less late -- MB x's own rows
// 12..15 when the MB below filters no top edge (top_on), whole MBs in
// row_drain -- the rule is conservative.  A store moved later in row_pp must
// move these.
#define DEPC_SAME_ROW 2
#define DEPC_ROW_BELOW 1
// a row wave publishes its progress every PROG_EVERY of its MBs
#ifndef PROG_EVERY
#define PROG_EVERY 2
#endif
#define CHK_RING    64u
#define CHK_RING_WR 128u
#define CHK_REGION  256u
#define CHK_PROG    512u
#define CHK_REFROW  1024u
#define CHK_NODB    2048u   // a PD_NO_DEBLOCK picture holds an MB that filters (row_drain)

__constant__ uint8_t cZigzag[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
__constant__ uint8_t cLevelScale[6][3] = {
    {10, 16, 13}, {11, 18, 14}, {13, 20, 16}, {14, 23, 18}, {16, 25, 20}, {18, 29, 23}};
__constant__ uint8_t cAlpha[52] = {
    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 4, 4, 5, 6, 7, 8, 9, 10,
    12, 13, 15, 17, 20, 22, 25, 28, 32, 36, 40, 45, 50, 56, 63, 71, 80, 90,
    101, 113, 127, 144, 162, 182, 203, 226, 255, 255};
__constant__ uint8_t cBeta[52] = {
    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 2, 2, 3, 3, 3, 3, 4,
    4, 4, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13, 14, 14,
    15, 15, 16, 16, 17, 17, 18, 18};
__constant__ uint8_t cTc0[52][3] = {
    {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0},
    {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0},
    {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 1}, {0, 0, 1}, {0, 0, 1}, {0, 0, 1},
    {0, 1, 1}, {0, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 1, 2},
    {1, 1, 2}, {1, 1, 2}, {1, 1, 2}, {1, 2, 3}, {1, 2, 3}, {2, 2, 3}, {2, 2, 4},
    {2, 3, 4}, {2, 3, 4}, {3, 3, 5}, {3, 4, 6}, {3, 4, 6}, {4, 5, 7}, {4, 5, 8},
    {4, 6, 9}, {5, 7, 10}, {6, 8, 11}, {6, 8, 13}, {7, 10, 14}, {8, 11, 16},
    {9, 12, 18}, {10, 13, 20}, {11, 15, 23}, {13, 17, 25}};

// Per-wave register tables: lane i holds entry i, looked up with
// ds_bpermute (an LDS-crossbar lane shuffle: LDS latency, no VMEM).  A
// per-lane index into a __constant__ array would be a VMEM load, and since
// vmcnt retires in order, waiting for it would also wait for every
// reference-window load issued before it.  Lookups run with all lanes active.
struct Tabs {
    uint32_t ab;    // lane i < 52: alpha[i] | beta[i] << 8 | tc0[i][0] << 16 | tc0[i][1] << 24
    uint32_t c2;    // lane i < 52: tc0[i][2]
    uint32_t ls;    // lane i < 18: levelScale[i / 3][i % 3]
};
__device__ __forceinline__ Tabs load_tabs(int lane)
{
    Tabs t;
    const int i = lane < 52 ? lane : 0;
    t.ab = cAlpha[i] | (uint32_t)cBeta[i] << 8 | (uint32_t)cTc0[i][0] << 16 | (uint32_t)cTc0[i][1] << 24;
    t.c2 = cTc0[i][2];
    t.ls = lane < 18 ? cLevelScale[lane / 3][lane % 3] : 0;
    return t;
}
__device__ __forceinline__ uint32_t tab_at(uint32_t reg, int idx)
{
    return (uint32_t)__builtin_amdgcn_ds_bpermute(idx << 2, (int)reg);
}

// ordering of LDS traffic between the lanes of one wave
// A wave's LDS instructions execute in issue order, so lanes of one wave see
// each other's LDS writes once the compiler keeps program order: a compiler
// barrier is enough (no s_waitcnt, which would also drain in-flight global
// prefetches because vmcnt retires in order).
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

// write-through (sc1) stores and L1-bypassing loads for data another CU
// consumes within the same launch (MI355X_MICROARCH.md, inter-workgroup
// visibility, table row 1)
__device__ __forceinline__ uint32_t ld_sc1_u32(const uint32_t *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_sc1_u32(uint32_t *p, uint32_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
template <bool SC1> __device__ __forceinline__ uint32_t ld32(const void *p)
{
    return SC1 ? ld_sc1_u32((const uint32_t *)p) : *(const uint32_t *)p;
}
template <bool SC1> __device__ __forceinline__ void st32(void *p, uint32_t v)
{
    if (SC1) st_sc1_u32((uint32_t *)p, v);
    else *(uint32_t *)p = v;
}
// pin a uniform pointer to SGPRs, so that base[32-bit lane offset] becomes a
// saddr access (no per-lane 64-bit address arithmetic)
// (global address space kept explicit: a generic pointer would turn the
// access into a FLAT one, counted by lgkmcnt as well)
typedef const __attribute__((address_space(1))) uint8_t *gcu8p;
__device__ __forceinline__ gcu8p uni(const void *p)
{
    gcu8p g = (gcu8p)p;
    asm volatile("" : "+s"(g));
    return g;
}
__device__ __forceinline__ uint32_t ldg32(gcu8p base, uint32_t off)
{
    return *(const __attribute__((address_space(1))) uint32_t *)(base + off);
}
__device__ __forceinline__ void drain_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ int clip255(int v) { return min(max(v, 0), 255); }
__device__ __forceinline__ int clip3(int lo, int hi, int v) { return min(max(v, lo), hi); }
__device__ __forceinline__ int blk_x(int b) { return ((b >> 2) & 1) * 2 + (b & 1); }
__device__ __forceinline__ int blk_y(int b) { return ((b >> 3) & 1) * 2 + ((b >> 1) & 1); }
__device__ __forceinline__ int blk_of(int x4, int y4) { return ((y4 >> 1) * 2 + (x4 >> 1)) * 4 + (y4 & 1) * 2 + (x4 & 1); }

// ---------------------------------------------------------------------------
// residual: dequant + inverse transforms (transform.c:94-398) for one MB.
// Residual hand-off k_prep -> k_wgpp, compact: only the 4x4 blocks that can
// carry a residual travel, 32 B each, in cbits bit order, from the start of
// the MB's 768-B slot.  res_mask: AC-coded blocks plus every block of a plane
// whose DC transform is coded (I16 luma DC, chroma DC of that plane).
__device__ __forceinline__ uint32_t res_mask(int type, uint32_t cbits)
{
    uint32_t m = cbits & 0xFFFFFFu;
    if (type == MBT_I16 && ((cbits >> 24) & 1)) m |= 0xFFFFu;
    if ((cbits >> 25) & 1) m |= 0xF0000u;
    if ((cbits >> 26) & 1) m |= 0xF00000u;
    return m;
}

// res: the MB's compact residual slot (global, res_mask blocks in bit order,
// 16 raster int16 each).  dc: LDS int32[24].
// Returns (through *err) a nonzero flag if a sample leaves [-512,511].
// ---------------------------------------------------------------------------
// base: the MB's coded blocks in cbits order (staged in LDS by the caller).
// ls: the levelScale register table (Tabs::ls).
__device__ void mb_residual(const MbRec &r, const int16_t *base, int16_t *res,
                            int32_t *dc, int lane, int *range_err, uint32_t ls, uint32_t m)
{
    const uint32_t cb = r.cbits;
    const bool i16 = r.type == MBT_I16;
    // levelScale lookups (all lanes active): luma DC scale, chroma DC scale,
    // and this lane's three AC scales (luma lanes qp, chroma lanes qpc)
    const int qp_l = r.qp, qp_c = r.qpc;
    const int ls_ldc = (int)tab_at(ls, (qp_l % 6) * 3), ls_cdc = (int)tab_at(ls, (qp_c % 6) * 3);
    const int qm_mine = (lane < 16 ? qp_l : qp_c) % 6;
    const int ls_ac0 = (int)tab_at(ls, qm_mine * 3), ls_ac1 = (int)tab_at(ls, qm_mine * 3 + 1),
              ls_ac2 = (int)tab_at(ls, qm_mine * 3 + 2);
    if (lane < 16) {
        int32_t v = 0;
        if (i16 && (cb & (1u << 24))) {
            const int16_t *d = base + __popc(cb & 0xFFFFFFu) * 16;
            const int i = lane >> 2, j = lane & 3;
            // f = A c A with A = [[1,1,1,1],[1,1,-1,-1],[1,-1,-1,1],[1,-1,1,-1]]:
            // A[i][k] = (-1)^popcount(k & m(i)), m = {0, 2, 3, 1}
            const int mi = i == 1 ? 2 : i == 2 ? 3 : i == 3 ? 1 : 0;
            const int mj = j == 1 ? 2 : j == 2 ? 3 : j == 3 ? 1 : 0;
            int32_t s = 0;
#pragma unroll
            for (int sp = 0; sp < 16; sp++) {
                const int rr = sp == 0 ? 0 : sp == 1 ? 1 : sp == 2 ? 4 : sp == 3 ? 8 : sp == 4 ? 5 : sp == 5 ? 2 :
                               sp == 6 ? 3 : sp == 7 ? 6 : sp == 8 ? 9 : sp == 9 ? 12 : sp == 10 ? 13 :
                               sp == 11 ? 10 : sp == 12 ? 7 : sp == 13 ? 11 : sp == 14 ? 14 : 15;
                const int neg = (__popc((rr >> 2) & mi) + __popc((rr & 3) & mj)) & 1;
                s += neg ? -(int32_t)d[sp] : (int32_t)d[sp];
            }
            const int q6 = r.qp / 6;
            const int32_t x = s * ls_ldc;
            v = q6 >= 2 ? x << (q6 - 2) : ((x << q6) + 2) >> 2;
        }
        dc[lane] = v;
    } else if (lane < 24) {
        const int comp = (lane - 16) >> 2, b = (lane - 16) & 3;
        int32_t f = 0;
        const uint32_t bit = 1u << (25 + comp);
        if (cb & bit) {
            const int16_t *d = base + __popc(cb & (bit - 1)) * 16;
            const int32_t c0 = d[0], c1 = d[1], c2 = d[2], c3 = d[3];
            f = b == 0 ? c0 + c1 + c2 + c3 : b == 1 ? c0 - c1 + c2 - c3 : b == 2 ? c0 + c1 - c2 - c3 : c0 - c1 - c2 + c3;
            f = ((f * ls_cdc) << (r.qpc / 6)) >> 1;
        }
        dc[lane] = f;
    }
    wave_sync();
    if (lane < 24) {
        const bool luma = lane < 16;
        const int qp = luma ? r.qp : r.qpc;
        const int q6 = qp / 6, qm = qp % 6;
        int32_t d[16];
#pragma unroll
        for (int i = 0; i < 16; i++) d[i] = 0;
        bool nz = false;
        const uint32_t bit = 1u << lane;
        if (cb & bit) {
            const int16_t *c = base + __popc(cb & (bit - 1)) * 16;
            const bool skip0 = !luma || i16;
#pragma unroll
            for (int s = 0; s < 16; s++) {
                // raster position of scan position s (compile-time)
                const int rr = s == 0 ? 0 : s == 1 ? 1 : s == 2 ? 4 : s == 3 ? 8 : s == 4 ? 5 : s == 5 ? 2 :
                               s == 6 ? 3 : s == 7 ? 6 : s == 8 ? 9 : s == 9 ? 12 : s == 10 ? 13 :
                               s == 11 ? 10 : s == 12 ? 7 : s == 13 ? 11 : s == 14 ? 14 : 15;
                const int cls = (!(rr & 1) && !((rr >> 2) & 1)) ? 0 : (((rr & 1) && ((rr >> 2) & 1)) ? 1 : 2);
                if (s == 0 && skip0) continue;
                d[rr] = (int32_t)c[s] * ((cls == 0 ? ls_ac0 : cls == 1 ? ls_ac1 : ls_ac2) << q6);
            }
            nz = true;
        }
        if (luma) {
            if (i16) { d[0] = dc[blk_y(lane) * 4 + blk_x(lane)]; nz |= d[0] != 0; }
        } else {
            d[0] = dc[lane];
            nz |= d[0] != 0;
        }
        int32_t o[16];
        if (nz) {
            int32_t t[16];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int32_t a = d[4 * i] + d[4 * i + 2], b = d[4 * i] - d[4 * i + 2];
                const int32_t c = (d[4 * i + 1] >> 1) - d[4 * i + 3], e = d[4 * i + 1] + (d[4 * i + 3] >> 1);
                t[4 * i] = a + e; t[4 * i + 1] = b + c; t[4 * i + 2] = b - c; t[4 * i + 3] = a - e;
            }
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int32_t a = t[j] + t[8 + j], b = t[j] - t[8 + j];
                const int32_t c = (t[4 + j] >> 1) - t[12 + j], e = t[4 + j] + (t[12 + j] >> 1);
                o[j] = (a + e + 32) >> 6; o[4 + j] = (b + c + 32) >> 6;
                o[8 + j] = (b - c + 32) >> 6; o[12 + j] = (a - e + 32) >> 6;
            }
            bool bad = false;
#pragma unroll
            for (int i = 0; i < 16; i++) bad |= (o[i] < -512) | (o[i] > 511);
            if (bad) *range_err = 1;
        } else {
#pragma unroll
            for (int i = 0; i < 16; i++) o[i] = 0;
        }
        // compact hand-off: the block's 16 samples (raster) at its rank
        // among the MB's res_mask blocks, 32 B straight from registers
        if ((m >> lane) & 1) {
            uint32_t w[8];
#pragma unroll
            for (int i = 0; i < 8; i++) w[i] = ((uint32_t)o[2 * i] & 0xFFFFu) | ((uint32_t)o[2 * i + 1] << 16);
            uint4 *q = (uint4 *)(res + __popc(m & ((1u << lane) - 1)) * 16);
            q[0] = make_uint4(w[0], w[1], w[2], w[3]);
            q[1] = make_uint4(w[4], w[5], w[6], w[7]);
        }
    }
}

// ---------------------------------------------------------------------------
// inter prediction (h264bsdPredictSamples, reconstruct.c:1819-1941): luma
// 6-tap from a 9x9 window per 4x4 block (the 16 positions of
// h264bsdInterpolate*, :1004-1381), chroma bilinear from a 3x3 window per
// 2x2 block (h264bsdInterpolateChromaHorVer and friends, :302-404).
//
// Packed arithmetic (round 6): four samples travel as the bytes of one
// dword, two intermediate values as the 16-bit halves of one (v_pk_*_i16),
// and the 6-tap sums are dot products:
//   - horizontal half samples b of a row: v_dot4_i32_i8 of the row's bytes
//     (biased by ^0x80 into int8; sum of taps 32 -> +4096) with the taps
//     shifted to each output column, 9 dot products for 4 outputs;
//   - vertical 6-tap sums V of columns 0..8 over the lane's six window rows:
//     one v_pk_mad_i16 chain per column pair (u8 pairs from v_perm_b32);
//   - centre j = the horizontal 6-tap over V (exact: the filter is linear),
//     v_dot2_i32_i16 on the column pairs, 3-4 per output;
//   - every output is (A + B + 1) >> 1 of two of {G, b, h, j} (A = B for
//     the full / half positions): one v_lerp_u8 for the lane's four samples.
// What no lane of the wave needs (b of row +0 / +1, h of column +0 / +1, j)
// is skipped wave-uniformly: most inter MBs carry one MV (skip, 16x16), so
// their waves compute one or two candidates.
// ---------------------------------------------------------------------------
typedef short s2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ s2v s2of(uint32_t x) { return __builtin_bit_cast(s2v, x); }
__device__ __forceinline__ uint32_t uof(s2v x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) { return __builtin_amdgcn_perm(hi, lo, sel); }
// two 16-bit lanes clipped to [0, 255] (v_pk_max_i16, v_pk_min_i16)
__device__ __forceinline__ s2v clip_pk(s2v v)
{
    return __builtin_elementwise_min(__builtin_elementwise_max(v, (s2v){0, 0}), (s2v){255, 255});
}
// the low bytes of two clipped pairs -> four bytes (lo.x, lo.y, hi.x, hi.y)
__device__ __forceinline__ uint32_t pack4(s2v lo, s2v hi) { return perm(uof(hi), uof(lo), 0x06040200u); }
// four clipped int32 -> four bytes
__device__ __forceinline__ uint32_t pack4i(int a, int b, int c, int d)
{
    return perm(perm((uint32_t)d, (uint32_t)c, 0x0C0C0400u), perm((uint32_t)b, (uint32_t)a, 0x0C0C0400u), 0x05040100u);
}
constexpr uint32_t w4(int a, int b, int c, int d)
{
    return (uint32_t)(a & 255) | (uint32_t)(b & 255) << 8 | (uint32_t)(c & 255) << 16 | (uint32_t)(d & 255) << 24;
}
constexpr uint32_t w2(int a, int b) { return (uint32_t)(a & 0xFFFF) | (uint32_t)(b & 0xFFFF) << 16; }
__device__ __forceinline__ int sdot4(uint32_t a, uint32_t b, int c) { return __builtin_amdgcn_sdot4((int)a, (int)b, c, false); }
__device__ __forceinline__ int sdot2(s2v a, uint32_t b, int c) { return __builtin_amdgcn_sdot2(a, s2of(b), c, false); }

// b of output columns 0..3 of one window row (bytes = columns 0..8, x..z):
// clip((tap6(col x .. x+5) + 16) >> 5), four bytes
__device__ __forceinline__ uint32_t hb4(uint32_t x, uint32_t y, uint32_t z)
{
    const uint32_t X = x ^ 0x80808080u, Y = y ^ 0x80808080u, Z = z ^ 0x80808080u;
    const int k = 4096 + 16;            // 128 * (sum of taps) + rounding
    const int b0 = sdot4(X, w4(1, -5, 20, 20), sdot4(Y, w4(-5, 1, 0, 0), k));
    const int b1 = sdot4(X, w4(0, 1, -5, 20), sdot4(Y, w4(20, -5, 1, 0), k));
    const int b2 = sdot4(X, w4(0, 0, 1, -5), sdot4(Y, w4(20, 20, -5, 1), k));
    const int b3 = sdot4(X, w4(0, 0, 0, 1), sdot4(Y, w4(-5, 20, 20, -5), sdot4(Z, w4(1, 0, 0, 0), k)));
    return pack4i(clip255(b0 >> 5), clip255(b1 >> 5), clip255(b2 >> 5), clip255(b3 >> 5));
}

// one lane's four luma samples: row yy of 4x4 block b at fractional position
// (fx, fy); R[i] = window row yy + i (bytes = columns 0..8).  Returns them
// as four bytes (before the residual).  nb2 / nb3 / nh / nhx / nj: wave-
// uniform, some lane needs b of row 2 / row 3, h of columns 2..5 / 3..6, j.
__device__ __forceinline__ uint32_t luma_pred4(const uint4 (&R)[6], int fx, int fy, bool nb2, bool nb3, bool nh,
                                               bool nhx, bool nj)
{
    const uint32_t G2 = __builtin_amdgcn_alignbyte(R[2].y, R[2].x, 2u);     // row 2, columns 2..5
    const uint32_t G2x = __builtin_amdgcn_alignbyte(R[2].y, R[2].x, 3u);    // row 2, columns 3..6
    const uint32_t G3 = __builtin_amdgcn_alignbyte(R[3].y, R[3].x, 2u);     // row 3, columns 2..5
    uint32_t B2 = 0, B3 = 0, Hc = 0, Hx = 0, J = 0;
    if (nb2) B2 = hb4(R[2].x, R[2].y, R[2].z);
    if (nb3) B3 = hb4(R[3].x, R[3].y, R[3].z);
    if (nh || nhx || nj) {
        // V of column pairs (0,1) (2,3) (4,5) (6,7) (8,-) over rows 0..5
        s2v V[5];
#pragma unroll
        for (int m = 0; m < 5; m++) {
            if (!nj && (m == 0 || m == 4)) { V[m] = (s2v){0, 0}; continue; }
            s2v P[6];
#pragma unroll
            for (int i = 0; i < 6; i++) {
                const uint32_t src = m < 2 ? R[i].x : m < 4 ? R[i].y : R[i].z;
                P[i] = s2of(m == 4 ? (src & 255u) : perm(0u, src, (m & 1) ? 0x0C030C02u : 0x0C010C00u));
            }
            V[m] = (P[0] + P[5]) + (P[2] + P[3]) * (short)20 - (P[1] + P[4]) * (short)5;
        }
        if (nh || nhx) {
            const s2v h1 = clip_pk((V[1] + (short)16) >> (short)5), h2 = clip_pk((V[2] + (short)16) >> (short)5);
            Hc = pack4(h1, h2);
            if (nhx) {
                const s2v h3 = clip_pk((V[3] + (short)16) >> (short)5);
                Hx = __builtin_amdgcn_alignbyte(uof(h3), Hc, 1u);
            }
        }
        if (nj) {
            const int j0 = sdot2(V[0], w2(1, -5), sdot2(V[1], w2(20, 20), sdot2(V[2], w2(-5, 1), 512)));
            const int j1 = sdot2(V[0], w2(0, 1), sdot2(V[1], w2(-5, 20), sdot2(V[2], w2(20, -5), sdot2(V[3], w2(1, 0), 512))));
            const int j2 = sdot2(V[1], w2(1, -5), sdot2(V[2], w2(20, 20), sdot2(V[3], w2(-5, 1), 512)));
            const int j3 = sdot2(V[1], w2(0, 1), sdot2(V[2], w2(-5, 20), sdot2(V[3], w2(20, -5), sdot2(V[4], w2(1, 0), 512))));
            J = pack4i(clip255(j0 >> 10), clip255(j1 >> 10), clip255(j2 >> 10), clip255(j3 >> 10));
        }
    }
    // the position's two operands (8.4.2.2.1, equations 8-250 .. 8-261)
    const bool fx0 = fx == 0, fy0 = fy == 0, half = fx == 2 || fy == 2;
    const uint32_t bs = fy == 3 ? B3 : B2, hs = fx == 3 ? Hx : Hc;
    uint32_t A, B;
    if (fx0 && fy0) { A = G2; B = G2; }
    else if (fy0) { A = B2; B = fx == 1 ? G2 : fx == 2 ? B2 : G2x; }
    else if (fx0) { A = Hc; B = fy == 1 ? G2 : fy == 2 ? Hc : G3; }
    else if (half) { A = J; B = (fx == 2 && fy == 2) ? J : (fy == 2 ? hs : bs); }
    else { A = bs; B = hs; }
    return __builtin_amdgcn_lerp(A, B, 0x01010101u);       // (A + B + 1) >> 1 per byte
}

// ---------------------------------------------------------------------------
// intra prediction tiles (intra_prediction.c, per MC wave in LDS): the MB's
// samples with a one-sample halo, every 4-sample group dword-aligned.  Luma
// sample (x, y) at ty[(y + 1) * TY_STRIDE + TX0 + x]; the left neighbour
// column at TX0 - 1; the row above in row 0 (top-left at TX0 - 1, top-right
// at TX0 + 16..19).  Chroma alike with TC_STRIDE (no top-right).
// ---------------------------------------------------------------------------
#define TY_STRIDE 24
#define TC_STRIDE 12
#define TX0 4

__device__ __forceinline__ int bs_of(const MbRec &p, int bp, const MbRec &q, int bq, bool mb_edge)
{
    if ((p.type >= MBT_I4x4) | (q.type >= MBT_I4x4) | (((p.dbf | q.dbf) & DBF_INTRA) != 0)) return mb_edge ? 4 : 3;
    if (((p.cbits >> bp) & 1) | ((q.cbits >> bq) & 1)) return 2;
    if (p.ref[bp >> 2] != q.ref[bq >> 2]) return 1;
    if (abs(p.mv[bp][0] - q.mv[bq][0]) >= 4 || abs(p.mv[bp][1] - q.mv[bq][1]) >= 4) return 1;
    return 0;
}

// ---------------------------------------------------------------------------
// deblocking record (computed by k_prep, consumed by k_wgpp): 64 B per MB
//   [0..15]  bS nibbles, index (dir*16 + seg*4 + edge): dir 0 = vertical edges;
//            the four edges crossed by one line are one 16-bit word
//   [16..63] 8 bytes per (plane*3 + class), plane 0 luma / 1 chroma, class
//            0 internal / 1 left MB edge / 2 top MB edge:
//            {alpha, beta, tc0(bS=1), tc0(bS=2), tc0(bS=3), indexA, 0, 0}
// Reference: GetBoundaryStrengths deblocking.c:1134-1370,
// GetLumaEdgeThresholds :1381-1449, GetChromaEdgeThresholds :1460-1532.
// ---------------------------------------------------------------------------
// computes the record into s_db (LDS, 64 B)
// Deblocking record of MB gmb (GetBoundaryStrengths, deblocking.c:1134-1370;
// thresholds :1381-1532).  The MB's record and its left / top neighbours'
// are staged in LDS (srec, 72 dwords) by one coalesced load per lane, so the
// per-lane bS decisions read LDS instead of issuing dependent global loads;
// the threshold-table loads are issued before the bS work.  srec is staged
// by the caller (stage_recs_load).
// the MB's, left and top records in LDS (srec: dwords 0..23, 24..47, 48..71)
__device__ void mb_dbrec(int lane, uint8_t *s_db, const uint32_t *srec, const Tabs &T)
{
    const MbRec *Q = (const MbRec *)srec;
    const bool fl = Q->avail & DB_LEFT, ft = Q->avail & DB_TOP;
    // thresholds: lanes 32..37 = luma classes 0..2 (internal, left, top), chroma 3..5
    const int k = lane - 32;
    const bool thr = k >= 0 && k < 6;
    const bool chroma = k >= 3;
    const int cls = chroma ? k - 3 : k;
    const MbRec *PN = (const MbRec *)(srec + ((cls == 1 && fl) ? 24 : (cls == 2 && ft) ? 48 : 0));
    const int qpp = chroma ? PN->qpc : PN->qp, qq = chroma ? Q->qpc : Q->qp;
    const int qpav = (qpp + qq + 1) >> 1;
    const int ia = clip3(0, 51, qpav + Q->offA), ib = clip3(0, 51, qpav + Q->offB);
    const uint32_t wa = tab_at(T.ab, ia), wb = tab_at(T.ab, ib), t2 = tab_at(T.c2, ia);
    const uint32_t al = wa & 255, be = (wb >> 8) & 255, t0 = (wa >> 16) & 255, t1 = wa >> 24;
    // bS: lanes 0..31 = (dir, line segment kk, edge e)
    int bS = 0;
    {
        const int dir = (lane >> 4) & 1, kk = (lane >> 2) & 3, e = lane & 3;
        const bool on = lane < 32 && (Q->avail & DB_INNER) && (e > 0 || (dir == 0 ? fl : ft));
        if (on) {
            const MbRec &pm = *(const MbRec *)(srec + (e > 0 ? 0 : dir == 0 ? 24 : 48));
            const int bq = dir == 0 ? blk_of(e, kk) : blk_of(kk, e);
            const int bp = e == 0 ? (dir == 0 ? blk_of(3, kk) : blk_of(kk, 3))
                                  : (dir == 0 ? blk_of(e - 1, kk) : blk_of(kk, e - 1));
            bS = bs_of(pm, bp, *Q, bq, e == 0);
        }
    }
    // pack two nibbles per byte: even lane owns the low nibble
    const int hi = __shfl_down(bS, 1, 64);
    if (lane < 32 && !(lane & 1)) s_db[lane >> 1] = (uint8_t)(bS | (hi << 4));
    if (thr) {
        uint32_t *o = (uint32_t *)(s_db + 16 + k * 8);
        o[0] = al | be << 8 | t0 << 16 | t1 << 24;
        o[1] = t2 | (uint32_t)ia << 8;
    }
    wave_sync();
}

// per-wave LDS scratch of the MB reconstruction (reference windows)
struct McScratch {
    int32_t dc[24];
    uint32_t srec[72];               // deblocking record inputs: this MB's, left and top records
    uint32_t coef[216];              // the MB's coded blocks (<= 27 x 32 B), staged by one coalesced load
    int16_t res[384];                // k_wgpp MC waves: the MB's residual (luma 16x16, Cb 8x8, Cr 8x8)
    union {
        struct {                         // inter: luma reference windows
            uint4 wrow[16][9];           // block, window row: columns 0..8 in bytes 0..8 (realigned)
        };
        struct {                         // intra (k_wg MC waves): prediction tiles with halo
            uint8_t ty[17 * TY_STRIDE], tu[9 * TC_STRIDE], tv[9 * TC_STRIDE];
            uint8_t junk[256];
        };
    };
};

// k_prep: the per-MB work that does not depend on any reconstructed sample --
// deblocking record (bS + thresholds) and residual (dequant + inverse
// transforms) -- for every MB of a batch, fully parallel (one wave per MB).
// It runs one batch ahead of k_wgpp, whose MC waves then only load its
// outputs: either as tail workgroups of the previous batch's k_wgpp launch
// (prep_mb from k_wgpp, started once enough of that launch's rows are done)
// or as its own launch (the first batch; host-staged batches).  Outputs:
// dbrec (64 B per MB; byte 63 = residual range error, a byte no consumer reads
// otherwise), res (384 x int16, for MBs with coded blocks).
struct PrepArgs {
    const MbRec *rec;
    const int16_t *coef;
    const PicDesc *pics;
    uint8_t *dbrec;
    int16_t *res;
    int nmbs_total;           // MBs of the batch (npics * w * h)
    int w, h;
};

__device__ __forceinline__ void prep_mb(const PrepArgs &a, int gidx, int lane, McScratch &Mw,
                                        uint8_t *s_db, const Tabs &T)
{
    const int nmbs = a.w * a.h;
    const int p = gidx / nmbs, mb = gidx - p * nmbs;
    const PicDesc &pd = a.pics[p];
    const int gmb = pd.rec_base + mb;
    {
        const int mbx = mb % a.w, mby = mb / a.w;
        const uint32_t *rq = (const uint32_t *)(a.rec + gmb);
        const uint32_t *rl = (const uint32_t *)(a.rec + (mbx > 0 ? gmb - 1 : gmb));
        const uint32_t *rt = (const uint32_t *)(a.rec + (mby > 0 ? gmb - a.w : gmb));
        Mw.srec[lane] = *(lane < 24 ? rq + lane : lane < 48 ? rl + (lane - 24) : rt + (lane - 48));
        if (lane < 8) Mw.srec[64 + lane] = rt[16 + lane];
    }
    wave_sync();
    const MbRec &r = *(const MbRec *)Mw.srec;
    const int rtype = __builtin_amdgcn_readfirstlane(r.type);
    const uint32_t rcbits = __builtin_amdgcn_readfirstlane(r.cbits);
    const bool has_res = rtype != MBT_IPCM && rcbits != 0;
    const int ncw = has_res ? __popc(rcbits & 0x7FFFFFFu) * 8 : 0;
    uint32_t cq0 = 0, cq1 = 0, cq2 = 0, cq3 = 0;
    {
        const uint32_t *csrc = (const uint32_t *)(a.coef + ((size_t)pd.coef_base + (uint32_t)__builtin_amdgcn_readfirstlane(r.coef)) * 16);
        if (lane < ncw) cq0 = csrc[lane];
        if (lane + 64 < ncw) cq1 = csrc[lane + 64];
        if (lane + 128 < ncw) cq2 = csrc[lane + 128];
        if (lane + 192 < ncw) cq3 = csrc[lane + 192];
    }
    mb_dbrec(lane, s_db, Mw.srec, T);
    int e = 0;
    if (has_res) {
        if (lane < ncw) Mw.coef[lane] = cq0;
        if (lane + 64 < ncw) Mw.coef[lane + 64] = cq1;
        if (lane + 128 < ncw) Mw.coef[lane + 128] = cq2;
        if (lane + 192 < ncw) Mw.coef[lane + 192] = cq3;
        wave_sync();
        mb_residual(r, (const int16_t *)Mw.coef, a.res + (size_t)gidx * 384, Mw.dc, lane, &e, T.ls,
                    res_mask(rtype, rcbits));
    }
    const int any_e = __builtin_amdgcn_ballot_w64(e != 0) != 0;
    if (lane < 16) {
        uint32_t w = ((const uint32_t *)s_db)[lane];
        if (lane == 15) w = (w & 0x00FFFFFFu) | (any_e ? 0x01000000u : 0u);
        ((uint32_t *)(a.dbrec + (size_t)gidx * 64))[lane] = w;     // batch position, not rec_base
    }
    wave_sync();
}

__global__ __launch_bounds__(256) void k_prep(PrepArgs a)
{
    __shared__ McScratch M[4];
    __shared__ uint8_t s_db[4][64];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int gidx = blockIdx.x * 4 + wv;
    if (gidx >= a.nmbs_total) return;            // wave-uniform; no workgroup barrier follows
    const Tabs T = load_tabs(lane);
    prep_mb(a, gidx, lane, M[wv], s_db[wv], T);
}

// ---------------------------------------------------------------------------
// intra reconstruction of one MB inside a wave-private tile whose 1-sample
// halo (top row incl. top-left/top-right, left column) is already filled.
// ---------------------------------------------------------------------------
// I4x4 sub-wavefront: 16 blocks in 10 steps, two per step where the
// dependencies allow (left, top, top-right, top-left blocks done first):
//   {0,-} {1,-} {4,2} {5,3} {6,8} {7,9} {12,10} {13,11} {14,-} {15,-}
__device__ constexpr int i4s0(int s) { return s < 2 ? s : s < 4 ? s + 2 : s < 6 ? s + 2 : s < 8 ? s + 6 : s + 6; }
__device__ constexpr int i4s1(int s) { return s == 2 ? 2 : s == 3 ? 3 : s == 4 ? 8 : s == 5 ? 9 : s == 6 ? 10 : s == 7 ? 11 : -1; }
static_assert(i4s0(0) == 0 && i4s0(2) == 4 && i4s0(4) == 6 && i4s0(6) == 12 && i4s0(9) == 15, "I4x4 schedule");

// Intra 4x4 prediction as a table (8.3.1.2.1-9): every mode and position is
// v = (A + wB*B + wC*C + rnd) >> sh over the block's 13 neighbours Sx[0..12]
// (Sx[3-k] = p[-1,k], Sx[4] = p[-1,-1], Sx[5+k] = p[k,-1]), or DC.  Entry:
// the tile offsets of A, B, C relative to the block's sample (0,0) as int8
// (the top-right samples p[4..7,-1] read as p[3,-1] when unavailable, avtr =
// 0 -- intra_prediction.c:789-792), wB (bits 24-25), wC (26), sh (27-28),
// DC flag (29).  Index ((avtr * 9 + mode) * 16 + y * 4 + x).
__device__ uint32_t i4_entry(int mode, int x, int y, int avtr)
{
    int a = 0, b = 0, c = 0, wb = 0, wc = 0, sh = 0;
    bool dc = false;
    auto copy = [&](int i) { a = b = c = i; wb = 0; wc = 0; sh = 0; };
    auto k11 = [&](int i, int j) { a = i; b = j; c = i; wb = 1; wc = 0; sh = 1; };
    auto k121 = [&](int i, int j, int k) { a = i; b = j; c = k; wb = 2; wc = 1; sh = 2; };
    auto k13 = [&](int i, int j) { a = i; b = j; c = i; wb = 3; wc = 0; sh = 2; };
    switch (mode) {
    case 0: copy(5 + x); break;                                   // vertical
    case 1: copy(3 - y); break;                                   // horizontal
    case 2: dc = true; copy(0); break;                            // DC
    case 3:                                                       // diagonal down left
        if (x == 3 && y == 3) k13(11, 12);
        else k121(5 + x + y, 6 + x + y, 7 + x + y);
        break;
    case 4: { const int d = x - y; k121(3 + d, 4 + d, 5 + d); break; }    // diagonal down right
    case 5: {                                                     // vertical right
        const int z = 2 * x - y, i = x - (y >> 1);
        if (z >= 0 && !(z & 1)) k11(4 + i, 5 + i);
        else if (z > 0) k121(3 + i, 4 + i, 5 + i);
        else if (z == -1) k121(3, 4, 5);
        else k121(4 - y, 5 - y, 6 - y);
        break;
    }
    case 6: {                                                     // horizontal down
        const int z = 2 * y - x, i = y - (x >> 1);
        if (z >= 0 && !(z & 1)) k11(4 - i, 3 - i);
        else if (z > 0) k121(5 - i, 4 - i, 3 - i);
        else if (z == -1) k121(3, 4, 5);
        else k121(4 + x, 3 + x, 2 + x);
        break;
    }
    case 7: {                                                     // vertical left
        const int i = x + (y >> 1);
        if (!(y & 1)) k11(5 + i, 6 + i);
        else k121(5 + i, 6 + i, 7 + i);
        break;
    }
    default: {                                                    // horizontal up
        const int z = x + 2 * y, i = y + (x >> 1);
        if (z > 5) copy(0);
        else if (z == 5) k13(1, 0);
        else if (!(z & 1)) k11(3 - i, 2 - i);
        else k121(3 - i, 2 - i, 1 - i);
        break;
    }
    }
    auto rel = [&](int i) {
        int r;
        if (i <= 3) r = (3 - i) * TY_STRIDE - 1;                  // p[-1, 3-i]
        else if (i == 4) r = -TY_STRIDE - 1;                      // p[-1, -1]
        else r = -TY_STRIDE + ((i - 5 > 3 && !avtr) ? 3 : i - 5); // p[i-5, -1]
        return (uint32_t)r & 255u;
    };
    return rel(a) | rel(b) << 8 | rel(c) << 16 | (uint32_t)wb << 24 | (uint32_t)wc << 26 | (uint32_t)sh << 27 |
           (dc ? 1u << 29 : 0u);
}
#define I4TAB_N (2 * 9 * 16)

// Cross-MB intra pipelining: the left neighbour MB's samples are read from
// its ring slot as they land there, not after it is complete.  LeftNb: that
// slot's samples and progress words (MbRing::lprog / cprog, tagged with the
// MB index) and this MB's own progress words.
template <bool LDSM> __device__ __forceinline__ unsigned long long ld_granT(const unsigned long long *p);
struct LeftNb {
    const uint8_t *lp;              // left MB's ring slot (samples), NULL when unavailable (no AV_A)
    const int *lprog, *cprog;       // its progress words
    int *my_lprog, *my_cprog;       // this MB's
    int ltag, mytag;                // (c - 1) << 4, c << 4
    unsigned *perr;
    bool chk;                       // dependency checker: the word must name the left MB
    // intra_tile CDEF: the above-right MB's granule (read by I4x4 block 5
    // only, step 3) is waited for there, not before the luma starts: lane
    // 32's pointer, last value and the tag it must carry; cdef wave-uniform
    const unsigned long long *cg;
    unsigned long long cgr;
    uint32_t ctag;
    bool cdef;
};
__device__ __forceinline__ void prog_wait(const int *p, int want, int lane, unsigned *perr, bool chk = false)
{
    unsigned spins = 0;
    int v;
    while ((v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))) < want) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 22)) { if (lane == 0) atomicOr(perr, 16u); break; }   // bounded wait
    }
    // a later MB in the same ring slot also passes `< want`
    if (chk && (v >> 4) != (want >> 4) && lane == 0) atomicOr(perr, CHK_PROG);
    wave_sync();
}
__device__ __forceinline__ void prog_set(int *p, int v, int lane)
{
    wave_sync();
    if (lane == 0) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Intra reconstruction of one MB from its tiles, whose top halo is filled;
// the left column comes from the left MB's ring slot, part by part (LeftNb):
// prediction + residual (res: the MB's residual staged in LDS) + clip, all
// written straight into the ring slot px (I4x4 luma into the tile as well:
// each block predicts from the blocks before it).  `part` 1 = luma, 2 =
// chroma (mc_intra runs luma first and publishes its bottom row before the
// chroma); chroma waits only for the left MB's chroma, an I4x4 block in
// column 0 for the left MB's block beside it, so the next MB's blocks follow
// this one's 3 steps behind.  Every lane issues all of its LDS reads of a
// phase before it uses any, so a phase costs one LDS round trip
// (Intra16x16 :626-686, Intra4x4 :700-832, IntraChroma :844-914,
// AddResidual :926-988).
template <bool UPL = false, bool CDEF = false>
__device__ __forceinline__ void intra_tile(int mbtype, int avail, int pred, uint64_t i4, const int16_t *res, bool has_res,
                                           uint8_t *ty, uint8_t *tu, uint8_t *tv, const uint32_t *i4tab, uint8_t *junk,
                                           uint8_t *px, int lane, const LeftNb &N, int part = 3)
{
    const bool aA = avail & AV_A, aB = avail & AV_B;
    if (part & 2) {   // chroma: lane -> (comp, row, pair), straight into the slot
        if (aA) {
            prog_wait(N.cprog, N.ltag | 1, lane, N.perr, N.chk);
            if (lane < 16) {
                const int k = lane & 7, comp = lane >> 3;
                (comp ? tv : tu)[(k + 1) * TC_STRIDE + TX0 - 1] = N.lp[256 + comp * 64 + k * 8 + 7];
            }
            wave_sync();
        }
        const int comp = lane >> 5, y = (lane >> 2) & 7, x0 = (lane & 3) * 2;
        const uint8_t *T = comp ? tv : tu;
        const int cmode = (pred >> 4) & 3;
        int pv[2];
        if (cmode == 0) {                                         // DC per 4x4 quadrant (:1175-1245)
            const int xo = x0 & 4, yo = y & 4;
            const uint32_t tw = *(const uint32_t *)&T[TX0 + xo];
            const int sl = T[(yo + 1) * TC_STRIDE + TX0 - 1] + T[(yo + 2) * TC_STRIDE + TX0 - 1] +
                           T[(yo + 3) * TC_STRIDE + TX0 - 1] + T[(yo + 4) * TC_STRIDE + TX0 - 1];
            const int st = (int)__builtin_amdgcn_sad_u8(tw, 0u, 0u);
            int pr;
            if ((xo == 0 && yo == 0) || (xo > 0 && yo > 0)) pr = (aA && aB) ? (st + sl + 4) >> 3 : aA ? (sl + 2) >> 2 : aB ? (st + 2) >> 2 : 128;
            else if (xo > 0) pr = aB ? (st + 2) >> 2 : aA ? (sl + 2) >> 2 : 128;
            else pr = aA ? (sl + 2) >> 2 : aB ? (st + 2) >> 2 : 128;
            pv[0] = pv[1] = pr;
        } else if (cmode == 1) {                                  // horizontal
            pv[0] = pv[1] = T[(y + 1) * TC_STRIDE + TX0 - 1];
        } else if (cmode == 2) {                                  // vertical
            pv[0] = T[TX0 + x0]; pv[1] = T[TX0 + x0 + 1];
        } else {                                                  // plane
            const uint32_t t0w = *(const uint32_t *)&T[TX0], t1w = *(const uint32_t *)&T[TX0 + 4];
            int lc[8];
#pragma unroll
            for (int k = 0; k < 8; k++) lc[k] = T[(k + 1) * TC_STRIDE + TX0 - 1];
            const int tl = T[TX0 - 1];
            auto Tt = [&](int k) { return k < 0 ? tl : (int)(((k < 4 ? t0w : t1w) >> ((k & 3) * 8)) & 255); };
            auto Lc = [&](int k) { return k < 0 ? tl : lc[k]; };
            int H = 0, V = 0;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                H += (i + 1) * (Tt(4 + i) - Tt(2 - i));
                V += (i + 1) * (Lc(4 + i) - Lc(2 - i));
            }
            const int pa = 16 * (Lc(7) + Tt(7)), pb = (34 * H + 32) >> 6, pc = (34 * V + 32) >> 6;
#pragma unroll
            for (int i = 0; i < 2; i++) pv[i] = clip255((pa + pb * (x0 + i - 3) + pc * (y - 3) + 16) >> 5);
        }
        const int o = 256 + comp * 64 + y * 8 + x0;
        if (has_res) {
            const uint32_t rr = *(const uint32_t *)&res[o];
            pv[0] = clip255(pv[0] + (int)(int16_t)(rr & 0xFFFF));
            pv[1] = clip255(pv[1] + (int)(int16_t)(rr >> 16));
        }
        *(uint16_t *)&px[o] = (uint16_t)(pv[0] | (pv[1] << 8));
        prog_set(N.my_cprog, N.mytag | 1, lane);
    }
    if (!(part & 1)) {
    } else if (mbtype == MBT_I16) {
        if (aA) {
            prog_wait(N.lprog, N.ltag | 10, lane, N.perr, N.chk);
            if (lane < 16) ty[(lane + 1) * TY_STRIDE + TX0 - 1] = N.lp[lane * 16 + 15];
            wave_sync();
        }
        const int mode = pred & 3;
        const int y = lane >> 2, x0 = (lane & 3) * 4;
        int pv[4];
        if (mode == 0) {                                          // vertical
            const uint32_t t = *(const uint32_t *)&ty[TX0 + x0];
#pragma unroll
            for (int i = 0; i < 4; i++) pv[i] = (t >> (8 * i)) & 255;
        } else if (mode == 1) {                                   // horizontal
            const int l = ty[(y + 1) * TY_STRIDE + TX0 - 1];
#pragma unroll
            for (int i = 0; i < 4; i++) pv[i] = l;
        } else {
            uint32_t tdw[4];
            int lc[16];
#pragma unroll
            for (int k = 0; k < 4; k++) tdw[k] = *(const uint32_t *)&ty[TX0 + 4 * k];
#pragma unroll
            for (int k = 0; k < 16; k++) lc[k] = ty[(k + 1) * TY_STRIDE + TX0 - 1];
            if (mode == 2) {                                      // DC
                int st = 0, sl = 0;
#pragma unroll
                for (int k = 0; k < 4; k++) st += (int)__builtin_amdgcn_sad_u8(tdw[k], 0u, 0u);
#pragma unroll
                for (int k = 0; k < 16; k++) sl += lc[k];
                const int dcv = (aA && aB) ? (st + sl + 16) >> 5 : aA ? (sl + 8) >> 4 : aB ? (st + 8) >> 4 : 128;
#pragma unroll
                for (int i = 0; i < 4; i++) pv[i] = dcv;
            } else {                                              // plane
                const int tl = ty[TX0 - 1];
                auto T = [&](int k) { return k < 0 ? tl : (int)((tdw[k >> 2] >> ((k & 3) * 8)) & 255); };
                auto Lc = [&](int k) { return k < 0 ? tl : lc[k]; };
                int H = 0, V = 0;
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    H += (i + 1) * (T(8 + i) - T(6 - i));
                    V += (i + 1) * (Lc(8 + i) - Lc(6 - i));
                }
                const int pa = 16 * (Lc(15) + T(15)), pb = (5 * H + 32) >> 6, pc = (5 * V + 32) >> 6;
#pragma unroll
                for (int i = 0; i < 4; i++) pv[i] = clip255((pa + pb * (x0 + i - 7) + pc * (y - 7) + 16) >> 5);
            }
        }
        uint32_t pk = 0;
        if (has_res) {
            const uint2 rr = *(const uint2 *)&res[y * 16 + x0];
            const int r4[4] = {(int)(int16_t)(rr.x & 0xFFFF), (int)(int16_t)(rr.x >> 16), (int)(int16_t)(rr.y & 0xFFFF),
                               (int)(int16_t)(rr.y >> 16)};
#pragma unroll
            for (int i = 0; i < 4; i++) pk |= (uint32_t)clip255(pv[i] + r4[i]) << (8 * i);
        } else {
#pragma unroll
            for (int i = 0; i < 4; i++) pk |= (uint32_t)pv[i] << (8 * i);
        }
        *(uint32_t *)&px[y * 16 + x0] = pk;
        prog_set(N.my_lprog, N.mytag | 10, lane);
    } else {
        // I4x4, lanes 0..15 = block of slot 0, 16..31 = slot 1 (lanes 32..63
        // mirror, writing to their junk bytes)
        const int slot = (lane >> 4) & 1, pos = lane & 15, px4 = pos & 3, py4 = pos >> 2;
        const bool lo = lane < 32;
        // blocks whose top-right neighbour is available: 2,6,8,9,10,12,14
        // always; 0,1,4 from the MB above; 5 from the MB above-right
        const uint32_t trmask = 0x5744u | ((avail & AV_B) ? 0x13u : 0u) | ((avail & AV_C) ? 0x20u : 0u);
        // every step's table entry and residual sample, issued up front: they
        // do not depend on the reconstruction
        uint32_t ent[10];
        int rv[10];
#pragma unroll
        for (int s = 0; s < 10; s++) {
            const int b0 = i4s0(s), b1 = i4s1(s) < 0 ? i4s0(s) : i4s1(s);
            const int m0 = (int)(i4 >> (b0 * 4)) & 15, m1 = (int)(i4 >> (b1 * 4)) & 15;
            const int e0 = ((int)(trmask >> b0) & 1) * 9 + (m0 < 9 ? m0 : 0);
            const int e1 = ((int)(trmask >> b1) & 1) * 9 + (m1 < 9 ? m1 : 0);
            ent[s] = i4tab[(slot ? e1 : e0) * 16 + pos];
            const int o0 = blk_y(b0) * 64 + blk_x(b0) * 4, o1 = blk_y(b1) * 64 + blk_x(b1) * 4;
            rv[s] = has_res ? (int)res[(slot ? o1 : o0) + py4 * 16 + px4] : 0;
        }
        // CDEF: lane 32 re-reads the above-right granule now, so that the load
        // has landed by step 3
        unsigned long long cgv = CDEF ? N.cgr : 0ull;
        if (CDEF && N.cdef && lane == 32 && (uint32_t)(cgv >> 32) != N.ctag) cgv = ld_granT<UPL>(N.cg);
#pragma unroll
        for (int s = 0; s < 10; s++) {
            const int b0 = i4s0(s), b1 = i4s1(s);
            if (CDEF && s == 3 && N.cdef) {     // block 5 reads the above-right MB's bottom row
                const bool need = lane == 32;
                unsigned spins = 0;
                while (__builtin_amdgcn_ballot_w64(need && (uint32_t)(cgv >> 32) != N.ctag) != 0) {
                    __builtin_amdgcn_s_sleep(1);
                    if (++spins > (1u << 20)) { if (lane == 0) atomicOr(N.perr, 2u); break; }   // bounded wait
                    if (need) cgv = ld_granT<UPL>(N.cg);
                }
                if (need) *(uint32_t *)&ty[TX0 + 16] = (uint32_t)cgv;
                wave_sync();
            }
            // a block in column 0 (steps 0, 2, 4, 6: blocks 0, 2, 8, 10) reads
            // the left MB's block beside it (5, 7, 13, 15: its steps 3, 5, 7, 9)
            if ((s & 1) == 0 && s <= 6 && aA) {
                const int by = s == 0 ? 0 : s == 2 ? 1 : s == 4 ? 2 : 3;
                prog_wait(N.lprog, N.ltag | (s + 4), lane, N.perr, N.chk);
                if (lane < 4) ty[(by * 4 + lane + 1) * TY_STRIDE + TX0 - 1] = N.lp[(by * 4 + lane) * 16 + 15];
                wave_sync();
            }
            const int t0c = (blk_y(b0) * 4 + 1) * TY_STRIDE + TX0 + blk_x(b0) * 4;
            const int t1c = b1 >= 0 ? (blk_y(b1) * 4 + 1) * TY_STRIDE + TX0 + blk_x(b1) * 4 : t0c;
            const int p0c = blk_y(b0) * 64 + blk_x(b0) * 4;
            const int p1c = b1 >= 0 ? blk_y(b1) * 64 + blk_x(b1) * 4 : p0c;
            const bool valid = lo && (slot == 0 || b1 >= 0);
            const int t0 = slot ? t1c : t0c;
            const uint32_t e = ent[s];
            const int A = ty[t0 + (int)(int8_t)(e & 255)];
            const int B = ty[t0 + (int)(int8_t)((e >> 8) & 255)];
            const int C = ty[t0 + (int)(int8_t)((e >> 16) & 255)];
            const int sh = (int)((e >> 27) & 3);
            int v = (A + (int)((e >> 24) & 3) * B + (int)((e >> 26) & 1) * C + ((1 << sh) >> 1)) >> sh;
            // DC: only in steps where some block is DC (wave-uniform)
            const int m0 = (int)(i4 >> (b0 * 4)) & 15, m1 = b1 >= 0 ? (int)(i4 >> (b1 * 4)) & 15 : 0;
            if (m0 == 2 || (b1 >= 0 && m1 == 2)) {
                const uint32_t tw = *(const uint32_t *)&ty[t0 - TY_STRIDE];
                const int sl = ty[t0 - 1] + ty[t0 - 1 + TY_STRIDE] + ty[t0 - 1 + 2 * TY_STRIDE] + ty[t0 - 1 + 3 * TY_STRIDE];
                const int st = (int)__builtin_amdgcn_sad_u8(tw, 0u, 0u);
                const int bb = slot && b1 >= 0 ? b1 : b0;
                const bool avT = blk_y(bb) > 0 || aB, avL = blk_x(bb) > 0 || aA;
                const int dsum = (avT ? st : 0) + (avL ? sl : 0);
                const int dsh = (avT && avL) ? 3 : 2;
                const int dcv = (avT || avL) ? (dsum + (1 << (dsh - 1))) >> dsh : 128;
                v = (e >> 29) & 1 ? dcv : v;
            }
            v = clip255(v + rv[s]);
            *(valid ? &ty[t0 + py4 * TY_STRIDE + px4] : &junk[lane]) = (uint8_t)v;
            *(valid ? &px[(slot ? p1c : p0c) + py4 * 16 + px4] : &junk[64 + lane]) = (uint8_t)v;
            prog_set(N.my_lprog, N.mytag | (s + 1), lane);
        }
    }
    wave_sync();
}

#define RY_S 20       // region luma stride (cols -4..15)
#define RC_S 20       // region chroma stride (cols -4..7, padded to the luma stride)


__device__ __forceinline__ int absd(int a, int b) { return (int)__builtin_amdgcn_sad_u8((unsigned)a, (unsigned)b, 0u); }

// one sample line across edge k (p3..q3 = v[4k..4k+7]); chroma lines only
// use p1..q1.  filterSamples / bS<4 / bS==4 of deblocking.c:1543-1736.  The
// bS==4 arithmetic runs only when some lane of the wave has bS==4 on this
// edge (wave-uniform branch); everything else is select-based.
// keep a value computed where it stands: the filter updates below are cheap
// enough to compute for every lane and select, instead of the compiler
// sinking them into exec-masked blocks (each costs more scalar work than it
// saves)
#define MATERIALIZE(x) asm volatile("" : "+v"(x))
// median of three = clamp lo <= x <= hi for lo <= hi, in this form one
// v_med3_i32 (min(max(x, lo), hi) is two instructions unless both bounds are
// constants)
__device__ __forceinline__ int med3i(int x, int lo, int hi) { return min(max(x, lo), max(min(x, lo), hi)); }
// c - 2 * x in one v_mad_i32_i24 (the compiler emits a shift and a subtract)
__device__ __forceinline__ int mad_m2(int x, int c)
{
    int r;
    asm("v_mad_i32_i24 %0, %1, -2, %2" : "=v"(r) : "v"(x), "v"(c));
    return r;
}

// One edge of one line (8.7.2.3 / 8.7.2.4).  Per-lane constants: alpha,
// beta; beta_ap = beta for luma, 0 for chroma (so a_p / a_q are false and
// the p1 / q1 updates off); tcs = tc0 by bS in bytes 1..3 (+1 for chroma,
// where tc = tc0 + 1), byte 0 = 0.  MBEDGE: the MB edge, the only one that
// can carry bS = 4.
template <bool MBEDGE>
__device__ __forceinline__ void filt_line(int (&v)[20], const int k, const int bS, const int alpha, const int beta,
                                          const int beta_ap, const uint32_t tcs)
{
    const int o = 4 * k;
    const int p2 = v[o + 1], p1 = v[o + 2], p0 = v[o + 3];
    const int q0 = v[o + 4], q1 = v[o + 5], q2 = v[o + 6];
    const int d0 = absd(p0, q0);
    // filterSamples as one sign test: v_sad_u8 subtracts each threshold in
    // its addend, one v_max3 joins the three
    const int m0 = (int)__builtin_amdgcn_sad_u8((uint32_t)p0, (uint32_t)q0, (uint32_t)-alpha);
    const int m1 = (int)__builtin_amdgcn_sad_u8((uint32_t)p1, (uint32_t)p0, (uint32_t)-beta);
    const int m2 = (int)__builtin_amdgcn_sad_u8((uint32_t)q1, (uint32_t)q0, (uint32_t)-beta);
#ifndef FILT_SHORTCIRCUIT
    // (bitwise: a short-circuit && became an exec-masked block around the
    // sign test -- scalar exec bookkeeping on the chain, every edge)
    const bool f = (bS != 0) & (max(m0, max(m1, m2)) < 0);
#else
    const bool f = bS != 0 && max(m0, max(m1, m2)) < 0;
#endif
    const bool ap = absd(p2, p0) < beta_ap, aq = absd(q2, q0) < beta_ap;
    // bS < 4
    const int tc0 = (int)__builtin_amdgcn_ubfe(tcs, (uint32_t)bS << 3, 8);    // bS = 4: offset 32 -> byte 0 (unused)
    const int tc = tc0 + (int)ap + (int)aq;
    const int d = med3i((((q0 - p0) << 2) + (p1 - q1) + 4) >> 3, -tc, tc);
    const int avg = (int)__builtin_amdgcn_lerp((uint32_t)p0, (uint32_t)q0, 1u);    // (p0 + q0 + 1) >> 1 (v_lerp_u8)
    const int ntc0 = -tc0;
    int n_p1 = p1 + med3i((mad_m2(p1, p2) + avg) >> 1, ntc0, tc0);
    int n_q1 = q1 + med3i((mad_m2(q1, q2) + avg) >> 1, ntc0, tc0);
    int n_p0 = clip255(p0 + d), n_q0 = clip255(q0 - d);
    MATERIALIZE(n_p1); MATERIALIZE(n_q1); MATERIALIZE(n_p0); MATERIALIZE(n_q0);
    int r_p2 = p2, r_q2 = q2;
    int r_p1 = f && ap ? n_p1 : p1;
    int r_q1 = f && aq ? n_q1 : q1;
    int r_p0 = f ? n_p0 : p0;
    int r_q0 = f ? n_q0 : q0;
    if (MBEDGE) {
        // bS == 4: MB edges next to intra MBs only -- skipped unless some lane needs it
        const bool b4 = f & (bS >= 4);
        if (__builtin_amdgcn_ballot_w64(b4) != 0) {
            const int p3 = v[o], q3 = v[o + 7];
            const bool strong = d0 < ((alpha >> 2) + 2);
            const bool sp = ap && strong, sq = aq && strong;
            int s_p0 = (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3, w_p0 = (2 * p1 + p0 + q1 + 2) >> 2;
            int s_q0 = (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3, w_q0 = (2 * q1 + q0 + p1 + 2) >> 2;
            int s_p1 = (p2 + p1 + p0 + q0 + 2) >> 2, s_q1 = (p0 + q0 + q1 + q2 + 2) >> 2;
            int s_p2 = (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3, s_q2 = (2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3;
            MATERIALIZE(s_p0); MATERIALIZE(w_p0); MATERIALIZE(s_q0); MATERIALIZE(w_q0);
            MATERIALIZE(s_p1); MATERIALIZE(s_q1); MATERIALIZE(s_p2); MATERIALIZE(s_q2);
            r_p0 = b4 ? (sp ? s_p0 : w_p0) : r_p0;
            r_q0 = b4 ? (sq ? s_q0 : w_q0) : r_q0;
            r_p1 = b4 ? (sp ? s_p1 : p1) : r_p1;
            r_q1 = b4 ? (sq ? s_q1 : q1) : r_q1;
            r_p2 = b4 && sp ? s_p2 : r_p2;
            r_q2 = b4 && sq ? s_q2 : r_q2;
        }
    }
    v[o + 1] = r_p2; v[o + 2] = r_p1; v[o + 3] = r_p0;
    v[o + 4] = r_q0; v[o + 5] = r_q1; v[o + 6] = r_q2;
}

// all edges of one direction: lanes 0..15 = luma lines, 16..31 = chroma
// lines (comp = bit 3, index = bits 0..2).  dir 0: lines are rows, edges are
// the 4 (chroma 2) vertical edges, left to right; dir 1: columns / horizontal
// edges, top to bottom.  Each lane owns its line for all edges of the
// direction, so no cross-lane ordering is needed inside a direction.  Lanes
// 32..63 mirror lanes 0..31 (same addresses, same values) so that every
// access is unconditional.
struct NoMid { __device__ __forceinline__ void operator()() const {} };
// Mid (dir 0): called once the MB edge (edge 0) is filtered and its samples
// (region cols -4..-1, the left MB's cols 12..15, now final) are written back
// -- the row hand-off publishes from there without waiting for the internal
// edges (edges 1..3 touch only this MB's columns 1..14)
// One pass's per-line filter parameters, from the MB's deblocking record:
// this line's four bS nibbles (chroma: its edges 0, 1 sit on luma edges 0,
// 2) and the two threshold sets {alpha, beta, tc0(bS 1..3)} of the MB edge
// and the internal edges.  They depend on nothing the chain produces, so the
// row waves compute them off the chain (before the hdone / top waits).
struct DbPar {
    uint32_t bsw, tcs_e, tcs_i;
    int alpha_e, beta_e, alpha_i, beta_i;
};
__device__ __forceinline__ DbPar dbpar(const int dir, const uint8_t *db, int lane, bool mb_edge_on)
{
    const int li = lane & 31;
    const bool chroma = li >= 16;
    const int idx = chroma ? (li & 7) : (li & 15);
    const int seg = chroma ? idx >> 1 : idx >> 2;
    DbPar P;
    uint32_t bsw = *(const uint16_t *)(db + dir * 8 + seg * 2);
    if (chroma) bsw = (bsw & 15) | ((bsw >> 4) & 0xF0);
    if (!mb_edge_on) bsw &= ~15u;
    P.bsw = bsw;
    const uint8_t *pe = db + 16 + ((chroma ? 3 : 0) + 1 + dir) * 8;    // MB edge class
    const uint8_t *pi = db + 16 + (chroma ? 3 : 0) * 8;                  // internal class
    const uint2 te = *(const uint2 *)pe, ti = *(const uint2 *)pi;
    const uint32_t cplus = chroma ? 0x01010100u : 0u;
    P.alpha_e = te.x & 255; P.beta_e = (te.x >> 8) & 255; P.alpha_i = ti.x & 255; P.beta_i = (ti.x >> 8) & 255;
    P.tcs_e = (((te.x >> 8) & 0xFFFF00u) | (te.y << 24)) + cplus;
    P.tcs_i = (((ti.x >> 8) & 0xFFFF00u) | (ti.y << 24)) + cplus;
    return P;
}

// pre (dir 0): the line's columns 0..15 (dwords 1..4 of its region row),
// read off the chain; only the left halo (dword 0) is read here
// use_halo (dir 0): the line's left halo (dword 0) is `halo`, already in a
// register (passed by value: a pointer chosen at run time would put it in
// scratch memory)
template <class Mid = NoMid>
__device__ __forceinline__ void deblock_dir(const int dir, const DbPar &P, uint8_t *ry, uint8_t *ru, uint8_t *rv,
                                            uint8_t *junk, int lane, const uint32_t *pre = nullptr,
                                            bool use_halo = false, uint32_t halo = 0, const Mid &mid = Mid())
{
    const int li = lane & 31;
    const bool chroma = li >= 16;
    const int idx = chroma ? (li & 7) : (li & 15);
    uint8_t *D = chroma ? ((li & 8) ? rv : ru) : ry;
    const uint32_t bsw = P.bsw, tcs_e = P.tcs_e, tcs_i = P.tcs_i;
    const int alpha_e = P.alpha_e, beta_e = P.beta_e, alpha_i = P.alpha_i, beta_i = P.beta_i;
    // one stride for both planes (RC_S == RY_S): every access below is
    // base + immediate.  Chroma lines read past their 12/10 samples into
    // neighbouring LDS (values unused) and write back only what they own.
    static_assert(RC_S == RY_S, "deblock_dir assumes one region stride");
    int v[20];
    if (dir == 0) {
        const uint32_t *row = (const uint32_t *)(D + (idx + (chroma ? 2 : 4)) * RY_S);
#pragma unroll
        for (int j = 0; j < 5; j++) {
            const uint32_t w = (pre && j > 0) ? pre[j - 1] : (j == 0 && use_halo) ? halo : row[j];
            v[4 * j] = w & 255; v[4 * j + 1] = (w >> 8) & 255; v[4 * j + 2] = (w >> 16) & 255; v[4 * j + 3] = w >> 24;
        }
    } else {
        // v[j] = sample row j-4 of this column (chroma region row 0 = sample row -2)
        const uint8_t *col = D + idx + 4 - (chroma ? 2 * RY_S : 0);
#pragma unroll
        for (int j = 0; j < 20; j++) v[j] = col[j * RY_S];
    }
    {
        const int b = (int)(bsw & 15);
        if (__builtin_amdgcn_ballot_w64(b != 0) != 0)     // wave-uniform skip
            filt_line<true>(v, 0, b, alpha_e, beta_e, chroma ? 0 : beta_e, tcs_e);
    }
    if (dir == 0) {
        // cols -4..-1 are final after the MB edge: write them back now, then
        // let the caller publish
        uint32_t *row = (uint32_t *)(D + (idx + (chroma ? 2 : 4)) * RY_S);
        row[0] = (uint32_t)v[0] | ((uint32_t)v[1] << 8) | ((uint32_t)v[2] << 16) | ((uint32_t)v[3] << 24);
        wave_sync();
        mid();
    }
#pragma unroll
    for (int k = 1; k < 4; k++) {
        const int b = (int)((bsw >> (4 * k)) & 15);
        if (__builtin_amdgcn_ballot_w64(b != 0) == 0) continue;
        filt_line<false>(v, k, b, alpha_i, beta_i, chroma ? 0 : beta_i, tcs_i);
    }
    // write-back without divergence: samples a lane does not own go to its
    // junk slot; lanes 32..63 store exactly what lanes 0..31 store
    if (dir == 0) {
        uint32_t *row = (uint32_t *)(D + (idx + (chroma ? 2 : 4)) * RY_S);
        uint32_t *jk = (uint32_t *)(junk + lane * 4);
#pragma unroll
        for (int j = 1; j < 5; j++) {
            const uint32_t w = (uint32_t)v[4 * j] | ((uint32_t)v[4 * j + 1] << 8) | ((uint32_t)v[4 * j + 2] << 16) | ((uint32_t)v[4 * j + 3] << 24);
            *((!chroma || j < 3) ? row + j : jk) = w;
        }
    } else {
        uint8_t *col = D + idx + 4 - (chroma ? 2 * RY_S : 0);
        uint8_t *jk = junk + lane * 4;
#pragma unroll
        for (int j = 1; j < 19; j++)
            *((!chroma || j == 3 || j == 4 || j == 7 || j == 8) ? col + j * RY_S : jk) = (uint8_t)v[j];
    }
}

// (global address space explicit: a generic pointer would make these FLAT
// accesses, which lgkmcnt counts too -- every LDS wait would then wait for them)
typedef __attribute__((address_space(1))) unsigned long long g_u64;
__device__ __forceinline__ unsigned long long ld_gran(const unsigned long long *p)
{
    return __hip_atomic_load((const g_u64 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_gran(unsigned long long *p, uint32_t v, uint32_t tag)
{
    __hip_atomic_store((g_u64 *)p, ((unsigned long long)tag << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the same granules in LDS, between the two rows of one workgroup (k_wgpp
// RPW = 2): one 8-B LDS access each, no L2 round trip
typedef __attribute__((address_space(3))) unsigned long long l_u64;
template <bool LDSM> __device__ __forceinline__ unsigned long long ld_granT(const unsigned long long *p)
{
    if (LDSM) return __hip_atomic_load((const l_u64 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return ld_gran(p);
}
template <bool LDSM> __device__ __forceinline__ void st_granT(unsigned long long *p, uint32_t v, uint32_t tag)
{
    if (LDSM) __hip_atomic_store((l_u64 *)p, ((unsigned long long)tag << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else st_gran(p, v, tag);
}

// LDS hand-off ring between the MC waves of a row workgroup and its row
// unit: slot c % RK holds MB c's MC samples (residual added) and deblocking
// record; flag[slot] = c + 1 once filled, consumed = c + 1 once the row unit
// no longer reads MB c's slot.  LDS instructions of one wave execute in
// order, so a flag written after the data (compiler barrier between) is
// seen after it by every other wave of the workgroup.
// ring slots per row: a single-row workgroup (RPW = 1) gets a deep ring, so
// its MC waves run far ahead of the row's deblocking chain and their
// reference loads are mostly done before the chain reaches the row (fewer
// loads queued in front of the chain's mailbox polls); row groups keep a
// small one (LDS)
#ifndef RING1
#define RING1 64
#endif
#ifndef RINGG
#define RINGG 16
#endif
// the 2-MC-wave single-row shape's ring (its LDS decides how many of its
// workgroups share a CU, with WGPP2_WAVES_PER_EU); 32 slots, the 3-MC
// shape keeps RING1
#ifndef RING1_2MC
#define RING1_2MC 32
#endif
template <int RK>
struct __attribute__((aligned(16))) MbRing {
    static_assert(RK > 0 && (RK & (RK - 1)) == 0, "ring depth must be a power of two: slot = c & (RK - 1)");
    uint8_t px[RK][384];
    uint8_t db[RK][64];
    int flag[RK];
    // intra progress of the MB in the slot, tagged (c << 4) | n: lprog n =
    // I4x4 steps whose samples are in px (10: all luma), cprog n = 1 once its
    // chroma is -- the next MB's intra reads its left neighbours as they land
    int lprog[RK], cprog[RK];
    int consumed;
    int claim;          // the next MB an MC wave takes (MC_DYN; NMC .. w)
};

__device__ __forceinline__ int lds_ld(const int *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ void lds_st(int *p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }

// k_wg MC wave, intra MB c of row r: unfiltered neighbours -> prediction
// tile -> the MB's ring slot (reconstruction runs ahead of the deblocking
// row unit; intra prediction reads unfiltered samples only).  Left: MB c-1's
// slot, once its flag shows it reconstructed.  Top: the row above's mailbox
// entries c-1..c+1, dwords 24..31 (unfiltered bottom rows, published by that
// row's MC waves), polled until their tags carry this launch's epoch.
// (out of line to keep the kernel's VGPR count for 3 workgroups per CU; the
// arguments are plain values: a reference to the kernel's ReconArgs would
// force the whole argument block into private memory)
// The LDS objects come in as address-space-3 pointers and the record and the
// error word as address-space-1 ones: a noinline function's generic pointer
// arguments would turn every access inside into a FLAT instruction (counted
// by vmcnt and lgkmcnt alike, at far more than LDS latency per dependent
// access -- measured, 4.7 us per intra MB).  The generic views below are
// addrspacecasts of those arguments, which the compiler folds back into
// ds_* / global_* accesses.
typedef __attribute__((address_space(3))) McScratch lds_McScratch;
typedef const __attribute__((address_space(3))) uint32_t lds_cu32;
typedef const __attribute__((address_space(1))) MbRec g_MbRec;
typedef __attribute__((address_space(1))) unsigned g_u32;
// LF (the 6-MC-wave intra-heavy instance): luma first, its bottom row
// published before the chroma runs (below).  PROF builds pass the MB's
// profiling stamps in `pq` (and the caller publishes the luma bottom row with
// the chroma); LF builds pass where this MB's luma bottom row goes (the row
// below's mailbox entry, NULL in the last row) -- one pointer argument either
// way: a second one costs the callers' spills.  The other instances keep
// chroma first and one wait for the row above (luma-first measured slower in
// P pictures: configs[3] 295.1 vs 287.9 us per step, profiles/r167_*)
template <bool UPL, bool MEL, int RK, bool CHK, bool PROF, bool LF>
__device__ __attribute__((noinline)) void mc_intra(g_MbRec *mbrec, const unsigned long long *mbx_up, g_u32 *perr_g,
                                                   int W, int c, uint32_t tag, bool has_up, int lane, lds_McScratch *Ml,
                                                   __attribute__((address_space(3))) MbRing<RK> *Rl, lds_cu32 *i4tab_l,
                                                   unsigned long long *pq)
{
    __attribute__((address_space(1))) unsigned long long *const pst = PROF ? (__attribute__((address_space(1))) unsigned long long *)pq : nullptr;
    unsigned long long *const pub = PROF || !LF ? nullptr : pq;
    // pst (profiling build): [0] left ready | top ready, [1] prediction done | slot written
    unsigned long long st0 = 0, st1 = 0;
    McScratch &M = *(McScratch *)Ml;
    MbRing<RK> &R = *(MbRing<RK> *)Rl;
    const uint32_t *i4tab = (const uint32_t *)i4tab_l;
    unsigned *perr = (unsigned *)perr_g;
    // the record's fields, wave-uniform (scalar branches below)
    const uint32_t *rw = (const uint32_t *)mbrec;
    const uint32_t d0 = __builtin_amdgcn_readfirstlane(rw[0]), d1 = __builtin_amdgcn_readfirstlane(rw[1]);
    const uint32_t cbits = __builtin_amdgcn_readfirstlane(rw[2]);
    // (readfirstlane returns int: widen through uint32_t, or a mode >= 8 in
    // block 7 sign-extends into blocks 8..15)
    const uint64_t i4 = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(rw[4]) |
                        (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(rw[5]) << 32;
    const int qtype = d0 & 255, avail = d0 >> 24, pred = d1 & 255;
    const int slot = c & (RK - 1);
    const bool aA = avail & AV_A, aB = avail & AV_B, aC = avail & AV_C, aD = avail & AV_D;
    // the row above's entries first: lanes 24..31 entry c dwords 24..31 (B),
    // 32 entry c+1 dword 24 (C), 33..35 entry c-1 dwords 27/29/31 (D).  The
    // loads are issued before the wait for the left MB, so their L2 round
    // trip overlaps it; re-polled only if some granule is still stale
    // the above-right MB (C) is read by one prediction only: I4x4 block 5
    // in Diagonal_Down_Left or Vertical_Left (8.3.1.2.4 / .7); every other MB
    // skips its granule, so the MC chain of the row below waits on MB c of
    // this row, not c + 1 (the wavefront's slope: one in-row step per row)
    const int m5 = (int)(i4 >> 20) & 15;
    const bool needC = aC && qtype == MBT_I4x4 && (m5 == 3 || m5 == 7);
    const bool need_top = has_up && (aB || needC || aD);
    const int dsel = lane == 32 ? 1 : (lane > 32 && lane < 36) ? -1 : 0;
    const int dw = lane < 32 ? (lane & 31) : lane == 32 ? 24 : lane < 36 ? 27 + 2 * (lane - 33) : 24;
    const unsigned long long *g = mbx_up + min(max(c + dsel, 0), W - 1) * 32 + dw;
    const bool mine = need_top && ((lane >= 24 && lane < 32 && aB) || (lane == 32 && needC) || (lane >= 33 && lane < 36 && aD));
    unsigned long long gr = need_top ? ld_granT<UPL>(g) : 0ull;
    if constexpr (!LF) {
        if (pst) st0 = wall_clock64();
        // the above-right granule (needC) only before I4x4 step 3 (intra_tile CDEF)
        const bool minew = mine && !(needC && lane == 32);
        if (need_top) {
            unsigned spins = 0;
            while (__builtin_amdgcn_ballot_w64(minew && (uint32_t)(gr >> 32) != tag) != 0) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > (1u << 20)) { if (lane == 0) atomicOr(perr, 2u); break; }   // bounded wait
                if (minew) gr = ld_granT<UPL>(g);
            }
        }
        const uint32_t top = (uint32_t)gr;
        if (pst) st0 = (st0 & 0xFFFFFFFFull) | (wall_clock64() << 32);
        {   // tile halo: the row above (dwords), its top-left / top-right (the left
            // column is read from the left MB's slot as it lands, intra_tile)
            if (lane >= 24 && lane < 32) {
                const int k = lane - 24;
                if (aB) *(uint32_t *)(k < 4 ? &M.ty[TX0 + k * 4] : k < 6 ? &M.tu[TX0 + (k - 4) * 4] : &M.tv[TX0 + (k - 6) * 4]) = top;
            } else if (lane == 32) {
            } else if (lane < 36) {
                if (aD) (lane == 33 ? M.ty[TX0 - 1] : lane == 34 ? M.tu[TX0 - 1] : M.tv[TX0 - 1]) = (uint8_t)(top >> 24);
            }
        }
        wave_sync();
        uint8_t *px = R.px[slot];
        const int ls = (c - 1) & (RK - 1);
        LeftNb N;
        N.lp = R.px[ls];
        N.lprog = &R.lprog[ls]; N.cprog = &R.cprog[ls];
        N.my_lprog = &R.lprog[slot]; N.my_cprog = &R.cprog[slot];
        N.ltag = (c - 1) << 4; N.mytag = c << 4;
        N.perr = perr;
        N.chk = CHK;
        N.cg = g; N.cgr = gr; N.ctag = tag; N.cdef = needC;
        intra_tile<UPL, true>(qtype, avail, pred, i4, M.res, cbits != 0, M.ty, M.tu, M.tv, i4tab, M.junk, px, lane, N);
    } else {
        if (pst) st0 = wall_clock64();
        // luma first: its top granules (B dwords 24..27, C, D's luma byte) are
        // waited for and its bottom row is published before the chroma runs, so
        // the row below's luma -- the intra chain from row to row -- does not
        // wait behind this MB's chroma; the chroma granules follow
        const bool lumal = (lane >= 24 && lane < 28) || lane == 32 || lane == 33;
        auto top_wait = [&](bool mine_part) {
            unsigned spins = 0;
            while (__builtin_amdgcn_ballot_w64(mine_part && (uint32_t)(gr >> 32) != tag) != 0) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > (1u << 20)) { if (lane == 0) atomicOr(perr, 2u); break; }   // bounded wait
                if (mine_part) gr = ld_granT<UPL>(g);
            }
        };
        // the above-right granule (needC: I4x4 block 5 in modes 3 / 7) is
        // taken before step 3 only (intra_tile CDEF)
        const bool cdef = needC;
        if (need_top) top_wait(mine && lumal && !(cdef && lane == 32));
        if (pst) st0 = (st0 & 0xFFFFFFFFull) | (wall_clock64() << 32);
        {   // luma tile halo: the row above (dwords), its top-left / top-right (the
            // left column is read from the left MB's slot as it lands, intra_tile)
            const uint32_t top = (uint32_t)gr;
            if (lane >= 24 && lane < 28) {
                if (aB) *(uint32_t *)&M.ty[TX0 + (lane - 24) * 4] = top;
            } else if (lane == 32) {
                if (needC && !cdef) *(uint32_t *)&M.ty[TX0 + 16] = top;
            } else if (lane == 33) {
                if (aD) M.ty[TX0 - 1] = (uint8_t)(top >> 24);
            }
        }
        wave_sync();
        uint8_t *px = R.px[slot];
        const int ls = (c - 1) & (RK - 1);
        LeftNb N;
        N.lp = R.px[ls];
        N.lprog = &R.lprog[ls]; N.cprog = &R.cprog[ls];
        N.my_lprog = &R.lprog[slot]; N.my_cprog = &R.cprog[slot];
        N.ltag = (c - 1) << 4; N.mytag = c << 4;
        N.perr = perr;
        N.chk = CHK;
        N.cg = g; N.cgr = gr; N.ctag = tag; N.cdef = cdef;
        intra_tile<UPL, true>(qtype, avail, pred, i4, M.res, cbits != 0, M.ty, M.tu, M.tv, i4tab, M.junk, px, lane, N, 1);
        if (pub && lane < 4)        // luma bottom row -> the row below (entry c, dwords 24..27)
            st_granT<MEL>(pub + 24 + lane, *(const uint32_t *)&px[240 + lane * 4], tag);
        if (need_top) top_wait(mine && !lumal);
        {   // chroma tile halo
            const uint32_t top = (uint32_t)gr;
            if (lane >= 28 && lane < 32) {
                const int k = lane - 24;
                if (aB) *(uint32_t *)(k < 6 ? &M.tu[TX0 + (k - 4) * 4] : &M.tv[TX0 + (k - 6) * 4]) = top;
            } else if (lane == 34 || lane == 35) {
                if (aD) (lane == 34 ? M.tu[TX0 - 1] : M.tv[TX0 - 1]) = (uint8_t)(top >> 24);
            }
        }
        wave_sync();
        intra_tile(qtype, avail, pred, i4, M.res, cbits != 0, M.ty, M.tu, M.tv, i4tab, M.junk, px, lane, N, 2);
    }
    if (pst) st1 = wall_clock64();
    if (pst && lane == 0) { pst[0] = st0; pst[1] = (st1 & 0xFFFFFFFFull) | (wall_clock64() << 32); }
}

// ---------------------------------------------------------------------------
// k_wgpp: k_wg with TWO row-unit waves per MB row, ping-pong: wave w
// deblocks the MBs c with c % 2 == w.  The deblocking chain along a row is
// strictly sequential (V(c) reads MB c-1's columns 12..15 after H(c-1); H(c)
// follows V(c)), but each MB also carries work off that chain: taking its
// samples and deblocking record out of the MC ring, the speculative
// row-above read, the frame stores, the provisional mailbox entry.  With two
// waves, MB c+1's wave does its off-chain part while MB c's wave runs the
// chain, so the row advances at the chain's pace (copy + V + top + H) rather
// than at the pace of everything one wave does per MB.
//
// Each wave owns one LDS region (the MB's samples with a 4-column left and
// 4-row top halo) used for its MBs in turn.  Hand-offs (LDS flags, both
// monotonic):
//   hdone  = c + 1  once H(c) is done: MB c's region holds its final columns
//                   12..15 for V(c+1), and its rows 12..15 (provisional
//                   mailbox entry, columns 0..11 final)
//   copied = c + 1  once MB c+1's wave has read both: MB c's region is free
// The row hand-off to the row below (mailbox granules) and the frame stores
// are exactly those of row_unit (each sample stored once, by the MB that
// finalises it).  Reference: h264bsdFilterPicture (deblocking.c:574-639),
// filter order per MB vertical then horizontal edges (:603-637).
// ---------------------------------------------------------------------------
struct __attribute__((aligned(16))) PPRegion {
    uint8_t db[64];
    uint8_t ry[20 * RY_S];      // rows -4..15, cols -4..15
    uint8_t ru[10 * RC_S];      // rows -2..7, cols -4..7
    uint8_t rv[10 * RC_S];
};
struct __attribute__((aligned(16))) PPLds {
    PPRegion G[2];
    uint8_t junk[2][256];
    int hdone, copied, pdone, fin;
    uint32_t i4tab[I4TAB_N];
    unsigned long long ptw1[8];     // PROF: wave 1's phase sums, added by wave 0
};

// UPL / MEL: the row above's mailbox (mbx_up) / this row's (mbx_me) is the
// workgroup's LDS one (k_wgpp RPW = 2: the upper row of the pair publishes to
// LDS, the lower one reads from there)
// COLP (frame-pipelined launches): when a later step of the launch reads
// this picture (pubp), the frame stores are write-through (sc1) and the wave
// publishes its store progress, a granule {c, epoch} at the top of each MB c
// behind an s_waitcnt vmcnt(0): every MB of its parity below c is in memory
// (MI355X_MICROARCH.md, valid forms: sc1 payload, drained, sc1 flag).  A
// sample of MB row r, column x is final once row r's MBs 0..x+1 and row
// r+1's MBs 0..x have stored (row r+1 stores row r's rows 12..15 after its
// top-edge filter; MB x+1 stores MB x's columns 12..15 after its left edge).
// row_pp's path for rows without deblocking (see there): store each MB's
// ring slot to the frame as its MC lands, release the slot before it (the
// intra prediction of MB c has read MB c - 1's), and -- when a later step of
// the launch reads this picture (wt: write-through stores) -- publish both
// row waves' store progress.  Out of line, so that it leaves row_pp's
// register allocation alone; LDS and global pointers address-space typed
// (a generic pointer argument would make every access FLAT).  ydst / cdst:
// this lane's luma / chroma dword of MB 0 in the frame.
typedef __attribute__((address_space(1))) uint8_t *g_u8p;
typedef __attribute__((address_space(1))) unsigned long long *g_u64p;
template <int RK, bool CHK>
__device__ __attribute__((noinline)) void row_drain(__attribute__((address_space(3))) MbRing<RK> *Rl, g_u8p ydst, g_u8p cdst,
                                                    int W, bool wt, g_u64p prog0, g_u64p prog1, uint32_t tag, g_u32 *perr_g,
                                                    int lane, const __attribute__((address_space(1))) uint32_t *recw)
{
    MbRing<RK> &R = *(MbRing<RK> *)Rl;
    unsigned *perr = (unsigned *)perr_g;
    const int orow = lane >> 2, oq = lane & 3, li = lane & 31;
    const int ccomp = (li >> 4) & 1, crow = (li >> 1) & 7, cq = li & 1;
    for (int c = 0; c < W; c++) {
        const int slot = c & (RK - 1);
        if (wt && c >= 2 && (c & 1) == 0) {
            // MBs 0..c-1 stored and drained: both parities' progress
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0) { st_gran((unsigned long long *)prog0, (uint32_t)c, tag); st_gran((unsigned long long *)prog1, (uint32_t)c, tag); }
        }
        unsigned spins = 0;
        while (__builtin_amdgcn_readfirstlane(lds_ld(&R.flag[slot])) != c + 1) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > (1u << 22)) { if (lane == 0) atomicOr(perr, 16u); break; }
        }
        wave_sync();
        if (CHK && __builtin_amdgcn_readfirstlane(*(const uint16_t *)&R.db[slot][CHK_TAG_OFF]) != c && lane == 0)
            atomicOr(perr, CHK_RING);
        // (checker: the host's PD_NO_DEBLOCK -- this MB filters nothing)
        if (CHK && ((recw[c * 24] >> 24) & DB_INNER) && lane == 0) atomicOr(perr, CHK_NODB);
        const uint32_t vy = *(const uint32_t *)&R.px[slot][orow * 16 + oq * 4];
        const uint32_t vc = *(const uint32_t *)&R.px[slot][256 + ccomp * 64 + crow * 8 + cq * 4];
        if (wt) st_sc1_u32((uint32_t *)(ydst + c * 16), vy);
        else *(__attribute__((address_space(1))) uint32_t *)(ydst + c * 16) = vy;
        if (lane < 32) {
            if (wt) st_sc1_u32((uint32_t *)(cdst + c * 8), vc);
            else *(__attribute__((address_space(1))) uint32_t *)(cdst + c * 8) = vc;
        }
        wave_sync();
        // MB c done: the intra prediction of MB c has read MB c - 1's slot
        if (lane == 0) lds_st(&R.consumed, c);
    }
    if (lane == 0) lds_st(&R.consumed, W);
    if (wt) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) { st_gran((unsigned long long *)prog0, (uint32_t)W, tag); st_gran((unsigned long long *)prog1, (uint32_t)W, tag); }
    }
}

template <bool PROF, bool UPL, bool MEL, int RK, bool CHK, bool COLP = false>
__device__ void row_pp(const ReconArgs &a, int p, int r, PPLds &L, const int w, const int lane, MbRing<RK> *R,
                       const unsigned long long *mbx_up, unsigned long long *mbx_me, bool pubp = false)
{
    const int W = a.w, H = a.h;
    if (PROF && a.prof_mode == 1) {     // role split (see ReconArgs::prof_mode): drain the ring only
        if (w == 0)
            for (int c = 0; c < W; c++) {
                unsigned spins = 0;
                while (__builtin_amdgcn_readfirstlane(lds_ld(&R->flag[c & (RK - 1)])) != c + 1) {
                    __builtin_amdgcn_s_sleep(1);
                    if (++spins > (1u << 22)) break;
                }
                if (lane == 0) lds_st(&R->consumed, c + 1);
            }
        // a later step's DEP_COLS waits read this row's store progress: the
        // row counts as stored (nothing is, in this study mode), so that they
        // do not poll to their bounded-wait limit
        if (COLP && pubp && lane == 0) st_gran(PROG_AT(a.prog, p, H, r, w), (uint32_t)W, a.epoch);
        return;
    }
    const PicDesc *pdp = a.pics + p;
    const int rec_base = __builtin_amdgcn_readfirstlane(pdp->rec_base);
    const int fslot = __builtin_amdgcn_readfirstlane(pdp->frame_base + pdp->cur_slot);
    const int W16 = W * 16, H16 = H * 16, CP = a.cpitch, CH = H16 / 2;
    uint8_t *cur = a.frames + (unsigned long long)fslot * a.frame_bytes;
    uint8_t *curU = cur + (size_t)W16 * H16;
    unsigned *perr = a.err + p;
    const uint32_t tag = a.epoch;
    const bool has_up = r > 0, has_down = r + 1 < H;
    const bool last_row = r == H - 1;
    typedef const __attribute__((address_space(4))) uint32_t *cu32p;
    const cu32p recw = (cu32p)(const void *)(a.rec + rec_base + r * W);   // 24 dwords per record
    PPRegion &G = L.G[w];
    const PPRegion &Gp = L.G[w ^ 1];
    uint8_t *const junk = L.junk[w];
    uint8_t *const Lb = (uint8_t *)&G;

    const int orow = lane >> 2, oq = lane & 3;                                   // luma 16x16 dwords
    const int li = lane & 31;
    const int ccomp = (li >> 4) & 1, crow = (li >> 1) & 7, cq = li & 1;          // chroma dwords (32..63 mirror)
    const int le = li < 24 ? li : li - 8;                                        // mailbox entry dword
    uint8_t *const ybase = cur + (size_t)r * 16 * W16;
    uint8_t *const cbase = curU + (size_t)r * 8 * CP;
    const uint32_t yoff = (uint32_t)(orow * W16 + oq * 4);
    const uint32_t coff = (uint32_t)(ccomp * CP * CH + crow * CP + cq * 4);
    // common-case frame store maps (as row_unit): offsets in the region /
    // relative to (row r*16-4 | r*8-2, col -4) of MB c
    uint32_t sa_lds, sa_glb, sb_lds, sb_glb;
    bool sa_left, sa_top, sb_left, sb_top;
    {
        const int Lry = (int)(G.ry - Lb), Lru = (int)(G.ru - Lb), Lrv = (int)(G.rv - Lb);
        int row, col;
        if (lane < 36) { row = lane / 3; col = (lane % 3) * 4; }
        else if (lane < 48) { row = lane - 36; col = -4; }
        else { row = -4 + ((lane - 48) >> 2); col = ((lane - 48) & 3) * 4; }
        sa_lds = (uint32_t)(Lry + (row + 4) * RY_S + 4 + col);
        sa_glb = (uint32_t)((row + 4) * W16 + col + 4);
        sa_left = lane >= 36 && lane < 48;
        sa_top = lane >= 48;
        int comp;
        const int k = lane & 31;
        if (k < 12) { comp = k / 6; row = k % 6; col = 0; }
        else if (k < 24) { comp = (k - 12) / 6; row = (k - 12) % 6; col = -4; }
        else { comp = (k - 24) >> 2; row = -2 + (((k - 24) >> 1) & 1); col = ((k - 24) & 1) * 4; }
        sb_lds = (uint32_t)((comp ? Lrv : Lru) + (row + 2) * RC_S + 4 + col);
        sb_glb = (uint32_t)(comp * CP * CH + (row + 2) * CP + col + 4);
        sb_left = k >= 12 && k < 24;
        sb_top = k >= 24;
    }
    // left-halo copy from the partner's region: lanes 0..15 luma rows, 16..31
    // chroma rows (cols 12..15 / 4..7 -> -4..-1); lanes 32..63 into junk
    // (lanes 32..63 read what lanes 0..31 read -- the vertical pass takes
    // the copied dword as its line's halo, and its lanes 32..63 mirror)
    uint32_t cp_src, cp_dst;
    {
        int off, step;
        const uint8_t *D;
        const int cl = lane & 31;
        if (cl < 16) { D = Gp.ry; off = (cl + 4) * RY_S; step = 16; }
        else { const int k = cl - 16; D = (k >> 3) ? Gp.rv : Gp.ru; off = ((k & 7) + 2) * RC_S; step = 8; }
        cp_src = (uint32_t)((int)(D - (const uint8_t *)&Gp) + off + step);
        cp_dst = lane < 32 ? (uint32_t)((int)(D - (const uint8_t *)&Gp) + off) : (uint32_t)((int)(junk - Lb) + lane * 4);
    }
    // publishing: slot ls = le (0..23; lanes 24..63 repeat slots 16..23 /
    // 0..23 with the same values) stores granule gi(ls).  Slots 0..7 are the
    // 8 granules MB c+1's left edge patches (luma rows 12..15 / Cb, Cr rows
    // 6..7, the dword holding columns 12..15 / 4..7) -- patch lane pj = ls
    // publishes its own result, no cross-lane move; slots 8..23 the others.
    uint32_t prov_off;      // the granule's provisional dword in the region (rows 12..15, cols 0..15)
    uint32_t ent_glb;       // ... and its frame offset (rows 12..15 / chroma 6..7)
    int gi;
    {
        const int ls = le;
        int yrow, yq, comp, row, qq;
        bool luma;
        if (ls < 8) {
            luma = ls < 4;
            yrow = ls & 3; yq = 3;
            comp = (ls >> 1) & 1; row = ls & 1; qq = 1;
        } else if (ls < 20) {
            luma = true;
            yrow = (ls - 8) / 3; yq = (ls - 8) % 3;
            comp = row = qq = 0;
        } else {
            luma = false;
            yrow = yq = 0;
            comp = (ls - 20) >> 1; row = (ls - 20) & 1; qq = 0;
        }
        gi = luma ? yrow * 4 + yq : 16 + comp * 4 + row * 2 + qq;
        // its place in the frame, from MB c's luma / chroma origin
        ent_glb = luma ? (uint32_t)((12 + yrow) * W16 + yq * 4) : (uint32_t)(comp * CP * CH + (6 + row) * CP + qq * 4);
        prov_off = luma ? (uint32_t)((int)(G.ry - Lb) + (16 + yrow) * RY_S + 4 + yq * 4)
                        : (uint32_t)((int)((comp ? G.rv : G.ru) - Lb) + (8 + row) * RC_S + 4 + qq * 4);
    }
    // ---- the hand-off to the row below, made by the wave that ran H(c):
    //      MB c's rows 12..15 are final except columns 13..15, which MB c+1's
    //      left edge (V(c+1) edge 0) still changes.  That edge reads MB c's
    //      columns 12..15 (this region, now final w.r.t. H(c)) and MB c+1's
    //      unfiltered columns 0..3 (its ring slot), with MB c+1's bS and
    //      left-edge thresholds (its deblocking record, also in the slot) --
    //      so this wave applies it to those 8 lines (lanes 0..7: luma rows
    //      12..15, Cb rows 6/7, Cr rows 6/7) and publishes the final rows
    //      without waiting for the partner's V(c+1).
    const int pj = lane & 7;
    const bool pchroma = pj >= 4;
    int pq_off;             // q side: cols 0..3 of the ring slot's MB (p side: the lane's own provisional dword)
    {
        const int comp = (pj >> 1) & 1, row = pj & 1;
        pq_off = !pchroma ? (12 + pj) * 16 : 256 + comp * 64 + (6 + row) * 8;
    }
    const bool is_patch = le < 8;
    // the vertical pass's line in the region (deblock_dir dir 0): luma rows
    // for lanes 0..15, Cb / Cr rows for 16..31 (32..63 mirror)
    uint32_t vrow_lds;
    {
        const int vl = lane & 31, vch = vl >= 16, vidx = vch ? (vl & 7) : (vl & 15);
        const uint8_t *D = vch ? ((vl & 8) ? G.rv : G.ru) : G.ry;
        vrow_lds = (uint32_t)((int)(D - Lb) + (vidx + (vch ? 2 : 4)) * RY_S);
    }
    // own samples from the ring slot: luma all lanes, chroma lanes 0..31
    const uint32_t own_y_lds = (uint32_t)((int)(G.ry - Lb) + (orow + 4) * RY_S + 4 + oq * 4);
    const uint32_t own_c_lds = lane < 32 ? (uint32_t)((int)((ccomp ? G.rv : G.ru) - Lb) + (crow + 2) * RC_S + 4 + cq * 4)
                                         : (uint32_t)((int)(junk - Lb) + lane * 4);
    const uint32_t db_lds = lane < 16 ? (uint32_t)(lane * 4) : (uint32_t)((int)(junk - Lb) + lane * 4);
    // top halo lanes 0..23: entry dword lane -> region rows 0..3 / chroma rows 0..1
    uint32_t top_lds;
    {
        const int k = lane - 16, comp = k >> 2, row = (k >> 1) & 1, qq = k & 1;
        top_lds = lane < 16 ? (uint32_t)((int)(G.ry - Lb) + orow * RY_S + 4 + oq * 4)
                : lane < 24 ? (uint32_t)((int)((comp ? G.rv : G.ru) - Lb) + row * RC_S + 4 + qq * 4)
                            : (uint32_t)((int)(junk - Lb) + lane * 4);
    }
    unsigned long long *const sink = a.gjunk + ((p * H + r) & 127) * 64 + lane;
    const bool wt = COLP && pubp;       // write-through frame stores + progress granules
    unsigned long long *const prog_me = PROG_AT(a.prog, p, H, r, w);
    auto fst = [&](void *ptr, uint32_t v) {
        if (wt) st32<true>(ptr, v);
        else st32<false>(ptr, v);
    };

    unsigned long long pt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const bool prof = PROF && a.prof != nullptr;
    unsigned long long tc0 = 0, tc1, tva = 0, tvd = 0;
#define PPT(i) do { if (prof) { tc1 = clock64(); pt[i] += tc1 - tc0; tc0 = tc1; } } while (0)
    if (prof && w == 0 && lane == 0) {
        a.prof[((size_t)r * a.npics + p) * 16] = wall_clock64();
        // placement: HW_REG_HW_ID (CU / SH / SE of this wave) and HW_REG_XCC_ID
        a.prof[((size_t)r * a.npics + p) * 16 + 10] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
        a.prof[((size_t)r * a.npics + p) * 16 + 11] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);
    }

    for (int c = w; c < W; c += 2) {
        if (a.row_prio_split) __builtin_amdgcn_s_setprio(1);
        if (wt && c >= 2 && ((c >> 1) % PROG_EVERY) == 0) {
            // MB c - 2's write-through stores (issued one MB of the partner
            // earlier) drained: publish this wave's progress, off the chain
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0) st_gran(prog_me, (uint32_t)c, tag);
        }
        if (prof) tc0 = clock64();
        // per-MB stamps (100 MHz wall clock): [0] row-above entry c in hand (H(c)
        // may start); [1] V(c) start (after the hdone wait and halo copy) in
        // bits 0..31, V(c) end in bits 32..63; [2] entry c published in bits
        // 0..31, H(c) end (hdone = c + 1) in bits 32..63
        unsigned long long *pmb = prof ? a.prof + (size_t)a.npics * H * 16 + ((size_t)(p * H + r) * W + c) * PROF_MB : nullptr;
        const cu32p rw = recw + c * 24;
        const uint32_t h0 = rw[0];
        // MB c+1's record dword 0 (avail), for the hand-off patch (a VMEM load:
        // an SMEM one would couple to every LDS wait through lgkmcnt)
        const uint32_t avn = ldg32(uni(a.rec + rec_base + r * W + min(c + 1, W - 1)), 0);
        const int avail = (h0 >> 24) & 255;
        const bool dbf = avail & DB_INNER;
        // The top MB edge is filtered (filterTopMbEdgeFlag, deblocking.c:
        // 288-319): only then does H(c) need the row above's final rows
        // 12..15, and only then does this MB store them (after its top-edge
        // filter).  Otherwise -- disable_deblocking_filter_idc 1, or 2 with
        // the MB above in another slice -- the MB above stores them itself
        // and this MB does not wait on the row above at all.
        const bool top_on = has_up && (avail & DB_INNER) && (avail & DB_TOP);
        // the MB below's record dword 0 (its top-edge flags: who stores this
        // MB's rows 12..15); a VMEM load, like avn
        const uint32_t avd = has_down ? ldg32(uni(a.rec + rec_base + (r + 1) * W + c), 0) : 0u;
        // speculative read of the row above's entry c (lanes 0..23 used)
        const unsigned long long *tga = mbx_up + c * 32 + (lane < 24 ? lane : (lane & 15));
        unsigned long long gr = top_on ? ld_granT<UPL>(tga) : 0ull;
        // ---- off the chain: my region is free once MB c-1's wave read MB c-2's
        {
            unsigned spins = 0;
            while (c >= 2 && __builtin_amdgcn_readfirstlane(lds_ld(&L.copied)) < c - 1) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > (1u << 22)) { if (lane == 0) atomicOr(perr, 16u); break; }
            }
        }
        PPT(6);
        const int slot = c & (RK - 1);
        {
            unsigned spins = 0;
            while (__builtin_amdgcn_readfirstlane(lds_ld(&R->flag[slot])) != c + 1) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > (1u << 22)) { if (lane == 0) atomicOr(perr, 16u); break; }
            }
        }
        wave_sync();
        PPT(7);
        if (CHK && __builtin_amdgcn_readfirstlane(*(const uint16_t *)&R->db[slot][CHK_TAG_OFF]) != c && lane == 0)
            atomicOr(perr, CHK_RING);
        {
            const uint32_t oy = *(const uint32_t *)&R->px[slot][orow * 16 + oq * 4];
            const uint32_t oc = *(const uint32_t *)&R->px[slot][256 + ccomp * 64 + crow * 8 + cq * 4];
            const uint32_t od = ((const uint32_t *)R->db[slot])[lane & 15];
            *(uint32_t *)(Lb + own_y_lds) = oy;
            *(uint32_t *)(Lb + own_c_lds) = oc;
            *(uint32_t *)(Lb + db_lds) = od;
        }
        // both passes' filter parameters, off the chain (the record just
        // copied in; a wave's LDS accesses complete in order)
        wave_sync();
        const DbPar Pv = dbpar(0, G.db, lane, avail & DB_LEFT);
        const DbPar Ph = dbpar(1, G.db, lane, avail & DB_TOP);
        // the vertical pass's own columns 0..15 of the lane's line (only its
        // left halo arrives on the chain)
        uint32_t vpre[4];
        {
            const uint32_t *row = (const uint32_t *)(Lb + vrow_lds);
#pragma unroll
            for (int j = 0; j < 4; j++) vpre[j] = row[1 + j];
        }
        // the hand-off patch's inputs (below): MB c+1's unfiltered columns
        // 0..3 and its left-edge bS / thresholds, from its ring slot -- its MC
        // is normally long done, so they are read here, off the chain, and
        // only re-read after H(c) if its flag was not set yet (one LDS round
        // trip: the MC wave writes the slot before the flag)
        const int s1 = (c + 1) & (RK - 1);
        const bool pmore = has_down && c + 1 < W;
        bool p_ready = false;
        int p_bS = 0, p_alpha = 0, p_beta = 0;
        uint32_t p_q = 0, p_tcs = 0;
        auto patch_in = [&](int fl) {
            const uint32_t *dbn = (const uint32_t *)R->db[s1];
            p_q = *(const uint32_t *)&R->px[s1][pq_off];
            const uint32_t bsw = dbn[1], t0 = dbn[pchroma ? 12 : 6], t1 = dbn[pchroma ? 13 : 7];
            const uint32_t avb = avn >> 24;
            const bool on = (avb & DB_INNER) && (avb & DB_LEFT);
            p_bS = on ? (int)((bsw >> 16) & 15) : 0;      // byte 6 low nibble: dir 0, seg 3, edge 0
            p_alpha = t0 & 255; p_beta = (t0 >> 8) & 255;
            p_tcs = (((t0 >> 8) & 0xFFFF00u) | (t1 << 24)) + (pchroma ? 0x01010100u : 0u);
            p_ready = __builtin_amdgcn_readfirstlane(fl) == c + 2;
        };
        if (pmore) {
            const int fl = lds_ld(&R->flag[s1]);
            wave_sync();
            patch_in(fl);
        }
        PPT(0);
        if (a.row_prio_split) __builtin_amdgcn_s_setprio(3);
        // ---- the chain: MB c-1's H pass done -> its columns 12..15
        uint32_t vhalo = 0;     // the vertical pass's left halo (MB c-1's columns 12..15), c > 0
        if (c > 0) {
            unsigned spins = 0;
            while (__builtin_amdgcn_readfirstlane(lds_ld(&L.hdone)) < c) {
                // (no sleep: the partner's hdone store is the chain's next step)
                if (++spins > (1u << 22)) { if (lane == 0) atomicOr(perr, 16u); break; }
            }
            wave_sync();
            PPT(3);
            if (CHK && __builtin_amdgcn_readfirstlane(*(const uint16_t *)&Gp.db[CHK_TAG_OFF]) != c - 1 && lane == 0)
                atomicOr(perr, CHK_REGION);
            if (prof && lane == 0) tva = wall_clock64();
            const uint32_t hv = *(const uint32_t *)((const uint8_t *)&Gp + cp_src);
            *(uint32_t *)(Lb + cp_dst) = hv;
            vhalo = hv;
            wave_sync();
            if (lane == 0) { lds_st(&L.copied, c); lds_st(&R->consumed, c); }
        } else {
            wave_sync();
            if (lane == 0) lds_st(&R->consumed, 0);
        }
        // ---- vertical edges
        // (measured: reading the left halo straight from the partner's region
        // inside V and releasing it after the MB
        // edge was 3 us per launch slower than this copy)
#ifdef STUDY_V_DELAY
        // study build: lengthen the vertical pass (the own chain only: the
        // hand-off to the row below leaves after H)
        __builtin_amdgcn_s_sleep(STUDY_V_DELAY);
#endif
        if (dbf) deblock_dir(0, Pv, G.ry, G.ru, G.rv, junk, lane, vpre, c > 0, vhalo);
        wave_sync();
        PPT(1);
        if (prof && lane == 0) { if (c == 0) tva = wall_clock64(); pmb[1] = (tva & 0xFFFFFFFFull) | (wall_clock64() << 32); }
        // ---- top halo (row above's entry c final), horizontal edges
        if (top_on) {
            unsigned spins = 0;
            const bool mine = lane < 24;
            // (measured: four staggered polls in flight made the hand-off
            // slower -- median 0.83 vs 0.68 us; the poll's latency is the
            // consumer CU's memory queue, MI355X_MICROARCH.md handoff-1to1)
            while (__builtin_amdgcn_ballot_w64(mine && (uint32_t)(gr >> 32) != tag) != 0) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > (1u << 20)) { if (lane == 0) atomicOr(perr, 2u); break; }
                if (mine) gr = ld_granT<UPL>(tga);
            }
            *(uint32_t *)(Lb + top_lds) = (uint32_t)gr;
            wave_sync();
        }
        if (prof && lane == 0) pmb[0] = wall_clock64();
        PPT(5);
        if (dbf) {
            deblock_dir(1, Ph, G.ry, G.ru, G.rv, junk, lane);
            wave_sync();
        }
#ifdef STUDY_CHAIN_DELAY
        // study build: lengthen the in-row chain by a fixed delay per MB (how
        // much of the own chain reaches the launch time)
        __builtin_amdgcn_s_sleep(STUDY_CHAIN_DELAY);
#endif
        if (lane == 0) lds_st(&L.hdone, c + 1);
        if (prof && lane == 0) tvd = wall_clock64();
        PPT(2);
        if (has_down) {
            const bool more = c + 1 < W;
            uint32_t ent = *(const uint32_t *)(Lb + prov_off);
            if (more) {
                if (!p_ready) {
                    unsigned spins = 0;
                    while (__builtin_amdgcn_readfirstlane(lds_ld(&R->flag[s1])) != c + 2) {
                        __builtin_amdgcn_s_sleep(1);
                        if (++spins > (1u << 22)) { if (lane == 0) atomicOr(perr, 16u); break; }
                    }
                    wave_sync();
                    patch_in(c + 2);
                }
                if (CHK && __builtin_amdgcn_readfirstlane(*(const uint16_t *)&R->db[s1][CHK_TAG_OFF]) != c + 1 && lane == 0)
                    atomicOr(perr, CHK_RING);
                const uint32_t pdw = ent;
                int v[20];
#pragma unroll
                for (int x = 0; x < 4; x++) { v[x] = (pdw >> (8 * x)) & 255; v[4 + x] = (p_q >> (8 * x)) & 255; }
#pragma unroll
                for (int x = 8; x < 20; x++) v[x] = 0;
                filt_line<true>(v, 0, p_bS, p_alpha, p_beta, pchroma ? 0 : p_beta, p_tcs);
                const uint32_t newp = (uint32_t)v[0] | ((uint32_t)v[1] << 8) | ((uint32_t)v[2] << 16) | ((uint32_t)v[3] << 24);
                if (is_patch) ent = newp;
            }
            // rows 12..15 (chroma 6..7) are final: to the MB below, which
            // filters its top edge and stores them, or straight to the frame
            const uint32_t bflags = (uint32_t)__builtin_amdgcn_readfirstlane((int)avd) >> 24;
            // (lanes 0..23 hold the 24 granules once; the lanes above would
            // store duplicates of them)
            if ((bflags & (DB_INNER | DB_TOP)) == (DB_INNER | DB_TOP)) { if (lane < 24) st_granT<MEL>(mbx_me + (size_t)c * 32 + gi, ent, tag); }
            else if (lane < 24) fst((gi < 16 ? ybase + c * 16 : cbase + c * 8) + ent_glb, ent);
            if (prof && lane == 0) pmb[2] = (wall_clock64() & 0xFFFFFFFFull) | (tvd << 32);
        }
        // ---- off the chain again: frame stores, once per sample
        if (a.row_prio_split) __builtin_amdgcn_s_setprio(1);
        if (!last_row && c != W - 1) {
            const uint32_t va = *(const uint32_t *)(Lb + sa_lds);
            const uint32_t vb = *(const uint32_t *)(Lb + sb_lds);
            uint8_t *const yb = ybase + c * 16 - 4 * W16 - 4;
            uint8_t *const cb = cbase + c * 8 - 2 * CP - 4;
            const bool oka = (!sa_left || c > 0) && (!sa_top || top_on);
            const bool okb = (!sb_left || c > 0) && (!sb_top || top_on);
            fst(oka ? (void *)(yb + sa_glb) : (void *)sink, va);
            fst(okb ? (void *)(cb + sb_glb) : (void *)((uint32_t *)sink + 1), vb);
        } else {
            const int yrows = last_row ? 16 : 12;
            const int crows = last_row ? 8 : 6;
            const bool last_col = c == W - 1;
            if (orow < yrows && (oq < 3 || last_col))
                fst(ybase + c * 16 + yoff, *(const uint32_t *)&G.ry[(orow + 4) * RY_S + 4 + oq * 4]);
            if (lane < 32 && crow < crows && (cq == 0 || last_col))
                fst(cbase + c * 8 + coff, *(const uint32_t *)&(ccomp ? G.rv : G.ru)[(crow + 2) * RC_S + 4 + cq * 4]);
            if (c > 0) {
                if (lane < 16) {
                    if (lane < yrows)
                        fst(ybase + c * 16 - 4 + lane * W16, *(const uint32_t *)&G.ry[(lane + 4) * RY_S]);
                } else if (lane < 32) {
                    const int k = lane - 16, comp = k >> 3, row = k & 7;
                    if (row < crows)
                        fst(cbase + c * 8 - 4 + comp * CP * CH + row * CP, *(const uint32_t *)&(comp ? G.rv : G.ru)[(row + 2) * RC_S]);
                }
            }
            if (top_on) {
                if (lane >= 32 && lane < 48) {
                    const int k = lane - 32;
                    fst(ybase + c * 16 + (k & 3) * 4 + (-4 + (k >> 2)) * W16, *(const uint32_t *)&G.ry[(k >> 2) * RY_S + 4 + (k & 3) * 4]);
                } else if (lane >= 48 && lane < 56) {
                    const int k = lane - 48, comp = k >> 2, row = (k >> 1) & 1, qq = k & 1;
                    fst(cbase + c * 8 + qq * 4 + comp * CP * CH + (row - 2) * CP, *(const uint32_t *)&(comp ? G.rv : G.ru)[row * RC_S + 4 + qq * 4]);
                }
            }
        }
        wave_sync();
        PPT(4);
    }
    if (wt) {
        // the row's last MBs of this parity: every MB of the wave stored
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) st_gran(prog_me, (uint32_t)W, tag);
    }
    if (prof) {
        unsigned long long *o = a.prof + ((size_t)r * a.npics + p) * 16;
        if (lane == 0 && ((W - 1) & 1) == w) o[1] = wall_clock64();
        if (w == 1) {
            if (lane == 0) {
                for (int i = 0; i < 8; i++) L.ptw1[i] = pt[i];
                wave_sync();
                lds_st(&L.pdone, 1);
            }
        } else {
            unsigned spins = 0;
            while (__builtin_amdgcn_readfirstlane(lds_ld(&L.pdone)) == 0 && ++spins < (1u << 22)) __builtin_amdgcn_s_sleep(1);
            wave_sync();
            if (lane == 0)
                for (int i = 0; i < 8; i++) o[2 + i] = pt[i] + L.ptw1[i];
        }
    }
#undef PPT
}

// ---------------------------------------------------------------------------
// Software-pipelined MC for k_wgpp (k_prep outputs, single-picture launches):
// mc_issue issues every HBM load of one MB -- its k_prep outputs (deblocking
// record, residual) and its reference windows -- from the MB's record held
// one dword per lane (lane i < 24: dword i), so an MC wave issues MB c+NMC's
// loads right after finishing MB c and they land while it waits for a free
// ring slot; mc_finish stages them into LDS and interpolates.  Same
// arithmetic as mc_core (reconstruct.c:1819-1941, :2222-2314).
// ---------------------------------------------------------------------------
struct McLoad {
    uint32_t lw[3][3], cw[2][2];     // reference windows (luma rows lsub+4k; chroma rows yy, yy+1)
    uint32_t dbw, r0, r1, r2, r3;    // k_prep outputs (r*: half a residual block, lanes 0..47)
    uint32_t mvl, mvc;               // the lane's luma / chroma block MV (x | y << 16)
    int l_x0, l_ax, c_x0, c_ax;      // window geometry (per lane)
};

// dword vectors at 4-byte alignment (the windows start on any dword)
typedef uint32_t u32x3a4 __attribute__((ext_vector_type(3), aligned(4)));
typedef uint32_t u32x2a4 __attribute__((ext_vector_type(2), aligned(4)));
__device__ __forceinline__ uint32_t rec_dw(uint32_t v0, int i) { return (uint32_t)__builtin_amdgcn_readlane((int)v0, i); }

// Reference windows are addressed from the stream's first slot (a uniform
// 64-bit base in SGPRs) with 32-bit per-lane offsets: slot * frame_bytes
// (frame_bytes a multiple of 256, so one 24-bit multiply) + row * pitch +
// column, one v_mad_u32_u24 per row.  A stream's slots span far less than
// 4 GiB (17 slots of 2160p: 211 MB).
__device__ __forceinline__ void mc_issue(const ReconArgs &a, const PicDesc &pd, int p, int mb, uint32_t v0, int lane,
                                         McLoad &L, uint32_t *tsd = nullptr)
{
    // k_prep outputs are indexed by the MB's position in the batch (picture p
    // of the launch), not by PicDesc.rec_base: records may sit anywhere in
    // the record pool
    const int gmb = p * (a.w * a.h) + mb;
    const uint32_t d0 = rec_dw(v0, 0), cbits = rec_dw(v0, 2), refs = rec_dw(v0, 6);
    const int rtype = d0 & 255;
    const bool has_res = rtype != MBT_IPCM && cbits != 0;
    const gcu8p pdb = uni(a.dbrec + (size_t)gmb * 64);
    const gcu8p pres = uni(a.res + (size_t)gmb * 384);
    if (rtype < MBT_I4x4) {
        const int mbx = mb % a.w, mby = mb / a.w;
        const int W16 = a.w * 16, H16 = a.h * 16, CW = W16 / 2, CH = H16 / 2;
        const gcu8p sb = uni(a.frames + (unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane(pd.frame_base) * a.frame_bytes);
        const uint32_t fbu = (uint32_t)(a.frame_bytes >> 8);
        const int lb = lane >> 2, lsub = lane & 3;
        const uint32_t mvl = (uint32_t)__builtin_amdgcn_ds_bpermute((7 + lb) << 2, (int)v0);
        L.mvl = mvl;
        const int mvx = (int)(int16_t)(mvl & 0xFFFF), mvy = (int)(int16_t)(mvl >> 16);
        L.l_x0 = mbx * 16 + blk_x(lb) * 4 + (mvx >> 2) - 2;
        const int l_y0 = mby * 16 + blk_y(lb) * 4 + (mvy >> 2) - 2;
        L.l_ax = clip3(0, W16 - 12, L.l_x0 & ~3);
        if (tsd) tsd[0] = (uint32_t)wall_clock64();
        {
            const uint32_t rs = __builtin_amdgcn_ubfe(refs, (uint32_t)(lb >> 2) * 8, 8);
            const uint32_t o = (__umul24(rs, fbu) << 8) + (uint32_t)L.l_ax;
#pragma unroll
            for (int k = 0; k < 3; k++) {
                const int y = clip3(0, H16 - 1, l_y0 + min(lsub + 4 * k, 8));
                const u32x3a4 t = *(const __attribute__((address_space(1))) u32x3a4 *)(sb + (o + __umul24((uint32_t)y, (uint32_t)W16)));
                L.lw[k][0] = t.x; L.lw[k][1] = t.y; L.lw[k][2] = t.z;       // one dwordx3 load
            }
        }
        if (tsd) tsd[1] = (uint32_t)wall_clock64();
        // chroma: lane -> block cb, component lane & 1; lanes 0..31 load
        // window rows 0, 1 (output row 0), lanes 32..63 rows 1, 2 (output row 1)
        const int cb = (lane & 31) >> 1, ccomp = lane & 1, cyy = lane >> 5;
        const uint32_t mvc = (uint32_t)__builtin_amdgcn_ds_bpermute((7 + cb) << 2, (int)v0);
        L.mvc = mvc;
        const int cmx = (int)(int16_t)(mvc & 0xFFFF), cmy = (int)(int16_t)(mvc >> 16);
        L.c_x0 = mbx * 8 + blk_x(cb) * 2 + (cmx >> 3);
        const int c_y0 = mby * 8 + blk_y(cb) * 2 + (cmy >> 3) + cyy;
        L.c_ax = clip3(0, CW - 8, L.c_x0 & ~3);
        {
            const uint32_t rs = __builtin_amdgcn_ubfe(refs, (uint32_t)(cb >> 2) * 8, 8);
            const uint32_t o = (__umul24(rs, fbu) << 8) + (uint32_t)(W16 * H16) +
                               (uint32_t)(ccomp * a.cpitch * CH) + (uint32_t)L.c_ax;
#pragma unroll
            for (int wy = 0; wy < 2; wy++) {
                const int y = clip3(0, CH - 1, c_y0 + wy);
                const u32x2a4 t = *(const __attribute__((address_space(1))) u32x2a4 *)(sb + (o + __umul24((uint32_t)y, (uint32_t)a.cpitch)));
                L.cw[wy][0] = t.x; L.cw[wy][1] = t.y;                      // one dwordx2 load
            }
        }
    }
    if (tsd) tsd[2] = (uint32_t)wall_clock64();
    L.dbw = ldg32(pdb, (uint32_t)(lane & 15) * 4);
    L.r0 = L.r1 = L.r2 = L.r3 = 0;
    // lane 2b + h (< 48) takes rows 2h, 2h+1 of block bit b: 16 B of the
    // compact residual (one dwordx4 load), zero if the block has none
    const int rb = lane >> 1;
    if (has_res && lane < 48 && ((res_mask(rtype, cbits) >> rb) & 1)) {
        const int k = __popc(res_mask(rtype, cbits) & ((1u << rb) - 1));
        const uint4 t = *(const uint4 *)(a.res + (size_t)gmb * 384 + (k * 2 + (lane & 1)) * 8);
        L.r0 = t.x; L.r1 = t.y; L.r2 = t.z; L.r3 = t.w;
    }
}

// returns the MB type; inter MBs end with their samples in px
__device__ __forceinline__ int mc_finish(const ReconArgs &a, int p, uint32_t v0, int lane, const McLoad &L, McScratch &M,
                                         uint8_t *px, int16_t *s_res, uint8_t *db)
{
    const uint32_t d0 = rec_dw(v0, 0), cbits = rec_dw(v0, 2);
    const int rtype = d0 & 255;
    const bool has_res = rtype != MBT_IPCM && cbits != 0;
    if (lane < 16) ((uint32_t *)db)[lane] = L.dbw;
    if (lane == 15 && (L.dbw >> 24)) atomicOr(a.err + p, 1u);        // k_prep's range-error byte
    if (has_res && lane < 48) {
        const int b = lane >> 1, h = lane & 1;
        uint32_t *d = (uint32_t *)s_res;
        const int o = b < 16 ? (blk_y(b) * 4 + h * 2) * 8 + blk_x(b) * 2
                             : 128 + ((b - 16) >> 2) * 32 + ((((b - 16) >> 1) & 1) * 4 + h * 2) * 4 + (b & 1) * 2;
        const int st = b < 16 ? 8 : 4;
        *(uint2 *)(d + o) = make_uint2(L.r0, L.r1);
        *(uint2 *)(d + o + st) = make_uint2(L.r2, L.r3);
    }
    if (rtype >= MBT_I4x4) { wave_sync(); return rtype; }
    const int W16 = a.w * 16, CW = W16 / 2;
    const int lb = lane >> 2, lsub = lane & 3;
    // luma windows realigned into LDS: row wy of block lb = columns 0..8 in
    // bytes 0..8 (h264bsdFillBlock's clamp, reconstruct.c:2222-2314, for
    // windows that leave the picture horizontally; rows were clamped by the
    // loads)
    const bool l_in = L.l_x0 >= 0 && L.l_x0 + 8 <= W16 - 1;
    uint4 own[3];
    {
        const uint32_t xo = (uint32_t)(L.l_x0 - L.l_ax);
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const uint32_t e0 = L.lw[k][0], e1 = L.lw[k][1], e2 = L.lw[k][2];
            uint4 o;
            o.x = __builtin_amdgcn_alignbyte(e1, e0, xo);
            o.y = __builtin_amdgcn_alignbyte(e2, e1, xo);
            o.z = __builtin_amdgcn_alignbyte(0u, e2, xo);
            o.w = 0;
            if (!l_in) {
                uint32_t q[3] = {0, 0, 0};
#pragma unroll
                for (int i = 0; i < 9; i++) {
                    const int kk = clip3(0, W16 - 1, L.l_x0 + i) - L.l_ax;
                    const uint32_t w = kk < 4 ? e0 : (kk < 8 ? e1 : e2);
                    q[i >> 2] |= ((w >> ((kk & 3) * 8)) & 255u) << ((i & 3) * 8);
                }
                o.x = q[0]; o.y = q[1]; o.z = q[2];
            }
            own[k] = o;
            if (k < 2 || lsub == 0) M.wrow[lb][lsub + 4 * k] = o;
        }
    }
    wave_sync();
    uint32_t res_any = has_res;
    {   // luma: lane -> (block b, row yy) = (lb, lsub): window rows yy .. yy + 5
        const int b = lb, yy = lsub;
        const int fx = L.mvl & 3, fy = (L.mvl >> 16) & 3;
        // which candidates some lane needs, by position bit fy * 4 + fx:
        // b of row 2 (fx != 0, fy < 2), b of row 3 (fx != 0, fy == 3), h of
        // columns 2..5 (fy != 0, fx < 2), 3..6 (fy != 0, fx == 3), j (a half
        // position off the axes)
        const uint32_t pm = 1u << (fy * 4 + fx);
        const bool nb2 = __builtin_amdgcn_ballot_w64((pm & 0x00EEu) != 0) != 0;
        const bool nb3 = __builtin_amdgcn_ballot_w64((pm & 0xE000u) != 0) != 0;
        const bool nh = __builtin_amdgcn_ballot_w64((pm & 0x3330u) != 0) != 0;
        const bool nhx = __builtin_amdgcn_ballot_w64((pm & 0x8880u) != 0) != 0;
        const bool nj = __builtin_amdgcn_ballot_w64((pm & 0x4E40u) != 0) != 0;
        uint4 R[6];
        R[0] = own[0];
        R[4] = own[1];
        R[2] = M.wrow[b][yy + 2];
        R[3] = M.wrow[b][yy + 3];
        if (nh || nhx || nj) {
            R[1] = M.wrow[b][yy + 1];
            R[5] = M.wrow[b][yy + 5];
        } else {
            R[1] = R[5] = make_uint4(0, 0, 0, 0);
        }
        uint32_t pk = luma_pred4(R, fx, fy, nb2, nb3, nh, nhx, nj);
        const int bx = blk_x(b) * 4, by = blk_y(b) * 4 + yy;
        if (res_any) {
            const uint2 rr = *(const uint2 *)&s_res[by * 16 + bx];
            const s2v lo = s2of(perm(0u, pk, 0x0C010C00u)) + s2of(rr.x);
            const s2v hi = s2of(perm(0u, pk, 0x0C030C02u)) + s2of(rr.y);
            pk = pack4(clip_pk(lo), clip_pk(hi));
        }
        *(uint32_t *)&px[by * 16 + bx] = pk;
    }
    {   // chroma: lane -> (block cb, comp, row cyy), 2 samples, from the
        // lane's own window rows (no LDS staging)
        const int cb = (lane & 31) >> 1, comp = lane & 1, cyy = lane >> 5;
        const int fx = L.mvc & 7, fy = (L.mvc >> 16) & 7;
        const bool c_in = L.c_x0 >= 0 && L.c_x0 + 2 <= CW - 1;
        // (xo reaches 5 at the right edge: c_ax stops at CW - 8; a 64-bit
        // shift, not v_alignbyte, whose shift is taken mod 4)
        const uint32_t xo8 = (uint32_t)(L.c_x0 - L.c_ax) * 8u;
        uint32_t a0 = (uint32_t)((((uint64_t)L.cw[0][1] << 32) | L.cw[0][0]) >> xo8);
        uint32_t a1 = (uint32_t)((((uint64_t)L.cw[1][1] << 32) | L.cw[1][0]) >> xo8);
        if (!c_in) {
            uint32_t q0 = 0, q1 = 0;
#pragma unroll
            for (int i = 0; i < 3; i++) {
                const int kk = clip3(0, CW - 1, L.c_x0 + i) - L.c_ax;
                const uint32_t w0 = kk < 4 ? L.cw[0][0] : L.cw[0][1], w1 = kk < 4 ? L.cw[1][0] : L.cw[1][1];
                q0 |= ((w0 >> ((kk & 3) * 8)) & 255u) << (i * 8);
                q1 |= ((w1 >> ((kk & 3) * 8)) & 255u) << (i * 8);
            }
            a0 = q0; a1 = q1;
        }
        // (A, B, C, D) of output columns 0 and 1 as bytes; weights alike
        const uint32_t q0 = perm(a1, a0, 0x05040100u), q1 = perm(a1, a0, 0x06050201u);
        const uint32_t gx = 8 - fx, gy = 8 - fy;
        const uint32_t wts = (gx * gy) | (fx * gy) << 8 | (gx * fy) << 16 | (fx * fy) << 24;
        const uint32_t v0 = __builtin_amdgcn_udot4(q0, wts, 32u, false) >> 6, v1 = __builtin_amdgcn_udot4(q1, wts, 32u, false) >> 6;
        uint32_t pr = v0 | (v1 << 16);
        const int cx = blk_x(cb) * 2, cy = blk_y(cb) * 2 + cyy;
        const int po = 256 + comp * 64 + cy * 8 + cx;
        if (res_any) pr = uof(clip_pk(s2of(pr) + s2of(*(const uint32_t *)&s_res[po])));
        *(uint16_t *)&px[po] = (uint16_t)perm(0u, pr, 0x0C0C0200u);
    }
    wave_sync();
    return rtype;
}

// Frame-pipelined launches (a.P > 1): before MB mb's reference loads are
// issued, wait until every 128-B line they touch is final in the slots that
// earlier steps of this launch reconstruct.  Each lane takes the windows it
// loads itself (mc_issue's geometry: luma block lane >> 2, window rows
// lane & 3 .. 8; chroma block (lane & 31) >> 1, component lane & 1): the MB
// rows R_lo..R_hi their lines hold and the last MB column X of those lines.
// They need rows R_lo..R_hi final through column X -- those row workgroups'
// stores through MB X + 1 -- and row R_hi + 1's through MB X (row_pp).  A
// line is only read once all of its bytes are final, so no CU's L1 and no
// XCD's L2 ever holds a stale copy of it (the frame stores are write-through;
// lines from earlier launches were dropped at kernel start), and the loads
// themselves stay plain.  Luma rows whose 128-B lines also hold the end of
// the row above (w % 8 != 0) need that row to its last column.
//
// The producer of a block's reference is the earlier step whose picture of
// this stream writes that slot (at most one: no picture of a launch writes a
// slot an earlier one reads or writes).  Its store progress is read from its
// granules (one per row wave, 8 B: {MBs stored, epoch}); what the row's MC
// waves have seen is kept in the workgroup's LDS (values only grow, so any
// value a wave stores is a valid lower bound), so most MBs need no load.
#define PC_ROWS 136         // MB rows of a producer the LDS progress cache holds (2160p: 135)
// k_wgpp's dependency modes (template DEPM): none (one step per launch), whole
// rows, or (MB row, MB column) cells
enum { DEP_NONE = 0, DEP_ROWS = 1, DEP_COLS = 2 };
struct DepState {
    int n;                 // in-launch producers: steps j - 1 .. j - n (0: none)
    uint32_t slots;        // DEP_COLS: their target slots, 8 bits each (step j - 1 - k at bits 8k)
    uint32_t mask;         // DEP_ROWS: their target slots, a bit each (< 32)
    int pic;               // DEP_ROWS: the step j - 1 picture
    int known;             // DEP_ROWS: its leading rows seen done by this wave
};
typedef __attribute__((address_space(3))) unsigned long long lds_u2;   // {wave 0, wave 1} progress

// rows R_lo..R_hi of producer k final through MB column X (and R_hi + 1
// through X - 1); load: poll the granules the LDS cache cannot vouch for
__device__ __forceinline__ bool dep_rows_ok(const ReconArgs &a, int p, int k, int rlo, int rhi, int X, bool load,
                                            lds_u2 *pc)
{
    const int pk = p - (k + 1) * a.S;
    bool ok = true;
    for (int R = rlo; R <= rhi + 1 && R < a.h; R++) {
        const uint32_t need = (uint32_t)min(R <= rhi ? X + DEPC_SAME_ROW : X + DEPC_ROW_BELOW, a.w);
        const unsigned long long c = R < PC_ROWS ? pc[k * PC_ROWS + R] : 0ull;
        uint32_t vx = (uint32_t)c, vy = (uint32_t)(c >> 32);
        if (min(vx, vy) < need && load) {
            const unsigned long long g0 = ld_gran(PROG_AT(a.prog, pk, a.h, R, 0)), g1 = ld_gran(PROG_AT(a.prog, pk, a.h, R, 1));
            if ((uint32_t)(g0 >> 32) == a.epoch) vx = max(vx, (uint32_t)g0);
            if ((uint32_t)(g1 >> 32) == a.epoch) vy = max(vy, (uint32_t)g1);
            if (R < PC_ROWS) pc[k * PC_ROWS + R] = (unsigned long long)vx | ((unsigned long long)vy << 32);
        }
        ok &= min(vx, vy) >= need;
    }
    return ok;
}

template <bool CHK>
__device__ __forceinline__ void dep_wait_cols(const ReconArgs &a, int p, int mb, uint32_t v0, int lane, const DepState &D,
                                              lds_u2 *pc)
{
    const uint32_t d0 = rec_dw(v0, 0), refs = rec_dw(v0, 6);
    if ((d0 & 255) >= MBT_I4x4) return;
#ifdef STUDY_DEP_NOPOLL
    return;                             // study build (output not valid): no in-launch wait
#endif
    const int W16 = a.w * 16, H16 = a.h * 16, CW = W16 / 2, CH = H16 / 2;
    const int mbx = mb % a.w, mby = mb / a.w;
    auto producer = [&](uint32_t rs) -> int {
        int k = -1;
        for (int i = 0; i < D.n; i++)
            if (((D.slots >> (i * 8)) & 255) == rs) k = i;
        return k;
    };
    // luma: block lb, window rows lsub .. 8 (mc_issue)
    int kl, lrlo, lrhi, lx;
    {
        const int lb = lane >> 2, lsub = lane & 3;
        const uint32_t mvl = (uint32_t)__builtin_amdgcn_ds_bpermute((7 + lb) << 2, (int)v0);
        kl = producer((refs >> ((lb >> 2) * 8)) & 255);
        const int mvx = (int)(int16_t)(mvl & 0xFFFF), mvy = (int)(int16_t)(mvl >> 16);
        const int x0 = clip3(0, W16 - 12, (mbx * 16 + blk_x(lb) * 4 + (mvx >> 2) - 2) & ~3);
        const int y0 = mby * 16 + blk_y(lb) * 4 + (mvy >> 2) - 2;
        const int ya = clip3(0, H16 - 1, y0 + lsub), yb = clip3(0, H16 - 1, y0 + 8);
        if ((W16 & 127) == 0) {             // rows end on lines: a line holds one row's bytes
            lrlo = ya >> 4; lrhi = yb >> 4;
            lx = min((x0 + 11) | 127, W16 - 1) >> 4;
        } else {                            // a line can hold the end of earlier rows: to their last column
            const uint32_t ls = ((uint32_t)ya * W16 + x0) & ~127u, le = ((uint32_t)yb * W16 + x0 + 11) | 127u;
            lrlo = (int)(ls / (uint32_t)W16) >> 4;
            lrhi = min((int)(le / (uint32_t)W16), H16 - 1) >> 4;
            lx = a.w - 1;
        }
    }
    // chroma: block cb, component lane & 1, rows 0..2 (chroma rows padded to 128 B)
    int kc, crlo, crhi, cx;
    {
        const int cb = (lane & 31) >> 1;
        const uint32_t mvc = (uint32_t)__builtin_amdgcn_ds_bpermute((7 + cb) << 2, (int)v0);
        kc = producer((refs >> ((cb >> 2) * 8)) & 255);
        const int cmx = (int)(int16_t)(mvc & 0xFFFF), cmy = (int)(int16_t)(mvc >> 16);
        const int x0 = clip3(0, CW - 8, (mbx * 8 + blk_x(cb) * 2 + (cmx >> 3)) & ~3);
        const int y0 = mby * 8 + blk_y(cb) * 2 + (cmy >> 3);
        crlo = clip3(0, CH - 1, y0) >> 3; crhi = clip3(0, CH - 1, y0 + 2) >> 3;
        cx = min((x0 + 7) | 127, CW - 1) >> 3;
    }
    if (CHK && a.chk_short_cols) { lx = max(lx - a.chk_short_cols, 0); cx = max(cx - a.chk_short_cols, 0); }
    if (CHK && a.chk_short_rows) {
        lrhi = max(lrhi - a.chk_short_rows, 0); crhi = max(crhi - a.chk_short_rows, 0);
        lrlo = min(lrlo, lrhi); crlo = min(crlo, crhi);
    }
    bool okl = kl < 0, okc = kc < 0;
    unsigned spins = 0;
    for (int pass = 0;; pass++) {
        if (!okl) okl = dep_rows_ok(a, p, kl, lrlo, lrhi, lx, pass > 0, pc);
        if (!okc) okc = dep_rows_ok(a, p, kc, crlo, crhi, cx, pass > 0, pc);
        if (__builtin_amdgcn_ballot_w64(!(okl && okc)) == 0) break;
        if (pass > 0) {
            __builtin_amdgcn_s_sleep(4);
            if (++spins > (1u << 21)) { if (lane == 0) atomicOr(a.err + p, 32u); break; }
        }
    }
    // order the reference loads after the polls (compiler: the polls are
    // relaxed atomics; hardware: the wave issues in order)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// DEP_ROWS: the whole-row rule of round 4.  The host records per inter MB
// and 8x8 partition the last reference MB row its lines touch (MbRec.i4 of
// an inter MB, capture.c set_ref_rows), and row workgroup r of a picture
// tags done[p][r] = epoch once its frame stores drained and an agent-scope
// release wrote its XCD's L2 back.  MB row R of a slot is final once rows
// 0..R+1 are done (row R+1 stores row R's rows 12..15).  The done tags are
// chained (row r of step j only after row r of step j - 1), so the step j - 1
// picture's leading rows seen done imply the same rows of every earlier step:
// a partition whose reference slot is any earlier step's target (the mask)
// waits on step j - 1's tags.  For the configs[3] streams, whose windows
// reach the bottom and right picture edges in most rows (5 % off-picture
// MVs), this is as early as the data allows (tools/dep_sim.py) and keeps the
// later pictures' rows idle until then (less contention than DEP_COLS).
template <bool CHK>
__device__ __forceinline__ void dep_wait_rows(const ReconArgs &a, int p, uint32_t v0, int lane, DepState &D)
{
    const uint32_t d0 = rec_dw(v0, 0);
    if ((d0 & 255) >= MBT_I4x4) return;
    const uint32_t rw01 = rec_dw(v0, 4), rw23 = rec_dw(v0, 5), refs = rec_dw(v0, 6);
    int need = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint32_t row = ((q < 2 ? rw01 : rw23) >> ((q & 1) * 16)) & 0xFFFF;
        const uint32_t rs = (refs >> (q * 8)) & 255;
        const uint32_t hit = rs < 32 ? (D.mask >> rs) & 1 : 0;
        need = max(need, hit ? (int)row + 2 : 0);
    }
    if (CHK && a.chk_short_rows) need = max(need - a.chk_short_rows, 0);
    need = min(need, a.h);
    unsigned spins = 0;
    while (need > D.known) {
        const int idx = D.known + lane;
        const bool ok = idx >= a.h || ld_sc1_u32(a.done + (size_t)D.pic * a.h + idx) == a.epoch;
        const unsigned long long m = __builtin_amdgcn_ballot_w64(ok);
        const int adv = __builtin_amdgcn_readfirstlane(~m ? __builtin_ctzll(~m) : 64);
        D.known = min(D.known + adv, a.h);
        if (adv == 0) {
            __builtin_amdgcn_s_sleep(2);
            if (++spins > (1u << 22)) { if (lane == 0) atomicOr(a.err + p, 32u); D.known = a.h; }
        }
    }
    // order the reference loads after the polls (compiler: the polls are
    // relaxed atomics; hardware: the wave issues in order)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// its checker: the rows of the in-launch producer picture that MB mb's
// reference loads need final, from the loads' own geometry (mc_issue's
// windows at 128-B line granularity), must all be among the leading rows
// dep_wait_rows saw done (D.known) -- i.e. set_ref_rows covered every line
// the kernel reads.  Rows 0..R+1 done make MB row R's bytes final.
__device__ __forceinline__ int chk_rows_need(uint32_t o, uint32_t ysz, int W16, int CP, int h)
{
    // MB rows whose workgroups must be done for byte o of a slot to be final
    // (chroma rows padded to CP: no line crosses a plane)
    const uint32_t csz = (uint32_t)CP * (uint32_t)(h * 8);
    const int R = o < ysz ? (int)(o / (uint32_t)W16) >> 4 : (int)(((o - ysz) % csz) / (uint32_t)CP) >> 3;
    return min(R + 2, h);
}
__device__ __forceinline__ void chk_ref_rows_rows(const ReconArgs &a, int p, int mb, uint32_t v0, int lane, const DepState &D)
{
    const uint32_t d0 = rec_dw(v0, 0), refs = rec_dw(v0, 6);
    if ((d0 & 255) >= MBT_I4x4) return;
    const int W16 = a.w * 16, H16 = a.h * 16, CW = W16 / 2, CH = H16 / 2, CP = a.cpitch;
    const uint32_t ysz = (uint32_t)W16 * H16, csz = (uint32_t)CP * CH;
    const int mbx = mb % a.w, mby = mb / a.w;
    int need = 0;
    {   // luma: lane -> block lb, window rows lsub + 4k (mc_issue)
        const int lb = lane >> 2, lsub = lane & 3;
        const uint32_t mvl = (uint32_t)__builtin_amdgcn_ds_bpermute((7 + lb) << 2, (int)v0);
        if (const uint32_t rs = (refs >> ((lb >> 2) * 8)) & 255; rs < 32 && ((D.mask >> rs) & 1)) {
            const int mvx = (int)(int16_t)(mvl & 0xFFFF), mvy = (int)(int16_t)(mvl >> 16);
            const int x0 = clip3(0, W16 - 12, (mbx * 16 + blk_x(lb) * 4 + (mvx >> 2) - 2) & ~3);
            const int y0 = mby * 16 + blk_y(lb) * 4 + (mvy >> 2) - 2;
#pragma unroll
            for (int k = 0; k < 3; k++) {
                const int y = clip3(0, H16 - 1, y0 + min(lsub + 4 * k, 8));
                const uint32_t o = (uint32_t)(y * W16 + x0);
                need = max(need, chk_rows_need(min((o + 11) | 127u, ysz - 1), ysz, W16, CP, a.h));
            }
        }
    }
    {   // chroma: lane -> block cb, component
        const int cb = (lane & 31) >> 1, ccomp = lane & 1;
        const uint32_t mvc = (uint32_t)__builtin_amdgcn_ds_bpermute((7 + cb) << 2, (int)v0);
        if (const uint32_t rs = (refs >> ((cb >> 2) * 8)) & 255; rs < 32 && ((D.mask >> rs) & 1)) {
            const int cmx = (int)(int16_t)(mvc & 0xFFFF), cmy = (int)(int16_t)(mvc >> 16);
            const int x0 = clip3(0, CW - 8, (mbx * 8 + blk_x(cb) * 2 + (cmx >> 3)) & ~3);
            const int y0 = mby * 8 + blk_y(cb) * 2 + (cmy >> 3);
#pragma unroll
            for (int wy = 0; wy < 3; wy++) {
                const int y = clip3(0, CH - 1, y0 + wy);
                const uint32_t base = ysz + (uint32_t)ccomp * csz;
                const uint32_t o = base + (uint32_t)(y * CP + x0);
                need = max(need, chk_rows_need(min((o + 7) | 127u, base + csz - 1), ysz, W16, CP, a.h));
            }
        }
    }
    if (__builtin_amdgcn_ballot_w64(need > D.known) != 0 && lane == 0) atomicOr(a.err + p, CHK_REFROW);
}

// k_wgpp tail workgroup: waves 0..NMC-1 run the next batch's k_prep over a
// grid-stride share of its MBs, in the LDS of the MC scratch and ring (unused
// by a tail workgroup), once enough row workgroups of this and earlier
// launches have finished (their CUs are idle then; k_prep's memory traffic
// beside live row chains would lengthen the chains' L2 hand-offs).  Tail
// workgroups come after every row workgroup in dispatch order, so no row
// ever waits for them; the poll is bounded.
// NW waves take MBs: the NM of them with a McScratch of M, the others
// (single-row layout: the two row waves' slots) one carved from the unused
// ring samples.  The extra waves only for batches of 4 and more pictures:
// measured, 1080p S = 8 +0.5 % frames/s, 2160p S = 1 658 vs 646 us
// (profiles/r31_*)
template <int NW, int NM, int RK>
__device__ __forceinline__ void prep_tail(const ReconArgs &a, McScratch *M, MbRing<RK> &R, int row_wgs)
{
    static_assert(NW <= RK && (NW - NM) * sizeof(McScratch) <= sizeof(R.px), "tail scratch");
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int nw = a.S >= 4 ? NW : NM;
    if (wid >= nw) return;
    McScratch *const Mx = (McScratch *)(void *)R.px;
    unsigned spins = 0;
    while (__hip_atomic_load(a.rows_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < a.prep_target) {
        __builtin_amdgcn_s_sleep(64);
        if (++spins > (1u << 16)) break;            // bounded: ~0.5 s
    }
    PrepArgs pa;
    pa.rec = a.n_rec; pa.coef = a.n_coef; pa.pics = a.n_pics; pa.dbrec = a.n_dbrec; pa.res = a.n_res;
    pa.nmbs_total = a.n_nmbs_total; pa.w = a.w; pa.h = a.h;
    const Tabs T = load_tabs(lane);
    const int t = blockIdx.x - row_wgs;
    for (int g = t * nw + wid; g < pa.nmbs_total; g += a.prep_wgs * nw)
        prep_mb(pa, g, lane, wid < NM ? M[wid] : Mx[wid - NM], R.db[wid], T);
}

// Dependency checker, frame-pipelined launches: every 128-B line MB mb's
// reference loads touch (mc_issue's windows, recomputed from the loads' own
// geometry) must already be final in its in-launch producer picture --
// (MB row, MB column) by (MB row, MB column) of the bytes it holds, read from
// the producers' progress granules just before the loads are issued (values
// only grow: what is final then is final when the loads run).  This checks
// the host's set_ref_rows encoding and dep_wait together.
__device__ __forceinline__ bool chk_row_final(const ReconArgs &a, int pk, int R, uint32_t need)
{
    if (R >= a.h || need == 0) return true;
    const unsigned long long g0 = ld_gran(PROG_AT(a.prog, pk, a.h, R, 0)), g1 = ld_gran(PROG_AT(a.prog, pk, a.h, R, 1));
    const uint32_t v0 = (uint32_t)(g0 >> 32) == a.epoch ? (uint32_t)g0 : 0u;
    const uint32_t v1 = (uint32_t)(g1 >> 32) == a.epoch ? (uint32_t)g1 : 0u;
    return min(v0, v1) >= need;
}
// the bytes [o, o + len) of a plane at pbase (pitch, rows, width bytes; MB
// mbh rows x mbw bytes): every line they touch final in producer pk
__device__ __forceinline__ bool chk_access(const ReconArgs &a, int pk, uint32_t o, int len, uint32_t pbase, int pitch,
                                           int rows, int width, int mbh, int mbw)
{
    bool ok = true;
    for (uint32_t l = o >> 7; l <= (o + len - 1) >> 7; l++) {
        const uint32_t s0 = (l << 7) - pbase, e = (l << 7) + 127 - pbase;
        const int ya = (int)(s0 / (uint32_t)pitch);
        const int yb = min((int)(e / (uint32_t)pitch), rows - 1);
        const int xe = ya == yb ? min((int)(e % (uint32_t)pitch), width - 1) / mbw : (width - 1) / mbw;
        for (int R = ya / mbh; R <= yb / mbh; R++)
            ok &= chk_row_final(a, pk, R, (uint32_t)min(xe + DEPC_SAME_ROW, a.w)) &&
                  chk_row_final(a, pk, R + 1, (uint32_t)min(xe + DEPC_ROW_BELOW, a.w));
    }
    return ok;
}
// (inline: an out-of-line call with the kernel arguments by reference
// fails instruction selection -- a divergent copy into SGPRs)
__device__ __forceinline__ void chk_ref_rows(const ReconArgs &a, int p, int mb, uint32_t v0, int lane, const DepState &D)
{
    const uint32_t d0 = rec_dw(v0, 0), refs = rec_dw(v0, 6);
    if ((d0 & 255) >= MBT_I4x4) return;
    const int W16 = a.w * 16, H16 = a.h * 16, CW = W16 / 2, CH = H16 / 2, CP = a.cpitch;
    const uint32_t ysz = (uint32_t)W16 * H16, csz = (uint32_t)CP * CH;
    const int mbx = mb % a.w, mby = mb / a.w;
    // the in-launch producer of slot rs (or -1)
    auto producer = [&](uint32_t rs) -> int {
        for (int k = 0; k < D.n; k++)
            if (((D.slots >> (k * 8)) & 255) == rs) return p - (k + 1) * a.S;
        return -1;
    };
    bool ok = true;
    {   // luma: lane -> block lb, window rows lsub + 4k (mc_issue)
        const int lb = lane >> 2, lsub = lane & 3;
        const uint32_t mvl = (uint32_t)__builtin_amdgcn_ds_bpermute((7 + lb) << 2, (int)v0);
        const int pk = producer((refs >> ((lb >> 2) * 8)) & 255);
        if (pk >= 0) {
            const int mvx = (int)(int16_t)(mvl & 0xFFFF), mvy = (int)(int16_t)(mvl >> 16);
            const int x0 = clip3(0, W16 - 12, (mbx * 16 + blk_x(lb) * 4 + (mvx >> 2) - 2) & ~3);
            const int y0 = mby * 16 + blk_y(lb) * 4 + (mvy >> 2) - 2;
            for (int k = 0; k < 3; k++) {
                const int y = clip3(0, H16 - 1, y0 + min(lsub + 4 * k, 8));
                ok &= chk_access(a, pk, (uint32_t)(y * W16 + x0), 12, 0, W16, H16, W16, 16, 16);
            }
        }
    }
    {   // chroma: lane -> block cb, component
        const int cb = (lane & 31) >> 1, ccomp = lane & 1;
        const uint32_t mvc = (uint32_t)__builtin_amdgcn_ds_bpermute((7 + cb) << 2, (int)v0);
        const int pk = producer((refs >> ((cb >> 2) * 8)) & 255);
        if (pk >= 0) {
            const int cmx = (int)(int16_t)(mvc & 0xFFFF), cmy = (int)(int16_t)(mvc >> 16);
            const int x0 = clip3(0, CW - 8, (mbx * 8 + blk_x(cb) * 2 + (cmx >> 3)) & ~3);
            const int y0 = mby * 8 + blk_y(cb) * 2 + (cmy >> 3);
            const uint32_t pb = ysz + (uint32_t)ccomp * csz;
            for (int wy = 0; wy < 3; wy++) {
                const int y = clip3(0, CH - 1, y0 + wy);
                ok &= chk_access(a, pk, pb + (uint32_t)(y * CP + x0), 8, pb, CP, CH, CW, 8, 8);
            }
        }
    }
    if (__builtin_amdgcn_ballot_w64(!ok) != 0 && lane == 0) atomicOr(a.err + p, CHK_REFROW);
}

// MC waves of one row (picture p, MB row r): MB c0 first (c0 = the wave's
// index), then -- in P pictures -- the MBs the waves claim from the row's
// counter R.claim, in order, into the row's LDS ring: a wave held up by an
// intra MB (which waits for its left neighbour, then predicts 16 blocks in
// sequence) no longer holds up the MBs that would statically be the other
// waves' turn behind it.  A wave claims its next MB when it starts the
// current one, so its record load is in flight meanwhile.  Intra-heavy
// pictures (PicDesc PD_INTRA_HEAVY) keep the static c0, c0 + NMC, ... walk:
// their MBs wait on each other in order anyway, and the claims measured
// slower there (profiles/r77_ab_mc_claim.txt).  Every wait (ring slot, intra
// neighbours, reference rows) is on a lower-numbered MB, which some wave
// already holds.  UPL / MEL as row_pp: where the row above's unfiltered
// bottom rows come from (intra) / where this row's go.
#ifndef MC_DYN
#define MC_DYN 1
#endif
template <int NMC, bool PROF, bool UPL, bool MEL, int RK, bool CHK, int DEPM>
__device__ __forceinline__ void mc_row(const ReconArgs &a, int p, int r, int c0, int lane, McScratch &Mw, MbRing<RK> &R,
                                       const uint32_t *i4tab, const unsigned long long *mbx_up, unsigned long long *mbx_me,
                                       lds_u2 *pc)
{
    const PicDesc pd = a.pics[p];
    const uint32_t *recrow = (const uint32_t *)(a.rec + pd.rec_base + r * a.w);
    DepState D;
    D.n = 0; D.slots = 0; D.mask = 0; D.pic = 0; D.known = 0;
    if (DEPM != DEP_NONE && a.P > 1) {
        // the earlier steps of this stream in the launch (at most
        // H264MI_MAX_STEPS - 1) and the slots their pictures write
        const int j = p / a.S;
        uint32_t m = 0, mk = 0;
#pragma unroll
        for (int k = 1; k < 4; k++)
            if (k <= j) {
                const uint32_t cs = a.pics[p - k * a.S].cur_slot;
                m |= (cs & 255) << ((k - 1) * 8);
                mk |= 1u << (cs & 31);
            }
        D.n = __builtin_amdgcn_readfirstlane(min(j, 3));
        D.slots = __builtin_amdgcn_readfirstlane(m);
        D.mask = __builtin_amdgcn_readfirstlane(mk);
        D.pic = p - a.S;
    }
    // the next MB of this wave: the row counter's (dynamic) or c + NMC.  The
    // claim is one lane's LDS atomic, exec = lane 0 inside the asm, its
    // result read from lane 0 by v_readlane whatever the caller's exec (no
    // divergent branch in the IR feeding the index; an atomic from all 64
    // lanes on one address serialises: +35 % per launch).  The static walk
    // runs the same block with a zero increment: its wait and compiler
    // barrier at the top of each MB measured 1.4 % faster than without
    // (r77_ab_mc_claim.txt).
    const bool dyn = MC_DYN && !(__builtin_amdgcn_readfirstlane(pd.flags) & PD_INTRA_HEAVY);
    auto next_mb = [&](int c) -> int {
        const unsigned addr = (unsigned)(size_t)(__attribute__((address_space(3))) int *)&R.claim;
        const int inc = dyn ? 1 : 0;
        int u, tmp;
        unsigned long long saved;
        asm volatile("s_mov_b64 %1, exec\n\t"
                     "s_mov_b64 exec, 1\n\t"
                     "ds_add_rtn_u32 %2, %3, %4\n\t"
                     "s_waitcnt lgkmcnt(0)\n\t"
                     "s_mov_b64 exec, %1\n\t"
                     "v_readlane_b32 %0, %2, 0"
                     : "=s"(u), "=&s"(saved), "=&v"(tmp) : "v"(addr), "v"(inc) : "memory");
        return dyn ? u : c + NMC;
    };
    // MB c0's record (lane i < 24: dword i) and loads
    int c = c0;
    uint32_t v0 = c < a.w ? recrow[(size_t)c * 24 + (lane < 24 ? lane : 0)] : 0;
    McLoad ld;
    if (DEPM == DEP_COLS && c < a.w && D.n) dep_wait_cols<CHK>(a, p, r * a.w + c, v0, lane, D, pc);
    if (DEPM == DEP_COLS && CHK && c < a.w && D.n) chk_ref_rows(a, p, r * a.w + c, v0, lane, D);
    if (DEPM == DEP_ROWS && c < a.w && D.n) dep_wait_rows<CHK>(a, p, v0, lane, D);
    if (DEPM == DEP_ROWS && CHK && c < a.w && D.n) chk_ref_rows_rows(a, p, r * a.w + c, v0, lane, D);
    if (c < a.w) mc_issue(a, pd, p, r * a.w + c, v0, lane, ld);

    const int lead = a.mc_lead > 0 && a.mc_lead < RK ? a.mc_lead : RK;
    const int lead0 = a.mc_lead0 > 0 && a.mc_lead0 < lead ? a.mc_lead0 : lead;
    while (c < a.w) {
        const int slot = c & (RK - 1);
        // claim the next MB now and fetch its record
        const int cn = next_mb(c);
        // conditional: the waitcnt pass then makes mc_finish wait for this
        // fresh load too (vmcnt(0)), which measured faster than letting the MC
        // run on (an unconditional, clamped load: vmcnt(1), 317 vs 301 us per
        // step, profiles/r119_ab_nv0.txt) -- the MC waves' pace is not what
        // binds, their share of the CU is
#ifndef MC_NV0_UNCOND
        const uint32_t nv0 = cn < a.w ? recrow[(size_t)cn * 24 + (lane < 24 ? lane : 0)] : 0;
#else
        const uint32_t nv0 = recrow[(size_t)min(cn, a.w - 1) * 24 + (lane < 24 ? lane : 0)];
#endif
        if (c >= lead0) {
            // slot free (ring depth) and at most lead MBs ahead; before the
            // row's chain has begun (consumed < 1: MB 1 not taken yet) at
            // most lead0 -- with the defaults (lead0 = lead = RK) exactly
            // the ring's own condition
            const int need = max(c - lead + 1, lead0 < lead ? 1 : 0);
            unsigned spins = 0;
            while (__builtin_amdgcn_readfirstlane(lds_ld(&R.consumed)) < need) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > (1u << 22)) { if (lane == 0) atomicOr(a.err + p, 16u); break; }
            }
            wave_sync();
        }
        // the slot held MB c - RK: the row waves must have released it
        if (CHK && c >= RK && __builtin_amdgcn_readfirstlane(lds_ld(&R.consumed)) < c - RK + 1 && lane == 0)
            atomicOr(a.err + p, CHK_RING_WR);
        const unsigned long long t0 = PROF ? wall_clock64() : 0;      // MB c's MC start (ring slot free)
        if (NMC == 2) {
            // urgency (2-MC-wave workgroups, 3 per CU): an MC wave whose row
            // unit is within 8 MBs of it issues ahead of the MC waves of rows
            // whose deblocking is far off -- the rows sharing a CU all start
            // their MC at once, and the top rows' MC gates their chains
            // (measured: P-only 350 vs 354 us per launch; 3 MC waves: slower)
            if (c - __builtin_amdgcn_readfirstlane(lds_ld(&R.consumed)) < a.mc_urgency) {
                if (r < a.mc_top) __builtin_amdgcn_s_setprio(3);
                else __builtin_amdgcn_s_setprio(2);
            } else __builtin_amdgcn_s_setprio(0);
        }
        // PROF stamps [4] / [5] of inter MBs (intra MBs: mc_intra's): loads
        // landed (a drain the normal kernel leaves to the loads' first use),
        // samples reconstructed into the slot
        unsigned long long t_ld = 0;
        if (PROF) { drain_vm(); t_ld = wall_clock64(); }
        const int type = mc_finish(a, p, v0, lane, ld, Mw, R.px[slot], Mw.res, R.db[slot]);
        if (PROF && type < MBT_I4x4 && lane == 0) {
            unsigned long long *pm = a.prof + (size_t)a.npics * a.h * 16 + ((size_t)(p * a.h + r) * a.w + c) * PROF_MB;
            pm[4] = (t0 & 0xFFFFFFFFull) | (t_ld << 32);
            pm[5] = wall_clock64() & 0xFFFFFFFFull;
        }
        if (type == MBT_IPCM) {
            const uint32_t *src = (const uint32_t *)(a.coef + ((size_t)pd.coef_base + a.rec[pd.rec_base + r * a.w + c].coef) * 16);
            ((uint32_t *)R.px[slot])[lane] = src[lane];
            if (lane < 32) ((uint32_t *)R.px[slot])[64 + lane] = src[64 + lane];
        } else if (type >= MBT_I4x4) {
            mc_intra<UPL, MEL, RK, CHK, PROF, NMC == 6>((g_MbRec *)(a.rec + pd.rec_base + r * a.w + c), mbx_up, (g_u32 *)(a.err + p), a.w, c, a.epoch,
                              r > 0, lane, (lds_McScratch *)&Mw, (__attribute__((address_space(3))) MbRing<RK> *)&R,
                              (lds_cu32 *)i4tab,
                              PROF ? (unsigned long long *)(a.prof + (size_t)a.npics * a.h * 16 + ((size_t)(p * a.h + r) * a.w + c) * PROF_MB + 4)
                                   : NMC == 6 && r + 1 < a.h ? mbx_me + c * 32 : nullptr);
        }
        wave_sync();
        {   // unfiltered bottom row -> the row below's intra neighbours (entry c,
            // dwords 24..31; an intra MB published its luma dwords 24..27 itself)
            const int kk = lane & 7;
            const uint8_t *px = R.px[slot];
            const uint32_t v = *(const uint32_t *)&px[kk < 4 ? 240 + kk * 4 : kk < 6 ? 312 + (kk - 4) * 4 : 376 + (kk - 6) * 4];
            const int k0 = NMC == 6 && !PROF && (type == MBT_I4x4 || type == MBT_I16) ? 4 : 0;
            if (r + 1 < a.h && lane < 8 && kk >= k0) st_granT<MEL>(mbx_me + c * 32 + 24 + kk, v, a.epoch);
        }
        // PROF stamp [3]: MC start in bits 0..31, flag set (slot final) in bits 32..63 (100 MHz)
        if (PROF && lane == 0)
            a.prof[(size_t)a.npics * a.h * 16 + ((size_t)(p * a.h + r) * a.w + c) * PROF_MB + 3] = (t0 & 0xFFFFFFFFull) | (wall_clock64() << 32);
        if (lane == 0) {
            if (CHK) *(uint16_t *)&R.db[slot][CHK_TAG_OFF] = (uint16_t)(c ^ (a.chk_inject == 1 && c == 5 ? 1 : 0));
            lds_st(&R.lprog[slot], (c << 4) | 10);
            lds_st(&R.cprog[slot], (c << 4) | 1);
            lds_st(&R.flag[slot], c + 1);
        }
        c = cn;
        v0 = nv0;
        const unsigned long long tdw = PROF ? wall_clock64() : 0;
        if (DEPM == DEP_COLS && c < a.w && D.n) dep_wait_cols<CHK>(a, p, r * a.w + c, v0, lane, D, pc);
        if (DEPM == DEP_ROWS && c < a.w && D.n) dep_wait_rows<CHK>(a, p, v0, lane, D);
        // PROF stamp [6] of the next MB: its in-launch dependency wait (100 MHz ticks)
        if (PROF && DEPM != DEP_NONE && c < a.w && lane == 0)
            a.prof[(size_t)a.npics * a.h * 16 + ((size_t)(p * a.h + r) * a.w + c) * PROF_MB + 6] = wall_clock64() - tdw;
        if (DEPM == DEP_COLS && CHK && c < a.w && D.n) chk_ref_rows(a, p, r * a.w + c, v0, lane, D);
        if (DEPM == DEP_ROWS && CHK && c < a.w && D.n) chk_ref_rows_rows(a, p, r * a.w + c, v0, lane, D);
        const unsigned long long tis = PROF ? wall_clock64() : 0;
        uint32_t tsd[3] = {0, 0, 0};
        if (c < a.w) mc_issue(a, pd, p, r * a.w + c, v0, lane, ld, PROF ? tsd : nullptr);
        // PROF stamp [7] of the next MB: its loads' issue began (bits 0..31) / ended (32..63)
        if (PROF && c < a.w && lane == 0) {
            const unsigned long long te = wall_clock64();
            a.prof[(size_t)a.npics * a.h * 16 + ((size_t)(p * a.h + r) * a.w + c) * PROF_MB + 7] =
                (tis & 0xFFFFFFFFull) | (te << 32);
            // [6] with one step per launch (no dependency wait): issue phases, 16 bits each
            // (100 MHz ticks from the issue start): address set-up, luma loads, chroma loads
            if (DEPM == DEP_NONE)
                a.prof[(size_t)a.npics * a.h * 16 + ((size_t)(p * a.h + r) * a.w + c) * PROF_MB + 6] =
                    (unsigned long long)((tsd[0] - (uint32_t)tis) & 0xFFFF) | ((unsigned long long)((tsd[1] - (uint32_t)tis) & 0xFFFF) << 16) |
                    ((unsigned long long)((tsd[2] - (uint32_t)tis) & 0xFFFF) << 32);
        }
    }
}

// RPW MB rows per workgroup (1..3), each with its own NMC MC waves, two row
// waves, ring and region LDS.  Inside the group a row hands its bottom rows
// to the next one through an LDS mailbox (dynamic shared memory, w * 256 B
// per inner boundary) instead of an L2 round trip: (RPW - 1) / RPW of the
// picture's row-to-row hand-offs become LDS ones.
//
// LDS: one dynamic block, [RPW regions | RPW * NMC MC scratch | RPW rings |
// (RPW - 1) mailboxes], sized on the host by WgppLds::bytes.  Dynamic rather
// than static so that the compiler's occupancy check, which reads only
// static LDS, accepts any register budget (WGPP_WAVES_PER_EU).  Residency
// (tools/ubench/census.hip): 320-thread (5-wave) workgroups are admitted 2
// per CU at 117 VGPRs and 3 at 93; 256-thread ones 3 at 117.  A 1080p
// picture's 68 rows on one XCD's 32 CUs need 3 per CU: with 3 MC waves
// (5-wave workgroups, 128 VGPRs) rows 64..67 wait for a free slot (~180 us
// into the launch); a 96-VGPR budget admits them but spills and slows every
// MB (396 vs 366 us per launch), so that variant stays a build option.
template <int NMC, int RPW>
struct WgppLds {
    static constexpr int RK = RPW == 1 ? (NMC == 2 ? RING1_2MC : RING1) : RINGG;
    static constexpr size_t a16(size_t x) { return (x + 15) & ~(size_t)15; }
    static constexpr size_t offM = a16(sizeof(PPLds) * RPW);
    // MC scratch per row: NMC, plus one for row wave 1 of the 2-MC single-row
    // shape, which turns MC wave in pictures without deblocking (k_wgpp)
    static constexpr int NMS = NMC + (NMC == 2 && RPW == 1 ? 1 : 0);
    static constexpr size_t offR = offM + a16(sizeof(McScratch) * RPW * NMS);
    static constexpr size_t offX = offR + a16(sizeof(MbRing<RK>) * RPW);
    static size_t bytes(int w, bool dep3 = false)
    {
        return offX + (size_t)(RPW - 1) * w * 256 + (dep3 ? 3 * PC_ROWS * 8 : 0);
    }
};
#ifndef WGPP_WAVES_PER_EU
#define WGPP_WAVES_PER_EU 4
#endif
// the 2-MC-wave single-row shape's register budget: 4 waves per SIMD (128
// VGPRs, no spill) -- with its 32-slot ring (RING1_2MC, ~28 KB of LDS) four
// four-wave workgroups share a CU: 1,024 row slots, against 768 at 3 (162
// VGPRs, 64 slots).  A two-step launch's 1,088 rows nearly all start at once:
// 307 vs 321 us per step on the configs[3] GOP mix, launches holding an IDR
// 614 vs 669 us (profiles/r82_ab_occupancy.txt); 5 per SIMD spills (448).
#ifndef WGPP2_WAVES_PER_EU
#define WGPP2_WAVES_PER_EU 4
#endif

// DEPM: frame-pipelined launches (two or more steps per stream), DEP_ROWS or
// DEP_COLS (dep_wait_rows / dep_wait_cols); separate instances, so that
// single-step launches carry none of it
template <int NMC, bool PROF, bool PREP, int RPW, bool CHK = false, int DEPM = DEP_NONE>
__global__ __launch_bounds__(64 * (NMC + 2) * RPW)
__attribute__((amdgpu_waves_per_eu(NMC == 3 && RPW == 1 ? WGPP_WAVES_PER_EU : NMC >= 3 || RPW > 1 ? 4 : WGPP2_WAVES_PER_EU))) void k_wgpp(ReconArgs a)
{
    using Lay = WgppLds<NMC, RPW>;
    constexpr int RK = Lay::RK;
    static_assert(RK >= NMC * RPW, "tail workgroups use one ring db entry per wave as k_prep scratch");
    extern __shared__ __attribute__((aligned(16))) unsigned char wg_lds[];
    PPLds *const L = (PPLds *)wg_lds;
    McScratch *const M = (McScratch *)(wg_lds + Lay::offM);
    MbRing<RK> *const R = (MbRing<RK> *)(wg_lds + Lay::offR);
    unsigned long long *const lmbx = (unsigned long long *)(wg_lds + Lay::offX);
    const int S = a.S;
    const int hg = (a.h + RPW - 1) / RPW;
    // blockIdx = (j * hg + g) * S + s: step j's pictures (one per stream)
    // come before step j + 1's, and within a step the S pictures' row group
    // g are dispatched together, groups in order -- so a row's workgroup
    // only waits on earlier ones (the row above, an earlier step's rows)
    if (blockIdx.x >= a.npics * hg) {  // tail workgroup: the next batch's k_prep
        prep_tail<RPW == 1 ? NMC + 2 : NMC * RPW, NMC * RPW, RK>(a, M, R[0], a.npics * hg);
        return;
    }
    const int jg = blockIdx.x / S, s = blockIdx.x - jg * S;
    const int j = jg / hg, g = jg - j * hg, p = j * S + s;
    // a picture without deblocking (PD_NO_DEBLOCK; see below) in the 2-MC
    // single-row shape: its rows are MC-bound, so row wave 1 runs as a third
    // MC wave (MB claims only: P pictures, not intra-heavy ones)
    const uint32_t pflags = __builtin_amdgcn_readfirstlane(a.pics[p].flags);
    const int xmc = (Lay::NMS > NMC && (pflags & PD_NO_DEBLOCK) && !(pflags & PD_INTRA_HEAVY) && MC_DYN) ? 1 : 0;
    for (int q = 0; q < RPW; q++) {
        if (threadIdx.x < RK) { R[q].flag[threadIdx.x] = 0; R[q].lprog[threadIdx.x] = -1; R[q].cprog[threadIdx.x] = -1; }
        if (threadIdx.x == 0) { R[q].consumed = 0; R[q].claim = NMC + xmc; L[q].hdone = 0; L[q].copied = 0; L[q].pdone = 0; L[q].fin = 0; }
    }
    for (int e = threadIdx.x; e < I4TAB_N; e += 64 * (NMC + 2) * RPW)
        L[0].i4tab[e] = i4_entry((e >> 4) % 9, e & 3, (e >> 2) & 3, e >= 9 * 16);
    // frame-pipelined launches: the producers' progress cache (dep_wait)
    lds_u2 *const pc = (lds_u2 *)(__attribute__((address_space(3))) unsigned char *)(wg_lds + Lay::offX);
    if (DEPM == DEP_COLS)
        for (int e = threadIdx.x; e < 3 * PC_ROWS; e += 64 * (NMC + 2) * RPW) pc[e] = 0ull;
    if (RPW > 1)        // granule tags from an earlier workgroup on this CU must not match
        for (int e = threadIdx.x; e < (RPW - 1) * a.w * 32; e += 64 * (NMC + 2) * RPW) lmbx[e] = 0;
    __syncthreads();
    const int wid0 = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int q = RPW == 1 ? 0 : wid0 / (NMC + 2), wid = wid0 - q * (NMC + 2);
    const int r = g * RPW + q;
    if (r >= a.h) return;
    if (PROF && RPW == 1 && wid0 >= 1 && lane == 0)    // placement of waves 1..4 (wave 0: row_pp)
        a.prof[((size_t)r * a.npics + p) * 16 + 11 + wid0] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
    const size_t W32 = (size_t)a.w * 32;
    // mailboxes: the group's first row reads the row above from L2, its last
    // row publishes there; inner boundaries use lmbx[(q - 1) * W32 ..]
    const bool upl = q > 0, mel = q < RPW - 1;
    unsigned long long *const up = upl ? lmbx + (q - 1) * W32 : a.mbx + ((size_t)p * a.h + (r > 0 ? r - 1 : 0)) * W32;
    unsigned long long *const me = mel ? lmbx + q * W32 : a.mbx + ((size_t)p * a.h + r) * W32;
    if (wid < 2) {
        __builtin_amdgcn_s_setprio(3);
        // pictures without deblocking (PicDesc PD_NO_DEBLOCK: no MB filters
        // any edge -- every slice disable_deblocking_filter_idc 1, the
        // reference's recommended `-flags -loop` encode, README.markdown:
        // 32-35; GetMbFilteringFlags drops every edge, deblocking.c:288-319).
        // Every MB's MC output is then final: row wave 0 stores each ring slot
        // straight to the frame as it lands (row_drain: no region, no in-row
        // chain, no row above), row wave 1 has nothing to do.  A host flag,
        // not a scan of the records here: any load on the row waves' way in
        // measurably delays the filtered pictures' first rows.
        const bool nodb = pflags & PD_NO_DEBLOCK;
        if (nodb) {
            if (wid == 0) {
                const int fslot = __builtin_amdgcn_readfirstlane(a.pics[p].frame_base + a.pics[p].cur_slot);
                const int W16 = a.w * 16, CP = a.cpitch, CH = a.h * 8;
                uint8_t *cur = a.frames + (unsigned long long)fslot * a.frame_bytes;
                const int orow = lane >> 2, oq = lane & 3, li = lane & 31;
                const int ccomp = (li >> 4) & 1, crow = (li >> 1) & 7, cq = li & 1;
                uint8_t *ydst = cur + (size_t)r * 16 * W16 + orow * W16 + oq * 4;
                uint8_t *cdst = cur + (size_t)W16 * a.h * 16 + (size_t)r * 8 * CP + ccomp * CP * CH + crow * CP + cq * 4;
                const bool wt = DEPM == DEP_COLS && j + 1 < a.P;
                row_drain<RK, CHK>((__attribute__((address_space(3))) MbRing<RK> *)&R[q], (g_u8p)ydst, (g_u8p)cdst, a.w, wt,
                                   (g_u64p)PROG_AT(a.prog, p, a.h, r, 0), (g_u64p)PROG_AT(a.prog, p, a.h, r, 1), a.epoch,
                                   (g_u32 *)(a.err + p), lane,
                                   (const __attribute__((address_space(1))) uint32_t *)(a.rec + a.pics[p].rec_base + r * a.w));
            } else if (xmc) {
                // the third MC wave: MB NMC first, then claims (R.claim starts at NMC + 1)
                if (RPW == 1)
                    mc_row<NMC, PROF, false, false, RK, CHK, DEPM>(a, p, r, NMC, lane, M[Lay::NMS - 1], R[q], L[0].i4tab, up, me, pc);
            }
        } else if (DEPM == DEP_COLS) row_pp<PROF, false, false, RK, CHK, true>(a, p, r, L[q], wid, lane, &R[q], up, me, j + 1 < a.P);
        else if (!upl && !mel) row_pp<PROF, false, false, RK, CHK>(a, p, r, L[q], wid, lane, &R[q], up, me);
        else if (!upl) row_pp<PROF, false, true, RK, CHK>(a, p, r, L[q], wid, lane, &R[q], up, me);
        else if (mel) row_pp<PROF, true, true, RK, CHK>(a, p, r, L[q], wid, lane, &R[q], up, me);
        else row_pp<PROF, true, false, RK, CHK>(a, p, r, L[q], wid, lane, &R[q], up, me);
        // row finished: progress for the tail workgroups' start
        if (wid == 0 && lane == 0 && a.rows_done)
            __hip_atomic_fetch_add(a.rows_done, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (DEPM == DEP_ROWS && j + 1 < a.P) {
            // a later step of this launch may read this picture: once both
            // row waves' frame stores have completed, the second wave writes
            // the XCD's L2 back and tags the row done -- chained (row r of
            // step j - 1 first; normally long done, this picture's rows
            // having waited on it)
            if (j > 0) {
                const uint32_t *pd = a.done + (size_t)(p - S) * a.h + r;
                unsigned spins = 0;
                while (__builtin_amdgcn_readfirstlane(ld_sc1_u32(pd)) != a.epoch) {
                    __builtin_amdgcn_s_sleep(2);
                    if (++spins > (1u << 22)) { if (lane == 0) atomicOr(a.err + p, 32u); break; }
                }
            }
            drain_vm();
            int last = 0;
            if (lane == 0) last = __hip_atomic_fetch_add(&L[q].fin, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            last = __builtin_amdgcn_readfirstlane(last);
            if (last == 1 && lane == 0) {
#ifndef STUDY_NO_WBL2
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
#endif
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                st_sc1_u32(a.done + (size_t)p * a.h + r, a.epoch);
            }
        }
        return;
    }
    static_assert(PREP, "k_wgpp's MC waves take k_prep outputs");
    McScratch &Mw = M[q * Lay::NMS + wid - 2];
    if (!upl && !mel) mc_row<NMC, PROF, false, false, RK, CHK, DEPM>(a, p, r, wid - 2, lane, Mw, R[q], L[0].i4tab, up, me, pc);
    else if (!upl) mc_row<NMC, PROF, false, true, RK, CHK, DEPM>(a, p, r, wid - 2, lane, Mw, R[q], L[0].i4tab, up, me, pc);
    else if (mel) mc_row<NMC, PROF, true, true, RK, CHK, DEPM>(a, p, r, wid - 2, lane, Mw, R[q], L[0].i4tab, up, me, pc);
    else mc_row<NMC, PROF, true, false, RK, CHK, DEPM>(a, p, r, wid - 2, lane, Mw, R[q], L[0].i4tab, up, me, pc);
}
template __global__ void k_wgpp<3, false, true, 1>(ReconArgs);
template __global__ void k_wgpp<3, true, true, 1>(ReconArgs);
template __global__ void k_wgpp<3, false, true, 2>(ReconArgs);
template __global__ void k_wgpp<3, true, true, 2>(ReconArgs);
template __global__ void k_wgpp<3, false, true, 3>(ReconArgs);
template __global__ void k_wgpp<2, false, true, 2>(ReconArgs);
template __global__ void k_wgpp<2, true, true, 1>(ReconArgs);
template __global__ void k_wgpp<3, true, true, 3>(ReconArgs);
// intra-heavy single-step launches whose rows all fit two workgroups per CU:
// six MC waves per row (engine launch_nmc)
template __global__ void k_wgpp<6, false, true, 1>(ReconArgs);
template __global__ void k_wgpp<6, true, true, 1>(ReconArgs);
// dependency-checker instantiations (H264MI_CHECK=1)
template __global__ void k_wgpp<3, false, true, 1, true>(ReconArgs);
template __global__ void k_wgpp<2, false, true, 1, true>(ReconArgs);
template __global__ void k_wgpp<3, false, true, 2, true>(ReconArgs);
template __global__ void k_wgpp<2, false, true, 2, true>(ReconArgs);
template __global__ void k_wgpp<3, false, true, 3, true>(ReconArgs);
template __global__ void k_wgpp<6, false, true, 1, true>(ReconArgs);
// frame-pipelined launches (single-row, 2 MC waves: launch_batch), by
// dependency mode; the profiling builds for tools/prof_steps.py
template __global__ void k_wgpp<2, false, true, 1, false, DEP_ROWS>(ReconArgs);
template __global__ void k_wgpp<2, false, true, 1, true, DEP_ROWS>(ReconArgs);
template __global__ void k_wgpp<2, true, true, 1, false, DEP_ROWS>(ReconArgs);
template __global__ void k_wgpp<2, false, true, 1, false, DEP_COLS>(ReconArgs);
template __global__ void k_wgpp<2, false, true, 1, true, DEP_COLS>(ReconArgs);
template __global__ void k_wgpp<2, true, true, 1, false, DEP_COLS>(ReconArgs);
