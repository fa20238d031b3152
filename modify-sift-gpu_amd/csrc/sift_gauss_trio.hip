// sift_gauss_trio.hip -- three consecutive Gaussian levels per launch ("trio"), gfx950.
//
// Levels k+1 = V(H(level k)), k+2 = V(H(level k+1)) and k+3 = V(H(level k+2)) (FilterH<FW> then
// FilterV<FW>, ProgramCU.cu:115-222, driven per level by PyramidCU::BuildPyramid,
// PyramidCU.cpp:979-1044) in one pass over level k, plus level k+3's 2x decimation into the next
// octave's level 0 (DownsampleKernel<1>, ProgramCU.cu:287-298; PyramidCU.cpp:1024): 17 B of HBM
// traffic per pixel for the three levels (read level k, write k+1, k+2, k+3 and the quarter-size
// decimation) instead of the 25 B of a paired-level launch (k_gauss_duo) plus a single level.
//
// The paired-level kernel's scheme (sift_gauss_duo.hip) with a third stage:
//   * a wave owns SW output columns of all three levels and walks a band of rows top to bottom,
//     one row pair per step;
//   * stage A: the input row pair (128 + 2 RA columns, clamped) arrives in a wave-private LDS ring
//     by LDS-DMA, NIN - 1 steps ahead; H1 (lane l: mid-A columns mA0 + 2l, + 1, packed over the
//     row pair) reads it with ds_read_b128 and its rows are pushed into the V1 accumulators;
//   * stage B: H2 of the mid-A row pair that stage A completed in the previous step (an LDS mid
//     slot; lane l: mid-B columns mB0 + 2l, + 1), pushed into the V2 accumulators;
//   * stage C: H3 of the mid-B pair that stage B completed in the previous step (lane l: output
//     columns x0 + 2l, + 1), pushed into the V3 accumulators;
//   * every push adds a row into the FW accumulators of the rows it contributes to, in the
//     reference's tap order i = 0 .. FW-1 (one fma each: bit for bit the pull form's sum); the
//     three rings are arrays indexed (row - base) mod P with the step loop unrolled by P / 2;
//   * clamp-to-edge: stage A's rows and columns are clamped in the DMA addresses; rows above 0 /
//     below H-1 of the mid levels read extra LDS pairs -- (mid 0, mid 0) of both mid levels,
//     computed by a prologue in the top band, and (mid H-1, mid H-1), captured during the walk --
//     and mid columns outside the image take the edge column's value by v_readlane.
//
// As in the paired-level kernel every VMEM instruction of a step is issued unconditionally (rows
// outside the band store to a per-wave scratch block), so one s_waitcnt vmcnt(OPS (NIN - 1))
// waits for exactly the step's DMA.  Levels are bit-identical to three k_gauss_lean launches
// (tests/test_gpu_gauss.py).
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <utility>

#include "sift_gauss_ring.h"
#include "sift_kernels.h"

// the DMA asm names M0 as clobbered (gring::dma_pair5): clang warns that M0 is reserved; nothing
// else in this file uses M0
#pragma clang diagnostic ignored "-Winline-asm"

namespace sgk {
namespace {

using namespace gring;

constexpr int kTrioWaves = 4;      // waves per workgroup (each wave works alone: no barriers)
constexpr int kTrioSlot = 256;     // floats of one mid row pair: 128 columns x (row, row + 1)
constexpr int kTrioTrash = 1024;   // floats of scratch per wave slot (1024 slots)
// a compiler barrier between the stages' H passes (their LDS reads are not hoisted above the
// previous stage's pushes: fewer live registers)
#ifndef SGK_TRIO_FENCE
#define SGK_TRIO_FENCE 1
#endif
constexpr bool kTrioFence = SGK_TRIO_FENCE != 0;

// output columns of a wave: the largest multiple of 32 (rows start on 128-B lines, as the duo's
// strips) for which stage B's lanes cover what stage C reads and read inside the 128-column mid-A
// slot: stage C's last lane reads mid-B float2 SW - 2 + OBC + FWC, so stage B needs
// NB = (SW - 2 + OBC + FWC) / 2 + 1 lanes, whose last reads mid-A float2 2 (NB - 1) + OBB + FWB
constexpr int trio_nb(int sw, int obc, int fwc) { return (sw - 2 + obc + fwc) / 2 + 1; }
constexpr int trio_sw(int obb, int fwb, int obc, int fwc) {
    int sw = 128;
    while (sw > 0 && !(trio_nb(sw, obc, fwc) <= 64 && 2 * (trio_nb(sw, obc, fwc) - 1) + obb + fwb <= 127))
        sw -= 32;
    return sw;
}

template <int FWA, int FWB, int FWC>
struct TrioGeom {
    static constexpr int RA = FWA / 2, RB = FWB / 2, RC = FWC / 2;
    // mid-B column of lane 0 = x0 - MOFFC, mid-A column of lane 0 = that - MOFFB (both even:
    // column pairs 8-B aligned); stage B's H2 reads start OBB float2 past its lane's pair, stage
    // C's H3 OBC
    static constexpr int MOFFC = RC + (RC & 1), OBC = MOFFC - RC;
    static constexpr int MOFFB = RB + (RB & 1), OBB = MOFFB - RB;
    static constexpr int SW = trio_sw(OBB, FWB, OBC, FWC);
    static constexpr int NB = trio_nb(SW, OBC, FWC);
    static constexpr int IN_W = 128 + 2 * RA;         // input columns of stage A
    static constexpr int NDMA = (IN_W + 31) / 32;     // dword DMAs per row pair (32 columns each)
    static constexpr int IN_SLOT = NDMA * 64;         // floats of one input row pair
    static constexpr int PMAX = FWA > FWB ? (FWA > FWC ? FWA : FWC) : (FWB > FWC ? FWB : FWC);
    static constexpr int P = (PMAX + 1) & ~1;         // accumulator ring period (rows), even
    static constexpr int U = P / 2;                   // steps per unrolled iteration
};

struct TrioJob {
    const float* src;            // level k
    int src_stride;
    long long src_img;
    float* dst1;                 // level k + 1
    float* dst2;                 // level k + 2
    float* dst3;                 // level k + 3 (rows W apart, images dst_img apart)
    long long dst_img;
    int W, H;
    Taps ta, tb, tc;             // the three filters (widths FWA, FWB, FWC)
    float* ds;                   // level k + 3 decimated into the next octave's level 0
    int dsw, dsh;                // (an odd H's last row decimates into no row when dsh = H / 2)
    long long ds_img;
    int strips, nsy, rows_per_band, total_waves;
    float* trash;                // kTrioTrash floats per wave slot (1024 slots): stores of rows
                                 // outside the band and the DMA prologue's count-keeping stores
};

template <int FWA, int FWB, int FWC, int NIN>
__device__ __forceinline__ void trio_wave(const TrioJob& J, int gw, float* s_in, float* s_ma,
                                          float* s_mb) {
    using G = TrioGeom<FWA, FWB, FWC>;
    constexpr int RA = G::RA, RB = G::RB, RC = G::RC, SW = G::SW, NB = G::NB;
    constexpr int NDMA = G::NDMA, IN_SLOT = G::IN_SLOT, P = G::P, U = G::U;
    constexpr int MOFFB = G::MOFFB, MOFFC = G::MOFFC, OBB = G::OBB, OBC = G::OBC;
    static_assert(SW >= 32 && NDMA == 5, "geometry");
    // VMEM instructions per step: the DMAs, 3 x 2 stores, the decimated row's store
    constexpr int OPS = NDMA + 6 + 1;
    static_assert(NIN >= 2 && OPS * (NIN - 1) < 64, "DMA ring (vmcnt field)");
    static_assert(NIN * IN_SLOT >= 4 * kTrioSlot, "the top prologue's mid-A rows fit the input ring");
    const int lane = threadIdx.x & 63;
    const int W = J.W, H = J.H;
    const int sx = gw % J.strips, rest = gw / J.strips;
    const int sy = rest % J.nsy, b = rest / J.nsy;
    const int x0 = sx * SW;
    const int yb = sy * J.rows_per_band, ye = min(H, yb + J.rows_per_band);
    const int mB0 = x0 - MOFFC;    // mid-B column of lane 0's first column (even)
    const int mA0 = mB0 - MOFFB;   // mid-A column of lane 0's first column (even)
    const int a0 = mA0 - RA;       // input column of the input slot's float2 0
    const float* src = J.src + (long long)b * J.src_img;
    float* d1 = J.dst1 + (long long)b * J.dst_img;
    float* d2 = J.dst2 + (long long)b * J.dst_img;
    float* d3 = J.dst3 + (long long)b * J.dst_img;
    float* trash = J.trash + (size_t)(gw & 1023) * kTrioTrash;

    // ---- DMA lane map (the duo's): instruction q, lane i -> input column a0 + 32 q + i / 2
    // (clamped), row i & 1 of the pair
    uint32_t coff[NDMA];
#pragma unroll
    for (int q = 0; q < NDMA; q++) coff[q] = 4u * (uint32_t)clampd(a0 + 32 * q + (lane >> 1), 0, W - 1);
    const uint32_t rsel = (lane & 1) ? 4u * (uint32_t)J.src_stride : 0u;
    auto dma = [&](int rho, float* slot) __attribute__((always_inline)) {
        const int r0 = clampd(rho, 0, H - 1), r1 = clampd(rho + 1, 0, H - 1);
        const char* base = uniform_ptr(reinterpret_cast<const char*>(src) +
                                       (uint32_t)r0 * (4u * (uint32_t)J.src_stride));
        const uint32_t ro = r1 != r0 ? rsel : 0u;
        const uint32_t lds = __builtin_amdgcn_readfirstlane(
            (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)slot);
        dma_pair5(base, lds, coff, ro);
    };

    // ---- lane roles
    const int ca = mA0 + 2 * lane;                              // stage A: mid-A columns ca, ca + 1
    const bool ownA = ca >= x0 && ca < x0 + SW && ca < W;
    const int lb = lane < NB ? lane : NB - 1;                   // stage B lane (idle lanes repeat)
    const int cb = mB0 + 2 * lb;                                // mid-B columns cb, cb + 1
    const bool ownB = lane < NB && cb >= x0 && cb < x0 + SW && cb < W;
    const int lc = lane < SW / 2 ? lane : SW / 2 - 1;           // stage C lane
    const int e = x0 + 2 * lc;                                  // output columns e, e + 1
    const bool ownC = lane < SW / 2 && e < W;
    // edge strips (uniform): the lanes holding column 0 (as .x) and W - 1 (as .y) of each mid
    // level; 0 when there is no such edge (no lane then has a column outside the image)
    const bool edgeA = mA0 < 0 || mA0 + 128 > W;
    const int lAl = mA0 < 0 ? (-mA0) >> 1 : 0, lAr = mA0 + 128 > W ? (W - 2 - mA0) >> 1 : 0;
    const bool edgeB = mB0 < 0 || mB0 + 2 * NB > W;
    const int lBl = mB0 < 0 ? (-mB0) >> 1 : 0, lBr = mB0 + 2 * NB > W ? (W - 2 - mB0) >> 1 : 0;
    auto fixA = [&](f2v& v) __attribute__((always_inline)) {
        const float el = readlane_f(v.x, lAl), er = readlane_f(v.y, lAr);
        v = ca < 0 ? f2v{el, el} : (ca >= W ? f2v{er, er} : v);
    };
    auto fixB = [&](f2v& v) __attribute__((always_inline)) {
        const float el = readlane_f(v.x, lBl), er = readlane_f(v.y, lBr);
        v = cb < 0 ? f2v{el, el} : (cb >= W ? f2v{er, er} : v);
    };
    // the taps' distinct halves as wave-uniform scalars (symmetric bit for bit, as the duo's)
    float ka[RA + 1], kb[RB + 1], kc[RC + 1];
#pragma unroll
    for (int i = 0; i <= RA; i++) ka[i] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(J.ta.k[i])));
#pragma unroll
    for (int i = 0; i <= RB; i++) kb[i] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(J.tb.k[i])));
#pragma unroll
    for (int i = 0; i <= RC; i++) kc[i] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(J.tc.k[i])));
    auto tapa = [&](int i) __attribute__((always_inline)) { return ka[i <= RA ? i : FWA - 1 - i]; };
    auto tapb = [&](int i) __attribute__((always_inline)) { return kb[i <= RB ? i : FWB - 1 - i]; };
    auto tapc = [&](int i) __attribute__((always_inline)) { return kc[i <= RC ? i : FWC - 1 - i]; };
    // H1 of the input slot: columns ca, ca + 1 packed over the row pair
    auto h1 = [&](const float* slot, f2v& o0, f2v& o1) __attribute__((always_inline)) {
        o0 = f2v{0.f, 0.f};
        o1 = f2v{0.f, 0.f};
        const float4* p = reinterpret_cast<const float4*>(slot) + lane;
#pragma unroll
        for (int q = 0; q <= RA; q++) {
            const float4 v = p[q];
            const f2v ev[2] = {f2v{v.x, v.y}, f2v{v.z, v.w}};
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const int m = 2 * q + u;   // input float2 2l + m: tap m of column ca, m-1 of ca+1
                if (m < FWA) o0 = pkf(ev[u], tapa(m), o0);
                if (m >= 1 && m <= FWA) o1 = pkf(ev[u], tapa(m - 1), o1);
            }
        }
    };
    // H of a mid slot for lane li: columns (2 li + OB) + (0 .. FW) of the slot's float2s
    auto hmid = [&](auto FWK, auto OBK, auto tap, const float* slot, int li, f2v& o0, f2v& o1)
        __attribute__((always_inline)) {
        constexpr int FW = decltype(FWK)::value, OB = decltype(OBK)::value;
        o0 = f2v{0.f, 0.f};
        o1 = f2v{0.f, 0.f};
        f2v ev[FW + 2];
        if constexpr (OB == 0) {
            const float4* p = reinterpret_cast<const float4*>(slot) + li;
#pragma unroll
            for (int q = 0; 2 * q <= FW; q++) {
                const float4 v = p[q];
                ev[2 * q] = f2v{v.x, v.y};
                ev[2 * q + 1] = f2v{v.z, v.w};
            }
        } else {   // one float2, then 16-B aligned float4s, then a last float2 when needed
            const f2v* p2 = reinterpret_cast<const f2v*>(slot) + 2 * li + 1;
            const float4* p4 = reinterpret_cast<const float4*>(slot) + li + 1;
            ev[0] = p2[0];
#pragma unroll
            for (int q = 0; 2 * q + 2 <= FW; q++) {
                const float4 v = p4[q];
                ev[2 * q + 1] = f2v{v.x, v.y};
                ev[2 * q + 2] = f2v{v.z, v.w};
            }
            if constexpr ((FW & 1) == 1) ev[FW] = p2[FW];
        }
#pragma unroll
        for (int m = 0; m <= FW; m++) {
            if (m < FW) o0 = pkf(ev[m], tap(m), o0);
            if (m >= 1) o1 = pkf(ev[m], tap(m - 1), o1);
        }
    };
    using IFWB = std::integral_constant<int, FWB>;
    using IFWC = std::integral_constant<int, FWC>;
    using IOBB = std::integral_constant<int, OBB>;
    using IOBC = std::integral_constant<int, OBC>;
    // mid slots per level: 0, 1 alternate (written in step t & 1, read in step t + 1), 2 = (mid 0,
    // mid 0), 3 = (mid H-1, mid H-1)
    float* const ma_top = s_ma + 2 * kTrioSlot;
    float* const ma_bot = s_ma + 3 * kTrioSlot;
    float* const mb_top = s_mb + 2 * kTrioSlot;
    float* const mb_bot = s_mb + 3 * kTrioSlot;
    auto put_mid = [&](float* slot, f2v r0, f2v r1) __attribute__((always_inline)) {
        reinterpret_cast<float4*>(slot)[lane] = make_float4(r0.x, r1.x, r0.y, r1.y);
    };

    // ---- top band: mid-A row 0 and mid-B row 0 (the rows above 0 clamp to them) before the walk.
    // Mid-A rows 0 .. RB as pull sums over the clamped input rows in tap order (input row q = 0
    // takes taps 0 .. RA - r of mid-A row r, row q >= 1 tap RA - r + q), one rolled loop over
    // the input row pairs; then mid-B row 0 = taps 0 .. RB on H2(mid-A 0), taps RB + r on
    // H2(mid-A r).  The mid-A rows pass through the input ring's LDS (free until the walk's DMAs).
    if (yb - RB - RC < 0) {
        auto tap_at = [&](int idx) __attribute__((always_inline)) {
            float t = 0.f;
#pragma unroll
            for (int j = 0; j < FWA; j++) t = idx == j ? tapa(j) : t;
            return t;
        };
        f2v acc[RB + 1];
#pragma unroll
        for (int r = 0; r <= RB; r++) acc[r] = f2v{0.f, 0.f};
#pragma unroll 1
        for (int p = 0; 2 * p <= RA + RB; p++) {
            dma(2 * p, s_in);
            wait_vm<0>();
            asm volatile("" ::: "memory");
            f2v o0, o1;
            h1(s_in, o0, o1);
            const f2v rows[2] = {f2v{o0.x, o1.x}, f2v{o0.y, o1.y}};   // input rows 2p, 2p + 1
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const int q = 2 * p + u;
                if (q > RA + RB) break;
                if (q == 0) {
#pragma unroll
                    for (int r = 0; r <= RB; r++)
#pragma unroll
                        for (int j = 0; j <= RA - r; j++) acc[r] = pkf(rows[0], tapa(j), acc[r]);
                } else {
#pragma unroll
                    for (int r = 0; r <= RB; r++) {
                        const int j = RA - r + q;
                        if (j >= 0 && j < FWA) acc[r] = pkf(rows[u], tap_at(j), acc[r]);
                    }
                }
            }
            wait_lgkm0();
            asm volatile("" ::: "memory");
        }
#pragma unroll
        for (int r = 0; r <= RB; r++)
            if (edgeA) fixA(acc[r]);
        put_mid(ma_top, acc[0], acc[0]);
        // mid-A rows (2 t, 2 t + 1) into slot t of the input ring (row RB + 1 repeats row RB)
#pragma unroll
        for (int t = 0; 2 * t <= RB; t++)
            put_mid(s_in + t * kTrioSlot, acc[2 * t], acc[2 * t + 1 <= RB ? 2 * t + 1 : RB]);
        asm volatile("" ::: "memory");
        f2v mz{0.f, 0.f};
#pragma unroll
        for (int t = 0; 2 * t <= RB; t++) {
            f2v q0, q1;
            hmid(IFWB{}, IOBB{}, tapb, s_in + t * kTrioSlot, lb, q0, q1);
            const f2v g[2] = {f2v{q0.x, q1.x}, f2v{q0.y, q1.y}};   // H2 of mid-A rows 2t, 2t + 1
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const int r = 2 * t + u;
                if (r > RB) break;
                if (r == 0) {
#pragma unroll
                    for (int i = 0; i <= RB; i++) mz = pkf(g[0], tapb(i), mz);
                } else {
                    mz = pkf(g[u], tapb(RB + r), mz);
                }
            }
        }
        if (edgeB) fixB(mz);
        put_mid(mb_top, mz, mz);
        wait_lgkm0();
        asm volatile("" ::: "memory");
    }

    // ---- the walk.  Step t: stage A pushes input rows rho0 + 2t, + 1 and completes mid-A pair
    // mcA = rho - RA; stage B pushes mid-A pair muA = mcA - 2 (completed in step t - 1) and
    // completes mid-B pair mcB = muA - RB; stage C pushes mid-B pair muB = mcB - 2 and completes
    // output pair y = muB - RC.
    const int rho0 = yb - RA - RB - RC;
    const int ntau = (ye - yb) + 2 * (RA + RB + RC) + 4;
    const int nsteps = (ntau + 1) / 2;
    const int niter = (nsteps + U - 1) / U;
    f2v accA[P], accB[P], accC[P];
#pragma unroll
    for (int i = 0; i < P; i++) {
        accA[i] = f2v{0.f, 0.f};
        accB[i] = f2v{0.f, 0.f};
        accC[i] = f2v{0.f, 0.f};
    }
    // the first NIN - 1 steps' DMAs, each followed by 7 scratch stores in place of the stores of
    // the step that issues it (distinct 512-B blocks: the compiler neither drops nor merges them)
#pragma unroll
    for (int k = 0; k < NIN - 1; k++) {
        dma(rho0 + 2 * k, s_in + k * IN_SLOT);
#pragma unroll
        for (int j = 0; j < 7; j++)
            *reinterpret_cast<f2v*>(trash + 128 * (j + 1) + 2 * lane) = f2v{0.f, 0.f};
    }
    asm volatile("" ::: "memory");
    const uint32_t voffA = 4u * (uint32_t)ca, voffB = 4u * (uint32_t)cb, voffC = 4u * (uint32_t)e;
    const uint32_t vtr = 8u * (uint32_t)lane;
    const uint32_t W4 = 4u * (uint32_t)W;
    uint32_t rowA = (uint32_t)(rho0 - RA) * W4;                       // row mcA of step 0
    uint32_t rowB = (uint32_t)(rho0 - RA - 2 - RB) * W4;              // row mcB of step 0
    uint32_t rowC = (uint32_t)(rho0 - RA - 2 - RB - 2 - RC) * W4;     // row y of step 0 (even)
    char* const bA = reinterpret_cast<char*>(d1);
    char* const bB = reinterpret_cast<char*>(d2);
    char* const bC = reinterpret_cast<char*>(d3);
    char* const bT = reinterpret_cast<char*>(trash);
    char* const bD = reinterpret_cast<char*>(J.ds + (long long)b * J.ds_img);
    const uint32_t DW4 = 4u * (uint32_t)J.dsw;
    uint32_t rowD = (uint32_t)((rho0 - RA - 2 - RB - 2 - RC) / 2) * DW4;
    const uint32_t voffD = 2u * (uint32_t)e;
    int slot_use = 0, slot_dma = NIN - 1, curA = 0, curB = 0;
    for (int it = 0; it < niter; it++) {
        unroll_seq(std::make_integer_sequence<int, U>{}, [&](auto KI) __attribute__((always_inline)) {
            constexpr int k = decltype(KI)::value;
            const int t = it * U + k;
            const int rho = rho0 + 2 * t;
            const int mcA = rho - RA, muA = mcA - 2, mcB = muA - RB, muB = mcB - 2, y = muB - RC;
            asm volatile("" ::: "memory");
            dma(rho + 2 * (NIN - 1), s_in + slot_dma * IN_SLOT);
            slot_dma = slot_dma == NIN - 1 ? 0 : slot_dma + 1;
            // every older VMEM instruction but the OPS (NIN - 1) youngest has completed: step t's
            // DMA has landed
            wait_vm<OPS * (NIN - 1)>();
            asm volatile("" ::: "memory");
            const int ma_off = muA <= -1 ? 2 * kTrioSlot : (muA >= H - 1 ? 3 * kTrioSlot : (curA ^ 1) * kTrioSlot);
            const int mb_off = muB <= -1 ? 2 * kTrioSlot : (muB >= H - 1 ? 3 * kTrioSlot : (curB ^ 1) * kTrioSlot);
            f2v o0, o1, q0, q1, p0, p1;
            h1(s_in + slot_use * IN_SLOT, o0, o1);
            slot_use = slot_use == NIN - 1 ? 0 : slot_use + 1;
            // V1 push of input rows rho (ring row 2k) and rho + 1
            const f2v r0{o0.x, o1.x}, r1{o0.y, o1.y};
#pragma unroll
            for (int i = 0; i < FWA; i++) {
                const int s = ((2 * k - i) % P + P) % P;
                accA[s] = pkf(r0, tapa(i), i == 0 ? f2v{0.f, 0.f} : accA[s]);
            }
            f2v A0 = accA[((2 * k - (FWA - 1)) % P + P) % P];
#pragma unroll
            for (int i = 0; i < FWA; i++) {
                const int s = ((2 * k + 1 - i) % P + P) % P;
                accA[s] = pkf(r1, tapa(i), i == 0 ? f2v{0.f, 0.f} : accA[s]);
            }
            f2v A1 = accA[((2 * k + 1 - (FWA - 1)) % P + P) % P];
            if constexpr (kTrioFence) asm volatile("" ::: "memory");
            hmid(IFWB{}, IOBB{}, tapb, s_ma + ma_off, lb, q0, q1);
            // V2 push of mid-A rows muA (ring row 2k) and muA + 1
            const f2v g0{q0.x, q1.x}, g1{q0.y, q1.y};
#pragma unroll
            for (int i = 0; i < FWB; i++) {
                const int s = ((2 * k - i) % P + P) % P;
                accB[s] = pkf(g0, tapb(i), i == 0 ? f2v{0.f, 0.f} : accB[s]);
            }
            f2v B0 = accB[((2 * k - (FWB - 1)) % P + P) % P];
#pragma unroll
            for (int i = 0; i < FWB; i++) {
                const int s = ((2 * k + 1 - i) % P + P) % P;
                accB[s] = pkf(g1, tapb(i), i == 0 ? f2v{0.f, 0.f} : accB[s]);
            }
            f2v B1 = accB[((2 * k + 1 - (FWB - 1)) % P + P) % P];
            if constexpr (kTrioFence) asm volatile("" ::: "memory");
            hmid(IFWC{}, IOBC{}, tapc, s_mb + mb_off, lc, p0, p1);
            // V3 push of mid-B rows muB (ring row 2k) and muB + 1
            const f2v h0{p0.x, p1.x}, h1r{p0.y, p1.y};
#pragma unroll
            for (int i = 0; i < FWC; i++) {
                const int s = ((2 * k - i) % P + P) % P;
                accC[s] = pkf(h0, tapc(i), i == 0 ? f2v{0.f, 0.f} : accC[s]);
            }
            const f2v C0 = accC[((2 * k - (FWC - 1)) % P + P) % P];
#pragma unroll
            for (int i = 0; i < FWC; i++) {
                const int s = ((2 * k + 1 - i) % P + P) % P;
                accC[s] = pkf(h1r, tapc(i), i == 0 ? f2v{0.f, 0.f} : accC[s]);
            }
            const f2v C1 = accC[((2 * k + 1 - (FWC - 1)) % P + P) % P];
            // the completed mid pairs into their slots (t & 1) and the bottom pairs: edge columns
            // clamped, an odd H's pair (H-1, H) as (H-1, H-1)
            if (mcA == H - 1) A1 = A0;
            if (mcB == H - 1) B1 = B0;
            if (edgeA) {
                fixA(A0);
                fixA(A1);
            }
            if (edgeB) {
                fixB(B0);
                fixB(B1);
            }
            put_mid(s_ma + curA * kTrioSlot, A0, A1);
            put_mid(s_mb + curB * kTrioSlot, B0, B1);
            curA ^= 1;
            curB ^= 1;
            if (mcA <= H - 1 && mcA + 1 >= H - 1) {
                const f2v v = mcA == H - 1 ? A0 : A1;
                put_mid(ma_bot, v, v);
            }
            if (mcB <= H - 1 && mcB + 1 >= H - 1) {
                const f2v v = mcB == H - 1 ? B0 : B1;
                put_mid(mb_bot, v, v);
            }
            asm volatile("" ::: "memory");
            // levels k+1 rows mcA, + 1; k+2 rows mcB, + 1; k+3 rows y, + 1 and the decimated row
            // y / 2: the wave's own columns; rows outside the band into the scratch block
            {
                const bool a0ok = mcA >= yb && mcA < ye, a1ok = mcA + 1 >= yb && mcA + 1 < ye;
                const bool b0ok = mcB >= yb && mcB < ye, b1ok = mcB + 1 >= yb && mcB + 1 < ye;
                const bool c0ok = y >= yb && y < ye, c1ok = y + 1 >= yb && y + 1 < ye;
                if (ownA) {
                    *reinterpret_cast<f2v*>((a0ok ? bA : bT) + (a0ok ? rowA + voffA : vtr)) = A0;
                    *reinterpret_cast<f2v*>((a1ok ? bA : bT) + (a1ok ? rowA + W4 + voffA : vtr)) = A1;
                }
                if (ownB) {
                    *reinterpret_cast<f2v*>((b0ok ? bB : bT) + (b0ok ? rowB + voffB : vtr)) = B0;
                    *reinterpret_cast<f2v*>((b1ok ? bB : bT) + (b1ok ? rowB + W4 + voffB : vtr)) = B1;
                }
                if (ownC) {
                    *reinterpret_cast<f2v*>((c0ok ? bC : bT) + (c0ok ? rowC + voffC : vtr)) = C0;
                    *reinterpret_cast<f2v*>((c1ok ? bC : bT) + (c1ok ? rowC + W4 + voffC : vtr)) = C1;
                    // DownsampleKernel<1>: ds(r, cc) = level(2 r, 2 cc) (y is even)
                    const bool dok = c0ok && (y >> 1) < J.dsh;
                    *reinterpret_cast<float*>((dok ? bD : bT) + (dok ? rowD + voffD : vtr)) = C0.x;
                }
                rowA += 2 * W4;
                rowB += 2 * W4;
                rowC += 2 * W4;
                rowD += DW4;
            }
        });
    }
    // no DMA may land after the workgroup's LDS is handed to another workgroup
    wait_vm<0>();
}

// waves per SIMD the register allocation must allow: 2 (173 VGPRs, no spill); at 3 (168) the
// allocator spilled 5 VGPRs and 63 SGPRs and the launch took 1,921 against ~1,360 us
#ifndef SGK_TRIO_WPE
#define SGK_TRIO_WPE 2
#endif
template <int FWA, int FWB, int FWC, int NIN>
__global__ __launch_bounds__(64 * kTrioWaves) __attribute__((amdgpu_waves_per_eu(SGK_TRIO_WPE))) void k_gauss_trio(const TrioJob J) {
    using G = TrioGeom<FWA, FWB, FWC>;
    __shared__ __attribute__((aligned(16))) float s_in_all[kTrioWaves][NIN * G::IN_SLOT];
    __shared__ __attribute__((aligned(16))) float s_ma_all[kTrioWaves][4 * kTrioSlot];
    __shared__ __attribute__((aligned(16))) float s_mb_all[kTrioWaves][4 * kTrioSlot];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int gw = ring_block(blockIdx.x, gridDim.x) * kTrioWaves + wave;
    if (gw >= J.total_waves) return;   // uniform per wave
    trio_wave<FWA, FWB, FWC, NIN>(J, gw, s_in_all[wave], s_ma_all[wave], s_mb_all[wave]);
}

// input row pairs in LDS: the DMA runs NIN - 1 steps ahead; NIN 4 leaves 13,312 B of LDS per
// wave, 3 workgroups per CU (the registers allow 2 waves per SIMD)
#ifndef SGK_TRIO_NIN
#define SGK_TRIO_NIN 4
#endif
// waves a launch aims for (bands of one image added until the grid has as many)
#ifndef SGK_TRIO_WAVES
#define SGK_TRIO_WAVES 4096
#endif
static long long trio_waves_target() {
    static const long long v = [] {
        const char* e = getenv("SGPU_TRIO_WAVES");
        return e && atoll(e) > 0 ? atoll(e) : (long long)SGK_TRIO_WAVES;
    }();
    return v;
}

template <int FWA, int FWB, int FWC>
hipError_t trio_launch(const LevelOp& a, const LevelOp& b, const LevelOp& c, hipStream_t stream,
                       int rows_hint, float* trash) {
    using G = TrioGeom<FWA, FWB, FWC>;
    TrioJob J{};
    J.src = a.src;
    J.src_stride = a.src_stride;
    J.src_img = a.src_img_stride;
    J.dst1 = a.dst;
    J.dst2 = b.dst;
    J.dst3 = c.dst;
    J.dst_img = a.dst_img_stride;
    J.W = a.w;
    J.H = a.h;
    J.ta = a.taps;
    J.tb = b.taps;
    J.tc = c.taps;
    J.ds = c.ds_dst;
    J.dsw = c.ds_w;
    J.dsh = c.ds_h;
    J.ds_img = c.ds_img_stride;
    J.strips = (a.w + G::SW - 1) / G::SW;
    const long long per_band = (long long)J.strips * a.batch;
    // bands: as many as the grid needs for trio_waves_target() waves; each band re-walks
    // 2 (RA + RB + RC) + 4 halo rows, so bands stay >= 64 rows
    int nsy = 1;
    const long long want = trio_waves_target();
    if (rows_hint > 0) {
        nsy = (a.h + rows_hint - 1) / rows_hint;
    } else if (per_band < want) {
        nsy = (int)std::min<long long>((want + per_band - 1) / per_band, std::max(1, a.h / 64));
    }
    int rows = (a.h + nsy - 1) / nsy;
    rows = (rows + 7) / 8 * 8;
    J.nsy = (a.h + rows - 1) / rows;
    J.rows_per_band = rows;
    J.total_waves = (int)(per_band * J.nsy);
    J.trash = trash;
    const unsigned nb = (unsigned)((J.total_waves + kTrioWaves - 1) / kTrioWaves);
    hipLaunchKernelGGL((k_gauss_trio<FWA, FWB, FWC, SGK_TRIO_NIN>), dim3(nb), dim3(64 * kTrioWaves), 0, stream, J);
    return hipGetLastError();
}

}  // namespace

bool gauss_trio_supported(const LevelOp& a, const LevelOp& b, const LevelOp& c) {
    // f32 levels k -> k+1 -> k+2 -> k+3 with widths (11, 13, 17) and level k+3 decimated into the
    // next octave's level 0
    const bool widths = a.fw == 11 && b.fw == 13 && c.fw == 17;
    const bool ds = c.ds_dst && (a.w % 2) == 0 && c.ds_w * 2 == a.w &&
                    (c.ds_h == (a.h + 1) / 2 || c.ds_h == a.h / 2) &&
                    c.ds_img_stride >= (long long)c.ds_w * c.ds_h;
    const bool zeroes = (a.zero.n[0] | a.zero.n[1] | a.zero.n[2] | b.zero.n[0] | b.zero.n[1] |
                         b.zero.n[2] | c.zero.n[0] | c.zero.n[1] | c.zero.n[2]) != 0;
    return widths && ds && !zeroes && a.src && !a.src_u8 && !b.src_u8 && !c.src_u8 &&
           a.src_stride >= a.w && !a.ds_dst && !b.ds_dst && b.src == a.dst && c.src == b.dst &&
           a.w == b.w && a.w == c.w && a.h == b.h && a.h == c.h && a.batch == b.batch &&
           a.batch == c.batch && a.w >= 8 && a.h >= 8 && (a.w % 4) == 0 &&
           b.src_stride == a.w && c.src_stride == a.w && a.dst_img_stride == b.dst_img_stride &&
           a.dst_img_stride == c.dst_img_stride && b.src_img_stride == a.dst_img_stride &&
           c.src_img_stride == a.dst_img_stride && a.dst_img_stride >= (long long)a.w * a.h;
}

hipError_t launch_gauss_trio(const LevelOp& a, const LevelOp& b, const LevelOp& c,
                             hipStream_t stream, int rows_hint, float* trash) {
    if (!trash || !gauss_trio_supported(a, b, c)) return hipErrorInvalidValue;
    return trio_launch<11, 13, 17>(a, b, c, stream, rows_hint, trash);
}

}  // namespace sgk
