// sift_gauss_duo.hip -- two consecutive Gaussian levels per launch ("duo"), gfx950.
//
// Levels k+1 = V(H(level k)) and k+2 = V(H(level k+1)) (FilterH<FW> then FilterV<FW>,
// ProgramCU.cu:115-222, driven per level by PyramidCU::BuildPyramid, PyramidCU.cpp:979-1044) in one
// pass over level k: 12 B of HBM traffic per pixel for the two levels (read level k, write k+1 and
// k+2) instead of the 16 B of two single-level launches.  Round 3's two-level kernel kept both
// H results in LDS rings and lost to its LDS footprint (4 waves per CU); here both
// vertical passes are register-resident ("push" form), so a wave's LDS is its input rows and
// one mid row pair:
//
//   * a wave owns SW = 128 - 2 RB output columns of both levels (RB = FWB / 2) and walks a band
//     of rows top to bottom, two rows (one row pair) per step;
//   * stage A: the input row pair (128 + 2 RA columns, clamped to the image) arrives in LDS by
//     LDS-DMA NIN - 1 steps ahead of its use -- no staging registers.  Pairs of < 40 taps
//     (SGK_DUO_X4): two global_load_lds_dwordx4 (16 B per lane) into a row-major slot, H1 (lane
//     l: mid columns m0 + 2l, m0 + 2l + 1 of each row, packed over the column pair) reads
//     8-B pairs; the edge strips, whose slots hold columns outside the image, keep 5 per-column
//     clamped dword DMAs into the same layout (a second copy of the walk with its own counted
//     wait).  (21, 25): 5 dword DMAs into (row 2p, row 2p+1) pairs, H1 packed over the row pair
//     reads ds_read_b128;
//   * the V1 pass is pushed: each H1 row is multiplied into the FWA accumulators of the mid rows
//     it contributes to, so mid row m receives input rows m - RA .. m + RA in that order -- the
//     reference's tap order i = 0 .. FW-1, one fma each, bit for bit the pull form's sum.  The
//     accumulators are an array indexed by (row - base) mod P, P = the ring period, with the
//     step loop unrolled by P / 2 so every index is a compile-time constant (registers, no
//     rotation copies at the loop back edge);
//   * a completed mid row pair is written to HBM (level k+1, the wave's own SW columns) and, all
//     128 columns, to the wave's mid slot in LDS; stage B's H2 reads it there (lane l: output
//     columns x0 + 2l, x0 + 2l + 1) and pushes into the V2 accumulators; completed rows of level
//     k+2 go to HBM;
//   * clamp-to-edge: stage A's rows and columns are clamped in the DMA addresses; stage B's rows
//     above 0 / below H-1 read two extra LDS pairs, (mid 0, mid 0) -- computed by a short
//     prologue in the top band -- and (mid H-1, mid H-1); stage B's columns outside the image
//     take the edge mid column's value by v_readlane in the two edge strips.
//
// Every VMEM instruction of a step is issued unconditionally (rows outside the band store to a
// per-wave scratch area), so the count of memory operations younger than a step's DMA is a
// constant and one `s_waitcnt vmcnt(OPS (NIN - 1))` waits for exactly that DMA.  Levels are
// bit-identical to two k_gauss_lean launches (tests/test_gpu_gauss.py).  Pairs: (11, 13),
// (21, 25), (17, 21) decimating its first level, (13, 17) decimating its second, the u8 ingest
// pair (13, 11).
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <utility>

#include "sift_gauss_ring.h"
#include "sift_kernels.h"

// the DMA asm names M0 as clobbered: clang warns that M0 is reserved; nothing else in this file
// uses M0 (no builtin LDS-DMA, no indirect register indexing), see duo_wave's dma()
#pragma clang diagnostic ignored "-Winline-asm"

namespace sgk {
namespace {

using namespace gring;

// the two H passes of a step in one scheduling region (their fma chains interleave) or kept
// apart by a compiler barrier (SGK_DUO_INTERLEAVE=0)
#ifndef SGK_DUO_INTERLEAVE
#define SGK_DUO_INTERLEAVE 1
#endif
constexpr bool kDuoInterleave = SGK_DUO_INTERLEAVE != 0;
// timing experiments only (wrong levels, tests/diag): 1 = DMA lanes row-contiguous (lanes 0-31 row
// 2p, 32-63 row 2p+1), 2 = no H / V arithmetic (one LDS read per pass), 3 = the row pair as two
// 16-B-per-lane DMAs (global_load_lds_dwordx4, 128 lane addresses instead of 320), 4 = the same
// with the second on 8 lanes (72 lane addresses), 0 = the kernel
#ifndef SGK_DUO_EXP
#define SGK_DUO_EXP 0
#endif
// f32 input rows by 16-B-per-lane DMA (global_load_lds_dwordx4: 2 instructions, ~74 lane
// addresses per row pair instead of 5 x 64) into row-major slots, read by a column-packed H1: 1;
// the per-column dword DMA into (row 2p, row 2p+1)-interleaved slots (round 5): 0
#ifndef SGK_DUO_X4
#define SGK_DUO_X4 1
#endif
constexpr int kDuoWaves = 4;      // waves per workgroup (each wave works alone: no barriers)
constexpr int kMidSlot = 256;     // floats of one mid row pair: 128 columns x (row, row + 1)

// 32: strips of 96 columns for both compiled pairs; 128 x 1080p, (11, 13): 784 us against 905 for
// the unaligned 116-column strips (tests/diag/r05e.sh; 16, 64-B lines: 820)
#ifndef SGK_DUO_SWALIGN
#define SGK_DUO_SWALIGN 32
#endif
template <int FWA, int FWB>
struct DuoGeom {
    static constexpr int RA = FWA / 2, RB = FWB / 2;
    // mid column of lane 0 = x0 - MOFF: even (stage A's pairs of mid columns are 8-B aligned in
    // LDS and in the level k + 1 rows); stage B's H2 reads start OB = MOFF - RB float2 past its
    // lane's pair
    static constexpr int MOFF = RB + (RB & 1), OB = MOFF - RB;
    // output columns of a wave: 128 - 2 MOFF, rounded down to SGK_DUO_SWALIGN columns so that
    // the strips' rows start on 128-B lines (a strip boundary inside a line leaves two waves
    // writing parts of it)
    static constexpr int SW = (128 - 2 * MOFF) / SGK_DUO_SWALIGN * SGK_DUO_SWALIGN;
    static constexpr int IN_W = 128 + 2 * RA;         // input columns of stage A
    static constexpr int NDMA = (IN_W + 31) / 32;     // dword DMAs per row pair (32 columns each)
    static constexpr int IN_SLOT = (SGK_DUO_EXP == 3 ? 8 : NDMA) * 64;   // floats of one input row pair
    static constexpr int PMAX = FWA > FWB ? FWA : FWB;
    static constexpr int P = (PMAX + 1) & ~1;         // accumulator ring period (rows), even
    static constexpr int U = P / 2;                   // steps per unrolled iteration
    static constexpr int NQ = IN_W / 4;               // u8 input: dword quads per row
    // X4 slots: a row's quads start at column c0 = a0 - D (16-B aligned: x0 is a multiple of 32),
    // NQ4 per row (lane l's H1 reads floats D + 2 l .. D + 2 l + FWA of each row), row 2p + 1
    // 4 NQ4 floats after row 2p
    static constexpr int D = (-(MOFF + RA)) & 3;
    static constexpr int NQ4 = (D + 128 + FWA + 3) / 4;
};

struct DuoJob {
    const float* src;            // level k (f32), or
    const uint8_t* src8;         // the u8 image (level k = the ingest level's input)
    int src_stride;
    long long src_img;
    float* dst1;                 // level k + 1
    float* dst2;                 // level k + 2 (both rows W apart, images dst_img apart)
    long long dst_img;
    int W, H;
    Taps ta, tb;                 // the two filters (widths FWA, FWB)
    float* ds;                   // level k + 1 (DS 1) or k + 2 (DS 2) decimated into the next
    int dsw, dsh;                // octave's level 0
    long long ds_img;
    int strips, nsy, rows_per_band, total_waves;
    float* trash;                // 3,072 B per wave slot (1024 slots): stores of rows outside
                                 // the band and the DMA prologue's count-keeping stores
    ZeroJob zero;                // buffers this launch zeroes (the extract's first launch)
};

// a ZeroJob over the whole grid (uint4 stores; the buffers are hipMalloc'ed, 16-B aligned), as
// k_gauss_lean's
__device__ __forceinline__ void duo_zero(const ZeroJob& z) {
    const size_t step = (size_t)gridDim.x * blockDim.x;
    const size_t t0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll
    for (int i = 0; i < 3; i++)
        for (size_t q = t0; q * 4 < z.n[i]; q += step) {
            if (q * 4 + 4 <= z.n[i]) {
                *reinterpret_cast<uint4*>(z.p[i] + q * 4) = make_uint4(0, 0, 0, 0);
            } else {
                for (size_t j = q * 4; j < z.n[i]; j++) z.p[i][j] = 0;
            }
        }
}

// DS: 0 no decimation, 1 level k + 1 (stage A) into the next octave's level 0, 2 level k + 2
// (stage B)
template <int FWA, int FWB, int NIN, bool U8, int DS>
__device__ __forceinline__ void duo_wave(const DuoJob& J, int gw, float* s_in, float* s_mid) {
    using G = DuoGeom<FWA, FWB>;
    constexpr int RA = G::RA, RB = G::RB, SW = G::SW, NDMA = G::NDMA, IN_SLOT = G::IN_SLOT;
    constexpr int P = G::P, U = G::U, MOFF = G::MOFF, OB = G::OB, NQ = G::NQ;
    static_assert(!U8 || ((MOFF + RA) % 4 == 0 && G::IN_W % 4 == 0 && NQ <= 64),
                  "u8 input: the strip's input quads are 4-column aligned");
    // VMEM instructions per step: the DMAs, 2 + 2 stores, the decimated row's store
    constexpr bool kX4 = SGK_DUO_EXP == 3 || SGK_DUO_EXP == 4;
    // the shipped 16-B DMA, for the pairs of < 40 taps: (21, 25)'s register budget (168 VGPRs at
    // 3 waves per SIMD) does not take the second walk copy (a VGPR spill, 1,265 vs 987 us)
    constexpr bool kRowX4 = SGK_DUO_X4 && !U8 && SGK_DUO_EXP == 0 && FWA + FWB < 40;
    constexpr int D = G::D, NQ4 = G::NQ4;
    static_assert(!kRowX4 || (8 * NQ4 <= IN_SLOT && 2 * NQ4 > 64 && 2 * NQ4 <= 128), "X4 slot");
    // (X4: the interior strips' 2 DMAs; the edge strips keep 5 per-column DMAs, OPSE)
    constexpr int OPS = (kX4 || kRowX4 ? 2 : NDMA) + 4 + (DS ? 1 : 0);
    constexpr int OPSE = (kX4 ? 2 : NDMA) + 4 + (DS ? 1 : 0);
    static_assert(NIN >= 2 && OPSE * (NIN - 1) < 64, "DMA ring (vmcnt field)");
    const int lane = threadIdx.x & 63;
    const int W = J.W, H = J.H;
    const int sx = gw % J.strips, rest = gw / J.strips;
    const int sy = rest % J.nsy, b = rest / J.nsy;
    const int x0 = sx * SW;
    const int yb = sy * J.rows_per_band, ye = min(H, yb + J.rows_per_band);
    const int m0 = x0 - MOFF;      // mid column of lane 0's first column (even)
    const int a0 = m0 - RA;        // input column of the input slot's float2 0
    const float* src = U8 ? nullptr : J.src + (long long)b * J.src_img;
    const uint8_t* src8 = U8 ? J.src8 + (long long)b * J.src_img : nullptr;
    float* d1 = J.dst1 + (long long)b * J.dst_img;
    float* d2 = J.dst2 + (long long)b * J.dst_img;
    float* trash = J.trash + (size_t)(gw & 1023) * 768;   // 6 x 512 B per wave slot

    // ---- DMA lane map: instruction q, lane i -> input column a0 + 32 q + i / 2 (clamped),
    // row i & 1 of the pair; LDS float 64 q + i of the slot = float2 index 32 q + i / 2
    uint32_t coff[NDMA];
#pragma unroll
    for (int q = 0; q < NDMA; q++)
        coff[q] = 4u * (uint32_t)clampd(a0 + 32 * q + (SGK_DUO_EXP == 1 ? (lane & 31) : (lane >> 1)), 0, W - 1);
    const uint32_t rsel = ((SGK_DUO_EXP == 1 ? lane >> 5 : lane) & 1) ? 4u * (uint32_t)J.src_stride : 0u;
    // the DMAs: gring::dma_pair5 / dma_pair_x4 (inline asm, waited for by the counted waits below
    // only; every LDS access of the wave stays inside its own slots)
    static_assert(NDMA == 5, "dma_pair5 issues 5 DMAs per row pair");
    const int c0 = a0 - D;         // X4: column of the slot rows' float 0
    const uint32_t qoff0 = 4u * (uint32_t)clampd(c0 + 4 * (lane < NQ4 ? lane : lane - NQ4), 0, W - 4);
    const uint32_t qoff1 = 4u * (uint32_t)clampd(c0 + 4 * min(64 - NQ4 + lane, NQ4 - 1), 0, W - 4);
    // X4 edge strips (a slot column outside the image, uniform): the row-major slot filled by 5
    // per-column dword DMAs, each column clamped to the image (lane i of instruction q: slot
    // float 64 q + i, row 2p + 1 from float 4 NQ4 on)
    const bool xedge = kRowX4 && (c0 < 0 || c0 + 4 * NQ4 > W);
    uint32_t ecoff[NDMA], erow[NDMA];
#pragma unroll
    for (int q = 0; q < NDMA; q++) {
        const int f = 64 * q + lane, r = f >= 4 * NQ4 ? 1 : 0;
        ecoff[q] = 4u * (uint32_t)clampd(c0 + f - 4 * NQ4 * r, 0, W - 1);
        erow[q] = r ? 4u * (uint32_t)J.src_stride : 0u;
    }
    auto dma = [&](int rho, float* slot, auto EDGE) __attribute__((always_inline)) {
        const int r0 = clampd(rho, 0, H - 1), r1 = clampd(rho + 1, 0, H - 1);
        const char* base = uniform_ptr(reinterpret_cast<const char*>(src) +
                                       (uint32_t)r0 * (4u * (uint32_t)J.src_stride));
        const uint32_t ro = r1 != r0 ? rsel : 0u;
        const uint32_t lds = __builtin_amdgcn_readfirstlane(
            (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)slot);
        if constexpr (kRowX4 && decltype(EDGE)::value) {
            const uint32_t rm = r1 != r0 ? ~0u : 0u;
            const uint32_t eo[NDMA] = {ecoff[0] + (erow[0] & rm), ecoff[1] + (erow[1] & rm),
                                       ecoff[2] + (erow[2] & rm), ecoff[3] + (erow[3] & rm),
                                       ecoff[4] + (erow[4] & rm)};
            dma_pair5(base, lds, eo, 0u);
        } else if constexpr (kRowX4) {
            // instruction 0: lanes < NQ4 quads of row 2p, the rest row 2p + 1's first quads;
            // instruction 1 (lanes < 2 NQ4 - 64): row 2p + 1's last quads (interior strips: every
            // quad inside the image)
            const uint32_t rr = r1 != r0 ? 4u * (uint32_t)J.src_stride : 0u;
            dma_pair_x4(base, lds, qoff0 + (lane < NQ4 ? 0u : rr), qoff1 + rr, true, lane,
                        2 * NQ4 - 64);
        } else if constexpr (kX4) {   // (timing only) quads of the aligned window: 36 per row
            const uint32_t rr = r1 != r0 ? 4u * (uint32_t)J.src_stride : 0u;
            const int a4 = a0 & ~3;
            const uint32_t o0 = 4u * (uint32_t)clampd(a4 + 4 * (lane < 36 ? lane : lane - 36), 0, W - 4) +
                                (lane < 36 ? 0u : rr);
            const uint32_t o1 = 4u * (uint32_t)clampd(a4 + 4 * min(28 + lane, 35), 0, W - 4) + rr;
            dma_pair_x4(base, lds, o0, o1, SGK_DUO_EXP == 4, lane, 8);
        } else {
            dma_pair5(base, lds, coff, ro);
        }
    };
    // u8 input (stage A of the ingest pair): lane j < NQ loads quad j (columns a0 + 4 j ..
    // + 3, whole quads: W % 4 == 0 and a0 % 4 == 0) of both rows of a pair into registers; the
    // conversion to f32 writes them into the input slot in the DMA's layout (float2 index =
    // column - a0, (row 2p, row 2p + 1)).  A quad left of column 0 repeats column 0, right of
    // W - 1 column W - 1 (clamp-to-edge, as k_gauss_lean's loaders).
    const int qcol = a0 + 4 * (lane < NQ ? lane : NQ - 1);
    const uint32_t qoff = (uint32_t)clampd(qcol, 0, W - 4);
    const bool qleft = qcol < 0, qright = qcol > W - 4;
    auto fetch8 = [&](int rho, uint32_t (&r)[2]) __attribute__((always_inline)) {
        const int r0 = clampd(rho, 0, H - 1), r1 = clampd(rho + 1, 0, H - 1);
        r[0] = *reinterpret_cast<const uint32_t*>(src8 + (size_t)r0 * J.src_stride + qoff);
        r[1] = *reinterpret_cast<const uint32_t*>(src8 + (size_t)r1 * J.src_stride + qoff);
    };
    auto stage8 = [&](const uint32_t (&r)[2], float* slot) __attribute__((always_inline)) {
        f2v pr[4];
#pragma unroll
        for (int t = 0; t < 4; t++) pr[t] = u8_pair_to_unit((r[0] >> (8 * t)) & 255u, (r[1] >> (8 * t)) & 255u);
        if (qleft || qright) {
            const f2v e0 = pr[0], e3 = pr[3];
#pragma unroll
            for (int t = 0; t < 4; t++) pr[t] = qleft ? e0 : e3;
        }
        if (lane < NQ) {
            float4* q = reinterpret_cast<float4*>(slot) + 2 * lane;
            q[0] = make_float4(pr[0].x, pr[0].y, pr[1].x, pr[1].y);
            q[1] = make_float4(pr[2].x, pr[2].y, pr[3].x, pr[3].y);
        }
    };

    // ---- lane roles
    const int c = m0 + 2 * lane;                       // mid columns c, c + 1 (stage A)
    const bool own1 = c >= x0 && c < x0 + SW && c < W; // stage A stores these columns
    const int le = lane < SW / 2 ? lane : SW / 2 - 1;  // stage B lane (idle lanes repeat the last)
    const int e = x0 + 2 * le;                         // output columns e, e + 1 (stage B)
    const bool own2 = lane < SW / 2 && e < W;
    const bool left = m0 < 0, right = m0 + 128 > W;    // uniform: edge strips
    const int l_left = left ? (-m0) >> 1 : 0;          // lane holding mid column 0 (as .x)
    const int l_right = right ? (W - 2 - m0) >> 1 : 0; // lane holding mid column W-1 (as .y)
    // mid row pair of one lane (columns c, c+1) clamped to the image's edge columns
    // (in the edge strips only: the lanes' columns outside the image; l_left / l_right are 0
    // when there is no such edge, and no lane then has c < 0 / c >= W)
    auto fix_edges = [&](f2v& v) __attribute__((always_inline)) {
        const float el = readlane_f(v.x, l_left), er = readlane_f(v.y, l_right);
        v = c < 0 ? f2v{el, el} : (c >= W ? f2v{er, er} : v);
    };
    // the taps' distinct half (symmetric bit for bit) as wave-uniform scalars: read once from the
    // kernel arguments (a reference into the argument struct made the compiler copy it to
    // scratch and keep the taps in VGPRs)
    float ka[RA + 1], kb[RB + 1];
#pragma unroll
    for (int i = 0; i <= RA; i++)
        ka[i] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(J.ta.k[i])));
#pragma unroll
    for (int i = 0; i <= RB; i++)
        kb[i] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(J.tb.k[i])));
    auto tapa = [&](int i) __attribute__((always_inline)) { return ka[i <= RA ? i : FWA - 1 - i]; };
    auto tapb = [&](int i) __attribute__((always_inline)) { return kb[i <= RB ? i : FWB - 1 - i]; };
    // H1 of the input slot: columns c, c + 1 packed over the row pair
    auto h1 = [&](const float* slot, f2v& o0, f2v& o1) __attribute__((always_inline)) {
        o0 = f2v{0.f, 0.f};
        o1 = f2v{0.f, 0.f};
        const float4* p = reinterpret_cast<const float4*>(slot) + lane;
        if constexpr (SGK_DUO_EXP == 2) {
            const float4 v = p[0];
            o0 = f2v{v.x, v.y};
            o1 = f2v{v.z, v.w};
            return;
        }
#pragma unroll
        for (int q = 0; q <= RA; q++) {
            const float4 v = p[q];
            const f2v ev[2] = {f2v{v.x, v.y}, f2v{v.z, v.w}};
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const int m = 2 * q + u;   // input float2 2l + m: tap m of column c, m-1 of c+1
                if (m < FWA) o0 = pkf(ev[u], tapa(m), o0);
                if (m >= 1 && m <= FWA) o1 = pkf(ev[u], tapa(m - 1), o1);
            }
        }
    };
    // H1 of an X4 slot, column-packed: row 2p's (c, c + 1) and row 2p + 1's, each the sum over
    // taps m = 0 .. FWA-1 of tap m times the columns (c - RA + m, c + 1 - RA + m), in tap order;
    // lane l's inputs are floats D + 2 l .. D + 2 l + FWA of each row, read as 8-B-aligned pairs,
    // the odd-offset operands formed from two neighbouring pairs
    auto h1rows = [&](int off, f2v& r0, f2v& r1) __attribute__((always_inline)) {
        constexpr int O = D & 1;                      // x[m] sits at pair float m + O
        constexpr int NP = (FWA + O) / 2 + 1;         // pairs read per row
#pragma unroll
        for (int r = 0; r < 2; r++) {
            const f2v* pp = reinterpret_cast<const f2v*>(s_in + off + r * 4 * NQ4 + D - O + 2 * lane);
            f2v pr[NP];
#pragma unroll
            for (int i = 0; i < NP; i++) pr[i] = pp[i];
            f2v o{0.f, 0.f};
#pragma unroll
            for (int m = 0; m < FWA; m++) {
                const int idx = m + O;
                const f2v op = (idx & 1) ? f2v{pr[idx >> 1].y, pr[(idx >> 1) + 1].x} : pr[idx >> 1];
                o = pkf(op, tapa(m), o);
            }
            (r ? r1 : r0) = o;
        }
    };
    // H2 of a mid slot: output columns e, e + 1 from mid float2 2 le + OB + m, m = 0 .. FWB
    auto h2 = [&](const float* slot, f2v& o0, f2v& o1) __attribute__((always_inline)) {
        o0 = f2v{0.f, 0.f};
        o1 = f2v{0.f, 0.f};
        if constexpr (SGK_DUO_EXP == 2) {
            const float4 v = reinterpret_cast<const float4*>(slot)[le];
            o0 = f2v{v.x, v.y};
            o1 = f2v{v.z, v.w};
            return;
        }
        f2v ev[FWB + 2];
        if constexpr (OB == 0) {
            const float4* p = reinterpret_cast<const float4*>(slot) + le;
#pragma unroll
            for (int q = 0; 2 * q <= FWB; q++) {
                const float4 v = p[q];
                ev[2 * q] = f2v{v.x, v.y};
                ev[2 * q + 1] = f2v{v.z, v.w};
            }
        } else {   // one float2, then 16-B aligned float4s, then a last float2 when needed
            const f2v* p2 = reinterpret_cast<const f2v*>(slot) + 2 * le + 1;
            const float4* p4 = reinterpret_cast<const float4*>(slot) + le + 1;
            ev[0] = p2[0];
#pragma unroll
            for (int q = 0; 2 * q + 2 <= FWB; q++) {
                const float4 v = p4[q];
                ev[2 * q + 1] = f2v{v.x, v.y};
                ev[2 * q + 2] = f2v{v.z, v.w};
            }
            if constexpr ((FWB & 1) == 1) ev[FWB] = p2[FWB];
        }
#pragma unroll
        for (int m = 0; m <= FWB; m++) {
            if (m < FWB) o0 = pkf(ev[m], tapb(m), o0);
            if (m >= 1) o1 = pkf(ev[m], tapb(m - 1), o1);
        }
    };
    // mid slots: 0, 1 alternate (stage A writes step t's pair into slot t & 1, stage B reads the
    // previous step's from the other), 2 = (mid 0, mid 0), 3 = (mid H-1, mid H-1)
    float* const mid_top = s_mid + 2 * kMidSlot;
    float* const mid_bot = s_mid + 3 * kMidSlot;
    auto put_mid = [&](float* slot, f2v r0, f2v r1) __attribute__((always_inline)) {
        reinterpret_cast<float4*>(slot)[lane] = make_float4(r0.x, r1.x, r0.y, r1.y);
    };

    // ---- top band: mid row 0 (the rows above 0 clamp to it) before the walk, as the pull sum
    // of rows 0 .. RA in tap order (taps 0 .. RA on row 0).  A rolled loop (one copy of the H1
    // code; unrolled, it pushed the main loop's register allocation into spills), the tap of a
    // row picked by uniform selects.
    if (yb - RB < 0) {
        auto tap_at = [&](int idx) __attribute__((always_inline)) {
            float t = 0.f;
#pragma unroll
            for (int j = RA + 1; j < FWA; j++) t = idx == j ? tapa(j) : t;
            return t;
        };
        f2v mz{0.f, 0.f};
#pragma unroll 1
        for (int p = 0; 2 * p <= RA; p++) {
            if constexpr (U8) {
                uint32_t r[2];
                fetch8(2 * p, r);
                stage8(r, s_in);
            } else {
                if (xedge) dma(2 * p, s_in, std::true_type{});
                else dma(2 * p, s_in, std::false_type{});
                wait_vm<0>();
            }
            asm volatile("" ::: "memory");
            f2v r0, r1;   // rows 2p, 2p + 1: columns (c, c + 1)
            if constexpr (kRowX4) {
                h1rows(0, r0, r1);
            } else {
                f2v o0, o1;
                h1(s_in, o0, o1);
                r0 = f2v{o0.x, o1.x};
                r1 = f2v{o0.y, o1.y};
            }
            if (p == 0) {
#pragma unroll
                for (int i = 0; i <= RA; i++) mz = pkf(r0, tapa(i), i == 0 ? f2v{0.f, 0.f} : mz);
            } else {
                mz = pkf(r0, tap_at(RA + 2 * p), mz);
            }
            if (2 * p + 1 <= RA) mz = pkf(r1, tap_at(RA + 2 * p + 1), mz);
            wait_lgkm0();
            asm volatile("" ::: "memory");
        }
        if (left || right) fix_edges(mz);
        put_mid(mid_top, mz, mz);
    }

    // ---- the walk.  Step t: stage A pushes input rows rho0 + 2t, + 1 and completes the mid pair
    // mc = rho0 + 2t - RA, + 1; stage B pushes the pair stage A completed in step t - 1 (mc - 2),
    // so the two H passes of a step are independent and their fma chains interleave.
    const int rho0 = yb - RB - RA;
    const int ntau = (ye - yb) + 2 * RA + 2 * RB + 2;
    const int nsteps = (ntau + 1) / 2;
    const int niter = (nsteps + U - 1) / U;
    f2v accA[P], accB[P];
#pragma unroll
    for (int i = 0; i < P; i++) {
        accA[i] = f2v{0.f, 0.f};
        accB[i] = f2v{0.f, 0.f};
    }
    // the first NIN - 1 steps' DMAs, each followed by 4 scratch stores in place of the stores of
    // the step that issues it, so that the wait below counts the same instructions from step 0
    // (distinct 512-B blocks: the compiler neither drops nor merges them)
    // (u8: the first U steps' quads into registers; the compiler's own waits cover them)
    uint32_t rg[U8 ? U : 1][2];
    if constexpr (U8) {
#pragma unroll
        for (int k = 0; k < U; k++) fetch8(rho0 + 2 * k, rg[k]);
    }
    // (f32: issued at the start of the walk, whose copy fixes the DMA form)
    // stores: uniform row pointers (the level's image base + row * W, updated per step) plus a
    // lane byte offset; rows outside the band go to the wave's scratch block at lane * 8
    const uint32_t voffA = 4u * (uint32_t)c, voffB = 4u * (uint32_t)e, vtr = 8u * (uint32_t)lane;
    // 32-bit byte offsets of the stored rows inside an image (a level image is < 4 GB): the
    // stores are base (SGPR pair) + offset (VGPR), with no 64-bit address arithmetic per step
    const uint32_t W4 = 4u * (uint32_t)W;
    uint32_t rowA = (uint32_t)(rho0 - RA) * W4;            // row mc of step 0 (mod 2^32)
    uint32_t rowB = (uint32_t)(rho0 - RA - 2 - RB) * W4;   // row y of step 0
    char* const bA = reinterpret_cast<char*>(d1);
    char* const bB = reinterpret_cast<char*>(d2);
    char* const bT = reinterpret_cast<char*>(trash);
    // DS 1: the even row of stage A's pair (mc + DSR; mc's parity is RB's, yb being even)
    // decimated into the next octave's level 0 -- DownsampleKernel<1> (ProgramCU.cu:287-298):
    // ds(r, cc) = level(2 r, 2 cc), stored by the lanes that own column c = 2 cc; DS 2: stage B's
    // row y (even: y - yb is a multiple of 2), by the lanes that own column e = 2 cc
    constexpr int DSR = RB & 1;
    char* const bD = DS ? reinterpret_cast<char*>(J.ds + (long long)b * J.ds_img) : nullptr;
    const uint32_t DW4 = DS ? 4u * (uint32_t)J.dsw : 0u;
    uint32_t rowD = DS == 1 ? (uint32_t)((rho0 - RA + DSR) / 2) * DW4            // (even)
                  : DS == 2 ? (uint32_t)((rho0 - RA - 2 - RB) / 2) * DW4 : 0u;   // (row y, even)
    const uint32_t voffD = 2u * (uint32_t)(DS == 2 ? e : c);
    int slot_use = 0;                 // input slot of step t (t mod NIN)
    int mid_cur = 0;                  // mid slot of step t's stage A (t & 1; U may be odd)
    int slot_dma = NIN - 1;           // input slot of step t + NIN - 1
    // the walk, in two copies: edge strips (X4: the slot columns outside the image replicated
    // after each DMA lands) and the rest (fewer live scalars)
    auto walk = [&](auto EDGE) __attribute__((always_inline)) {
        constexpr bool kEdge = decltype(EDGE)::value;
        constexpr int OPSW = kEdge ? OPSE : OPS;   // VMEM instructions per step of this copy
        if constexpr (!U8) {
#pragma unroll
            for (int k = 0; k < NIN - 1; k++) {
                dma(rho0 + 2 * k, s_in + k * IN_SLOT, EDGE);
#pragma unroll
                for (int j = 0; j < 4 + (DS ? 1 : 0); j++)
                    *reinterpret_cast<f2v*>(trash + 128 * (j + 1) + 2 * lane) = f2v{0.f, 0.f};
            }
        }
        asm volatile("" ::: "memory");
        for (int it = 0; it < niter; it++) {
            unroll_seq(std::make_integer_sequence<int, U>{}, [&](auto KI) __attribute__((always_inline)) {
                constexpr int k = decltype(KI)::value;
                const int t = it * U + k;
                const int rho = rho0 + 2 * t;
                const int mc = rho - RA;          // stage A's completed pair
                const int mu = mc - 2;            // stage B's pair
                asm volatile("" ::: "memory");
                if constexpr (U8) {
                    // step t's quads (loaded U steps ago) into the one input slot, then step t + U's
                    // loads into the same registers
                    stage8(rg[k], s_in);
                    fetch8(rho + 2 * U, rg[k]);
                } else {
                    dma(rho + 2 * (NIN - 1), s_in + slot_dma * IN_SLOT, EDGE);
                    slot_dma = slot_dma == NIN - 1 ? 0 : slot_dma + 1;
                    // every older VMEM instruction but the OPS (NIN - 1) youngest -- this step's DMA,
                    // the previous NIN - 2 steps' DMAs and stores, and the stores of the step that
                    // issued step t's DMA -- has completed: step t's DMA has landed
                    wait_vm<OPSW * (NIN - 1)>();
                }
                asm volatile("" ::: "memory");
                // both H passes: stage A on the input slot, stage B on the previous step's mid pair
                // (an offset from one base: a select between the slot pointers made the compiler
                // lose their LDS address space -- flat accesses through the lambdas' closure)
                const int mb_off = mu <= -1 ? 2 * kMidSlot : (mu >= H - 1 ? 3 * kMidSlot
                                                                          : (mid_cur ^ 1) * kMidSlot);
                const float* mb = s_mid + mb_off;
                f2v q0, q1, r0, r1;
                if constexpr (kRowX4) {
                    h1rows(slot_use * IN_SLOT, r0, r1);
                } else {
                    f2v o0, o1;
                    h1(s_in + (U8 ? 0 : slot_use * IN_SLOT), o0, o1);
                    r0 = f2v{o0.x, o1.x};
                    r1 = f2v{o0.y, o1.y};
                }
                slot_use = slot_use == NIN - 1 ? 0 : slot_use + 1;
                // V1 push of rows rho (ring row 2k) and rho + 1 (2k + 1)
    #pragma unroll
                for (int i = 0; i < (SGK_DUO_EXP == 2 ? 1 : FWA); i++) {
                    const int s = ((2 * k - i) % P + P) % P;
                    accA[s] = pkf(r0, tapa(i), i == 0 ? f2v{0.f, 0.f} : accA[s]);
                }
                f2v A0 = accA[((2 * k - (FWA - 1)) % P + P) % P];
    #pragma unroll
                for (int i = 0; i < (SGK_DUO_EXP == 2 ? 1 : FWA); i++) {
                    const int s = ((2 * k + 1 - i) % P + P) % P;
                    accA[s] = pkf(r1, tapa(i), i == 0 ? f2v{0.f, 0.f} : accA[s]);
                }
                f2v A1 = accA[((2 * k + 1 - (FWA - 1)) % P + P) % P];
                if constexpr (!kDuoInterleave) asm volatile("" ::: "memory");
                h2(mb, q0, q1);
                // V2 push of mid rows mu (ring row 2k) and mu + 1
                const f2v g0{q0.x, q1.x}, g1{q0.y, q1.y};
    #pragma unroll
                for (int i = 0; i < (SGK_DUO_EXP == 2 ? 1 : FWB); i++) {
                    const int s = ((2 * k - i) % P + P) % P;
                    accB[s] = pkf(g0, tapb(i), i == 0 ? f2v{0.f, 0.f} : accB[s]);
                }
                const f2v B0 = accB[((2 * k - (FWB - 1)) % P + P) % P];
    #pragma unroll
                for (int i = 0; i < (SGK_DUO_EXP == 2 ? 1 : FWB); i++) {
                    const int s = ((2 * k + 1 - i) % P + P) % P;
                    accB[s] = pkf(g1, tapb(i), i == 0 ? f2v{0.f, 0.f} : accB[s]);
                }
                const f2v B1 = accB[((2 * k + 1 - (FWB - 1)) % P + P) % P];
                // stage A's pair into mid slot t & 1 (and the bottom pair): edge columns clamped
                if (mc == H - 1) A1 = A0;   // odd H: the pair (H-1, H) is (H-1, H-1)
                if (left || right) {
                    fix_edges(A0);
                    fix_edges(A1);
                }
                put_mid(s_mid + mid_cur * kMidSlot, A0, A1);
                mid_cur ^= 1;
                if (mc <= H - 1 && mc + 1 >= H - 1) {
                    const f2v Bv = mc == H - 1 ? A0 : A1;
                    put_mid(mid_bot, Bv, Bv);
                }
                asm volatile("" ::: "memory");
                // level k + 1 rows mc, mc + 1 and level k + 2 rows y = mu - RB, y + 1: the wave's
                // own columns; rows outside the band into the scratch block
                {
                    const int y = mu - RB;
                    // (mc is odd for an odd RA + RB, as in the u8 pair: each row of a pair is tested)
                    const bool a0ok = mc >= yb && mc < ye, a1ok = mc + 1 >= yb && mc + 1 < ye;
                    const bool b0ok = y >= yb && y < ye, b1ok = y + 1 >= yb && y + 1 < ye;
                    if (own1) {
                        *reinterpret_cast<f2v*>((a0ok ? bA : bT) + (a0ok ? rowA + voffA : vtr)) = A0;
                        *reinterpret_cast<f2v*>((a1ok ? bA : bT) + (a1ok ? rowA + W4 + voffA : vtr)) = A1;
                        if constexpr (DS == 1) {
                            const int yd = mc + DSR;
                            const bool dok = yd >= yb && yd < ye;
                            *reinterpret_cast<float*>((dok ? bD : bT) + (dok ? rowD + voffD : vtr)) =
                                DSR ? A1.x : A0.x;
                        }
                    }
                    if (own2) {
                        *reinterpret_cast<f2v*>((b0ok ? bB : bT) + (b0ok ? rowB + voffB : vtr)) = B0;
                        *reinterpret_cast<f2v*>((b1ok ? bB : bT) + (b1ok ? rowB + W4 + voffB : vtr)) = B1;
                        if constexpr (DS == 2) {   // (an odd H's last row decimates into no row when dsh = H / 2)
                            const bool dok = b0ok && (y >> 1) < J.dsh;
                            *reinterpret_cast<float*>((dok ? bD : bT) + (dok ? rowD + voffD : vtr)) = B0.x;
                        }
                    }
                    rowA += 2 * W4;
                    rowB += 2 * W4;
                    if constexpr (DS) rowD += DW4;
                }
            });
        }
    };
    if (xedge) walk(std::true_type{});
    else walk(std::false_type{});
    // no DMA may land after the workgroup's LDS is handed to another workgroup
    wait_vm<0>();
}

// waves per SIMD the register allocation must allow: 3 (<= 168 VGPRs) for (21, 25), whose
// scheduler otherwise hoists both H passes' LDS reads (255 VGPRs, one wave per SIMD), and the
// other pairs of >= 30 taps; 4 (<= 128) for the narrower pairs
#ifndef SGK_DUO_WPE_WIDE
#define SGK_DUO_WPE_WIDE 3
#endif
#ifndef SGK_DUO_WPE_NARROW
#define SGK_DUO_WPE_NARROW 4
#endif
template <int FWA, int FWB, int NIN, bool U8, int DS>
__global__ __launch_bounds__(64 * kDuoWaves) __attribute__((amdgpu_waves_per_eu(FWA + FWB >= 30 ? SGK_DUO_WPE_WIDE : SGK_DUO_WPE_NARROW))) void k_gauss_duo(const DuoJob J) {
    using G = DuoGeom<FWA, FWB>;
    // u8 input: one input slot (the registers hold the prefetched rows)
    __shared__ __attribute__((aligned(16))) float s_in_all[kDuoWaves][(U8 ? 1 : NIN) * G::IN_SLOT];
    __shared__ __attribute__((aligned(16))) float s_mid_all[kDuoWaves][4 * kMidSlot];
    if (J.zero.n[0] | J.zero.n[1] | J.zero.n[2]) duo_zero(J.zero);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int gw = ring_block(blockIdx.x, gridDim.x) * kDuoWaves + wave;
    if (gw >= J.total_waves) return;   // uniform per wave
    duo_wave<FWA, FWB, NIN, U8, DS>(J, gw, s_in_all[wave], s_mid_all[wave]);
}

// input row pairs in LDS: the DMA runs NIN - 1 steps ahead (compiled: 4, 5 and 7; SGPU_DUO_NIN
// picks one, A/B hook).  NIN 7 and 5 (52,224 / 41,984 B per workgroup) leave 3 workgroups per
// CU, NIN 4 (36,864 B) 4
#ifndef SGK_DUO_NIN
#define SGK_DUO_NIN 7
#endif
static int duo_nin() {
    static const int v = [] {
        const char* e = getenv("SGPU_DUO_NIN");
        return e ? atoi(e) : SGK_DUO_NIN;
    }();
    return v == 5 ? 5 : v == 4 ? 4 : 7;
}
static int duo_bands_env() {
    static const int v = [] {
        const char* e = getenv("SGPU_DUO_BANDS");
        return e ? atoi(e) : 0;
    }();
    return v;
}
// waves a launch aims for (bands of one image added until the grid has as many): a duo wave is
// latency-bound, so the grid wants more than the 12 resident waves per CU; 128 x 1080p, (11, 13)
// at octave 0: 750 / 780 / 765 / 797 us for 4,096 / 6,144 / 8,192 / 12,288 (tests/diag/r05f.sh)
#ifndef SGK_DUO_WAVES
#define SGK_DUO_WAVES 4096
#endif
static long long duo_waves_target() {
    static const long long v = [] {
        const char* e = getenv("SGPU_DUO_WAVES");
        return e && atoll(e) > 0 ? atoll(e) : (long long)SGK_DUO_WAVES;
    }();
    return v;
}

template <int FWA, int FWB, bool U8, int DS>
hipError_t duo_launch(const LevelOp& a, const LevelOp& b, hipStream_t stream, int rows_hint,
                      float* trash) {
    using G = DuoGeom<FWA, FWB>;
    DuoJob J{};
    J.src = a.src;
    J.src8 = a.src_u8;
    J.zero = a.zero;
    J.src_stride = a.src_stride;
    J.src_img = a.src_img_stride;
    J.dst1 = a.dst;
    J.dst2 = b.dst;
    J.dst_img = a.dst_img_stride;
    J.W = a.w;
    J.H = a.h;
    J.ta = a.taps;
    J.tb = b.taps;
    const LevelOp& dl = DS == 2 ? b : a;   // the level op that decimates
    J.ds = dl.ds_dst;
    J.dsw = dl.ds_w;
    J.dsh = dl.ds_h;
    J.ds_img = dl.ds_img_stride;
    J.strips = (a.w + G::SW - 1) / G::SW;
    const long long per_band = (long long)J.strips * a.batch;
    // bands: as many as the grid needs for duo_waves_target() waves; each band re-walks
    // 2 (RA + RB) halo rows, so bands stay >= 64 rows
    int nsy = 1;
    const long long want = duo_waves_target();
    if (rows_hint > 0) {
        nsy = (a.h + rows_hint - 1) / rows_hint;
    } else if (duo_bands_env() > 0) {
        nsy = std::min(duo_bands_env(), std::max(1, a.h / 64));
    } else if (per_band < want) {
        nsy = (int)std::min<long long>((want + per_band - 1) / per_band, std::max(1, a.h / 64));
    }
    int rows = (a.h + nsy - 1) / nsy;
    rows = (rows + 7) / 8 * 8;
    J.nsy = (a.h + rows - 1) / rows;
    J.rows_per_band = rows;
    J.total_waves = (int)(per_band * J.nsy);
    J.trash = trash;
    const unsigned nb = (unsigned)((J.total_waves + kDuoWaves - 1) / kDuoWaves);
    if constexpr (U8)
        hipLaunchKernelGGL((k_gauss_duo<FWA, FWB, 2, true, DS>), dim3(nb), dim3(64 * kDuoWaves), 0, stream, J);
    else if (duo_nin() == 5)
        hipLaunchKernelGGL((k_gauss_duo<FWA, FWB, 5, false, DS>), dim3(nb), dim3(64 * kDuoWaves), 0, stream, J);
    else if (duo_nin() == 4)   // 36,864 B of LDS per workgroup: 4 workgroups (16 waves) per CU
        hipLaunchKernelGGL((k_gauss_duo<FWA, FWB, 4, false, DS>), dim3(nb), dim3(64 * kDuoWaves), 0, stream, J);
    else
        hipLaunchKernelGGL((k_gauss_duo<FWA, FWB, 7, false, DS>), dim3(nb), dim3(64 * kDuoWaves), 0, stream, J);
    return hipGetLastError();
}

}  // namespace

bool gauss_duo_supported(const LevelOp& a, const LevelOp& b) {
    // f32 pairs (11, 13), (21, 25), (17, 21) with level k + 1 decimated into the next octave,
    // (13, 17) with level k + 2 decimated; the u8 ingest pair (13, 11) (level 0 from the image,
    // level 1)
    const bool u8 = a.src_u8 != nullptr;
    const bool ds = a.ds_dst != nullptr, dsb = b.ds_dst != nullptr;
    const bool dsb_ok = dsb && a.fw == 13 && b.fw == 17 && (b.w % 2) == 0 && b.ds_w * 2 == b.w &&
                        (b.ds_h == (b.h + 1) / 2 || b.ds_h == b.h / 2) &&
                        b.ds_img_stride >= (long long)b.ds_w * b.ds_h;
    const bool pair = u8 ? (a.fw == 13 && b.fw == 11 && !ds && !dsb)
                    : dsb ? (dsb_ok && !ds)
                    : ds ? (a.fw == 17 && b.fw == 21 && (a.w % 2) == 0 && a.ds_w * 2 == a.w &&
                            a.ds_h == (a.h + 1) / 2 && a.ds_img_stride >= (long long)a.ds_w * a.ds_h)
                         : ((a.fw == 11 && b.fw == 13) || (a.fw == 21 && b.fw == 25));
    const bool src_ok = u8 ? (!a.src && (a.src_stride % 4) == 0 && (a.src_img_stride % 4) == 0 &&
                              ((uintptr_t)a.src_u8 % 4) == 0)
                           : (a.src && a.src_stride >= a.w);
    const bool b_zeroes = (b.zero.n[0] | b.zero.n[1] | b.zero.n[2]) != 0;
    const bool a_zeroes = (a.zero.n[0] | a.zero.n[1] | a.zero.n[2]) != 0;
    return pair && src_ok && !b_zeroes && (u8 || !a_zeroes) && (!b.ds_dst || dsb_ok) &&
           b.src == a.dst && !b.src_u8 && a.w == b.w && a.h == b.h && a.batch == b.batch &&
           a.w >= 8 && a.h >= 8 && (a.w % 4) == 0 && b.src_stride == a.w &&
           a.dst_img_stride == b.dst_img_stride && b.src_img_stride == a.dst_img_stride &&
           a.dst_img_stride >= (long long)a.w * a.h;
}

hipError_t launch_gauss_duo(const LevelOp& a, const LevelOp& b, hipStream_t stream, int rows_hint,
                            float* trash) {
    if (!trash || !gauss_duo_supported(a, b)) return hipErrorInvalidValue;
    if (a.src_u8) return duo_launch<13, 11, true, 0>(a, b, stream, rows_hint, trash);
    if (a.ds_dst) return duo_launch<17, 21, false, 1>(a, b, stream, rows_hint, trash);
    if (b.ds_dst) return duo_launch<13, 17, false, 2>(a, b, stream, rows_hint, trash);
#define SGK_DUO(A, B) \
    if (a.fw == A && b.fw == B) return duo_launch<A, B, false, 0>(a, b, stream, rows_hint, trash);
    SGK_DUO(11, 13) SGK_DUO(21, 25)
#undef SGK_DUO
    return hipErrorInvalidValue;
}

}  // namespace sgk
