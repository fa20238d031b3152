// sift_gauss_tile.hip -- Gaussian level filter in 2-D tiles, for cache-resident levels (gfx950).
//
// FilterH<FW> then FilterV<FW> (ProgramCU.cu:115-222) with the reference's clamp-to-edge, driven
// per level by PyramidCU::BuildPyramid (PyramidCU.cpp:979-1044), and the 2x point decimation of
// DownsampleKernel<1> (ProgramCU.cu:287-298) for the level that feeds the next octave.
//
// Why a second form: one 1080p image (SiftGPU::RunSIFT, BASELINE config C2) has levels of 0.13 to
// 8.3 MB that the previous launch left in the 256 MB Infinity Cache.  The wave-streaming
// k_gauss_lean walks a band of rows per wave -- band + lag chunks of 8 rows one after the other,
// each a dependent load -> LDS -> H -> ring -> V -> store step -- so such a level is a chain of
// memory latencies (7 to 12 us per launch for at most 17 MB of traffic, profiles/r05s_c2_*).  Here
// a workgroup owns a 64 x 32 output tile: it issues the loads of its whole input window (the tile
// plus the FW - 1 halo rows and columns, clamped) at once, filters every window row horizontally
// into LDS, then vertically from LDS, and stores.  One load round trip per workgroup, no serial
// walk; the halo re-reads come from L2 / the Infinity Cache.  Levels are bit-identical to
// k_gauss_lean: the same taps summed t = 0 .. FW-1 by fma in the same order per output
// (tests/test_gpu_gauss.py).
//
// LDS per workgroup: the input window as row PAIRS (row 2p, row 2p+1) of float2, so every H-pass
// FMA is a v_pk_fma_f32 on two rows (k_gauss_lean's layout: pair stride = 2 mod 32 float2), and
// the H results (window rows x 64 columns, padded to 68).  FW 25: 37 KB -> 4 workgroups per CU.
#include <cstdint>
#include <cstdlib>
#include <utility>

#include "sift_kernels.h"

namespace sgk {
namespace {

typedef float f2v __attribute__((ext_vector_type(2)));

constexpr int kTW = 64;      // output columns of a tile
constexpr int kTH = 32;      // output rows of a tile
constexpr int kTT = 256;     // threads per workgroup

__device__ __forceinline__ f2v tpk(f2v a, float k, f2v c) {
    return __builtin_elementwise_fma(a, f2v{k, k}, c);
}
__device__ __forceinline__ int tclamp(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// tap t of a width-FW filter (make_filter's taps are symmetric bit for bit: half the SGPRs)
template <int FW>
__device__ __forceinline__ float ttap(const Taps& k, int t) {
    return k.k[t < FW - 1 - t ? t : FW - 1 - t];
}

template <int FW, int TH = kTH>
struct TileGeom {
    static constexpr int HALF = FW >> 1;
    static constexpr int OFF = (-HALF) & 3;                  // LDS column of the window's first input
    static constexpr int IN_W = kTW + FW - 1 + OFF;          // input columns held per row
    static constexpr int NQ = (IN_W + 3) / 4;                // aligned quads per row
    static constexpr int SH = OFF & 1;                       // keeps the H-pass reads 16-B aligned
    static constexpr int IN_S0 = (4 * NQ + SH + 3) & ~3;
    static constexpr int IN_S = IN_S0 + ((2 - IN_S0) & 31);  // float2 per row pair (= 2 mod 32)
    static constexpr int ROWS = TH + FW - 1;                 // window rows (even: FW is odd)
    static constexpr int NPAIR = ROWS / 2;
    static constexpr int HS = kTW + 4;                       // H-result row stride (floats)
    static constexpr int IN_BYTES = NPAIR * IN_S * 8;
    static constexpr int LDS_BYTES = IN_BYTES + ROWS * HS * 4;
    static constexpr int NLOAD = NPAIR * NQ;                 // load items: one quad of a row pair
    static constexpr int LITEMS = (NLOAD + kTT - 1) / kTT;
    static constexpr int NH = NPAIR * (kTW / 4);             // H items: 2 rows x 4 columns
    static constexpr int HITEMS = (NH + kTT - 1) / kTT;
    static constexpr int NRD = (FW + 3) / 2;                 // ds_read_b128 per H item
    static_assert(FW % 2 == 1 && FW <= 33, "odd widths up to 33");
    static_assert(TH == 16 || TH == 32, "tile heights 16 and 32 (V pass: TH / 8 rows per thread)");
    static_assert(IN_S % 32 == 2 && 4 * NQ + SH <= IN_S, "row-pair stride");
};

struct TileJob {
    const float* src;       // f32 source level, or
    const uint8_t* src8;    // the u8 image (the ingest level)
    int src_stride;         // elements between source rows
    long long src_img;
    float* dst;             // rows W apart
    long long dst_img;
    int W, H;
    Taps taps;
    float* ds;              // the next octave's level 0 (DS), rows dsw apart
    int dsw, dsh;
    long long ds_img;
    float* dst2;            // tile duo: level k+2 (dst: level k+1; same geometry and strides)
    Taps taps2;             // tile duo: the second filter
    int tx, ty;             // tiles per row / per column
    int nblocks;            // tx * ty * batch
    ZeroJob zero;           // buffers this launch zeroes besides filtering (the extract's first)
};

// logical block of dispatch slot bid: blocks are dealt round-robin over the 8 XCDs (observed,
// speed only), so logical block xcd * q + k runs on XCD xcd and a run of neighbouring tiles shares
// one L2 for its halos (k_gauss_lean's xcd_block)
__device__ __forceinline__ int tile_order(int bid, int nb) {
    const int q = nb / 8, r = nb % 8, xcd = bid % 8, k = bid / 8;
    return xcd < r ? xcd * (q + 1) + k : r * (q + 1) + (xcd - r) * q + k;
}

__device__ __forceinline__ void tile_zero(const ZeroJob& z) {
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

// The input window of a tile into LDS row pairs: rows r0 .. r0 + 2 G::NPAIR - 1 and columns
// a0 .. a0 + 4 G::NQ - 1 of the source (u8 -> p / 255), clamped to the image (clamp-to-edge);
// column a0 + c lands at float2 index p G::IN_S + c + G::SH.  Every load is issued before any LDS
// store (one round trip).
template <class G, bool U8>
__device__ __forceinline__ void tile_window(const TileJob& J, int b, int a0, int r0, f2v* s_in) {
    constexpr int NQ = G::NQ, IN_S = G::IN_S, SH = G::SH;
    const int tid = threadIdx.x;
    const int W = J.W, H = J.H;
    struct Raw { float4 v0, v1; };   // rows 2p, 2p+1 of one quad (u8: .x holds the 4 bytes)
    Raw raw[G::LITEMS];
    const float* sf = U8 ? nullptr : J.src + (long long)b * J.src_img;
    const uint8_t* s8 = U8 ? J.src8 + (long long)b * J.src_img : nullptr;
#pragma unroll
    for (int i = 0; i < G::LITEMS; i++) {
        const int item = min(tid + kTT * i, G::NLOAD - 1);   // past the end: a valid repeat
        const int p = item / NQ, j = item - p * NQ;
        const int lq = tclamp(a0 + 4 * j, 0, W - 4);
        const long long ya = tclamp(r0 + 2 * p, 0, H - 1), yb = tclamp(r0 + 2 * p + 1, 0, H - 1);
        if (U8) {
            raw[i].v0.x = __uint_as_float(*reinterpret_cast<const uint32_t*>(s8 + ya * J.src_stride + lq));
            raw[i].v1.x = __uint_as_float(*reinterpret_cast<const uint32_t*>(s8 + yb * J.src_stride + lq));
        } else {
            raw[i].v0 = *reinterpret_cast<const float4*>(sf + ya * J.src_stride + lq);
            raw[i].v1 = *reinterpret_cast<const float4*>(sf + yb * J.src_stride + lq);
        }
    }
#pragma unroll
    for (int i = 0; i < G::LITEMS; i++) {
        const int item = tid + kTT * i;
        if (G::NLOAD % kTT != 0 && item >= G::NLOAD) break;
        const int p = item / NQ, j = item - p * NQ;
        const int gq = a0 + 4 * j;
        f2v pr[4];   // column t of the quad: (row 2p, row 2p+1)
        if (U8) {
            const uint32_t w0 = __float_as_uint(raw[i].v0.x), w1 = __float_as_uint(raw[i].v1.x);
            const float c = 1.0f / 255.0f;
#pragma unroll
            for (int t = 0; t < 4; t++) {
                // p / 255 correctly rounded (GLTexImage.cpp:818): q = x / 255, one fma correction
                const f2v x{(float)((w0 >> (8 * t)) & 255u), (float)((w1 >> (8 * t)) & 255u)};
                const f2v q = x * f2v{c, c};
                const f2v r = __builtin_elementwise_fma(-q, f2v{255.0f, 255.0f}, x);
                pr[t] = __builtin_elementwise_fma(r, f2v{c, c}, q);
            }
        } else {
            pr[0] = f2v{raw[i].v0.x, raw[i].v1.x};
            pr[1] = f2v{raw[i].v0.y, raw[i].v1.y};
            pr[2] = f2v{raw[i].v0.z, raw[i].v1.z};
            pr[3] = f2v{raw[i].v0.w, raw[i].v1.w};
        }
        // clamp-to-edge: a quad left of column 0 repeats column 0, right of W-1 column W-1 (W is a
        // multiple of 4, so a quad is wholly inside or wholly outside)
        if (gq < 0) {
            pr[1] = pr[0]; pr[2] = pr[0]; pr[3] = pr[0];
        } else if (gq > W - 4) {
            pr[0] = pr[3]; pr[1] = pr[3]; pr[2] = pr[3];
        }
        f2v* q = s_in + p * IN_S + 4 * j + SH;
        if (SH == 0) {
            reinterpret_cast<float4*>(q)[0] = make_float4(pr[0].x, pr[0].y, pr[1].x, pr[1].y);
            reinterpret_cast<float4*>(q)[1] = make_float4(pr[2].x, pr[2].y, pr[3].x, pr[3].y);
        } else {
#pragma unroll
            for (int t = 0; t < 4; t++) q[t] = pr[t];
        }
    }
}

// The H pass of a width-FW filter over LDS row pairs s_in (stride IN_S float2, window column
// c at c + SH, output column j reading window columns j + OFF + t): NP row pairs x NC columns
// into s_h (rows HS floats apart), 2 rows x 4 columns per item, taps t = 0 .. FW-1 in order.
template <int FW, int NP, int NC, int IN_S, int OFF, int SH, int HS>
__device__ __forceinline__ void tile_hpass(const Taps& taps, const f2v* s_in, float* s_h) {
    constexpr int NG = NC / 4, NH = NP * NG, ITEMS = (NH + kTT - 1) / kTT, NRD = (FW + 3) / 2;
    static_assert(NC % 4 == 0 && (OFF + SH) % 2 == 0 && IN_S % 2 == 0, "16-B aligned reads");
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < ITEMS; i++) {
        const int item = tid + kTT * i;
        if (NH % kTT != 0 && item >= NH) break;
        const int hp = item / NG, hc = (item - hp * NG) * 4;
        const f2v* h_rd = s_in + hp * IN_S + hc + OFF + SH;
        f2v a[4] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
        for (int q = 0; q < NRD; q++) {
            const float4 v = reinterpret_cast<const float4*>(h_rd)[q];
            const f2v e[2] = {f2v{v.x, v.y}, f2v{v.z, v.w}};
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const int m = 2 * q + u;
#pragma unroll
                for (int c = 0; c < 4; c++)
                    if (m - c >= 0 && m - c < FW) a[c] = tpk(e[u], ttap<FW>(taps, m - c), a[c]);
            }
        }
        float* h_wr = s_h + 2 * hp * HS + hc;
        *reinterpret_cast<float4*>(h_wr) = make_float4(a[0].x, a[1].x, a[2].x, a[3].x);
        *reinterpret_cast<float4*>(h_wr + HS) = make_float4(a[0].y, a[1].y, a[2].y, a[3].y);
    }
}

// The output tile from a window already in LDS (s_in, TileGeom<FW>'s layout, window column c =
// image column x0 - HALF - OFF + c): H pass into s_h, V pass, stores of level rows y0 .. y0 + 31
// (and the decimation into the next octave's level 0).
template <int FW, bool DS, int TH = kTH>
__device__ __forceinline__ void tile_hv(const TileJob& J, const Taps& taps, float* dst, int b,
                                        int x0, int y0, const f2v* s_in, float* s_h) {
    using G = TileGeom<FW, TH>;
    constexpr int RT = TH / 8;   // V-pass rows per thread
    constexpr int HS = G::HS;
    tile_hpass<FW, G::NPAIR, kTW, G::IN_S, G::OFF, G::SH, HS>(taps, s_in, s_h);
    __syncthreads();
    // V pass: tile rows vr .. vr + RT - 1, columns vc, vc + 1
    const int tid = threadIdx.x;
    const int W = J.W, H = J.H;
    const int vc = (tid & 31) * 2, vr = (tid >> 5) * RT;
    f2v acc[RT];
#pragma unroll
    for (int j = 0; j < RT; j++) acc[j] = f2v{0.f, 0.f};
#pragma unroll
    for (int m = 0; m < FW + RT - 1; m++) {
        const f2v v = *reinterpret_cast<const f2v*>(s_h + (vr + m) * HS + vc);
#pragma unroll
        for (int j = 0; j < RT; j++)
            if (m - j >= 0 && m - j < FW) acc[j] = tpk(v, ttap<FW>(taps, m - j), acc[j]);
    }
    const int x = x0 + vc;
    if (x >= W) return;
    float* d = dst + (long long)b * J.dst_img;
    float* dd = DS ? J.ds + (long long)b * J.ds_img : nullptr;
#pragma unroll
    for (int j = 0; j < RT; j++) {
        const int y = y0 + vr + j;
        if (y >= H) break;
        *reinterpret_cast<f2v*>(d + (long long)y * W + x) = acc[j];
        if (DS && !(y & 1) && (y >> 1) < J.dsh) {
            // DownsampleKernel<1>: dst(r, c) = src(2r, min(2c, W-1))
            float* drow = dd + (long long)(y >> 1) * J.dsw;
            if ((x >> 1) < J.dsw) drow[x >> 1] = acc[j].x;
            if (x + 1 == W - 1)
                for (int cc = W >> 1; cc < J.dsw; cc++) drow[cc] = acc[j].y;
        }
    }
}

// One 64 x TH output tile (logical block lb of job J) with the workgroup's LDS `smem`.
template <int FW, bool U8, bool DS, int TH = kTH>
__device__ __forceinline__ void tile_block(const TileJob& J, int lb, char* smem) {
    using G = TileGeom<FW, TH>;
    f2v* s_in = reinterpret_cast<f2v*>(smem);
    float* s_h = reinterpret_cast<float*>(smem + G::IN_BYTES);
    const int sx = lb % J.tx, rest = lb / J.tx;
    const int ty = rest % J.ty, b = rest / J.ty;
    const int x0 = sx * kTW, y0 = ty * TH;
    tile_window<G, U8>(J, b, x0 - G::HALF - G::OFF, y0 - G::HALF, s_in);
    __syncthreads();
    tile_hv<FW, DS, TH>(J, J.taps, J.dst, b, x0, y0, s_in, s_h);
}

// ------------------------------------------------------------------------------------------
// Two consecutive levels per tile ("tile duo"): levels k+1 = V(H(level k)) and k+2 from one load
// of level k's window -- half the launches of a single image's pyramid and one level's HBM round
// trip less.  Stage 1 filters level k into level k+1 over the region the FWB filter of stage 2
// needs (the tile plus RB halo rows and columns, TileGeom<FWB>'s window), straight into LDS in
// stage 2's row-pair layout, and stores the tile's own 64 x 32 of level k+1; stage 2 is the
// single-level tile_hv on that region.  Clamp-to-edge of level k+1: its values at positions
// outside the image are recomputed as copies of the edge row / column (in the edge tiles only),
// exactly what stage 2 of a separate launch reads there.  Bit-identical to two launches: every
// output is the same fma sequence of the same values.
template <int FWA, int FWB>
struct TileDuoGeom {
    using GB = TileGeom<FWB>;
    static constexpr int RA = FWA >> 1, RB = FWB >> 1;
    static constexpr int MROWS = GB::ROWS;              // level k+1 rows y0 - RB .. (stage 2 window)
    static constexpr int MC = 4 * GB::NQ;               // level k+1 columns aB .., aB = x0 - RB - GB::OFF
    // the level-k window of stage 1: rows from y0 - RB - RA, columns from aB - RA - OFF
    struct Win {
        static constexpr int OFF = (-RA) & 3;
        static constexpr int SH = OFF & 1;
        static constexpr int NQ = (MC + FWA - 1 + OFF + 3) / 4;
        static constexpr int IN_S0 = (4 * NQ + SH + 3) & ~3;
        static constexpr int IN_S = IN_S0 + ((2 - IN_S0) & 31);
        static constexpr int NPAIR = (MROWS + FWA - 1) / 2;
        static constexpr int NLOAD = NPAIR * NQ;
        static constexpr int LITEMS = (NLOAD + kTT - 1) / kTT;
    };
    static constexpr int H1S = MC + 4;                  // stage-1 H rows (floats)
    static constexpr int R0 = Win::NPAIR * Win::IN_S * 8 > GB::IN_BYTES ? Win::NPAIR * Win::IN_S * 8
                                                                         : GB::IN_BYTES;
    static constexpr int H1B = 2 * Win::NPAIR * H1S * 4, H2B = GB::ROWS * GB::HS * 4;
    static constexpr int LDS_BYTES = R0 + (H1B > H2B ? H1B : H2B);
    static_assert(MROWS % 2 == 0 && MC % 4 == 0, "row pairs, quads");
};

template <int FWA, int FWB, bool U8, bool DSB>
__device__ __forceinline__ void tile_duo_block(const TileJob& J, int lb, char* smem) {
    using D = TileDuoGeom<FWA, FWB>;
    using GB = typename D::GB;
    using WG = typename D::Win;
    constexpr int RB = D::RB, MC = D::MC, MROWS = D::MROWS, H1S = D::H1S;
    f2v* s_w = reinterpret_cast<f2v*>(smem);             // level-k window, then level k+1 (GB layout)
    float* s_h = reinterpret_cast<float*>(smem + D::R0);  // stage-1 H rows, then stage-2 H rows
    const int tid = threadIdx.x;
    const int W = J.W, H = J.H;
    const int sx = lb % J.tx, rest = lb / J.tx;
    const int ty = rest % J.ty, b = rest / J.ty;
    const int x0 = sx * kTW, y0 = ty * kTH;
    const int aB = x0 - RB - GB::OFF;   // level k+1 column of stage-2 window column 0
    const int mr0 = y0 - RB;            // level k+1 row of stage-2 window row 0
    tile_window<WG, U8>(J, b, aB - D::RA - WG::OFF, mr0 - D::RA, s_w);
    __syncthreads();
    // stage 1, H: every window row, level k+1 columns aB .. aB + MC - 1
    tile_hpass<FWA, WG::NPAIR, MC, WG::IN_S, WG::OFF, WG::SH, H1S>(J.taps, s_w, s_h);
    __syncthreads();
    // stage 1, V: level k+1 rows 2 rp, 2 rp + 1 (stage-2 window rows), columns 2 cp, 2 cp + 1, into
    // stage 2's row pairs; the tile's own 64 x 32 also to HBM
    {
        constexpr int NCP = MC / 2, NV = NCP * (MROWS / 2), ITEMS = (NV + kTT - 1) / kTT;
        float* d1 = J.dst + (long long)b * J.dst_img;
#pragma unroll 1
        for (int i = 0; i < ITEMS; i++) {
            const int item = tid + kTT * i;
            if (item >= NV) break;
            const int rp = item / NCP, cp = item - rp * NCP;
            const int j = 2 * cp;
            const float* h_rd = s_h + 2 * rp * H1S + j;
            f2v a0{0.f, 0.f}, a1{0.f, 0.f};   // rows 2 rp, 2 rp + 1 (columns j, j + 1)
#pragma unroll
            for (int m = 0; m <= FWA; m++) {
                const f2v v = *reinterpret_cast<const f2v*>(h_rd + m * H1S);
                if (m < FWA) a0 = tpk(v, ttap<FWA>(J.taps, m), a0);
                if (m >= 1) a1 = tpk(v, ttap<FWA>(J.taps, m - 1), a1);
            }
            f2v* q = s_w + rp * GB::IN_S + j + GB::SH;
            q[0] = f2v{a0.x, a1.x};
            q[1] = f2v{a0.y, a1.y};
            // (RB may be odd: the pair's rows can straddle the tile's first / last row)
            const int y = mr0 + 2 * rp, x = aB + j;
            if (x >= x0 && x < x0 + kTW && x < W) {
                if (y >= y0 && y < y0 + kTH && y < H) *reinterpret_cast<f2v*>(d1 + (long long)y * W + x) = a0;
                if (y + 1 >= y0 && y + 1 < y0 + kTH && y + 1 < H)
                    *reinterpret_cast<f2v*>(d1 + (long long)(y + 1) * W + x) = a1;
            }
        }
    }
    __syncthreads();
    // clamp-to-edge of level k+1 (edge tiles): columns outside the image take the edge column,
    // then rows outside take the edge row
    float* sm = reinterpret_cast<float*>(s_w);
    auto at = [&](int r, int c) -> float& {   // stage-2 window row r, column c (= aB + c)
        return sm[2 * ((r >> 1) * GB::IN_S + c + GB::SH) + (r & 1)];
    };
    const int cl = aB < 0 ? -aB : 0, cr = aB + MC > W ? aB + MC - W : 0;
    if (cl | cr) {
        for (int i = tid; i < MROWS * (cl + cr); i += kTT) {
            const int r = i / (cl + cr), k = i - r * (cl + cr);
            const int c = k < cl ? k : MC - cr + (k - cl);
            at(r, c) = at(r, k < cl ? cl : W - 1 - aB);
        }
        __syncthreads();
    }
    const int rt = mr0 < 0 ? -mr0 : 0, rbt = mr0 + MROWS > H ? mr0 + MROWS - H : 0;
    if (rt | rbt) {
        for (int i = tid; i < (rt + rbt) * MC; i += kTT) {
            const int k = i / MC, c = i - k * MC;
            const int r = k < rt ? k : MROWS - rbt + (k - rt);
            at(r, c) = at(k < rt ? rt : H - 1 - mr0, c);
        }
        __syncthreads();
    }
    // stage 2: level k+2 (and its decimation)
    tile_hv<FWB, DSB>(J, J.taps2, J.dst2, b, x0, y0, s_w, s_h);
}

template <int FW, bool U8, bool DS, int TH>
__global__ __launch_bounds__(kTT) void k_gauss_tile(const TileJob J) {
    __shared__ __attribute__((aligned(16))) char smem[TileGeom<FW, TH>::LDS_BYTES];
    if (J.zero.n[0] | J.zero.n[1] | J.zero.n[2]) tile_zero(J.zero);
    tile_block<FW, U8, DS, TH>(J, tile_order(blockIdx.x, gridDim.x), smem);
}

// Two independent level jobs in one launch (the diagonal schedule, DESIGN.md 4.4: octave o+1's
// level k beside octave o's level k + kds): blocks [0, nbB) job B (dispatched first), the rest job
// A; nbB is a multiple of 8, so both keep the XCD-aware order.  f32 levels without decimation.
template <int FWA, int FWB, int TH>
__global__ __launch_bounds__(kTT) void k_gauss_tile_diag(const TileJob A, const TileJob B, int nbB) {
    constexpr int LA = TileGeom<FWA, TH>::LDS_BYTES, LB = TileGeom<FWB, TH>::LDS_BYTES;
    __shared__ __attribute__((aligned(16))) char smem[LA > LB ? LA : LB];
    const int bid = blockIdx.x;
    if (bid < nbB) {
        const int lb = tile_order(bid, nbB);
        if (lb < B.nblocks) tile_block<FWB, false, false, TH>(B, lb, smem);
    } else {
        tile_block<FWA, false, false, TH>(A, tile_order(bid - nbB, (int)gridDim.x - nbB), smem);
    }
}

template <int FWA, int FWB, bool U8, bool DSB>
__global__ __launch_bounds__(kTT) void k_gauss_tile_duo(const TileJob J) {
    __shared__ __attribute__((aligned(16))) char smem[TileDuoGeom<FWA, FWB>::LDS_BYTES];
    if (J.zero.n[0] | J.zero.n[1] | J.zero.n[2]) tile_zero(J.zero);
    tile_duo_block<FWA, FWB, U8, DSB>(J, tile_order(blockIdx.x, gridDim.x), smem);
}

// A tile duo of octave o (job A) beside octave o+1's first level (job B, single, FWC) in one
// launch: blocks [0, nbB) job B, the rest job A (as k_gauss_tile_diag).
template <int FWA, int FWB, int FWC>
__global__ __launch_bounds__(kTT) void k_gauss_tile_duo_diag(const TileJob A, const TileJob B, int nbB) {
    constexpr int LA = TileDuoGeom<FWA, FWB>::LDS_BYTES, LB = TileGeom<FWC>::LDS_BYTES;
    __shared__ __attribute__((aligned(16))) char smem[LA > LB ? LA : LB];
    const int bid = blockIdx.x;
    if (bid < nbB) {
        const int lb = tile_order(bid, nbB);
        if (lb < B.nblocks) tile_block<FWC, false, false>(B, lb, smem);
    } else {
        tile_duo_block<FWA, FWB, false, false>(A, tile_order(bid - nbB, (int)gridDim.x - nbB), smem);
    }
}

TileJob make_job(const LevelOp& op, int th = kTH) {
    TileJob J{};
    J.src = op.src;
    J.src8 = op.src_u8;
    J.src_stride = op.src_stride;
    J.src_img = op.src_img_stride;
    J.dst = op.dst;
    J.dst_img = op.dst_img_stride;
    J.W = op.w;
    J.H = op.h;
    J.taps = op.taps;
    J.ds = op.ds_dst;
    J.dsw = op.ds_w;
    J.dsh = op.ds_h;
    J.ds_img = op.ds_img_stride;
    J.tx = (op.w + kTW - 1) / kTW;
    J.ty = (op.h + th - 1) / th;
    J.nblocks = J.tx * J.ty * op.batch;
    J.zero = op.zero;
    return J;
}

template <int FW, int TH>
hipError_t tile_launch_th(const LevelOp& op, hipStream_t stream) {
    const TileJob J = make_job(op, TH);
#define SGK_TILE(U8, DS) \
    hipLaunchKernelGGL((k_gauss_tile<FW, U8, DS, TH>), dim3((unsigned)J.nblocks), dim3(kTT), 0, stream, J)
    if (op.src_u8) {
        if (op.ds_dst) SGK_TILE(true, true); else SGK_TILE(true, false);
    } else {
        if (op.ds_dst) SGK_TILE(false, true); else SGK_TILE(false, false);
    }
#undef SGK_TILE
    return hipGetLastError();
}

// (16-row tiles for the larger levels measured slower: C2 0.225-0.229 vs 0.220-0.224 ms with 32,
// alternating processes, tests/diag/r06e.sh; TileGeom / tile_hv keep the height as a parameter)
template <int FW>
hipError_t tile_launch(const LevelOp& op, hipStream_t stream) {
    return tile_launch_th<FW, kTH>(op, stream);
}

template <int FWA, int FWB>
hipError_t tile_diag_launch(const LevelOp& a, const LevelOp& b, hipStream_t stream) {
    const TileJob A = make_job(a, kTH), B = make_job(b, kTH);
    const int nbBp = (B.nblocks + 7) / 8 * 8;
    hipLaunchKernelGGL((k_gauss_tile_diag<FWA, FWB, kTH>), dim3((unsigned)(nbBp + A.nblocks)),
                       dim3(kTT), 0, stream, A, B, nbBp);
    return hipGetLastError();
}

TileJob make_duo_job(const LevelOp& a, const LevelOp& b) {
    TileJob J = make_job(a);
    J.dst2 = b.dst;
    J.taps2 = b.taps;
    J.ds = b.ds_dst;
    J.dsw = b.ds_w;
    J.dsh = b.ds_h;
    J.ds_img = b.ds_img_stride;
    return J;
}

template <int FWA, int FWB, bool U8, bool DSB>
hipError_t tile_duo_launch(const LevelOp& a, const LevelOp& b, hipStream_t stream) {
    const TileJob J = make_duo_job(a, b);
    hipLaunchKernelGGL((k_gauss_tile_duo<FWA, FWB, U8, DSB>), dim3((unsigned)J.nblocks), dim3(kTT), 0,
                       stream, J);
    return hipGetLastError();
}

template <int FWA, int FWB, int FWC>
hipError_t tile_duo_diag_launch(const LevelOp& a, const LevelOp& b, const LevelOp& c,
                                hipStream_t stream) {
    const TileJob A = make_duo_job(a, b), B = make_job(c);
    const int nbBp = (B.nblocks + 7) / 8 * 8;
    hipLaunchKernelGGL((k_gauss_tile_duo_diag<FWA, FWB, FWC>), dim3((unsigned)(nbBp + A.nblocks)),
                       dim3(kTT), 0, stream, A, B, nbBp);
    return hipGetLastError();
}

bool tile_diag_ok(const LevelOp& op) {
    return !op.src_u8 && !op.ds_dst && !(op.zero.n[0] | op.zero.n[1] | op.zero.n[2]);
}

}  // namespace

bool gauss_tile_supported(const LevelOp& op) {
    const void* base = op.src_u8 ? (const void*)op.src_u8 : (const void*)op.src;
    const bool fw_ok = op.fw >= 5 && op.fw <= 33 && (op.fw & 1);
    return fw_ok && base && op.w >= 4 && op.h >= 1 && (op.w % 4) == 0 && op.batch >= 1 &&
           (op.src_stride % 4) == 0 && (op.src_img_stride % 4) == 0 &&
           ((uintptr_t)base % (op.src_u8 ? 4 : 16)) == 0 && op.src_stride >= op.w &&
           (!op.ds_dst || (op.ds_w >= 1 && op.ds_h >= 1)) &&
           (long long)((op.w + kTW - 1) / kTW) * ((op.h + kTH - 1) / kTH) * op.batch < (1ll << 31);
}

hipError_t launch_gauss_tile(const LevelOp& op, hipStream_t stream) {
    if (!gauss_tile_supported(op)) return hipErrorInvalidValue;
#define SGK_T(FW) case FW: return tile_launch<FW>(op, stream);
    switch (op.fw) {
        SGK_T(5) SGK_T(7) SGK_T(9) SGK_T(11) SGK_T(13) SGK_T(15) SGK_T(17) SGK_T(19) SGK_T(21)
        SGK_T(23) SGK_T(25) SGK_T(27) SGK_T(29) SGK_T(31) SGK_T(33)
        default: return hipErrorInvalidValue;
    }
#undef SGK_T
}

hipError_t launch_gauss_tile_two(const LevelOp& a, const LevelOp& b, hipStream_t stream,
                                 int* launches) {
    if (launches) *launches = 1;
    if (gauss_tile_supported(a) && gauss_tile_supported(b) && tile_diag_ok(a) && tile_diag_ok(b)) {
        // the default schedule's pairs (-d 3: octave o's levels 4 / 5 beside octave o + 1's
        // levels 1 / 2); the larger job is A
        const bool swap = (long long)a.w * a.h * a.batch < (long long)b.w * b.h * b.batch;
        const LevelOp& big = swap ? b : a;
        const LevelOp& small = swap ? a : b;
#define SGK_TD(A, B) \
        if (big.fw == A && small.fw == B) return tile_diag_launch<A, B>(big, small, stream);
        SGK_TD(21, 11) SGK_TD(25, 13)
#undef SGK_TD
    }
    if (launches) *launches = 2;
    const hipError_t e = launch_gauss_tile(a, stream);
    if (e != hipSuccess) return e;
    return launch_gauss_tile(b, stream);
}

}  // namespace sgk

namespace sgk {

// The compiled tile duos (the default -d 3 schedule: octave 0's (13 u8, 11), (13, 17 + decimation),
// (21, 25); octaves >= 1: (13, 17 [+ decimation]), (21, 25); (13, 11) from a float first level,
// (11, 13) and (17, 21) for other pairings).
bool gauss_tile_duo_supported(const LevelOp& a, const LevelOp& b) {
    if (!gauss_tile_supported(a) || !gauss_tile_supported(b)) return false;
    if (a.ds_dst || b.src_u8 || (b.zero.n[0] | b.zero.n[1] | b.zero.n[2])) return false;
    if (a.src_u8 && b.ds_dst) return false;
    const bool geo = b.src == a.dst && a.w == b.w && a.h == b.h && a.batch == b.batch &&
                     b.src_stride == a.w && a.dst_img_stride == b.dst_img_stride &&
                     b.src_img_stride == a.dst_img_stride && a.dst_img_stride >= (long long)a.w * a.h;
    if (!geo) return false;
    const int fa = a.fw, fb = b.fw;
    if (b.ds_dst) return fa == 13 && fb == 17;
    return (fa == 13 && fb == 11) || (fa == 13 && fb == 17) || (fa == 21 && fb == 25) ||
           (fa == 11 && fb == 13) || (fa == 17 && fb == 21);
}

hipError_t launch_gauss_tile_duo(const LevelOp& a, const LevelOp& b, hipStream_t stream) {
    if (!gauss_tile_duo_supported(a, b)) return hipErrorInvalidValue;
    const int fa = a.fw, fb = b.fw;
    if (a.src_u8) return fa == 13 && fb == 11 ? tile_duo_launch<13, 11, true, false>(a, b, stream)
                                              : tile_duo_launch<11, 13, true, false>(a, b, stream);
    if (b.ds_dst) return tile_duo_launch<13, 17, false, true>(a, b, stream);
#define SGK_TDUO(A, B) if (fa == A && fb == B) return tile_duo_launch<A, B, false, false>(a, b, stream);
    SGK_TDUO(13, 11) SGK_TDUO(13, 17) SGK_TDUO(21, 25) SGK_TDUO(11, 13) SGK_TDUO(17, 21)
#undef SGK_TDUO
    return hipErrorInvalidValue;
}

hipError_t launch_gauss_tile_duo_one(const LevelOp& a, const LevelOp& b, const LevelOp& c,
                                     hipStream_t stream, int* launches) {
    if (launches) *launches = 1;
    if (gauss_tile_duo_supported(a, b) && !a.src_u8 && !b.ds_dst && gauss_tile_supported(c) &&
        tile_diag_ok(c) && !(a.zero.n[0] | a.zero.n[1] | a.zero.n[2])) {
        if (a.fw == 21 && b.fw == 25 && c.fw == 11) return tile_duo_diag_launch<21, 25, 11>(a, b, c, stream);
    }
    if (launches) *launches = 2;
    const hipError_t e = launch_gauss_tile_duo(a, b, stream);
    if (e != hipSuccess) return e;
    return launch_gauss_tile(c, stream);
}

}  // namespace sgk
