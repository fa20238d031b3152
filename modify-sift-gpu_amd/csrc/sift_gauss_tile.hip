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

template <int FW>
struct TileGeom {
    static constexpr int HALF = FW >> 1;
    static constexpr int OFF = (-HALF) & 3;                  // LDS column of the window's first input
    static constexpr int IN_W = kTW + FW - 1 + OFF;          // input columns held per row
    static constexpr int NQ = (IN_W + 3) / 4;                // aligned quads per row
    static constexpr int SH = OFF & 1;                       // keeps the H-pass reads 16-B aligned
    static constexpr int IN_S0 = (4 * NQ + SH + 3) & ~3;
    static constexpr int IN_S = IN_S0 + ((2 - IN_S0) & 31);  // float2 per row pair (= 2 mod 32)
    static constexpr int ROWS = kTH + FW - 1;                // window rows (even: FW is odd)
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

// One 64 x 32 output tile (logical block lb of job J) with the workgroup's LDS `smem`.
template <int FW, bool U8, bool DS>
__device__ __forceinline__ void tile_block(const TileJob& J, int lb, char* smem) {
    using G = TileGeom<FW>;
    constexpr int HALF = G::HALF, OFF = G::OFF, NQ = G::NQ, SH = G::SH, IN_S = G::IN_S, HS = G::HS;
    f2v* s_in = reinterpret_cast<f2v*>(smem);
    float* s_h = reinterpret_cast<float*>(smem + G::IN_BYTES);
    const int tid = threadIdx.x;
    const int W = J.W, H = J.H;
    const int sx = lb % J.tx, rest = lb / J.tx;
    const int ty = rest % J.ty, b = rest / J.ty;
    const int x0 = sx * kTW, y0 = ty * kTH;
    const int a0 = x0 - HALF - OFF;   // input column of LDS column SH (16-B aligned)
    const int r0 = y0 - HALF;         // input row of window row 0

    // ---- the window: every load issued before any LDS store (one round trip)
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
    __syncthreads();

    // ---- H pass: window rows 2 hp, 2 hp + 1, tile columns hc .. hc + 3, taps t = 0 .. FW-1
#pragma unroll
    for (int i = 0; i < G::HITEMS; i++) {
        const int item = tid + kTT * i;
        if (G::NH % kTT != 0 && item >= G::NH) break;
        const int hp = item >> 4, hc = (item & 15) * 4;
        const f2v* h_rd = s_in + hp * IN_S + hc + OFF + SH;
        f2v a[4] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
        for (int q = 0; q < G::NRD; q++) {
            const float4 v = reinterpret_cast<const float4*>(h_rd)[q];
            const f2v e[2] = {f2v{v.x, v.y}, f2v{v.z, v.w}};
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const int m = 2 * q + u;
#pragma unroll
                for (int c = 0; c < 4; c++)
                    if (m - c >= 0 && m - c < FW) a[c] = tpk(e[u], ttap<FW>(J.taps, m - c), a[c]);
            }
        }
        float* h_wr = s_h + 2 * hp * HS + hc;
        *reinterpret_cast<float4*>(h_wr) = make_float4(a[0].x, a[1].x, a[2].x, a[3].x);
        *reinterpret_cast<float4*>(h_wr + HS) = make_float4(a[0].y, a[1].y, a[2].y, a[3].y);
    }
    __syncthreads();

    // ---- V pass: tile rows vr .. vr + 3, columns vc, vc + 1
    const int vc = (tid & 31) * 2, vr = (tid >> 5) * 4;
    f2v acc[4] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
    for (int m = 0; m < FW + 3; m++) {
        const f2v v = *reinterpret_cast<const f2v*>(s_h + (vr + m) * HS + vc);
#pragma unroll
        for (int j = 0; j < 4; j++)
            if (m - j >= 0 && m - j < FW) acc[j] = tpk(v, ttap<FW>(J.taps, m - j), acc[j]);
    }
    const int x = x0 + vc;
    if (x >= W) return;
    float* d = J.dst + (long long)b * J.dst_img;
    float* dd = DS ? J.ds + (long long)b * J.ds_img : nullptr;
#pragma unroll
    for (int j = 0; j < 4; j++) {
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

template <int FW, bool U8, bool DS>
__global__ __launch_bounds__(kTT) void k_gauss_tile(const TileJob J) {
    __shared__ __attribute__((aligned(16))) char smem[TileGeom<FW>::LDS_BYTES];
    if (J.zero.n[0] | J.zero.n[1] | J.zero.n[2]) tile_zero(J.zero);
    tile_block<FW, U8, DS>(J, tile_order(blockIdx.x, gridDim.x), smem);
}

// Two independent level jobs in one launch (the diagonal schedule, DESIGN.md 4.4: octave o+1's
// level k beside octave o's level k + kds): blocks [0, nbB) job B (dispatched first), the rest job
// A; nbB is a multiple of 8, so both keep the XCD-aware order.  f32 levels without decimation.
template <int FWA, int FWB>
__global__ __launch_bounds__(kTT) void k_gauss_tile_diag(const TileJob A, const TileJob B, int nbB) {
    constexpr int LA = TileGeom<FWA>::LDS_BYTES, LB = TileGeom<FWB>::LDS_BYTES;
    __shared__ __attribute__((aligned(16))) char smem[LA > LB ? LA : LB];
    const int bid = blockIdx.x;
    if (bid < nbB) {
        const int lb = tile_order(bid, nbB);
        if (lb < B.nblocks) tile_block<FWB, false, false>(B, lb, smem);
    } else {
        tile_block<FWA, false, false>(A, tile_order(bid - nbB, (int)gridDim.x - nbB), smem);
    }
}

TileJob make_job(const LevelOp& op) {
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
    J.ty = (op.h + kTH - 1) / kTH;
    J.nblocks = J.tx * J.ty * op.batch;
    J.zero = op.zero;
    return J;
}

template <int FW>
hipError_t tile_launch(const LevelOp& op, hipStream_t stream) {
    const TileJob J = make_job(op);
#define SGK_TILE(U8, DS) \
    hipLaunchKernelGGL((k_gauss_tile<FW, U8, DS>), dim3((unsigned)J.nblocks), dim3(kTT), 0, stream, J)
    if (op.src_u8) {
        if (op.ds_dst) SGK_TILE(true, true); else SGK_TILE(true, false);
    } else {
        if (op.ds_dst) SGK_TILE(false, true); else SGK_TILE(false, false);
    }
#undef SGK_TILE
    return hipGetLastError();
}

template <int FWA, int FWB>
hipError_t tile_diag_launch(const LevelOp& a, const LevelOp& b, hipStream_t stream) {
    const TileJob A = make_job(a), B = make_job(b);
    const int nbBp = (B.nblocks + 7) / 8 * 8;
    hipLaunchKernelGGL((k_gauss_tile_diag<FWA, FWB>), dim3((unsigned)(nbBp + A.nblocks)), dim3(kTT),
                       0, stream, A, B, nbBp);
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
