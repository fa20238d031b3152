// sift_kernels.hip -- gfx950 (MI355X / CDNA4) kernels of the SIFT hot path.
//
// Reference semantics: SiftGPU/ProgramCU.cu (kernels) and SiftGPU/PyramidCU.cpp (stage order).
// The structure is MI355X-first, not a translation:
//   * one launch per (octave, level) covers the whole image batch (grid.z = image);
//   * the separable Gaussian is one fused kernel (H pass into an LDS tile, V pass from LDS),
//     8 B/px of HBM traffic per level instead of the reference's 16, with the next octave's
//     2x downsample written from the same tile;
//   * DoG and gradient images are never stored: the extremum kernel forms the 5 DoG planes of
//     an octave in LDS from the 6 Gaussian planes, and the orientation / descriptor kernels
//     evaluate gradients from the Gaussian level on the fly;
//   * keypoint compaction is a 1-bit-per-pixel mask written with wave ballots plus per-row
//     counts; one exclusive scan over rows gives every keypoint its slot in the reference's
//     (image, octave, level, row, column) order -- no histogram pyramid, no host round trips.
// Floating-point conventions are those of oracle/sift_oracle.cpp (fma contractions written
// out, transcendentals from sift_math.h); the build uses -ffp-contract=off.
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <type_traits>
#include <utility>

#include "sift_kernels.h"
#include "sift_math.h"

using namespace sgm;

#include "sift_keys.h"

namespace sgk {
namespace {

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// ------------------------------------------------------------------------------------------
// Gaussian level: FilterH<FW> then FilterV<FW> (ProgramCU.cu:115-222) in one kernel.
// A 256-thread workgroup owns a 64-column strip of `rows_per_strip` output rows and walks it top
// to bottom in chunks of SR2 = 32 rows:
//   * the input rows of chunk c+2 are loaded into registers while chunk c is filtered
//     (register-staged prefetch, written to LDS after the V pass), so HBM loads overlap the
//     filter arithmetic;
//   * the input chunk is stored in LDS as row PAIRS, s_in[pair][col] = (row 2p, row 2p+1);
//   * every FMA is a v_pk_fma_f32 on two independent outputs (gfx950 issues packed FP32 at twice
//     the scalar rate): a thread's H pass covers 2 rows x 4 columns and its V pass 4 rows x 2
//     columns, so every value read from LDS feeds 4 packed FMAs;
//   * the H pass writes 32 filtered rows into a 64-row LDS ring; the V pass emits output chunk
//     c-1 from the ring (lag one chunk: FW - 1 <= 32).
// Each input row is read from HBM once per strip (vertical halo (FW-1)/rows_per_strip), the
// horizontal halo (FW-1)/64 comes through L2.  Each packed lane is an IEEE fma and the taps are
// summed i = 0..FW-1 in order, so the levels are bit-identical to the oracle.
constexpr int GT = 64;
typedef float f2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2v pk_fma(f2v a, float b, f2v c) {
    return __builtin_elementwise_fma(a, f2v{b, b}, c);
}

// Tap t of a width-FW filter.  make_filter's taps are symmetric bit for bit (tap i is
// exp(-i^2 / 2 sigma^2) / sum for i = t - FW/2), so the kernels holding two filters read only
// the first half: half the scalar registers (two full tap sets spilled SGPRs to VGPR lanes).
template <int FW>
__device__ __forceinline__ float tap(const Taps& taps, int t) {
    return taps.k[t < FW - 1 - t ? t : FW - 1 - t];
}

// p / 255.0f for an integer p in [0, 255] (GLTexImage.cpp:818: the reference's u8 -> float),
// correctly rounded without a division: q = p * (1/255) then one fma residual correction.  Exact
// for all 256 inputs (tests/test_oracle.py::test_u8_scale_is_exact_division).
__device__ __forceinline__ float u8_to_unit(uint32_t p) {
    const float x = (float)p, c = 1.0f / 255.0f;
    const float q = x * c;
    return fma_(fma_(-q, 255.0f, x), c, q);
}

constexpr int SR2 = 32;

// VEC: the input rows are fetched as 16-byte (f32) / 4-byte (u8) aligned quads instead of one
// element per lane: the strip's load window starts at a0 = x0 - HALF - OFF, OFF = (-HALF) & 3,
// so every quad is aligned, and quads left of column 0 / right of W-1 replicate the edge value
// (W is a multiple of 4, so a quad is entirely inside or entirely outside).  LDS column j holds
// input column a0 + j in both forms.
template <int FW, bool U8, bool VEC>
__global__ __launch_bounds__(256) void k_gauss_pk2(
    const float* __restrict__ src, const uint8_t* __restrict__ src8, int src_stride,
    long long src_img_stride, float* __restrict__ dst, long long dst_img_stride, int W, int H,
    Taps taps, float* __restrict__ ds, int dsw, int dsh, long long ds_img_stride,
    int rows_per_strip) {
    constexpr int HALF = FW >> 1;
    constexpr int OFF = VEC ? ((-HALF) & 3) : 0;      // LDS column of the strip's first input
    constexpr int IN_W = GT + FW - 1 + OFF;           // input columns held per row
    constexpr int NQ = (IN_W + 3) / 4;                // aligned quads per row (VEC)
    constexpr int NRD = (FW + 3) / 2;                 // ds_read_b128 per H-pass thread
    constexpr int IN_S = (GT + FW + 3 + OFF + 3) & ~3;   // float2 per row pair
    static_assert(!VEC || 4 * NQ <= IN_S, "quad stores stay inside the row pair");
    constexpr int RS = 64;                            // ring rows: (1 + 1) * 32 for FW <= 33
    constexpr int HS = GT + 4;                        // ring row stride (floats)
    constexpr int NLD = VEC ? ((SR2 / 2) * NQ + 255) / 256 : ((SR2 / 2) * IN_W + 255) / 256;
    constexpr int IN_SV = IN_S;                       // LDS row-pair stride
    static_assert(FW - 1 <= SR2, "ring holds one chunk of lag");
    __shared__ __attribute__((aligned(16))) f2v s_in[(SR2 / 2) * IN_SV];
    __shared__ __attribute__((aligned(16))) float s_h[RS * HS];

    const int tid = threadIdx.x;
    const int strips_x = (W + GT - 1) / GT;
    const int strips_y = (H + rows_per_strip - 1) / rows_per_strip;
    const int id = blockIdx.x;
    const int sx = id % strips_x, rest = id / strips_x;
    const int sy = rest % strips_y, b = rest / strips_y;
    const int x0 = sx * GT;
    const int yb = sy * rows_per_strip;
    const int ye = min(H, yb + rows_per_strip);
    const int nin = (ye - yb) + FW - 1;
    const int nchunk_in = (nin + SR2 - 1) / SR2;
    const int nchunk_out = (ye - yb + SR2 - 1) / SR2;

    const float* sf = U8 ? nullptr : src + (long long)b * src_img_stride;
    const uint8_t* s8 = U8 ? src8 + (long long)b * src_img_stride : nullptr;
    const int a0 = x0 - HALF - OFF;
    // stage element: VEC -> 4 pairs (rows 2p, 2p+1 of one aligned quad); else one pair
    typedef typename std::conditional<VEC, f2v[4], f2v[1]>::type Elem;
    Elem stA[NLD], stB[NLD];
    auto load_chunk = [&](Elem (&stage)[NLD], int c) {
#pragma unroll
        for (int m = 0; m < NLD; m++) {
            if (VEC) {
                const int e = min(tid + 256 * m, (SR2 / 2) * NQ - 1);
                const int p = e / NQ, j = e - p * NQ;
                const int gy0 = clampi(yb - HALF + c * SR2 + 2 * p, 0, H - 1);
                const int gy1 = clampi(yb - HALF + c * SR2 + 2 * p + 1, 0, H - 1);
                const int gq = a0 + 4 * j;                          // aligned first column
                const int lq = clampi(gq, 0, W - 4);
                float r0[4], r1[4];
                if (U8) {
                    const uint32_t w0 = *reinterpret_cast<const uint32_t*>(s8 + (long long)gy0 * src_stride + lq);
                    const uint32_t w1 = *reinterpret_cast<const uint32_t*>(s8 + (long long)gy1 * src_stride + lq);
#pragma unroll
                    for (int t = 0; t < 4; t++) {
                        r0[t] = u8_to_unit((w0 >> (8 * t)) & 255u);
                        r1[t] = u8_to_unit((w1 >> (8 * t)) & 255u);
                    }
                } else {
                    const float4 v0 = *reinterpret_cast<const float4*>(sf + (long long)gy0 * src_stride + lq);
                    const float4 v1 = *reinterpret_cast<const float4*>(sf + (long long)gy1 * src_stride + lq);
                    r0[0] = v0.x; r0[1] = v0.y; r0[2] = v0.z; r0[3] = v0.w;
                    r1[0] = v1.x; r1[1] = v1.y; r1[2] = v1.z; r1[3] = v1.w;
                }
                // clamp-to-edge: a quad left of column 0 repeats column 0, right of W-1 repeats W-1
                const bool left = gq < 0, right = gq > W - 4;
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    const float u0 = left ? r0[0] : (right ? r0[3] : r0[t]);
                    const float u1 = left ? r1[0] : (right ? r1[3] : r1[t]);
                    stage[m][t] = f2v{u0, u1};
                }
            } else {
                const int e = min(tid + 256 * m, (SR2 / 2) * IN_W - 1);
                const int p = e / IN_W, col = e - p * IN_W;
                const int gy0 = clampi(yb - HALF + c * SR2 + 2 * p, 0, H - 1);
                const int gy1 = clampi(yb - HALF + c * SR2 + 2 * p + 1, 0, H - 1);
                const int gx = clampi(a0 + col, 0, W - 1);
                if (U8) {
                    stage[m][0] = f2v{u8_to_unit(s8[(long long)gy0 * src_stride + gx]),
                                      u8_to_unit(s8[(long long)gy1 * src_stride + gx])};
                } else {
                    stage[m][0] = f2v{sf[(long long)gy0 * src_stride + gx],
                                      sf[(long long)gy1 * src_stride + gx]};
                }
            }
        }
    };
    auto store_chunk = [&](const Elem (&stage)[NLD]) {
#pragma unroll
        for (int m = 0; m < NLD; m++) {
            const int e = tid + 256 * m;
            if (VEC) {
                if (e < (SR2 / 2) * NQ) {
                    const int p = e / NQ, j = e - p * NQ;
                    float4* q = reinterpret_cast<float4*>(&s_in[p * IN_SV + 4 * j]);
                    q[0] = make_float4(stage[m][0].x, stage[m][0].y, stage[m][1].x, stage[m][1].y);
                    q[1] = make_float4(stage[m][2].x, stage[m][2].y, stage[m][3].x, stage[m][3].y);
                }
            } else if (e < (SR2 / 2) * IN_W) {
                const int p = e / IN_W, col = e - p * IN_W;
                s_in[p * IN_SV + col] = stage[m][0];
            }
        }
    };

    load_chunk(stA, 0);
    store_chunk(stA);
    if (1 < nchunk_in) load_chunk(stA, 1);
    __syncthreads();
    float* d = dst + (long long)b * dst_img_stride;
    float* dd = ds ? ds + (long long)b * ds_img_stride : nullptr;
    const int hp = tid >> 4, hc = (tid & 15) * 4;     // H pass: rows 2hp, 2hp+1; columns hc..hc+3
    const int vq = tid >> 5, vc = (tid & 31) * 2;     // V pass: rows 4vq..4vq+3; columns vc, vc+1
    const int x = x0 + vc;
    // iteration c: chunk c is in LDS, chunk c+1 in `cur` registers; load chunk c+2 into `nxt`
    auto step = [&](int c, Elem (&cur)[NLD], Elem (&nxt)[NLD]) {
        const bool has_in = c < nchunk_in, has_next = c + 1 < nchunk_in;
        if (c + 2 < nchunk_in) load_chunk(nxt, c + 2);
        if (has_in) {   // H pass of input chunk c -> ring rows c*SR2 .. c*SR2+31
            const f2v* rowp = &s_in[hp * IN_SV + hc + OFF];
            f2v a[4] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};   // columns hc+i
#pragma unroll
            for (int q = 0; q < NRD; q++) {
                f2v e[2];                            // pair columns hc+2q, hc+2q+1
                if (OFF % 2 == 0) {
                    const float4 v = reinterpret_cast<const float4*>(rowp)[q];
                    e[0] = f2v{v.x, v.y};
                    e[1] = f2v{v.z, v.w};
                } else {
                    e[0] = rowp[2 * q];
                    e[1] = rowp[2 * q + 1];
                }
#pragma unroll
                for (int u = 0; u < 2; u++) {
                    const int m = 2 * q + u;
#pragma unroll
                    for (int i = 0; i < 4; i++)
                        if (m - i >= 0 && m - i < FW) a[i] = pk_fma(e[u], taps.k[m - i], a[i]);
                }
            }
            const int r0 = (c * SR2 + 2 * hp) & (RS - 1);
            *reinterpret_cast<float4*>(&s_h[r0 * HS + hc]) = make_float4(a[0].x, a[1].x, a[2].x, a[3].x);
            *reinterpret_cast<float4*>(&s_h[(r0 + 1) * HS + hc]) = make_float4(a[0].y, a[1].y, a[2].y, a[3].y);
        }
        __syncthreads();
        const int kout = c - 1;
        if (kout >= 0) {   // V pass of output chunk kout (lag 1 chunk: FW - 1 <= SR2)
            const int t0 = kout * SR2 + 4 * vq;
            f2v acc[4] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};   // rows t0+j
#pragma unroll
            for (int m = 0; m < FW + 3; m++) {
                const f2v v = *reinterpret_cast<const f2v*>(&s_h[((t0 + m) & (RS - 1)) * HS + vc]);
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (m - j >= 0 && m - j < FW) acc[j] = pk_fma(v, taps.k[m - j], acc[j]);
            }
            // the sums are complete here: without this, each row's FMA chain is sunk into its
            // conditional store below and every ring value of the pass stays live until then
            // (+2 VGPRs per tap: a wave per SIMD of occupancy, pyramid +9 %)
#pragma unroll
            for (int j = 0; j < 4; j++) asm volatile("" : "+v"(acc[j]));
            if (x < W) {
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int y = yb + t0 + j;
                    if (y < ye) {
                        *reinterpret_cast<f2v*>(&d[(long long)y * W + x]) = acc[j];
                        // DownsampleKernel<1> (ProgramCU.cu:287-298) into the next octave's
                        // level 0: dst(r, c) = src(2r, min(2c, W-1)); x is even, W is even.
                        if (dd && !(y & 1) && (y >> 1) < dsh) {
                            float* drow = dd + (long long)(y >> 1) * dsw;
                            if ((x >> 1) < dsw) drow[x >> 1] = acc[j].x;
                            if (x + 1 == W - 1)
                                for (int cc = W >> 1; cc < dsw; cc++) drow[cc] = acc[j].y;
                        }
                    }
                }
            }
        }
        if (has_next) store_chunk(cur);
        __syncthreads();
    };
    const int nsteps = nchunk_out + 1;
    for (int c = 0; c < nsteps; c += 2) {
        step(c, stA, stB);
        if (c + 1 < nsteps) step(c + 1, stB, stA);
    }
}

// ------------------------------------------------------------------------------------------
// Gaussian level, wave-streaming form (k_gauss_lean below): the same H-then-V filter as
// k_gauss_pk2 (same taps, same summation order i = 0..FW-1, so bit-identical outputs), but every
// WAVE owns a 64-column strip band and walks it on its own with a wave-private LDS row-pair buffer
// and H ring -- no workgroup barriers, so each wave keeps its row loads in flight independently
// of the other waves of its workgroup (the extremum kernel gained 3.9 -> 5.9 TB/s from the same
// change).  Per step a wave:
//   * H-filters input chunk c (8 rows: 4 row pairs x 16 lanes x 4 columns, packed FMAs) from
//     the row-pair buffer into ring rows 8c .. 8c+7;
//   * V-filters output chunk c - L (L = ceil((FW-1)/8) chunks of lag: 2 row groups x 32 lanes
//     x 2 columns x 4 rows) from the ring and stores it (plus the decimated next-octave level);
//   * moves input chunk c+1 from registers into the row-pair buffer and issues the loads of
//     chunk c+4.
// LDS ops of one wave execute in issue order, so a wave needs no barrier between writing a
// buffer and reading what other lanes wrote; the empty asm statements only stop the compiler
// from moving LDS accesses across the phase boundaries.  Every LDS access of a wave stays inside
// its own buffers (round 3's pad-slot overrun, fixed in k_gauss_lean's loaders).
// XCD-aware block order: blocks are dealt round-robin over the 8 XCDs (observed placement,
// MI355X_MICROARCH.md; speed only, never correctness), so logical block xcd * q + k runs on XCD
// xcd and a run of consecutive logical blocks -- neighbouring image regions -- shares one L2.
__device__ __forceinline__ int xcd_block(int bid, int nb) {
    const int q = nb / 8, r = nb % 8, xcd = bid % 8, k = bid / 8;
    return xcd < r ? xcd * (q + 1) + k : r * (q + 1) + (xcd - r) * q + k;
}

// Grouped XCD order: G logically consecutive workgroups on one XCD, dispatched within 8 G slots
// of each other (workgroup b runs on XCD b % 8), the groups in dispatch order -- locality for
// neighbours without xcd_block's partition of the whole grid into 8 contiguous ranges (which
// leaves XCDs idle when the work per workgroup changes along the grid).  The last partial round
// of 8 G keeps the identity.
template <int G>
__device__ __forceinline__ int xcd_group(int bid, int nb) {
    const int full = nb / (8 * G) * (8 * G);
    if (bid >= full) return bid;
    const int m = bid / (8 * G), r = bid % (8 * G);
    return m * (8 * G) + (r % 8) * G + r / 8;
}

constexpr int WCH = 8;   // rows per chunk (wave kernel)

struct GaussWaveGrid {
    int strips_x, nsy, rows_per_band, total_waves;
};

#ifndef SGK_GW_WPB
#define SGK_GW_WPB 4
#endif
#ifndef SGK_GW_HSPAD
#define SGK_GW_HSPAD 4
#endif
// 1: conflict-free row-pair stores in k_gauss_lean (lane map, no pad slot):
// 128 x 1080p pyramid 3.402 / 3.434 vs 3.440 / 3.441 ms per step, C4 3.75 / 3.76 vs 3.77 / 3.73
// (two alternating pairs, tests/diag/g6.sh); 0: round 5's lane map
#ifndef SGK_GW_STMAP
#define SGK_GW_STMAP 1
#endif
constexpr int kGwWaves = SGK_GW_WPB;   // waves per workgroup of k_gauss_lean

// band height of the level kernel: rows_hint > 0 forces it (test / tuning hook), else bands of
// the whole image unless that leaves fewer than ~8 waves per CU, then as many bands as needed.
// A band re-reads the level's FW-1 halo rows, so bands stay >= 4 chunks high while the level
// streams from HBM; a level of at most SGK_SHORT_BAND_MB (one image of a small batch, or the
// upper octaves of a batch, largely still in the 256 MB Infinity Cache from the previous level)
// may go down to one chunk: its launches are
// latency-bound (a wave walks band + lag chunks one after the other), and shorter bands are
// fewer steps per wave.  Measured against 128 MB with ~8,192 waves on such levels (alternating
// processes, tests/diag/r03h.sh): pyramid 3.69 vs 3.73-3.76 ms per 128 x 1080p, C4 3.55 vs 3.65.
#ifndef SGK_SHORT_BAND_MB
#define SGK_SHORT_BAND_MB 64
#endif
static GaussWaveGrid gauss_wave_grid(int w, int h, int batch, int rows_hint, int nw,
                                     bool long_bands = false) {
    GaussWaveGrid g{};
    g.strips_x = (w + GT * nw - 1) / (GT * nw);
    const long long per_band = (long long)g.strips_x * nw * batch;   // waves per band
    int rows = h;
    if (rows_hint > 0) {
        rows = rows_hint;
    } else {
        // long_bands (A/B hook, per context: SGPU_DEBUG_GAUSS_LONG_BANDS, or SGPU_GAUSS_BANDS=long
        // read at context creation) keeps bands >= 4 chunks on every level (round 2)
        const bool short_ok = !long_bands && 4ll * w * h * batch <= ((long long)SGK_SHORT_BAND_MB << 20);
        const long long want = 8 * 256;
        const int nsy = (int)std::min<long long>((want + per_band - 1) / per_band,
                                                 std::max(1, h / ((short_ok ? 1 : 4) * WCH)));
        rows = (h + std::max(nsy, 1) - 1) / std::max(nsy, 1);
    }
    rows = std::max(WCH, (rows + WCH - 1) / WCH * WCH);
    g.rows_per_band = rows;
    g.nsy = (h + rows - 1) / rows;
    g.total_waves = (int)(per_band * g.nsy);
    return g;
}

// ------------------------------------------------------------------------------------------
// Gaussian level, lean form (the shipped kernel, FW <= 33): round 2's k_gauss_wave filter -- same
// strips, bands, chunks, row-pair buffer, H ring and lag, the same taps in the same order, so the
// levels are bit-identical -- with the per-step work that is not filtering taken off the vector
// ALU.  The kernel traces showed k_gauss_wave issuing ~150 non-FMA VALU instructions per 8-row
// step against 88 packed FMAs (FW 11): 64-bit load and store addresses, per-lane row clamps,
// clamp-to-edge selects, ring-row wrap arithmetic.  Here:
//   * the wave's geometry is uniform (readfirstlane of the wave index), so image, band and row
//     bases live in SGPRs and every global load / store is a uniform row pointer plus a lane
//     constant 32-bit offset (the saddr form);
//   * the loaders are laid out lane = 32 g + j: half-wave g loads the quads j of row pair 2m + g,
//     so a lane's column (and its clamp) is fixed for the whole kernel, and a chunk's rows are
//     uniform; only chunks that reach above row 0 or below row H-1 clamp per lane;
//   * clamp-to-edge column selects only in the strips at the image's left / right edge;
//   * the ring holds 4 chunk slots (RS = 32, LAG <= 3; 8 slots, RS = 64, for FW 27 .. 33) and the
//     step's slot is compile-time (the main loop is unrolled by the slot count), so ring reads and writes are lane-constant base + immediate
//     offset; the half-wave whose rows wrap first (vq = 1, 4 rows ahead) reads through a second
//     base for the 4 rows where only it has wrapped;
//   * u8 -> f32 (the ingest level) on row pairs with packed multiply / fma;
//   * the decimation into the next octave's level 0 is a template parameter.
#ifndef SGK_LEAN_R24
#define SGK_LEAN_R24 0   // 1: 3-slot ring for FW <= 17, 16 waves per CU: measured slower (3.76-3.77 vs 3.71-3.75 ms)
#endif
// f(integral_constant<int, I>) for I in the sequence, in order (compile-time step indices)
template <int... I, class F>
__device__ __forceinline__ void unrolled_steps(std::integer_sequence<int, I...>, F&& f) {
    (f(std::integral_constant<int, I>{}), ...);
}

// One level filter job of a launch: source (u8 or f32), destination, geometry, taps, the
// optional decimation into the next octave's level 0, and the wave grid.
struct GaussJob {
    const float* src;
    const uint8_t* src8;
    int src_stride;
    long long src_img_stride;
    float* dst;
    long long dst_img_stride;
    int W, H;
    Taps taps;
    float* ds;
    int dsw, dsh;
    long long ds_img_stride;
    GaussWaveGrid gg;
    ZeroJob zero;   // buffers this launch zeroes besides filtering (the extract's first launch)
};

__device__ __forceinline__ void zero_words(uint32_t* p, size_t n, size_t q) {
    if (q * 4 + 4 <= n) {
        *reinterpret_cast<uint4*>(p + q * 4) = make_uint4(0, 0, 0, 0);
    } else {
        for (size_t i = q * 4; i < n; i++) p[i] = 0;
    }
}

// a ZeroJob over the whole grid (uint4 stores; the buffers are hipMalloc'ed, 16-B aligned)
__device__ __forceinline__ void zero_job(const ZeroJob& z) {
    const size_t step = (size_t)gridDim.x * blockDim.x;
    const size_t t0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll
    for (int i = 0; i < 3; i++)
        for (size_t q = t0; q * 4 < z.n[i]; q += step) zero_words(z.p[i], z.n[i], q);
}

// LDS geometry of the level filter for width FW (per wave)
template <int FW>
struct LeanGeom {
    static constexpr int HALF = FW >> 1;
    static constexpr int OFF = (-HALF) & 3;                  // LDS column of the strip's first input
    static constexpr int IN_W = GT + FW - 1 + OFF;           // input columns held per row
    static constexpr int NQ = (IN_W + 3) / 4;                // aligned quads per row
    static constexpr int SH = OFF & 1;
    static constexpr int IN_S0 = (4 * NQ + SH + 3) & ~3;
    static constexpr int IN_S = IN_S0 + ((2 - IN_S0) & 31);  // float2 per row pair (= 2 mod 32)
    static constexpr int LAG = (FW - 1 + WCH - 1) / WCH;     // chunks between H and V of a row
    // ring rows: 3 slots of WCH for FW <= 17 (LAG <= 2; SGK_LEAN_R24), 4 for FW <= 25, 8 for
    // FW 27 .. 33 (LAG 4)
    static constexpr int RS = (SGK_LEAN_R24 && WCH * (LAG + 1) <= 24) ? 24
                            : WCH * (LAG + 1) <= 32 ? 32 : 64;
    static constexpr int HS = GT + SGK_GW_HSPAD;             // ring row stride (floats)
    static constexpr int IN_WORDS = (WCH / 2) * IN_S + 8;    // float2: row pairs + 2 pad slots
    static constexpr int RING_WORDS = RS * HS;               // floats
};

// The level filter of one wave (global wave index gw of job J) with its LDS buffers s_in / s_h.
template <int FW, bool U8, bool DS>
__device__ __forceinline__ void gauss_lean_wave(const GaussJob& J, int gw, f2v* s_in, float* s_h) {
    using G = LeanGeom<FW>;
    constexpr int HALF = G::HALF, OFF = G::OFF, NQ = G::NQ, SH = G::SH, IN_S = G::IN_S;
    static_assert(NQ <= 32, "a row's quads fit half a wave");
    constexpr int NRD = (FW + 3) / 2;                 // ds_read_b128 per H-pass lane
    static_assert(IN_S % 32 == 2 && 4 * NQ + SH <= IN_S, "row-pair stride");
    constexpr int LAG = G::LAG, RS = G::RS, HS = G::HS;
    constexpr int NSLOT = RS / WCH;
    static_assert(WCH * (LAG + 1) <= RS && FW <= 33, "the ring's chunk slots hold the lag");
    constexpr int NPAIR = WCH / 2;
#ifndef SGK_GW_NST_U8
#define SGK_GW_NST_U8 4
#endif
    constexpr int NST = U8 ? SGK_GW_NST_U8 : 4;       // chunks in registers (u8: 1 dword per row)
    const float* __restrict__ src = J.src;
    const uint8_t* __restrict__ src8 = J.src8;
    const int src_stride = J.src_stride;
    const long long src_img_stride = J.src_img_stride;
    float* __restrict__ dst = J.dst;
    const long long dst_img_stride = J.dst_img_stride;
    const int W = J.W, H = J.H;
    const Taps& taps = J.taps;
    float* __restrict__ ds = J.ds;
    const int dsw = J.dsw, dsh = J.dsh;
    const long long ds_img_stride = J.ds_img_stride;
    const GaussWaveGrid& gg = J.gg;

    const int lane = threadIdx.x & 63;
    if (gw >= gg.total_waves) return;                 // uniform per wave
    const int sx = gw % gg.strips_x, rest = gw / gg.strips_x;
    const int x0 = sx * GT;
    const int sy = rest % gg.nsy, b = rest / gg.nsy;
    const int yb = sy * gg.rows_per_band;
    const int ye = min(H, yb + gg.rows_per_band);
    const int nchunk_out = (ye - yb + WCH - 1) / WCH;

    const float* sf = U8 ? nullptr : src + (long long)b * src_img_stride;
    const uint8_t* s8 = U8 ? src8 + (long long)b * src_img_stride : nullptr;
    const int a0 = x0 - HALF - OFF;
    // loader lane: half-wave g, quad j (lanes past the row's last quad re-load the last quad and
    // store into a pad slot)
#if SGK_GW_STMAP
    // lane = 8 k + 4 g + i -> quad 4 k + i of row pair g: an 8-lane ds_write_b128 group covers
    // all 32 banks (rows 2p and 2p + 2's pairs are 2 IN_S = 4 mod 32 floats apart), and the lanes
    // past the row's last quad skip the row-pair store instead of sharing one pad slot
    const int lj0 = (lane & 3) | ((lane >> 3) << 2);
    const int lg = (lane >> 2) & 1, lj = min(lj0, NQ - 1);
    const bool lreal = lj0 < NQ;
#else
    const int lg = lane >> 5, lj = min(lane & 31, NQ - 1);
    const bool lreal = (lane & 31) < NQ;
#endif
    const int gq = a0 + 4 * lj;
    const int lq = clampi(gq, 0, W - 4);
    const bool left = gq < 0, right = gq > W - 4;
    const bool edge = a0 < 0 || a0 + 4 * NQ > W;      // uniform: this strip clamps columns
    // element offsets of the lane's quad in rows 2 g and 2 g + 1 of a row group
    const uint32_t loff0 = (uint32_t)(2 * lg * src_stride + lq), loff1 = loff0 + (uint32_t)src_stride;
    // LDS float2 index of the lane's quad in row pairs lg (m = 0) and lg + 2 (m = 1); a lane past
    // the row's last quad stores into its own pad slot per m.  (Round 3 used one pad slot and
    // added the m = 1 pair offset to it too: those stores landed 2 IN_S float2 past the wave's
    // buffer -- in the next wave's row-pair padding, or past the workgroup's LDS for the last
    // wave -- harmless only by layout; the same pattern made k_gauss_pair's aliased mid buffer
    // nondeterministic)
    const int s_off0 = lreal ? lg * IN_S + 4 * lj + SH : NPAIR * IN_S;
    const int s_off1 = lreal ? s_off0 + 2 * IN_S : NPAIR * IN_S + 4;

    struct Elem { float4 v0, v1; };   // the raw fetch of rows 2p, 2p+1 (u8: .x as the u32)
    Elem st[NST][2];
    auto load_chunk = [&](Elem (&stage)[2], int c) __attribute__((always_inline)) {
        const int rb = yb - HALF + WCH * c;           // first input row of chunk c (uniform)
        if (rb >= 0 && rb + WCH <= H) {
#pragma unroll
            for (int m = 0; m < 2; m++) {
                const long long ro = (long long)(rb + 4 * m) * src_stride;   // uniform
                if (U8) {
                    const uint8_t* r = s8 + ro;
                    stage[m].v0.x = __uint_as_float(*reinterpret_cast<const uint32_t*>(r + loff0));
                    stage[m].v1.x = __uint_as_float(*reinterpret_cast<const uint32_t*>(r + loff1));
                } else {
                    const float* r = sf + ro;
                    stage[m].v0 = *reinterpret_cast<const float4*>(r + loff0);
                    stage[m].v1 = *reinterpret_cast<const float4*>(r + loff1);
                }
            }
        } else {   // the band reaches above row 0 or below row H-1: rows clamp per lane
#pragma unroll
            for (int m = 0; m < 2; m++) {
                const int y0 = clampi(rb + 4 * m + 2 * lg, 0, H - 1);
                const int y1 = clampi(rb + 4 * m + 2 * lg + 1, 0, H - 1);
                if (U8) {
                    stage[m].v0.x = __uint_as_float(*reinterpret_cast<const uint32_t*>(s8 + (long long)y0 * src_stride + lq));
                    stage[m].v1.x = __uint_as_float(*reinterpret_cast<const uint32_t*>(s8 + (long long)y1 * src_stride + lq));
                } else {
                    stage[m].v0 = *reinterpret_cast<const float4*>(sf + (long long)y0 * src_stride + lq);
                    stage[m].v1 = *reinterpret_cast<const float4*>(sf + (long long)y1 * src_stride + lq);
                }
            }
        }
    };
    auto store_chunk = [&](const Elem (&stage)[2]) __attribute__((always_inline)) {
#pragma unroll
        for (int m = 0; m < 2; m++) {
            f2v pr[4];   // column t of the quad: (row 2p, row 2p+1)
            if (U8) {
                const uint32_t w0 = __float_as_uint(stage[m].v0.x), w1 = __float_as_uint(stage[m].v1.x);
                const float c = 1.0f / 255.0f;
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    // u8_to_unit on the pair: q = x / 255 rounded, then one fma correction
                    const f2v x{(float)((w0 >> (8 * t)) & 255u), (float)((w1 >> (8 * t)) & 255u)};
                    const f2v q = x * f2v{c, c};
                    const f2v r = __builtin_elementwise_fma(-q, f2v{255.0f, 255.0f}, x);
                    pr[t] = __builtin_elementwise_fma(r, f2v{c, c}, q);
                }
            } else {
                pr[0] = f2v{stage[m].v0.x, stage[m].v1.x};
                pr[1] = f2v{stage[m].v0.y, stage[m].v1.y};
                pr[2] = f2v{stage[m].v0.z, stage[m].v1.z};
                pr[3] = f2v{stage[m].v0.w, stage[m].v1.w};
            }
            if (edge) {   // clamp-to-edge: a quad left of column 0 repeats column 0, right of W-1 W-1
                const f2v e0 = pr[0], e3 = pr[3];
#pragma unroll
                for (int t = 0; t < 4; t++) pr[t] = left ? e0 : (right ? e3 : pr[t]);
            }
            f2v* q = s_in + (m ? s_off1 : s_off0);
            if (SGK_GW_STMAP && !lreal) continue;
            if (SH == 0) {
                reinterpret_cast<float4*>(q)[0] = make_float4(pr[0].x, pr[0].y, pr[1].x, pr[1].y);
                reinterpret_cast<float4*>(q)[1] = make_float4(pr[2].x, pr[2].y, pr[3].x, pr[3].y);
            } else {   // 8-byte aligned
#pragma unroll
                for (int t = 0; t < 4; t++) q[t] = pr[t];
            }
        }
    };

#pragma unroll
    for (int k = 0; k < NST; k++) load_chunk(st[k], k);
    store_chunk(st[0]);
    float* d = dst + (long long)b * dst_img_stride;
    float* dd = DS ? ds + (long long)b * ds_img_stride : nullptr;
    const int hp = lane >> 4, hc = (lane & 15) * 4;    // H pass: rows 2hp, 2hp+1; columns hc..hc+3
    const int vq = lane >> 5, vc = (lane & 31) * 2;    // V pass: rows 4vq..4vq+3; columns vc, vc+1
    const int x = x0 + vc;
    const bool active = x0 < W;                      // uniform
    const bool full_cols = x0 + GT <= W;             // uniform: every lane's columns exist
    const f2v* h_rd = s_in + hp * IN_S + hc + OFF + SH;
    float* h_wr = s_h + 2 * hp * HS + hc;
    const float* v_rd = s_h + 4 * vq * HS + vc;              // rows before the wrap
    const float* v_rd_amb = v_rd - (vq ? RS * HS : 0);       // rows where only vq = 1 wrapped
    const uint32_t st_off = (uint32_t)(4 * vq * W + x);      // lane offset of the V-pass stores
    const uint32_t ds_off = (uint32_t)(2 * vq * dsw + (x >> 1));
    // step c (ring slot K = c mod 4): H pass of input chunk c, V pass of output chunk c - LAG,
    // loads of chunk c + NST into `nxt`, chunk c + 1 (`cur`) into the row-pair buffer
    auto step = [&](int c, auto KC, Elem (&cur)[2], Elem (&nxt)[2]) __attribute__((always_inline)) {
        constexpr int K = decltype(KC)::value;
        {   // H pass -> ring rows 8K .. 8K+7
            f2v a[4] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};   // columns hc+i
#pragma unroll
            for (int q = 0; q < NRD; q++) {
                const float4 v = reinterpret_cast<const float4*>(h_rd)[q];
                const f2v e[2] = {f2v{v.x, v.y}, f2v{v.z, v.w}};
#pragma unroll
                for (int u = 0; u < 2; u++) {
                    const int m = 2 * q + u;
#pragma unroll
                    for (int i = 0; i < 4; i++)
                        if (m - i >= 0 && m - i < FW) a[i] = pk_fma(e[u], tap<FW>(taps, m - i), a[i]);
                }
            }
            *reinterpret_cast<float4*>(h_wr + WCH * K * HS) = make_float4(a[0].x, a[1].x, a[2].x, a[3].x);
            *reinterpret_cast<float4*>(h_wr + (WCH * K + 1) * HS) = make_float4(a[0].y, a[1].y, a[2].y, a[3].y);
        }
        asm volatile("" ::: "memory");
        const int kout = c - LAG;
        if (active && kout >= 0 && kout < nchunk_out) {   // V pass of output chunk kout (uniform)
            constexpr int KV = ((K - LAG) % NSLOT + NSLOT) % NSLOT;   // its ring slot
            f2v acc[4] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};   // rows t0+j
#pragma unroll
            for (int m = 0; m < FW + 3; m++) {
                const int rc = WCH * KV + m;                 // ring row of half-wave 0
                const float* p = rc < RS - 4 ? v_rd + rc * HS
                               : rc >= RS ? v_rd + (rc - RS) * HS : v_rd_amb + rc * HS;
                const f2v v = *reinterpret_cast<const f2v*>(p);
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (m - j >= 0 && m - j < FW) acc[j] = pk_fma(v, tap<FW>(taps, m - j), acc[j]);
            }
#pragma unroll
            for (int j = 0; j < 4; j++) asm volatile("" : "+v"(acc[j]));
            const int yu = yb + WCH * kout;                  // first row of the chunk (uniform)
            if (full_cols && yu + WCH <= ye && (!DS || (yu + WCH) / 2 <= dsh)) {
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    float* row = d + (long long)(yu + j) * W;             // uniform
                    *reinterpret_cast<f2v*>(row + st_off) = acc[j];
                    if (DS && !(j & 1)) {
                        // DownsampleKernel<1> (ProgramCU.cu:287-298): dst(r, c) = src(2r, min(2c, W-1))
                        float* drow = dd + (long long)((yu + j) >> 1) * dsw;   // uniform
                        if ((x >> 1) < dsw) drow[ds_off] = acc[j].x;
                        if (x + 1 == W - 1)
                            for (int cc = W >> 1; cc < dsw; cc++) drow[2 * vq * dsw + cc] = acc[j].y;
                    }
                }
            } else if (x < W) {
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int y = yu + 4 * vq + j;
                    if (y < ye) {
                        *reinterpret_cast<f2v*>(&d[(long long)y * W + x]) = acc[j];
                        if (DS && !(y & 1) && (y >> 1) < dsh) {
                            float* drow = dd + (long long)(y >> 1) * dsw;
                            if ((x >> 1) < dsw) drow[x >> 1] = acc[j].x;
                            if (x + 1 == W - 1)
                                for (int cc = W >> 1; cc < dsw; cc++) drow[cc] = acc[j].y;
                        }
                    }
                }
            }
        }
        asm volatile("" ::: "memory");
        load_chunk(nxt, c + NST);
        store_chunk(cur);
        asm volatile("" ::: "memory");
    };
    const int nsteps = nchunk_out + LAG;
    // slot K = c mod NSLOT, register set c mod NST (steps past the end filter clamped rows and
    // store nothing): the loop is unrolled by lcm(NSLOT, NST) steps
    constexpr int U = std::lcm(NSLOT, NST);
    for (int c = 0; c < nsteps; c += U) {
        unrolled_steps(std::make_integer_sequence<int, U>{}, [&](auto KI) __attribute__((always_inline)) {
            constexpr int k = decltype(KI)::value;
            step(c + k, std::integral_constant<int, k % NSLOT>{}, st[(k + 1) % NST], st[k % NST]);
        });
    }
}

// the level kernels' workgroup order: xcd_block (1, shipped) or xcd_group<SGK_GW_XCDG> (2)
#ifndef SGK_GW_XCD
#define SGK_GW_XCD 1
#endif
#ifndef SGK_GW_XCDG
#define SGK_GW_XCDG 4
#endif
__device__ __forceinline__ int gw_order(int bid, int nb) {
    return SGK_GW_XCD == 2 ? xcd_group<SGK_GW_XCDG>(bid, nb) : xcd_block(bid, nb);
}

template <int FW, bool U8, bool DS>
__global__ __launch_bounds__(64 * kGwWaves) void k_gauss_lean(const GaussJob J) {
    using G = LeanGeom<FW>;
    if (J.zero.n[0] | J.zero.n[1] | J.zero.n[2]) zero_job(J.zero);
    __shared__ __attribute__((aligned(16))) f2v s_in_all[kGwWaves][G::IN_WORDS];
    __shared__ __attribute__((aligned(16))) float s_h_all[kGwWaves][G::RING_WORDS];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // XCD-aware order (xcd_block)
    const int gw = gw_order(blockIdx.x, gridDim.x) * kGwWaves + wave;
    gauss_lean_wave<FW, U8, DS>(J, gw, s_in_all[wave], s_h_all[wave]);
}

// Two independent level jobs in one launch ("diagonal": octave o + 1's level k beside octave o's
// level k + kds): blocks [0, nbB) run job B (the small one, dispatched first),
// blocks [nbB, nbB + nbA) job A; nbB is a multiple of 8, so each job keeps the XCD-aware order.
// The LDS buffers are sized for the larger geometry; f32 levels without decimation only.
template <int FWA, int FWB>
__global__ __launch_bounds__(64 * kGwWaves) void k_gauss_diag(const GaussJob A, const GaussJob B,
                                                              int nbB) {
    using GA = LeanGeom<FWA>;
    using GB = LeanGeom<FWB>;
    constexpr int IW = GA::IN_WORDS > GB::IN_WORDS ? GA::IN_WORDS : GB::IN_WORDS;
    constexpr int RW = GA::RING_WORDS > GB::RING_WORDS ? GA::RING_WORDS : GB::RING_WORDS;
    __shared__ __attribute__((aligned(16))) f2v s_in_all[kGwWaves][IW];
    __shared__ __attribute__((aligned(16))) float s_h_all[kGwWaves][RW];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int bid = blockIdx.x;
    if (bid < nbB) {
        gauss_lean_wave<FWB, false, false>(B, gw_order(bid, nbB) * kGwWaves + wave,
                                           s_in_all[wave], s_h_all[wave]);
    } else {
        const int nbA = (int)gridDim.x - nbB;
        gauss_lean_wave<FWA, false, false>(A, gw_order(bid - nbB, nbA) * kGwWaves + wave,
                                           s_in_all[wave], s_h_all[wave]);
    }
}

template <int FW>
hipError_t gauss_dispatch(const float* src, const uint8_t* src8, int src_stride,
                          long long src_img_stride, float* dst, long long dst_img_stride, int w,
                          int h, const Taps& taps, int batch, float* ds, int dsw, int dsh,
                          long long ds_img_stride, hipStream_t stream, int wave_rows,
                          bool long_bands, const ZeroJob& zero) {
    const bool vec = (src_stride % 4) == 0 && (src_img_stride % 4) == 0 && (w % 4) == 0 &&
                     w >= 4 && ((uintptr_t)(src8 ? (const void*)src8 : (const void*)src) % 16) == 0;
    if (vec && wave_rows >= 0) {
        const GaussWaveGrid gg = gauss_wave_grid(w, h, batch, wave_rows, 1, long_bands);
        const dim3 wgrid((unsigned)((gg.total_waves + kGwWaves - 1) / kGwWaves));
        const GaussJob J{src, src8, src_stride, src_img_stride, dst, dst_img_stride, w, h, taps,
                         ds, dsw, dsh, ds_img_stride, gg, zero};
#define SGK_LEAN(U8, DS)                                                                      \
        hipLaunchKernelGGL((k_gauss_lean<FW, U8, DS>), wgrid, dim3(64 * kGwWaves), 0, stream, J)
        if (src8) {
            if (ds) SGK_LEAN(true, true); else SGK_LEAN(true, false);
        } else {
            if (ds) SGK_LEAN(false, true); else SGK_LEAN(false, false);
        }
#undef SGK_LEAN
        return hipGetLastError();
    }
    if (zero.n[0] | zero.n[1] | zero.n[2]) {   // the block kernel does not zero: its own launch
        const hipError_t ez = launch_zero(zero.p[0], zero.n[0], zero.p[1], zero.n[1], zero.p[2],
                                          zero.n[2], stream);
        if (ez != hipSuccess) return ez;
    }
    // bands of at most 17 chunks (544 rows), and at least 1024 workgroups when the image is
    // short (kernel traces: 2 bands of 540 rows beat 1 band of 1080 on 1080p, and 1 band beats 2
    // on the 540- and 270-row octaves)
    const int strips_x = (w + GT - 1) / GT;
    const long long per_col = (long long)strips_x * batch;
    int nsy = (h + 17 * SR2 - 1) / (17 * SR2);
    const int need = (int)std::min<long long>((1024 + per_col - 1) / per_col, (h + SR2 - 1) / SR2);
    nsy = std::max(std::max(nsy, need), 1);
    int rows = (h + nsy - 1) / nsy;
    rows = (rows + SR2 - 1) / SR2 * SR2;
    nsy = (h + rows - 1) / rows;
    const dim3 grid((unsigned)(strips_x * nsy * batch));
    // aligned quads need 4-element row strides and image strides, a 16-B aligned base and a
    // width that is a multiple of 4 (always true for pyramid levels)
#define SGK_PK2(U8, VEC)                                                                   \
    hipLaunchKernelGGL((k_gauss_pk2<FW, U8, VEC>), grid, dim3(256), 0, stream, src, src8,    \
                       src_stride, src_img_stride, dst, dst_img_stride, w, h, taps, ds, dsw,  \
                       dsh, ds_img_stride, rows)
    if (src8) {
        if (vec) SGK_PK2(true, true); else SGK_PK2(true, false);
    } else {
        if (vec) SGK_PK2(false, true); else SGK_PK2(false, false);
    }
#undef SGK_PK2
    return hipGetLastError();
}

// (ComputeKEY_Kernel's state machine key_test, the keypoint locate() / key_at(): sift_keys.h,
// shared with the test-hook library's candidate dump)

// ------------------------------------------------------------------------------------------
// Extremum detection, wave-streaming form.  Each WAVE owns a strip segment of one image/octave
// and walks it row by row on its own -- no workgroup barriers, so every wave keeps its loads in
// flight independently (a workgroup-synchronised tile walk reached ~3.9 TB/s, the same read
// pattern without barriers ~5.9 TB/s, tests/microbench).
//   * the d+3 Gaussian planes' rows are loaded into registers two rows ahead, turned into the
//     d+2 DoG rows (D_m = G_m - G_{m-1}) and written to a wave-private 4-row LDS ring;
//   * the 3-wide row max/min of each DoG row is computed once and kept in registers for the
//     three output rows it borders; a branch-free 3x3x3 max/min pre-filter selects candidates,
//     which are compacted per wave (ballot + mbcnt) and given the exact ComputeKEY test
//     (key_test) from the ring;
//   * accepted pixels set their bit in the zeroed mask (atomicOr) and count in their row.
struct ExtremaWaveGrid {
    int wave0[kMaxOctaves + 1];        // first global wave of octave o
    int seg_rows[kMaxOctaves];         // rows per strip segment
    int nseg[kMaxOctaves];             // segments per strip column
};

// Layout of the loop (k_extrema_wave2):
//   * A wave covers 62 output columns with 64 lanes: lane l holds column x0 - 1 + l, lanes 0
//     and 63 only feed their neighbours, so no lane issues a separate halo load (halo loads
//     behind a lane branch made the compiler's wait counting assume they were missing and wait
//     for every load in flight).
//   * Two register row sets alternate (the loop is unrolled by two and both halves always run;
//     the second half of the last pair tests no pixel).
//   * The octave's fields are read as scalars before the loop: read inside the candidate branch
//     they were vector loads whose vmcnt(0) waited for the rows in flight.
// Round 2: 1.94 -> 1.72 ms per 128 x 1080p against the one-row form.
#ifndef SGK_EXT2_WAVES
#define SGK_EXT2_WAVES 1
#endif
#ifndef SGK_EXT_XCD
#define SGK_EXT_XCD 2   // workgroup order: 0 launch order, 1 xcd_block, 2 xcd_group<SGK_EXT_XCDG>
#endif
// CPL = columns per lane.  CPL = 2: lane l holds the column pair x0 - 1 + 2l, x0 + 2l (one 8-byte
// load per plane and row instead of two 4-byte ones: the texture-address unit, ~88 % busy with
// 4-byte loads, handles a load per lane whatever its width), 126 tested columns per wave;
// x0 = 126 sx + 1 keeps the pairs 8-byte aligned.
template <int ND, int CPL>   // ND = number of DoG planes = d + 2
__global__ __launch_bounds__(256, SGK_EXT2_WAVES) void k_extrema_wave2(const float* __restrict__ pyr,
                                                       uint32_t* __restrict__ mask,
                                                       uint32_t* __restrict__ row_count,
                                                       const FeatureParams fp,
                                                       const ExtremaWaveGrid eg) {
    static_assert(CPL == 1 || CPL == 2, "one or two columns per lane");
    constexpr int TW = 64 * CPL - 2;                // tested columns per wave
    constexpr int RW = 64 * CPL + 2 * CPL + 2;      // ring row: column index i at i + CPL (+pad)
    constexpr int NJ = ND - 2;
    __shared__ __attribute__((aligned(8))) float s_ring[4][ND][4][RW];   // [wave][plane][row & 3][col]
    __shared__ uint16_t s_list[4][NJ * 64 * CPL];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // Workgroup order.  Two neighbouring 128-column windows (126 columns apart, not line-aligned)
    // share a cache line of every row; the 4 waves of a workgroup are 4 neighbouring strips, so
    // the lines at workgroup boundaries were fetched twice whenever the neighbour ran on another
    // XCD (another L2).  SGK_EXT_XCD = 2 (shipped): xcd_group<4>, 4 consecutive workgroups -- an
    // octave-0 segment row of 16 strips -- on one XCD, dispatched together: detect 1.55-1.56 vs
    // 1.60-1.63 ms (alternating processes, tests/diag/r04l.sh; groups of 2 / 8 / 16 workgroups:
    // 1.59 / 1.56 / 1.58).  SGK_EXT_XCD = 1, xcd_block's partition of the grid into 8 contiguous
    // ranges, measured 1.90 vs 1.67 ms: the ranges hold different octaves, whose waves differ in
    // work, so XCDs went idle.
#ifndef SGK_EXT_XCDG
#define SGK_EXT_XCDG 4
#endif
    const int gw = (SGK_EXT_XCD == 1 ? xcd_block(blockIdx.x, gridDim.x)
                    : SGK_EXT_XCD == 2 ? xcd_group<SGK_EXT_XCDG>(blockIdx.x, gridDim.x)
                                       : (int)blockIdx.x) * 4 + wave;
    if (gw >= eg.wave0[fp.n_octaves]) return;       // uniform per wave
    int o = 0;
    while (o + 1 < fp.n_octaves && gw >= eg.wave0[o + 1]) o++;
    // o is wave-uniform: said so, the octave's fields are scalar loads (lgkmcnt) instead of
    // vector loads from the argument block inside the candidate branch, whose vmcnt(0) would
    // wait for the rows in flight
    o = __builtin_amdgcn_readfirstlane(o);
    const OctaveDesc& od = fp.oct[o];
    const long long mask_off = od.mask_off, mask_lstride = od.mask_level_stride;
    const int nwords = od.nwords;
    const long long rc_base = fp.row_off[o];
    const int W = od.wa, H = od.h;
    const int strips_x = (W + TW - 1) / TW;
    const int id = gw - eg.wave0[o];
    const int sx = id % strips_x, rest = id / strips_x;
    const int sg = rest % eg.nseg[o], b = rest / eg.nseg[o];
    const int x0 = sx * TW + (CPL - 1);
    const int ys = sg * eg.seg_rows[o], ye = min(H, ys + eg.seg_rows[o]);
    const long long lstride = od.level_stride;
    const float* g0 = pyr + od.gauss_off + (long long)b * W * H;
    float(*ring)[4][RW] = s_ring[wave];
    uint16_t* list = s_list[wave];

    // this lane's columns x0 - 1 + CPL * lane + k; CPL = 2 loads the pair from column gx
    // (even; clamped to W - 2, W is even)
    const int xl = x0 - 1 + CPL * lane;
    const int gx = CPL == 1 ? clampi(xl, 0, W - 1) : min(xl, W - 2);
    bool out_col[CPL];
#pragma unroll
    for (int k = 0; k < CPL; k++) {
        const int i = CPL * lane + k, x = xl + k;
        out_col[k] = i >= 1 && i <= TW && x > 0 && x < W - 1;
    }
    struct Row { float m[ND + 1][CPL]; };
    Row rA, rB;
    auto fetch = [&](Row& r, int y) {   // G row y (clamped) into registers
        const float* q = g0 + (long long)clampi(y, 0, H - 1) * W + gx;
#pragma unroll
        for (int m = 0; m <= ND; m++) {
            if constexpr (CPL == 1) {
                r.m[m][0] = q[m * lstride];
            } else {
                const float2 v = *reinterpret_cast<const float2*>(q + m * lstride);
                r.m[m][0] = v.x;
                r.m[m][1] = v.y;
            }
        }
    };
    // Lanes exchange values through the wave-private ring and list.  LDS accesses of one wave
    // complete in issue order, but the compiler sees only per-lane addresses (a lane writes
    // its columns and reads its neighbours') and may reorder them: the empty asm statements keep
    // every write before the reads that follow it.
    // DoG row y into the ring (read by key_test for the rare candidates) and into dog[] (the
    // row max/min below take the neighbours' values by DPP wave shifts, not from LDS)
    float dog[ND][CPL];
    auto put = [&](const Row& r, int y) {
        float* rr = &ring[0][y & 3][CPL * lane + CPL];
#pragma unroll
        for (int m = 0; m < ND; m++) {
#pragma unroll
            for (int k = 0; k < CPL; k++) dog[m][k] = r.m[m + 1][k] - r.m[m][k];
            if constexpr (CPL == 1)
                rr[m * 4 * RW] = dog[m][0];
            else
                *reinterpret_cast<float2*>(&rr[m * 4 * RW]) = make_float2(dog[m][0], dog[m][1]);
        }
        asm volatile("" ::: "memory");
    };
    // rolling 3-wide row max/min of DoG rows y-1 and y (per plane), refreshed per step; the
    // wave's first and last columns get a neighbour from outside the wave (0) and are never
    // tested
    float hx0[ND][CPL], hn0[ND][CPL], hx1[ND][CPL], hn1[ND][CPL], cvx[ND][CPL];
    auto rowmm = [&](float (*mx)[CPL], float (*mn)[CPL], float (*cv)[CPL]) {   // of dog[]
#pragma unroll
        for (int m = 0; m < ND; m++) {
            float v[CPL + 2];   // columns left of, in and right of this lane's
#pragma unroll
            for (int k = 0; k < CPL; k++) v[k + 1] = dog[m][k];
            v[0] = __int_as_float(__builtin_amdgcn_update_dpp(
                0, __float_as_int(dog[m][CPL - 1]), 0x138, 0xf, 0xf, false));   // wave_shr:1
            v[CPL + 1] = __int_as_float(__builtin_amdgcn_update_dpp(
                0, __float_as_int(dog[m][0]), 0x130, 0xf, 0xf, false));         // wave_shl:1
#pragma unroll
            for (int k = 0; k < CPL; k++) {
                mx[m][k] = fmax_(fmax_(v[k], v[k + 1]), v[k + 2]);
                mn[m][k] = fmin_(fmin_(v[k], v[k + 1]), v[k + 2]);
                if (cv) cv[m][k] = v[k + 1];
            }
        }
    };
    auto body = [&](int y) {   // test row y: DoG rows y-1, y are rolled, y+1 is in dog[]
        float hx2[ND][CPL], hn2[ND][CPL], cnx[ND][CPL];
        rowmm(hx2, hn2, cnx);
        const bool row_ok = y < ye && y > 0 && y < H - 1;
        int ncand = 0;
#pragma unroll
        for (int j = 0; j < NJ; j++) {
#pragma unroll
            for (int k = 0; k < CPL; k++) {
                const float v = cvx[j + 1][k];
                float mx = hx0[j][k], mn = hn0[j][k];
#pragma unroll
                for (int m = j; m < j + 3; m++) {
                    mx = fmax_(mx, fmax_(fmax_(hx0[m][k], hx1[m][k]), hx2[m][k]));
                    mn = fmin_(mn, fmin_(fmin_(hn0[m][k], hn1[m][k]), hn2[m][k]));
                }
                const bool cand = row_ok && out_col[k] && fabs_(v) > fp.t0 && (v >= mx || v <= mn);
                const unsigned long long bal = __ballot(cand);
                if (cand) {
                    const int pos = ncand + __builtin_amdgcn_mbcnt_hi(
                                                (uint32_t)(bal >> 32),
                                                __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
                    list[pos] = (uint16_t)((j << 7) | (CPL * lane + k));
                }
                ncand += __popcll(bal);
            }
        }
        asm volatile("" ::: "memory");
        for (int c0 = 0; c0 < ncand; c0 += 64) {
            if (c0 + lane < ncand) {
                const int code = list[c0 + lane];
                const int j = code >> 7, cl = code & 127;
                auto get = [&](int m, int r, int c) {
                    return ring[j + m][(y + r - 1) & 3][cl + c - 1 + CPL];
                };
                if (key_test(get, fp.t0, fp.t, fp.edge, fp.subpixel).result != 0.f) {
                    const int xx = x0 - 1 + cl;
                    uint32_t* mrow = mask + mask_off + j * mask_lstride +
                                     ((long long)b * H + y) * nwords;
                    atomicOr(&mrow[xx >> 5], 1u << (xx & 31));
                    atomicAdd(&row_count[(long long)b * fp.rows_per_image + rc_base + j * H + y],
                              1u);
                }
            }
        }
#pragma unroll
        for (int m = 0; m < ND; m++)
#pragma unroll
            for (int k = 0; k < CPL; k++) {
                hx0[m][k] = hx1[m][k]; hn0[m][k] = hn1[m][k];
                hx1[m][k] = hx2[m][k]; hn1[m][k] = hn2[m][k];
                cvx[m][k] = cnx[m][k];
            }
        asm volatile("" ::: "memory");   // this row's list and ring reads before the next writes
    };
    fetch(rA, ys - 1);
    put(rA, ys - 1);
    rowmm(hx0, hn0, nullptr);
    fetch(rA, ys);
    put(rA, ys);
    rowmm(hx1, hn1, cvx);
    // rows past ye (the row below the segment's last tested row) feed no test: they are
    // fetched clamped to ye, a row already read (cache hit, no HBM bytes).  Round 3 read 2 more
    // rows per segment from HBM (1.19x the algorithmic bytes with 17-row segments).
    fetch(rA, min(ys + 1, ye));
    fetch(rB, min(ys + 2, ye));
    // each set is refetched after the row test that follows its put: the test's atomics (a
    // data-dependent number of them) then come before, not after, the loads that the next wait
    // must leave in flight
    for (int y = ys; y < ye; y += 2) {
        put(rA, y + 1);
        body(y);
        fetch(rA, min(y + 3, ye));
        put(rB, y + 2);
        body(y + 1);
        fetch(rB, min(y + 4, ye));
    }
}

// ------------------------------------------------------------------------------------------
// Extremum detection in 2-D tiles, for cache-resident pyramids (one image: C2).  The wave kernel's
// walk of a strip segment is a chain of row loads; a single 1080p image gives it ~2,700 waves
// that each wait for ~5 dependent row fetches (29 us, profiles/r06a).  Here a workgroup owns 64
// tested columns x 16 rows of one octave and image for all d levels: it issues the loads of the
// d + 3 Gaussian planes' window (18 rows x 72 columns, aligned quads) at once, stores the d + 2
// DoG planes D_m = G_{m+1} - G_m into LDS, and each wave tests 4 rows (a lane per column): the
// same branch-free 3x3x3 pre-filter superset as k_extrema_wave2, then ComputeKEY's exact state
// machine (key_test) on the LDS values for every candidate.  The tested pixels (1 .. W-2 x
// 1 .. H-2 per octave), the mask bits and the row counts are the wave kernel's; only the order of
// the commutative atomics differs.
struct ExtremaTileGrid {
    int tile0[kMaxOctaves + 1];   // first workgroup of octave o
    int tx[kMaxOctaves];          // tiles per row of octave o
    int ty[kMaxOctaves];          // tiles per column
};
constexpr int kEtW = 64, kEtH = 16, kEtLW = 72;   // tile columns / rows, LDS row (18 quads)

template <int ND>
__global__ __launch_bounds__(256) void k_extrema_tile(const float* __restrict__ pyr,
                                                      uint32_t* __restrict__ mask,
                                                      uint32_t* __restrict__ row_count,
                                                      const FeatureParams fp,
                                                      const ExtremaTileGrid eg) {
    constexpr int NJ = ND - 2, R = kEtH + 2, NQ = kEtLW / 4, NIT = R * NQ;
    constexpr int LITEMS = (NIT + 255) / 256;
    __shared__ __attribute__((aligned(16))) float s_d[ND][R][kEtLW];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int bid = blockIdx.x;
    int o = 0;
    while (o + 1 < fp.n_octaves && bid >= eg.tile0[o + 1]) o++;
    o = __builtin_amdgcn_readfirstlane(o);
    const OctaveDesc& od = fp.oct[o];
    const int W = od.wa, H = od.h;
    const int id = bid - eg.tile0[o];
    const int sx = id % eg.tx[o], rest = id / eg.tx[o];
    const int sy = rest % eg.ty[o], b = rest / eg.ty[o];
    const int x0 = sx * kEtW, y0 = sy * kEtH;
    const long long lstride = od.level_stride;
    const float* g0 = pyr + od.gauss_off + (long long)b * W * H;
    // the window: rows y0 - 1 .. y0 + 16 (clamped), columns x0 - 4 .. x0 + 67 as aligned quads
    // (clamped: the tested columns' neighbours x0 - 1 .. x0 + 64 are inside the plane wherever a
    // tested column exists)
    float4 gq[LITEMS][ND + 1];
#pragma unroll
    for (int i = 0; i < LITEMS; i++) {
        const int it = min(tid + 256 * i, NIT - 1);
        const int rr = it / NQ, q = it - rr * NQ;
        const int y = clampi(y0 - 1 + rr, 0, H - 1);
        const int xq = clampi(x0 - 4 + 4 * q, 0, W - 4);
        const float* p = g0 + (long long)y * W + xq;
#pragma unroll
        for (int m = 0; m <= ND; m++) gq[i][m] = *reinterpret_cast<const float4*>(p + m * lstride);
    }
#pragma unroll
    for (int i = 0; i < LITEMS; i++) {
        const int it = tid + 256 * i;
        if (NIT % 256 != 0 && it >= NIT) break;
        const int rr = it / NQ, q = it - rr * NQ;
#pragma unroll
        for (int m = 0; m < ND; m++) {
            const float4 a = gq[i][m], c = gq[i][m + 1];
            *reinterpret_cast<float4*>(&s_d[m][rr][4 * q]) =
                make_float4(c.x - a.x, c.y - a.y, c.z - a.z, c.w - a.w);
        }
    }
    __syncthreads();
    // wave w: tile rows 4 w .. 4 w + 3 (LDS rows 4 w + 1 .. 4 w + 4), lane = column x0 + lane
    // (LDS column lane + 4)
    const int x = x0 + lane;
    const bool col_ok = x > 0 && x < W - 1;
    const int lc = lane + 4;
    float hx[ND][6], hn[ND][6];   // 3-wide row max / min of LDS rows 4 w .. 4 w + 5
#pragma unroll
    for (int m = 0; m < ND; m++)
#pragma unroll
        for (int r = 0; r < 6; r++) {
            const float* row = &s_d[m][4 * wave + r][lc];
            const float a = row[-1], c = row[0], e = row[1];
            hx[m][r] = fmax_(fmax_(a, c), e);
            hn[m][r] = fmin_(fmin_(a, c), e);
        }
    uint32_t pend = 0;   // bit i * NJ + j: row i, level j passed the pre-filter
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int y = y0 + 4 * wave + i;
        const bool row_ok = y > 0 && y < H - 1;
#pragma unroll
        for (int j = 0; j < NJ; j++) {
            const float v = s_d[j + 1][4 * wave + 1 + i][lc];
            float mx = hx[j][i], mn = hn[j][i];
#pragma unroll
            for (int m = j; m < j + 3; m++) {
                mx = fmax_(mx, fmax_(fmax_(hx[m][i], hx[m][i + 1]), hx[m][i + 2]));
                mn = fmin_(mn, fmin_(fmin_(hn[m][i], hn[m][i + 1]), hn[m][i + 2]));
            }
            if (row_ok && col_ok && fabs_(v) > fp.t0 && (v >= mx || v <= mn)) pend |= 1u << (i * NJ + j);
        }
    }
    // every lane works through its candidates one per iteration (the wave loops while any lane
    // has one left): ComputeKEY on the LDS values, accepted pixels set their mask bit and count
    while (__ballot(pend != 0)) {
        if (pend) {
            const int bit = __ffs(pend) - 1;
            pend &= pend - 1;
            const int i = bit / NJ, j = bit - i * NJ;
            const int lr = 4 * wave + 1 + i;
            auto get = [&](int m, int r, int c) { return s_d[j + m][lr + r - 1][lc + c - 1]; };
            if (key_test(get, fp.t0, fp.t, fp.edge, fp.subpixel).result != 0.f) {
                const int y = y0 + 4 * wave + i;
                uint32_t* mrow = mask + od.mask_off + j * od.mask_level_stride +
                                 ((long long)b * H + y) * od.nwords;
                atomicOr(&mrow[x >> 5], 1u << (x & 31));
                atomicAdd(&row_count[(long long)b * fp.rows_per_image + fp.row_off[o] + j * H + y], 1u);
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// Exclusive scan (uint32), 1024 elements per block.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

__global__ __launch_bounds__(256) void k_scan_block(const uint32_t* __restrict__ in,
                                                    uint32_t* __restrict__ out, size_t n,
                                                    uint32_t* __restrict__ block_sums) {
    __shared__ uint32_t s_w[4];
    const size_t base = (size_t)blockIdx.x * 1024 + threadIdx.x * 4;
    uint32_t v[4];
#pragma unroll
    for (int i = 0; i < 4; i++) v[i] = (base + i < n) ? in[base + i] : 0u;
    uint32_t tsum = v[0] + v[1] + v[2] + v[3];
    uint32_t incl = wave_incl_scan(tsum);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    uint32_t wofs = 0, total = 0;
    for (int w = 0; w < 4; w++) {
        if (w < wave) wofs += s_w[w];
        total += s_w[w];
    }
    uint32_t run = wofs + incl - tsum;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        if (base + i < n) out[base + i] = run;
        run += v[i];
    }
    if (threadIdx.x == 0) {
        if (block_sums) block_sums[blockIdx.x] = total;
        else out[n] = total;   // single-block scan writes the total itself
    }
}

// Exclusive scan of a short array (a single image's rows or candidates: C2) by one workgroup
// in tiles of 4096, the running total carried across tiles: one launch instead of the three of
// the block scan (each a few microseconds of launch latency at these sizes).
__global__ __launch_bounds__(1024) void k_scan_single(const uint32_t* __restrict__ in,
                                                      uint32_t* __restrict__ out, size_t n) {
    // one pass: thread t owns the contiguous run [t c, t c + c), c = ceil(n / 1024) <= 32, loaded
    // at once (one round trip; round 5 walked 4,096-element tiles one after the other: a single
    // image's two scans took 6-7 us each)
    __shared__ uint32_t s_w[16];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const size_t c = (n + 1023) / 1024;
    const size_t base = (size_t)threadIdx.x * c;
    uint32_t v[32];
    uint32_t tsum = 0;
#pragma unroll
    for (int i = 0; i < 32; i++) {
        v[i] = ((size_t)i < c && base + i < n) ? in[base + i] : 0u;
        tsum += v[i];
    }
    const uint32_t incl = wave_incl_scan(tsum);
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    uint32_t wofs = 0, total = 0;
#pragma unroll
    for (int w = 0; w < 16; w++) {
        const uint32_t sw = s_w[w];
        wofs += w < wave ? sw : 0u;
        total += sw;
    }
    uint32_t run = wofs + incl - tsum;
#pragma unroll
    for (int i = 0; i < 32; i++) {
        if ((size_t)i < c && base + i < n) out[base + i] = run;
        run += v[i];
    }
    if (threadIdx.x == 0) out[n] = total;
}

__global__ __launch_bounds__(256) void k_scan_add(uint32_t* __restrict__ out, size_t n,
                                                  const uint32_t* __restrict__ block_ofs) {
    const size_t base = (size_t)blockIdx.x * 1024 + threadIdx.x * 4;
    const uint32_t add = block_ofs[blockIdx.x];
#pragma unroll
    for (int i = 0; i < 4; i++)
        if (base + i < n) out[base + i] += add;
    if (blockIdx.x == 0 && threadIdx.x == 0) out[n] = block_ofs[gridDim.x];
}

// ------------------------------------------------------------------------------------------
// Gradient of a Gaussian level at an interior pixel, as ComputeDOG_Kernel stores it
// (ProgramCU.cu:495-502): (0.5 |grad|, atan2(dy, dx)), atan2 skipped when the magnitude is 0.
__device__ __forceinline__ float2 grad_at(const float* __restrict__ g, int W, int x, int y) {
    const float* p = g + (long long)y * W + x;
    const float dx = p[1] - p[-1];
    const float dy = p[W] - p[-W];
    const float grd = 0.5f * sqrt_(fma_(dx, dx, dy * dy));
    const float rot = grd == 0.0f ? 0.0f : atan2_(dy, dx);
    return make_float2(grd, rot);
}


// ------------------------------------------------------------------------------------------
// Quad (4-lane) broadcast of lane S through DPP quad_perm [S,S,S,S]: no LDS traffic.
template <int S>
__device__ __forceinline__ int qbcast(int v) {
    return __builtin_amdgcn_mov_dpp(v, S * 0x55, 0xF, 0xF, false);
}
template <int S>
__device__ __forceinline__ float qbcastf(float v) {
    return as_float((uint32_t)qbcast<S>((int)as_uint(v)));
}

// Row-major walk of a window of ncols columns, advanced 4 samples at a time (one per quad lane).
struct Walk {
    int r, c;
    __device__ __forceinline__ void init(int i, int ncols) { r = i / ncols; c = i - r * ncols; }
    __device__ __forceinline__ void step(int ncols) {
        c += 4;
        while (c >= ncols) { c -= ncols; r++; }
    }
};

// ComputeOrientation_Kernel (ProgramCU.cu:813-977).  One quad (4 lanes) per keypoint: the
// lanes evaluate consecutive window samples (gradient, Gaussian weight, bin) in parallel and
// every lane then applies the quad's 4 votes in the reference's (y, x) order to the keypoint's
// 36-bin histogram in LDS, so each bin sees exactly the reference's sequence of float adds.
// Orientation histogram of ComputeOrientation_Kernel (ProgramCU.cu:857-903) for a keypoint
// (kx, ky, kz) of Gaussian level g (W x H): the quad's 4 lanes evaluate consecutive window
// samples and every lane applies the 4 votes in the reference's (y, x) order to the 36-bin LDS
// histogram; returns the 6-times smoothed histogram in vote[0..36] (vote[36] = vote[0]).
__device__ __forceinline__ void orientation_hist(const float* __restrict__ g, int W, int H,
                                                 float kx, float ky, float kz,
                                                 const FeatureParams& fp, int sub, float* vote_l,
                                                 float (&vote)[37]) {
    const float ten_degree_per_radius = (float)5.7295779513082320876798154814105;
    const float gsigma = kz * fp.gaussian_factor;
    const float win = fabs_(kz) * fp.sample_factor;
    const float dist_threshold = (float)((double)(win * win) + 0.5);
    const float factor = -0.5f / (gsigma * gsigma);
    const float xmin = fmax_(1.5f, floor_(kx - win) + 0.5f);
    const float ymin = fmax_(1.5f, floor_(ky - win) + 0.5f);
    const float xmax = fmin_(W - 1.5f, floor_(kx + win) + 0.5f);
    const float ymax = fmin_(H - 1.5f, floor_(ky + win) + 0.5f);
    for (int i = sub; i < 36; i += 4) vote_l[i] = 0.0f;
    const int ncols = xmax >= xmin ? (int)(xmax - xmin) + 1 : 0;
    const int nrows = ymax >= ymin ? (int)(ymax - ymin) + 1 : 0;
    const int total = ncols * nrows;
    // The 4 gradient neighbours of this lane's next sample are loaded one iteration ahead
    // (unconditionally: past the window's end a lane reads the window's first pixel), so a
    // sample's gathers overlap the previous sample's votes instead of starting after them.
    // Same values and the same arithmetic as grad_at.
    Walk wk;
    float nl = 0.f, nr = 0.f, nu = 0.f, nd = 0.f;
    const int x_safe = (int)xmin, y_safe = (int)ymin;
    auto fetch = [&](const Walk& w, bool ok) {
        const int x = ok ? (int)(xmin + (float)w.c) : x_safe;
        const int y = ok ? (int)(ymin + (float)w.r) : y_safe;
        const float* p = g + (long long)y * W + x;
        nl = p[-1];
        nr = p[1];
        nu = p[-W];
        nd = p[W];
    };
    if (total > 0) {
        wk.init(sub, ncols);
        fetch(wk, sub < total);
    }
    for (int base = 0; base < total; base += 4) {
        // this lane's sample: index base + sub
        const bool valid = base + sub < total;
        const float pl = nl, pr = nr, pu = nu, pd = nd;
        const float x = xmin + (float)wk.c, y = ymin + (float)wk.r;
        if (valid) wk.step(ncols);
        fetch(wk, base + 4 + sub < total);
        int bin = -1;
        float weight = 0.0f;
        if (valid) {
            const float dx = x - kx, dy = y - ky;
            const float sq = fma_(dx, dx, dy * dy);
            if (!(fp.circular && sq >= dist_threshold)) {
                const float gdx = pr - pl, gdy = pd - pu;   // grad_at (ProgramCU.cu:495-502)
                const float grd = 0.5f * sqrt_(fma_(gdx, gdx, gdy * gdy));
                const float rot = grd == 0.0f ? 0.0f : atan2_(gdy, gdx);
                weight = grd * exp_(sq * factor);
                bin = (int)floor_(rot * ten_degree_per_radius);
                if (bin < 0) bin += 36;
            }
        }
        // apply the 4 votes in sample order: lane 0 of the quad issues them as LDS float adds
        // (ds_add_f32, IEEE round-to-nearest like the VALU add), which the LDS performs in issue
        // order -- each bin sees the reference's sequence of adds, and no read-modify-write
        // round trip sits between one group of samples and the next
        const int b0 = qbcast<0>(bin), b1 = qbcast<1>(bin), b2 = qbcast<2>(bin), b3 = qbcast<3>(bin);
        const float w0 = qbcastf<0>(weight), w1 = qbcastf<1>(weight), w2 = qbcastf<2>(weight),
                    w3 = qbcastf<3>(weight);
        if (sub == 0) {
            auto add = [&](int bb, float ww) {
                __hip_atomic_fetch_add(&vote_l[bb], ww, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
            };
            if (b0 >= 0) add(b0, w0);
            if (b1 >= 0) add(b1, w1);
            if (b2 >= 0) add(b2, w2);
            if (b3 >= 0) add(b3, w3);
        }
    }
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < 36; ++i) vote[i] = vote_l[i];
    const float one_third = (float)(1.0 / 3.0);
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        vote[36] = vote[0];
        float pre = vote[35];
#pragma unroll
        for (int j = 0; j < 36; ++j) {
            const float temp = one_third * (pre + vote[j] + vote[j + 1]);
            pre = vote[j];
            vote[j] = temp;
        }
    }
    vote[36] = vote[0];
}

// The strongest orientation (ProgramCU.cu:904-919: num_orientation == 1 or a caller-supplied
// keypoint list), in radians of the reference's internal convention.
__device__ __forceinline__ float strongest_orientation(const float (&vote)[37]) {
    const float radius_per_ten_degrees = (float)(1.0 / 5.7295779513082320876798154814105);
    int index_max = 0;
    float max_vote = vote[0];
#pragma unroll
    for (int i = 1; i < 36; ++i) {
        index_max = vote[i] > max_vote ? i : index_max;
        max_vote = fmax_(max_vote, vote[i]);
    }
    float pre = vote[35], next = vote[1];
#pragma unroll
    for (int i = 1; i < 36; ++i)
        if (i == index_max) { pre = vote[i - 1]; next = vote[i + 1]; }
    const float off = 0.5f * ((next - pre) * (1.0f / (max_vote + max_vote - next - pre)));
    return radius_per_ten_degrees * (index_max + 0.5f + off);
}

// Keypoint of candidate f in octave coordinates (ComputeOrientation_Kernel's key, ProgramCU.cu:
// 838-851) and its info record; false when no orientation is computed (num_orientation == 0:
// the keypoint is written with orientation 0 here).
struct OriKey { float kx, ky, kz; const float* g; int W, H; };
// locate() by a whole wave (the one-wave-per-candidate orientation form): the same (image,
// octave, level, row, column) from 3 dependent loads instead of ~13 binary-search steps plus a
// serial scan over the mask row's words (up to 60 for a 1080p row) -- the latency chain of a
// single image's orientation launch.
//   * row: a 64-ary search for the last row whose scanned base is <= f -- the lanes probe 64
//     evenly spaced rows of the remaining range, the highest lane whose probe passes narrows it;
//   * column: lane l loads mask word l (64 at a time), a wave prefix sum of their popcounts picks
//     the word holding the k-th set bit, that lane finds the bit.
__device__ __forceinline__ KeyLoc locate_wave(uint32_t f, int lane, const uint32_t* __restrict__ row_base,
                                              int total_rows, const uint32_t* __restrict__ mask,
                                              const FeatureParams& fp) {
    int lo = 0, n = total_rows;   // the answer lies in [lo, lo + n); row_base[lo] <= f
    uint32_t base_lo = 0;         // row_base[lo] (row_base[0] = 0)
    while (n > 1) {
        const int step = (n + 63) / 64;
        const int i = lo + lane * step;
        const bool in = lane * step < n;
        const uint32_t v = in ? row_base[i] : 0xffffffffu;
        const unsigned long long bal = __ballot(in && v <= f);   // lane 0 always passes
        const int k = 63 - __clzll(bal);
        base_lo = (uint32_t)__builtin_amdgcn_readlane((int)v, k);
        const int end = lo + n;
        lo += k * step;
        n = min(step, end - lo);
    }
    KeyLoc L = row_loc(lo, fp);
    uint32_t k = f - base_lo;
    const OctaveDesc& od = fp.oct[L.o];
    const uint32_t* mrow = mask + od.mask_off + L.j * od.mask_level_stride +
                           ((long long)L.b * od.h + L.row) * od.nwords;
    int col = 0;
    for (int w0 = 0; w0 < od.nwords; w0 += 64) {
        const int w = w0 + lane;
        uint32_t m = w < od.nwords ? mrow[w] : 0u;
        const int c = __popc(m);
        int incl = c;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int u = __shfl_up(incl, d, 64);
            if (lane >= d) incl += u;
        }
        const int excl = incl - c;
        const unsigned long long hit = __ballot((uint32_t)excl <= k && k < (uint32_t)incl);
        if (hit) {
            const int hl = __ffsll((long long)hit) - 1;
            for (uint32_t q = 0; q < k - (uint32_t)excl && lane == hl; q++) m &= m - 1;
            col = __builtin_amdgcn_readlane(w * 32 + (__ffs(m) - 1), hl);
            break;
        }
        k -= (uint32_t)__builtin_amdgcn_readlane(incl, 63);
    }
    L.col = col;
    return L;
}

__device__ __forceinline__ bool orientation_key(uint32_t f, bool writer,
                                                const float* __restrict__ pyr,
                                                const uint32_t* __restrict__ mask,
                                                const uint32_t* __restrict__ row_base,
                                                int total_rows, const FeatureParams& fp,
                                                float4* __restrict__ out4,
                                                int2* __restrict__ info,
                                                uint32_t* __restrict__ ocount, OriKey& K,
                                                int wave_lane = -1) {
    // wave_lane >= 0: called by a whole wave for one candidate (locate_wave), else per lane
    const KeyLoc L = wave_lane >= 0 ? locate_wave(f, wave_lane, row_base, total_rows, mask, fp)
                                    : locate(f, row_base, total_rows, mask, fp);
    const KeyOut kv = key_at(pyr, fp, L);
    const OctaveDesc& od = fp.oct[L.o];

    float kx = L.col + 0.5f, ky = L.row + 0.5f, kz = fp.level_sigma[L.j];
    if (fp.subpixel) {
        kx += kv.dx;
        ky += kv.dy;
        kz *= pow_(fp.sigma_step, kv.ds);
    }
    if (fp.keep_sign) kz *= kv.result;
    if (writer) info[f] = make_int2(L.b, L.o * fp.d + L.j);
    if (fp.num_orientation == 0) {
        if (writer) {
            out4[f] = make_float4(kx, ky, kz, 0.0f);
            ocount[f] = 1;
        }
        return false;
    }
    // gradient of Gaussian level 1 + j (PyramidCU.cpp:1204)
    K.g = pyr + od.gauss_off + (long long)(1 + L.j) * od.level_stride + (long long)L.b * od.wa * od.h;
    K.W = od.wa;
    K.H = od.h;
    K.kx = kx;
    K.ky = ky;
    K.kz = kz;
    return true;
}

// Peaks of the smoothed histogram (ProgramCU.cu:904-977) -> the keypoint with its one or two
// orientations packed as u16 fractions of 2 pi, and the feature count it expands to
// (ReshapeFeatureListCPU, PyramidCU.cpp:560-578: drop "no orientation", keep a distinct second).
__device__ __forceinline__ void orientation_finish(uint32_t f, const float (&vote)[37],
                                                   const OriKey& K, const FeatureParams& fp,
                                                   float4* __restrict__ out4,
                                                   uint32_t* __restrict__ ocount) {
    if (fp.num_orientation == 1) {
        out4[f] = make_float4(K.kx, K.ky, K.kz, strongest_orientation(vote));
        ocount[f] = 1;
        return;
    }
    float max_vote = vote[0];
#pragma unroll
    for (int i = 1; i < 36; ++i) max_vote = fmax_(max_vote, vote[i]);
    const float vote_threshold = max_vote * 0.8f;
    float pre = vote[35];
    float rot0 = 0.f, rot1 = 0.f, vot0 = 0.f, vot1 = 0.f;
    int ocnt = 0;
#pragma unroll
    for (int i = 0; i < 36; ++i) {
        const float next = vote[i + 1];
        const float vi = vote[i];
        if (vi > vote_threshold && vi > pre && vi > next) {
            const float di = 0.5f * ((next - pre) * (1.0f / (vi + vi - next - pre)));
            const float rot = i + di + 0.5f;
            if (vi > vot1) {
                if (vi > vot0) { vot1 = vot0; rot1 = rot0; vot0 = vi; rot0 = rot; }
                else { vot1 = vi; rot1 = rot; }
                ocnt++;
            }
        }
        pre = vi;
    }
    float fr1 = rot0 / 36.0f;
    if (fr1 < 0) fr1 += 1.0f;
    const uint32_t us1 = ocnt == 0 ? 65535u : (uint32_t)(unsigned short)floor_(fr1 * 65535.0f);
    uint32_t us2 = 65535u;
    if (ocnt > 1) {
        float fr2 = rot1 / 36.0f;
        if (fr2 < 0) fr2 += 1.0f;
        us2 = (uint32_t)(unsigned short)floor_(fr2 * 65535.0f);
    }
    out4[f] = make_float4(K.kx, K.ky, K.kz, as_float((us2 << 16) | us1));
    ocount[f] = us1 == 65535u ? 0u : (1u + ((us2 != 65535u && us2 != us1) ? 1u : 0u));
}

__device__ __forceinline__ void orientation_one(uint32_t f, int sub, float* vote_l,
                                                const float* __restrict__ pyr,
                                                const uint32_t* __restrict__ mask,
                                                const uint32_t* __restrict__ row_base,
                                                int total_rows, const FeatureParams& fp,
                                                float4* __restrict__ out4,
                                                int2* __restrict__ info,
                                                uint32_t* __restrict__ ocount) {
    OriKey K;
    if (!orientation_key(f, sub == 0, pyr, mask, row_base, total_rows, fp, out4, info, ocount, K))
        return;
    float vote[37];
    orientation_hist(K.g, K.W, K.H, K.kx, K.ky, K.kz, fp, sub, vote_l, vote);
    if (sub != 0) return;
    orientation_finish(f, vote, K, fp, out4, ocount);
}

// The histogram of orientation_hist evaluated by a whole wave, for few candidates (a single
// image: ~1,500 candidates leave most SIMDs idle under the quad form, and each quad walks its
// window serially): 64 window samples at a time are evaluated in parallel, then lane b < 36
// adds the batch's votes for bin b in sample order.  Each bin sees the reference's sequence of
// float adds (the other samples add nothing: acc + 0.0f = acc, acc >= +0), so the histogram is
// orientation_hist's bit for bit.  Same window, sample arithmetic and smoothing.
__device__ __forceinline__ void orientation_hist_wave(const OriKey& K, const FeatureParams& fp,
                                                      int lane, float* s_v, float2* s_bw,
                                                      float (&vote)[37]) {
    const float ten_degree_per_radius = (float)5.7295779513082320876798154814105;
    const float gsigma = K.kz * fp.gaussian_factor;
    const float win = fabs_(K.kz) * fp.sample_factor;
    const float dist_threshold = (float)((double)(win * win) + 0.5);
    const float factor = -0.5f / (gsigma * gsigma);
    const float xmin = fmax_(1.5f, floor_(K.kx - win) + 0.5f);
    const float ymin = fmax_(1.5f, floor_(K.ky - win) + 0.5f);
    const float xmax = fmin_(K.W - 1.5f, floor_(K.kx + win) + 0.5f);
    const float ymax = fmin_(K.H - 1.5f, floor_(K.ky + win) + 0.5f);
    const int ncols = xmax >= xmin ? (int)(xmax - xmin) + 1 : 0;
    const int nrows = ymax >= ymin ? (int)(ymax - ymin) + 1 : 0;
#ifndef SGK_ORI_EXP
#define SGK_ORI_EXP 0   // timing experiment only (wrong orientations): 1 = no window samples
#endif
    const int total = SGK_ORI_EXP == 1 ? 0 : ncols * nrows;
    float acc = 0.0f;   // bin `lane`
    // sample base + lane: its pixel and the 4 gradient neighbours, fetched one batch ahead (the
    // loads are unconditional, at a clamped in-plane pixel, so the compiler waits only for the
    // batch it uses); `in` = inside the window and the circle
    struct Smp { float x, y, sq, a, b, c, d; bool in; };
    auto fetch = [&](int base, Smp& q) {
        const int sidx = base + lane;
        const bool valid = sidx < total;
        const int si = valid ? sidx : 0;
        const int r = si / max(ncols, 1), c = si - r * max(ncols, 1);
        q.x = xmin + (float)c;
        q.y = ymin + (float)r;
        const float dx = q.x - K.kx, dy = q.y - K.ky;
        q.sq = fma_(dx, dx, dy * dy);
        q.in = valid && total > 0 && !(fp.circular && q.sq >= dist_threshold);
        const int px = q.in ? (int)q.x : 1, py = q.in ? (int)q.y : 1;   // (1, 1): in-plane
        const float* p = K.g + (long long)py * K.W + px;
        q.a = p[1];
        q.b = p[-1];
        q.c = p[K.W];
        q.d = p[-K.W];
    };
    Smp cur, nxt;
    fetch(0, cur);
    for (int base = 0; base < total; base += 64) {
        fetch(base + 64, nxt);
        int bin = -1;
        float weight = 0.0f;
        if (cur.in) {
            const float gdx = cur.a - cur.b, gdy = cur.c - cur.d;   // grad_at
            const float grd = 0.5f * sqrt_(fma_(gdx, gdx, gdy * gdy));
            const float rot = grd == 0.0f ? 0.0f : atan2_(gdy, gdx);
            weight = grd * exp_(cur.sq * factor);
            bin = (int)floor_(rot * ten_degree_per_radius);
            if (bin < 0) bin += 36;
        }
        // the batch's (bin, weight) pairs through the wave's LDS (every lane writes one: samples
        // past the window have bin -1), read back as broadcasts of 4 pairs; lane b adds the
        // weights of bin b in sample order (the others add +0, which leaves acc >= +0 unchanged)
        const int nb = min(64, total - base);   // uniform
        s_bw[lane] = make_float2(__int_as_float(bin), weight);
        asm volatile("" ::: "memory");   // one wave: its LDS writes complete before its reads
        for (int k = 0; k < nb; k += 4) {
            const float4 q0 = *reinterpret_cast<const float4*>(&s_bw[k]);
            const float4 q1 = *reinterpret_cast<const float4*>(&s_bw[k + 2]);
            acc += __float_as_int(q0.x) == lane ? q0.y : 0.0f;
            acc += __float_as_int(q0.z) == lane ? q0.w : 0.0f;
            acc += __float_as_int(q1.x) == lane ? q1.y : 0.0f;
            acc += __float_as_int(q1.z) == lane ? q1.w : 0.0f;
        }
        asm volatile("" ::: "memory");   // read before the next batch overwrites them
        cur = nxt;
    }
    // the 6 smoothing passes, a bin per lane: each pass is a stencil over the previous pass's
    // values, (pre + vote[j]) + vote[j + 1] as the serial form, the ring through the wave's LDS
    const float one_third = (float)(1.0 / 3.0);
    const int jm = lane == 0 ? 35 : lane - 1, jp = lane == 35 ? 0 : lane + 1;
    float v = acc;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        if (lane < 36) s_v[lane] = v;
        asm volatile("" ::: "memory");   // one wave: its LDS writes complete before its reads
        const float pre = s_v[min(jm, 35)], nx = s_v[min(jp, 35)];
        asm volatile("" ::: "memory");
        v = one_third * (pre + v + nx);
    }
    if (lane < 36) s_v[lane] = v;
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < 36; ++i) vote[i] = s_v[i];
    asm volatile("" ::: "memory");
    vote[36] = vote[0];
}

// One wave per candidate, grid-stride (the few-candidates form of k_orientation; same outputs).
__global__ __launch_bounds__(256) void k_orientation_wave(const float* __restrict__ pyr,
                                                          const uint32_t* __restrict__ mask,
                                                          const uint32_t* __restrict__ row_base,
                                                          int total_rows,
                                                          const uint32_t* __restrict__ n_cand_dev,
                                                          uint32_t cap, const FeatureParams fp,
                                                          float4* __restrict__ out4,
                                                          int2* __restrict__ info,
                                                          uint32_t* __restrict__ ocount) {
    __shared__ float s_vote[4][64];
    __shared__ __attribute__((aligned(16))) float2 s_pair[4][64];
    const int lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t n = min(*n_cand_dev, cap);
    for (uint32_t f = blockIdx.x * 4 + wave; f < n; f += gridDim.x * 4) {   // uniform per wave
        OriKey K;
        if (!orientation_key(f, lane == 0, pyr, mask, row_base, total_rows, fp, out4, info,
                             ocount, K, lane))
            continue;
        float vote[37];
        orientation_hist_wave(K, fp, lane, s_vote[wave], s_pair[wave], vote);
        if (lane == 0) orientation_finish(f, vote, K, fp, out4, ocount);
        asm volatile("" ::: "memory");   // the next candidate's votes overwrite s_vote after
    }
}

// Grid-stride over the candidates (the grid is sized from the buffer capacity, the count is
// read on the device, so no host round trip sits between detection and orientation).
__global__ __launch_bounds__(256) void k_orientation(const float* __restrict__ pyr,
                                                     const uint32_t* __restrict__ mask,
                                                     const uint32_t* __restrict__ row_base,
                                                     int total_rows,
                                                     const uint32_t* __restrict__ n_cand_dev,
                                                     uint32_t cap, const FeatureParams fp,
                                                     float4* __restrict__ out4,
                                                     int2* __restrict__ info,
                                                     uint32_t* __restrict__ ocount) {
    __shared__ float s_vote[64 * 37];
    const int sub = threadIdx.x & 3, slot = threadIdx.x >> 2;
    const uint32_t n = min(*n_cand_dev, cap);
    float* vote_l = s_vote + slot * 37;
    for (uint32_t f = blockIdx.x * 64 + slot; f < n; f += gridDim.x * 64)   // uniform per quad
        orientation_one(f, sub, vote_l, pyr, mask, row_base, total_rows, fp, out4, info, ocount);
}

// ------------------------------------------------------------------------------------------
// -fo != 0: the first octave's input.  src value of input pixel k of the flat tw x h buffer
// the reference binds (_inputTex, PyramidCU.cpp:949-958): u8 -> p / 255.0f as the host
// conversion (GLTexImage.cpp:818); indices past the buffer read 0 (tex1Dfetch).
template <bool U8>
__device__ __forceinline__ float input_at(const float* sf, const uint8_t* s8, int stride, int tw,
                                          int h, long long k) {
    if (k >= (long long)tw * h) return 0.0f;
    const int r = (int)(k / tw), c = (int)(k - (long long)r * tw);
    return U8 ? u8_to_unit(s8[(long long)r * stride + c]) : sf[(long long)r * stride + c];
}

// DownsampleKernel (ProgramCU.cu:287-311): dst(r, c) = src(r << fo, min(c << fo, tw - 1)).
template <bool U8>
__global__ __launch_bounds__(256) void k_input_down(const float* __restrict__ src,
                                                    const uint8_t* __restrict__ src8, int stride,
                                                    long long src_img_stride, int tw, int h,
                                                    int fo, float* __restrict__ dst, int dw, int dh,
                                                    long long dst_img_stride) {
    const int b = blockIdx.z, r = blockIdx.y;
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= dw || r >= dh) return;
    const long long so = (long long)b * src_img_stride;
    const int sc = min(c << fo, tw - 1), sr = r << fo;
    const float v = U8 ? u8_to_unit(src8[so + (long long)sr * stride + sc])
                       : src[so + (long long)sr * stride + sc];
    dst[(long long)b * dst_img_stride + (long long)r * dw + c] = v;
}

// UpsampleKernel<s> (ProgramCU.cu:225-270): output row R blends source rows R >> s and
// (R >> s) + 1 with w1 = (R & (S-1)) / S; each source column c writes S outputs at
// (tw R + c) S interpolating c and c + 1 of the flat buffer.  a*b + c*d -> fma(a, b, c*d).
template <bool U8>
__global__ __launch_bounds__(256) void k_input_up(const float* __restrict__ src,
                                                  const uint8_t* __restrict__ src8, int stride,
                                                  long long src_img_stride, int tw, int h, int s,
                                                  float* __restrict__ dst,
                                                  long long dst_img_stride) {
    const int b = blockIdx.z, R = blockIdx.y;
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= tw) return;
    const int S = 1 << s;
    const float inv = 1.0f / float(S);
    const float* sf = U8 ? nullptr : src + (long long)b * src_img_stride;
    const uint8_t* s8 = U8 ? src8 + (long long)b * src_img_stride : nullptr;
    const int row = R >> s, helper = R & (S - 1);
    const long long index = (long long)row * tw + c;
    float v1, v2;
    if (helper) {
        const float v11 = input_at<U8>(sf, s8, stride, tw, h, index);
        const float v12 = input_at<U8>(sf, s8, stride, tw, h, index + 1);
        const float v21 = input_at<U8>(sf, s8, stride, tw, h, index + tw);
        const float v22 = input_at<U8>(sf, s8, stride, tw, h, index + tw + 1);
        const float w1 = inv * (float)helper, w2 = 1.0f - w1;   // (float)(1.0 - w1): exact
        v1 = fma_(v21, w1, w2 * v11);
        v2 = fma_(v22, w1, w2 * v12);
    } else {
        v1 = input_at<U8>(sf, s8, stride, tw, h, index);
        v2 = input_at<U8>(sf, s8, stride, tw, h, index + 1);
    }
    float* o = dst + (long long)b * dst_img_stride + ((long long)tw * R + c) * S;
    o[0] = v1;
    for (int i = 1; i < S; i++) {
        const float r2 = (float)i * inv, r1 = 1.0f - r2;
        o[i] = fma_(v1, r1, v2 * r2);
    }
}

// ------------------------------------------------------------------------------------------
// Color -> luminance: (19595 r + 38470 g + 7471 b) / (65535.0f * 255.0f).  The numerator is an
// exact integer below 2^24 and the denominator an exact float, so the IEEE division on the
// device gives the host conversion's bits.
template <int CH, bool BGR>
__global__ __launch_bounds__(256) void k_color_gray(const uint8_t* __restrict__ src, int tw, int h,
                                                    int stride, float* __restrict__ dst) {
    const int b = blockIdx.z, y = blockIdx.y;
    const int x = blockIdx.x * 256 + threadIdx.x;
    if (x >= tw) return;
    const uint8_t* p = src + ((long long)b * h + y) * stride + (long long)x * CH;
    const int r = BGR ? p[2] : p[0], g = p[1], bl = BGR ? p[0] : p[2];
    const int num = 19595 * r + 38470 * g + 7471 * bl;
    dst[((long long)b * h + y) * tw + x] = (float)num / (65535.0f * 255.0f);
}

// ------------------------------------------------------------------------------------------
// Feature expansion + image coordinates (PyramidCU.cpp:521-606 / 701-751).
// (io.off != nullptr: the grid's last block writes the readback record instead -- off[0] = the
// candidate count, off[1 + b] = image b's first feature for b in [0, batch] -- which one more
// launch after the descriptors wrote before; a single image's extract pays per launch)
// Candidate f's 0, 1 or 2 features at slots e0 .. e0 + n - 1 (ReshapeFeatureListCPU,
// PyramidCU.cpp:560-578): the orientations unpacked, the image-coordinate keys
// (PyramidCU.cpp:701-751).
__device__ __forceinline__ void expand_one(uint32_t f, uint32_t e0, uint32_t n,
                                           const float4* __restrict__ cand,
                                           const int2* __restrict__ info, const FeatureParams& fp,
                                           float4* __restrict__ feat, int2* __restrict__ feat_info,
                                           float4* __restrict__ keys) {
    const float4 c = cand[f];
    const int2 in = info[f];
    const int o = in.y / fp.d;
    const float oss = ldexpf(1.0f, o + fp.octave_min);   // os * 2^o, os = 2^octave_min
    const double twopi = 2.0 * 3.14159265358979323846;
    float ang[2];
    if (fp.num_orientation >= 2) {
        const double factor = 2.0 * 3.14159265358979323846 / 65535.0;
        const uint32_t pk = as_uint(c.w);
        ang[0] = (float)(factor * (double)(pk & 0xffffu));
        ang[1] = (float)(factor * (double)(pk >> 16));
    } else {
        ang[0] = ang[1] = c.w;
    }
    for (uint32_t q = 0; q < n; q++) {
        const uint32_t e = e0 + q;
        feat[e] = make_float4(c.x, c.y, c.z, ang[q]);
        feat_info[e] = in;
        keys[e] = make_float4(oss * (c.x - 0.5f) + fp.origin_offset,
                              oss * (c.y - 0.5f) + fp.origin_offset, oss * c.z,
                              (float)fmod(twopi - (double)ang[q], twopi));
    }
}

__global__ __launch_bounds__(256) void k_expand(const float4* __restrict__ cand,
                                                const int2* __restrict__ info,
                                                const uint32_t* __restrict__ eoff,
                                                const uint32_t* __restrict__ n_cand_dev,
                                                const FeatureParams fp, float4* __restrict__ feat,
                                                int2* __restrict__ feat_info,
                                                float4* __restrict__ keys, uint32_t cap,
                                                const ImageOffsetsArgs io) {
    int nblk = (int)gridDim.x;
    if (io.off) {
        nblk--;
        if ((int)blockIdx.x == nblk) {
            for (int b = threadIdx.x; b <= io.batch + 1; b += 256) {
                if (b == 0) {
                    io.off[0] = (int64_t)io.row_base[io.total_rows];
                } else {
                    const int r = b - 1 == io.batch ? io.total_rows : (b - 1) * io.rows_per_image;
                    io.off[b] = (int64_t)eoff[min(io.row_base[r], cap)];
                }
            }
            return;
        }
    }
    const uint32_t ncand = min(*n_cand_dev, cap);
    for (uint32_t f = blockIdx.x * 256 + threadIdx.x; f < ncand; f += (uint32_t)nblk * 256) {
        const uint32_t e0 = eoff[f], n = eoff[f + 1] - e0;
        if (n != 0) expand_one(f, e0, n, cand, info, fp, feat, feat_info, keys);
    }
}

// ------------------------------------------------------------------------------------------
// ComputeDescriptor_Kernel<false> (ProgramCU.cu:1013-1101) + NormalizeDescriptor_Kernel
// (:1173-1208).  16 lanes per feature (one 4x4 grid cell each, as the reference), 4 features
// per wave; normalisation sums are formed in the reference's sequential order via shuffles.
__device__ __forceinline__ float sq4(float a, float b, float c, float d) {
    float t = a * a;
    t = fma_(b, b, t);
    t = fma_(c, c, t);
    return fma_(d, d, t);
}

// RECT: ComputeDescriptorRECT_Kernel<false> (ProgramCU.cu:1104-1171) for keys given with
// keys_have_orientation == -1: the 4 x 4 grid spans the rectangle [x, x+z] x [y, y+w], cells
// are axis-aligned (nx = dx / sptx), no Gaussian window, theta = -angle.
template <bool RECT>
__device__ __forceinline__ void descriptor_one(uint32_t e, int lane,
                                               const float* __restrict__ pyr,
                                               const float4* __restrict__ feat,
                                               const int2* __restrict__ feat_info,
                                               const FeatureParams& fp,
                                               float* __restrict__ desc, uint32_t out) {
    // one wave per feature: lanes 4c..4c+3 own grid cell c (the reference's 16 threads per
    // feature, ProgramCU.cu:1017-1021); the quad evaluates consecutive window samples in
    // parallel and every lane applies the 4 contributions in the reference's (y, x) order, so
    // the 9 accumulators see the reference's exact sequence of fma's.
    const int cell = lane >> 2, sub = lane & 3;
    const int ix = cell & 3, iy = cell >> 2;
    // each quad lane owns two of the cell's 8 orientation bins (lane 0 also bin 8): every bin's
    // fma chain is the reference's, and a sample costs 4 compares instead of an 8-way select
    const int kb = 2 * sub;
    float acc0 = 0.0f, acc1 = 0.0f, acc8 = 0.0f;
    const float4 key = feat[e];
    const int2 in = feat_info[e];
    const int o = in.y / fp.d, j = in.y - o * fp.d;
    const OctaveDesc& od = fp.oct[o];
    const int W = od.wa, H = od.h;
    const float* g = pyr + od.gauss_off + (long long)(1 + j) * od.level_stride +
                     (long long)in.x * W * H;
    const float rpi = (float)(4.0 / 3.14159265358979323846);
    float spt = 0.f, anglef = 0.f, cspt = 0.f, sspt = 0.f, crspt = 0.f, srspt = 0.f;
    float ox = 0.f, oy = 0.f, ptx, pty, bszx, bszy;
    const float sptx = key.z * 0.25f, spty = key.w * 0.25f;   // RECT (exact: key * 0.25 double)
    if (RECT) {
        ptx = fma_(sptx, ix + 0.5f, key.x);
        pty = fma_(spty, iy + 0.5f, key.y);
        bszx = sptx;
        bszy = spty;
    } else {
        spt = fabs_(key.z * fp.window_factor);
        float s, c;
        sincos_(key.w, &s, &c);
        anglef = (double)key.w > 3.14159265358979323846
                     ? (float)((double)key.w - (2.0 * 3.14159265358979323846))
                     : key.w;
        cspt = c * spt;
        sspt = s * spt;
        crspt = c / spt;
        srspt = s / spt;
        ox = ix - 1.5f;
        oy = iy - 1.5f;
        ptx = fma_(cspt, ox, -(sspt * oy)) + key.x;
        pty = fma_(cspt, oy, sspt * ox) + key.y;
        bszx = bszy = fabs_(cspt) + fabs_(sspt);
    }
    const float xmin = fmax_(1.5f, floor_(ptx - bszx) + 0.5f);
    const float ymin = fmax_(1.5f, floor_(pty - bszy) + 0.5f);
    const float xmax = fmin_(W - 1.5f, floor_(ptx + bszx) + 0.5f);
    const float ymax = fmin_(H - 1.5f, floor_(pty + bszy) + 0.5f);
    const int ncols = xmax >= xmin ? (int)(xmax - xmin) + 1 : 0;
    const int nrows = ymax >= ymin ? (int)(ymax - ymin) + 1 : 0;
    // The reference visits every sample of the cell's axis-aligned box and keeps those with
    // |nx| < 1 and |ny| < 1 (the rotated square).  Only the samples it keeps contribute, so the
    // quad walks, row by row, a column span that covers the square with a 0.01-pixel margin
    // (the float bounds and the float test differ by ~1e-5 pixel; the exact test below still
    // decides each sample) -- same samples, same (y, x) order, ~45% fewer iterations.
    // (RECT: every column of the box; the exact test below decides)
    const bool use_c = !RECT && fabs_(crspt) > 1e-4f / spt;
    const bool use_s = !RECT && fabs_(srspt) > 1e-4f / spt;
    const float icr = use_c ? 1.0f / crspt : 0.0f, isr = use_s ? 1.0f / srspt : 0.0f;
    const float kInf = as_float(0x7f800000u);
    auto row_span = [&](int r, int& lo, int& len) {
        const float dy = (ymin + (float)r) - pty;
        float a = -kInf, bnd = kInf;
        if (use_c) {
            const float p = (-1.0f - srspt * dy) * icr, q = (1.0f - srspt * dy) * icr;
            a = fmax_(a, fmin_(p, q));
            bnd = fmin_(bnd, fmax_(p, q));
        }
        if (use_s) {
            const float p = (crspt * dy - 1.0f) * isr, q = (crspt * dy + 1.0f) * isr;
            a = fmax_(a, fmin_(p, q));
            bnd = fmin_(bnd, fmax_(p, q));
        }
        const float cl = fmax_(0.0f, ceilf(ptx + a - xmin - 0.01f));
        const float ch = fmin_((float)(ncols - 1), floor_(ptx + bnd - xmin + 0.01f));
        lo = (int)cl;
        len = ch >= cl ? (int)ch - lo + 1 : 0;
    };
    // lane sub starts at sample sub of the span sequence, then advances 4 samples per step
    int wr = 0, wc = sub, wlo = 0, wlen = 0;
    if (nrows > 0 && ncols > 0) row_span(0, wlo, wlen);
    else wr = nrows;
    auto normalize = [&]() {
        while (wr < nrows && wc >= wlen) {
            wc -= wlen;
            if (++wr < nrows) row_span(wr, wlo, wlen);
        }
    };
    normalize();
    for (;;) {
        // the quad's lane 0 holds its earliest sample: the quad stops together
        if (qbcast<0>(wr < nrows ? 1 : 0) == 0) break;
        int fidx = -1;
        float weight = 0.f, weight1 = 0.f, weight2 = 0.f;
        if (wr < nrows) {
            const float x = xmin + (float)(wlo + wc), y = ymin + (float)wr;
            const float dx = x - ptx, dy = y - pty;
            float nx, ny;
            if (RECT) {
                nx = dx / sptx;
                ny = dy / spty;
            } else {
                nx = fma_(crspt, dx, srspt * dy);
                ny = fma_(crspt, dy, -(srspt * dx));
            }
            const float nxn = fabs_(nx), nyn = fabs_(ny);
            if (nxn < 1.0f && nyn < 1.0f) {
                const float2 cc = grad_at(g, W, (int)x, (int)y);
                // (float)(1.0 - (double)n) of the reference: 1 - n is exact in double, so the
                // single float subtraction rounds to the same value
                const float wx = 1.0f - nxn, wy = 1.0f - nyn;
                float theta;
                if (RECT) {
                    weight = wx * wy * cc.x;
                    theta = (-cc.y) * rpi;
                } else {
                    const float dnx = nx + ox, dny = ny + oy;
                    const float ww = exp_mid_(-0.125f * fma_(dnx, dnx, dny * dny));   // in [-1.6, 0]
                    weight = ww * wx * wy * cc.x;
                    theta = (anglef - cc.y) * rpi;
                }
                if (theta < 0) theta += 8.0f;
                const float fo = floor_(theta);
                fidx = (int)fo;
                weight1 = fo + 1.0f - theta;
                weight2 = theta - fo;
            }
            wc += 4;
            normalize();
        }
        const int f4[4] = {qbcast<0>(fidx), qbcast<1>(fidx), qbcast<2>(fidx), qbcast<3>(fidx)};
        const float w4[4] = {qbcastf<0>(weight), qbcastf<1>(weight), qbcastf<2>(weight),
                             qbcastf<3>(weight)};
        const float a4[4] = {qbcastf<0>(weight1), qbcastf<1>(weight1), qbcastf<2>(weight1),
                             qbcastf<3>(weight1)};
        const float b4[4] = {qbcastf<0>(weight2), qbcastf<1>(weight2), qbcastf<2>(weight2),
                             qbcastf<3>(weight2)};
#pragma unroll
        for (int q = 0; q < 4; q++) {
            // sample q adds w1*w to bin f and w2*w to bin f+1, for f in 0..7 only (the
            // reference's unrolled k == fidx test drops fidx == 8 at theta == 8)
            // Branch-free: a non-matching bin adds fma(0, w, acc) = acc exactly (accumulators
            // and weights are >= +0, and an invalid sample has w = 0).
            const int f = f4[q];
            const float s0 = f == kb ? a4[q] : (f + 1 == kb ? b4[q] : 0.0f);
            const float s1 = f == kb + 1 ? a4[q] : (f == kb ? b4[q] : 0.0f);
            const float s8 = f == 7 ? b4[q] : 0.0f;
            acc0 = fma_(s0, w4[q], acc0);
            acc1 = fma_(s1, w4[q], acc1);
            acc8 = fma_(s8, w4[q], acc8);
        }
    }
    if (sub == 0) acc0 += acc8;   // des[0] += des[8]
    float des[8];
    des[0] = qbcastf<0>(acc0); des[1] = qbcastf<0>(acc1);
    des[2] = qbcastf<1>(acc0); des[3] = qbcastf<1>(acc1);
    des[4] = qbcastf<2>(acc0); des[5] = qbcastf<2>(acc1);
    des[6] = qbcastf<3>(acc0); des[7] = qbcastf<3>(acc1);
    if (fp.normalize) {
        // NormalizeDescriptor_Kernel: sums over the 32 float4s in order (cells 0..15)
        const int g0 = lane & ~63;
        float a = sq4(des[0], des[1], des[2], des[3]);
        float bq = sq4(des[4], des[5], des[6], des[7]);
        float norm1 = 0.f;
        for (int q = 0; q < 16; q++) {
            norm1 += __shfl(a, g0 + 4 * q, 64);
            norm1 += __shfl(bq, g0 + 4 * q, 64);
        }
        norm1 = rsqrt_(norm1);
#pragma unroll
        for (int i = 0; i < 8; i++) des[i] = fmin_(0.2f, des[i] * norm1);
        a = sq4(des[0], des[1], des[2], des[3]);
        bq = sq4(des[4], des[5], des[6], des[7]);
        float norm2 = 0.f;
        for (int q = 0; q < 16; q++) {
            norm2 += __shfl(a, g0 + 4 * q, 64);
            norm2 += __shfl(bq, g0 + 4 * q, 64);
        }
        norm2 = rsqrt_(norm2);
#pragma unroll
        for (int i = 0; i < 8; i++) des[i] *= norm2;
    }
    if (sub < 2) {
        float4* dst = reinterpret_cast<float4*>(desc + (size_t)out * 128 + cell * 8 + sub * 4);
        *dst = sub == 0 ? make_float4(des[0], des[1], des[2], des[3])
                        : make_float4(des[4], des[5], des[6], des[7]);
    }
}

// ------------------------------------------------------------------------------------------
// Relaxed-order descriptor (the shipped default).  Same samples, same weights, same bins as
// descriptor_one -- the reference's ComputeDescriptor_Kernel / ComputeDescriptorRECT_Kernel
// (ProgramCU.cu:1013-1171) -- but each sample's contribution is formed and accumulated by ONE
// lane, in any order:
//   * each of the quad's 4 lanes walks every 4th sample of its cell and keeps all 8 bins in
//     registers; the 4 partial histograms are summed by DPP at the end (descriptor_one instead
//     broadcasts every sample to the 4 lanes so that each bin sees the reference's fma order);
//   * the linear bin interpolation is the tent max(0, 1 - |theta - k|) per bin (bin 0 also
//     takes the wrap-around of bin 8, ProgramCU.cu:1094): 2 VALU + 1 fma per bin, no selects;
//   * gradient magnitude, atan2, the Gaussian window and the normalisation use the hardware
//     v_sqrt / v_rcp / v_exp (1 ulp) and a short atan2 series (|error| < 1e-6 rad), except
//     near the one discontinuity of the reference's binning (a sample whose theta rounds to
//     8.0 is dropped), where the oracle's atan2 decides.
// Every difference to the reference's arithmetic is continuous in the inputs and of the order of
// a float ulp, so descriptors agree with the oracle to L2 ~1e-6 (tests: < 1e-4, the north star's
// bound; descriptor_one stays the bit-exact test mode, SGPU_DEBUG_EXACT_DESCRIPTOR).
__device__ __forceinline__ float atan2_relaxed(float y, float x) {
    const float ax = fabs_(x), ay = fabs_(y);
    const float mx = fmax_(ax, ay), mn = fmin_(ax, ay);
    const bool red = mn > 0.414213562f * mx;           // reduce to |t| <= tan(pi/8)
    const float t = (red ? mn - mx : mn) * __builtin_amdgcn_rcpf(red ? mn + mx : mx);
    const float z = t * t;
    float p = -0.0909090909f;                           // odd series to t^11: |err| < 1e-6
    p = fma_(p, z, 0.111111111f);
    p = fma_(p, z, -0.142857143f);
    p = fma_(p, z, 0.2f);
    p = fma_(p, z, -0.333333333f);
    float r = fma_(p * z, t, t) + (red ? 0.785398163f : 0.0f);
    r = ay > ax ? 1.57079633f - r : r;
    r = (as_uint(x) >> 31) ? 3.14159265f - r : r;
    return (as_uint(y) >> 31) ? -r : r;
}

// Quad (xor) butterfly sum: every lane of the quad ends with the quad's total.
__device__ __forceinline__ float quad_sum(float v) {
    v += as_float((uint32_t)__builtin_amdgcn_mov_dpp((int)as_uint(v), 0xB1, 0xF, 0xF, false));  // [1,0,3,2]
    v += as_float((uint32_t)__builtin_amdgcn_mov_dpp((int)as_uint(v), 0x4E, 0xF, 0xF, false));  // [2,3,0,1]
    return v;
}

#ifndef SGK_DESC_RSTEP
#define SGK_DESC_RSTEP 4
#endif
static_assert(SGK_DESC_RSTEP == 0 || SGK_DESC_RSTEP == 1 || SGK_DESC_RSTEP == 2 ||
                  SGK_DESC_RSTEP == 4, "rows per quad step (0: flat strip order)");

template <bool RECT>
__device__ __forceinline__ void descriptor_fast(uint32_t e, int lane,
                                                const float* __restrict__ pyr,
                                                const float4* __restrict__ feat,
                                                const int2* __restrict__ feat_info,
                                                const FeatureParams& fp,
                                                float* __restrict__ desc, uint32_t out) {
    const int cell = lane >> 2, sub = lane & 3;
    const int ix = cell & 3, iy = cell >> 2;
    const float4 key = feat[e];
    const int2 in = feat_info[e];
    const int o = in.y / fp.d, j = in.y - o * fp.d;
    const OctaveDesc& od = fp.oct[o];
    const int W = od.wa, H = od.h;
    const float* g = pyr + od.gauss_off + (long long)(1 + j) * od.level_stride +
                     (long long)in.x * W * H;
    const float rpi = (float)(4.0 / 3.14159265358979323846);
    // cell geometry exactly as descriptor_one (so both visit the same samples)
    float spt = 0.f, anglef = 0.f, cspt = 0.f, sspt = 0.f, crspt = 0.f, srspt = 0.f;
    float ox = 0.f, oy = 0.f, ptx, pty, bszx, bszy;
    const float sptx = key.z * 0.25f, spty = key.w * 0.25f;
    if (RECT) {
        ptx = fma_(sptx, ix + 0.5f, key.x);
        pty = fma_(spty, iy + 0.5f, key.y);
        bszx = sptx;
        bszy = spty;
    } else {
        spt = fabs_(key.z * fp.window_factor);
        float s, c;
        sincos_(key.w, &s, &c);
        anglef = (double)key.w > 3.14159265358979323846
                     ? (float)((double)key.w - (2.0 * 3.14159265358979323846))
                     : key.w;
        cspt = c * spt;
        sspt = s * spt;
        crspt = c / spt;
        srspt = s / spt;
        ox = ix - 1.5f;
        oy = iy - 1.5f;
        ptx = fma_(cspt, ox, -(sspt * oy)) + key.x;
        pty = fma_(cspt, oy, sspt * ox) + key.y;
        bszx = bszy = fabs_(cspt) + fabs_(sspt);
    }
    const float xmin = fmax_(1.5f, floor_(ptx - bszx) + 0.5f);
    const float ymin = fmax_(1.5f, floor_(pty - bszy) + 0.5f);
    const float xmax = fmin_(W - 1.5f, floor_(ptx + bszx) + 0.5f);
    const float ymax = fmin_(H - 1.5f, floor_(pty + bszy) + 0.5f);
    const int ncols = xmax >= xmin ? (int)(xmax - xmin) + 1 : 0;
    const int nrows = ymax >= ymin ? (int)(ymax - ymin) + 1 : 0;
    const bool use_c = !RECT && fabs_(crspt) > 1e-4f / spt;
    const bool use_s = !RECT && fabs_(srspt) > 1e-4f / spt;
    // The row's column span as the intersection of the two slabs |nx| <= 1 and |ny| <= 1, each
    // linear in dy: descriptor_one's row_span refactored into 4 fma and no selects on the signs
    // of the coefficients (the 0.01-pixel margin absorbs the different rounding; the per-sample
    // test decides).  RECT: the whole row of the box.
    const float icr = use_c ? 1.0f / crspt : 0.0f, isr = use_s ? 1.0f / srspt : 0.0f;
    const float hu = use_c ? fabs_(icr) : 1e30f, su = use_c ? srspt * icr : 0.0f;
    const float hv = use_s ? fabs_(isr) : 1e30f, cv = use_s ? crspt * isr : 0.0f;
    const float k_lo = ptx - xmin - 0.01f, k_hi = ptx - xmin + 0.01f;
    const float dy0 = ymin - pty;
    auto row_span = [&](int r, int& lo, int& len) {
        const float dy = dy0 + (float)r;
        const float a = fmax_(fma_(-su, dy, -hu), fma_(cv, dy, -hv));
        const float bnd = fmin_(fma_(-su, dy, hu), fma_(cv, dy, hv));
        const float cl = fmax_(0.0f, ceilf(a + k_lo));
        const float ch = fmin_((float)(ncols - 1), floor_(bnd + k_hi));
        lo = (int)cl;
        len = ch >= cl ? (int)ch - lo + 1 : 0;
    };
    const float irx = RECT ? __builtin_amdgcn_rcpf(sptx) : 0.f;
    const float iry = RECT ? __builtin_amdgcn_rcpf(spty) : 0.f;
    const float kexp = -0.125f * 1.44269504f;           // e^(-x/8) = 2^(kexp x)
    const int ixmin = (int)xmin, iymin = (int)ymin;
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; k++) acc[k] = 0.0f;
    // One sample: its cell coordinates from the row offset dy and column offset dx (both from
    // the reference's rounded cell centre), its gradient (gx, gy); adds nothing when !valid.
    auto sample = [&](float dx, float dy, float gx, float gy, bool valid) {
        float nx, ny;
        if (RECT) {
            nx = dx * irx;
            ny = dy * iry;
        } else {
            nx = fma_(crspt, dx, srspt * dy);
            ny = fma_(crspt, dy, -(srspt * dx));
        }
        const float wx = 1.0f - fabs_(nx), wy = 1.0f - fabs_(ny);
        const float m2 = fma_(gx, gx, gy * gy);
        const float m = 0.5f * __builtin_amdgcn_sqrtf(m2);
        float rot = atan2_relaxed(gy, gx);   // NaN at (0, 0)
        // theta = (anglef - rot) * 4/pi, +8 if negative, is dropped when it rounds to 8.0
        // (ProgramCU.cu:1071-1090): a discontinuity at anglef - rot in (-2^-21, 0] and near +2pi.
        // Within 1e-5 rad of those points (rare) rot is recomputed with the oracle's atan2, so
        // the drop decisions are the reference's exactly; elsewhere |error| < 1e-6 cannot reach
        // them.
        const float dd = fabs_(anglef - rot);
        if (dd < 1e-5f || dd > 6.2831753f) rot = atan2_(gy, gx);
        rot = m2 == 0.0f ? 0.0f : rot;
        float w = m * wx * wy;
        float theta;
        if (RECT) {
            theta = -rot * rpi;
        } else {
            const float dnx = nx + ox, dny = ny + oy;
            w *= __builtin_amdgcn_exp2f(kexp * fma_(dnx, dnx, dny * dny));
            theta = (anglef - rot) * rpi;
        }
        if (theta < 0) theta += 8.0f;
        // outside the rotated square (|n| >= 1) or theta == 8 (the reference's fidx == 8 is
        // dropped) the sample adds nothing
        w = (valid && wx > 0.0f && wy > 0.0f && theta < 8.0f) ? w : 0.0f;
        acc[0] = fma_(__builtin_amdgcn_fmed3f(fmax_(1.0f - theta, theta - 7.0f), 0.0f, 1.0f), w,
                      acc[0]);
#pragma unroll
        for (int k = 1; k < 8; k++)
            acc[k] = fma_(__builtin_amdgcn_fmed3f(1.0f - fabs_(theta - (float)k), 0.0f, 1.0f), w,
                          acc[k]);
    };
    // Lane sub walks rows sub, sub + 4, ... of its cell's box, each row's span in strips of 4
    // consecutive samples: the strip's gradient neighbours come from 4 vector loads -- row y at
    // columns x-1 .. x+2 and x+1 .. x+4, rows y-1 and y+1 at x .. x+3 -- instead of 16 scalar
    // gathers (the gathers of 16 cells saturate the texture-address/L1 path: 42 cache-line
    // lookups per load instruction), and the 4 samples are independent dependency chains.
    const char* gb = reinterpret_cast<const char*>(g);
    typedef float f4v __attribute__((ext_vector_type(4)));
    auto ld4 = [&](uint32_t b) { return *reinterpret_cast<const f4v*>(gb + b); };
    // The strips are walked as one flat sequence with the next strip's 4 loads issued before the
    // current strip's samples (software pipelining: a strip's gathers overlap the previous
    // strip's arithmetic).  The loads are unconditional 16-byte loads: at the right edge a strip
    // may read up to 4 floats past the row end, which are the next row's (a sample is at most in
    // column W-2 and row H-2) and feed no valid sample; past the last strip a lane re-reads its
    // last strip.
    // DESC_RSTEP rows walked by the quad side by side: lanes per row LPR = 4 / RSTEP, lane
    // (rsub, csub) walks rows rsub, rsub + RSTEP, ... in strips starting 4 csub columns into the
    // span, 4 LPR apart (RSTEP 4: every lane its own rows; 2: two lanes on adjacent strips of one
    // row, so a load instruction touches half the cache lines)
    // RSTEP 0 (flat): the cell's strips in row-major order, strip f to lane f mod 4, so the
    // quad's 4 lanes read 16 consecutive columns of one row (or the end of one row and the start
    // of the next): one or two cache lines per quad and load instead of four, and no lane idles
    // on a short row.  Each lane keeps its own cursor (row r, strip s of the row) and moves it 4
    // strips per step.
    constexpr int RSTEP = SGK_DESC_RSTEP;
    constexpr int LPR = 4 / (RSTEP ? RSTEP : 4);
    const int rsub = RSTEP ? sub / LPR : 0, c4 = RSTEP ? 4 * (sub % LPR) : 0;
    int r = rsub, c = 0, lo = 0, len = 0, s = sub, ns = 0;
    auto next_row = [&]() {   // advance r (by RSTEP) to the next row with samples for this lane
        for (; r < nrows; r += RSTEP) {
            row_span(r, lo, len);
            if (len > c4) break;
        }
    };
    auto flat_norm = [&]() {   // move (r, s) forward over rows until strip s exists in row r
        while (s >= ns && r < nrows) {
            s -= ns;
            if (++r < nrows) {
                row_span(r, lo, len);
                ns = (len + 3) >> 2;
            }
        }
    };
    if (RSTEP == 0) {
        r = ncols > 0 ? 0 : nrows;
        if (r < nrows) {
            row_span(0, lo, len);
            ns = (len + 3) >> 2;
        }
        flat_norm();
        c = lo + 4 * s;
    } else {
        if (ncols > 0) next_row(); else r = nrows;
        c = lo + c4;
    }
    f4v na, nb, nu, nd;
    // the address loaded when no sample is left: row 1, column 1 of the plane, whose 4 loads
    // (columns 0 .. 5 of row 1, columns 1 .. 4 of rows 0 and 2) stay inside it for any feature --
    // a caller keypoint far outside the image has an empty box and unbounded ixmin / iymin
    uint32_t npo = 4u * (uint32_t)(W + 1);
    auto fetch = [&]() {
        if (r < nrows) npo = 4u * (uint32_t)((iymin + r) * W + ixmin + c);
        na = ld4(npo - 4u);            // x-1 .. x+2
        nb = ld4(npo + 4u);            // x+1 .. x+4
        nu = ld4(npo - 4u * W);        // row y-1, x .. x+3
        nd = ld4(npo + 4u * W);        // row y+1, x .. x+3
    };
    fetch();
    while (r < nrows) {
        const f4v a = na, b = nb, up = nu, dn = nd;
        const float dy = (ymin + (float)r) - pty;
        const int nv = lo + len - c;   // samples of this strip inside the span
        const float dx0 = (xmin + (float)c) - ptx;
        if (RSTEP == 0) {
            s += 4;
            flat_norm();
            c = lo + 4 * s;
        } else {
            c += 4 * LPR;
            if (c >= lo + len) {
                r += RSTEP;
                next_row();
                c = lo + c4;
            }
        }
        fetch();
        sample(dx0, dy, b.x - a.x, dn.x - up.x, true);
        sample(dx0 + 1.0f, dy, b.y - a.y, dn.y - up.y, nv > 1);
        sample(dx0 + 2.0f, dy, b.z - a.z, dn.z - up.z, nv > 2);
        sample(dx0 + 3.0f, dy, b.w - a.w, dn.w - up.w, nv > 3);
    }
#pragma unroll
    for (int k = 0; k < 8; k++) acc[k] = quad_sum(acc[k]);
    // lane sub owns bins 2 sub, 2 sub + 1 of its cell
    float b0 = acc[0], b1 = acc[1];
    b0 = sub == 1 ? acc[2] : b0; b1 = sub == 1 ? acc[3] : b1;
    b0 = sub == 2 ? acc[4] : b0; b1 = sub == 2 ? acc[5] : b1;
    b0 = sub == 3 ? acc[6] : b0; b1 = sub == 3 ? acc[7] : b1;
    if (fp.normalize) {
        float s = fma_(b0, b0, b1 * b1);
#pragma unroll
        for (int k = 32; k >= 1; k >>= 1) s += __shfl_xor(s, k, 64);
        const float n1 = __builtin_amdgcn_rsqf(s);
        b0 = fmin_(0.2f, b0 * n1);
        b1 = fmin_(0.2f, b1 * n1);
        s = fma_(b0, b0, b1 * b1);
#pragma unroll
        for (int k = 32; k >= 1; k >>= 1) s += __shfl_xor(s, k, 64);
        const float n2 = __builtin_amdgcn_rsqf(s);
        b0 *= n2;
        b1 *= n2;
    }
    *reinterpret_cast<float2*>(desc + (size_t)out * 128 + cell * 8 + sub * 2) = make_float2(b0, b1);
}

// ------------------------------------------------------------------------------------------
// Pixel-major descriptor (round 4, the shipped default for detected features).  descriptor_fast
// visits a window pixel once per cell whose rotated square holds it -- 2.56 times on average, up to
// 4 -- and pays the pixel's gradient magnitude, atan2, Gaussian weight and bin split on every visit,
// while only the spatial weight (1 - |nx|)(1 - |ny|) depends on the cell.  Here every pixel is
// evaluated once: the window |dnx|, |dny| < 2.5 (feature frame, cell units, dnx = nx + ox) is cut
// into the 5 x 5 "dual" cells of the half-cell-shifted grid, dual cell (a, b) = floor(dnx + 2.5),
// floor(dny + 2.5); a pixel of dual cell (a, b) lies in the squares of exactly the cells (a-1, b-1),
// (a, b-1), (a-1, b), (a, b), with the bilinear weights (1-u)(1-v), u(1-v), (1-u)v, uv (u, v its
// offsets inside the dual cell), which are the reference's (1 - |nx|)(1 - |ny|) for those cells
// (ProgramCU.cu:1044-1094).  Two lanes own each dual cell (lanes 0..49, alternate rows); a pixel's
// 8 contributions (4 cells x the 2 interpolated orientation bins) go to the wave's LDS histogram
// as no-return ds_add_f32 (IEEE adds in the LDS), laid out [bin][6 x 6 cells][lane copy]: the
// 6 x 6 grid gives the 4 cells of a dual cell constant offsets (0, 1, 6, 7 cells) and absorbs the
// border cells -1 and 4, which are never read; the two lanes of a dual cell add to their own copy,
// so no two lanes of an instruction hit one address.  Membership of a pixel is decided from dnx,
// dny, which every lane computes with the same operations, so each pixel is counted by exactly one
// lane.  Same samples, weights and bins as descriptor_fast (relaxed order and transcendentals):
// L2 ~1e-6 from the oracle; descriptor_one remains the bit-exact mode.
constexpr int kDualWords = 50 * 33;   // reduction words per wave
#ifndef SGK_DUAL_REF
#define SGK_DUAL_REF 1   // cell weights from the reference's rounded cell centres
#endif
// One wave per feature for every feature count.  Two-wave forms for few features (a single
// image) were measured in round 4: splitting each dual cell's rows between the
// pair (C2 30.9 vs 41 us) changes the sums' order, so a batch's descriptors no longer equalled a
// single image's; the bit-identical forms lost -- the pair splitting the bins 49.3 us (both waves
// walk every row), the one-wave kernel walking the pair's row groups in turn 1.786-1.80 vs
// 1.725-1.74 ms per 128 x 1080p step.
#ifndef SGK_DUAL_WPE
#define SGK_DUAL_WPE 4   // waves per SIMD the allocation must allow: 4 = <= 128 VGPRs, no spills (132 free)
#endif
#if SGK_DUAL_WPE
#define SGK_DUAL_ATTR __attribute__((amdgpu_waves_per_eu(SGK_DUAL_WPE)))
#else
#define SGK_DUAL_ATTR
#endif
__device__ __forceinline__ void descriptor_dual(uint32_t e, int lane, const float* __restrict__ pyr,
                                                const float4* __restrict__ feat,
                                                const int2* __restrict__ feat_info,
                                                const FeatureParams& fp, float* __restrict__ desc,
                                                uint32_t out, float* __restrict__ hist) {
    const float4 key = feat[e];
    const int2 in = feat_info[e];
    const int o = in.y / fp.d, j = in.y - o * fp.d;
    const OctaveDesc& od = fp.oct[o];
    const int W = od.wa, H = od.h;
    const float* g = pyr + od.gauss_off + (long long)(1 + j) * od.level_stride +
                     (long long)in.x * W * H;
    const float rpi = (float)(4.0 / 3.14159265358979323846);
    const float spt = fabs_(key.z * fp.window_factor);
    float s, c;
    sincos_(key.w, &s, &c);
    const float anglef = (double)key.w > 3.14159265358979323846
                             ? (float)((double)key.w - (2.0 * 3.14159265358979323846))
                             : key.w;
    const float cspt = c * spt, sspt = s * spt, crspt = c / spt, srspt = s / spt;
    // this lane's dual cell (a, b) and histogram copy; lanes 50..63 walk nothing
    const int q = lane >> 1, cp = lane & 1;
    const int a = q % 5, b = q / 5;
    const float fa = (float)a, fb = (float)b;
    // the dual cell's square: centre (a - 2, b - 2) cells from the keypoint, side spt
    const float fx = fa - 2.0f, fy = fb - 2.0f;
    const float cxi = key.x + fma_(cspt, fx, -(sspt * fy));
    const float cyi = key.y + fma_(sspt, fx, cspt * fy);
    const float hb = 0.5f * (fabs_(cspt) + fabs_(sspt)) + 0.01f;
    // pixel p has its sample at p + 0.5; rows and columns 1 .. H-2 / W-2 (the reference's box
    // clamp to [1.5, W - 1.5])
    // (clamped as floats first: a caller keypoint far outside the image must not saturate the
    // int conversion, whose y0 + 1 would wrap)
    const float fH = (float)H, fW = (float)W;
    const int y0 = (int)fmax_(1.0f, fmin_(fH, ceilf(cyi - hb - 0.5f)));
    int y1 = (int)fmin_(fH - 2.0f, fmax_(-1.0f, floor_(cyi + hb - 0.5f)));
    const int bx0 = (int)fmax_(1.0f, fmin_(fW, ceilf(cxi - hb - 0.5f)));
    const int bx1 = (int)fmin_(fW - 2.0f, fmax_(-1.0f, floor_(cxi + hb - 0.5f)));
    if (q >= 25 || !(spt > 0.0f)) y1 = y0 - 1;
    // row span: the columns whose u = dnx + 2.5 - a and v = dny + 2.5 - b can lie in [0, 1],
    // dnx = crspt dxk + srspt dyk, dny = crspt dyk - srspt dxk (dxk, dyk from the keypoint); the
    // 0.01-pixel margin absorbs rounding, the per-pixel test decides
    const bool use_c = fabs_(crspt) > 1e-4f / spt, use_s = fabs_(srspt) > 1e-4f / spt;
    const float icr = use_c ? 1.0f / crspt : 0.0f, isr = use_s ? 1.0f / srspt : 0.0f;
    auto row_span = [&](int py, int& lo, int& len) {
        const float dyk = ((float)py + 0.5f) - key.y;
        float l = -1e30f, h = 1e30f;
        if (use_c) {   // crspt dxk in [-Ku, 1 - Ku], Ku = srspt dyk + 2.5 - a
            const float p = -fma_(srspt, dyk, 2.5f - fa) * icr;
            l = fmax_(l, p + fmin_(0.0f, icr));
            h = fmin_(h, p + fmax_(0.0f, icr));
        }
        if (use_s) {   // -srspt dxk in [-Kv, 1 - Kv], Kv = crspt dyk + 2.5 - b
            const float p = fma_(crspt, dyk, 2.5f - fb) * isr;
            l = fmax_(l, p + fmin_(0.0f, -isr));
            h = fmin_(h, p + fmax_(0.0f, -isr));
        }
        const float xl = ceilf(l + key.x - 0.5f - 0.01f), xh = floor_(h + key.x - 0.5f + 0.01f);
        const int il = max(bx0, (int)fmax_(xl, -1.0f)), ih = min(bx1, (int)fmin_(xh, fW));
        lo = il;
        len = ih >= il ? ih - il + 1 : 0;
    };
    const float kexp = -0.125f * 1.44269504f;   // e^(-x/8) = 2^(kexp x)
    // lane-constant word offset of cell (a - 1, b - 1) in the 6 x 6 grid, own copy
#if SGK_DUAL_REF
    // The reference measures nx, ny from each cell's centre (ptx, pty), rounded to a float at
    // image-coordinate magnitude (ulp up to 1.2e-4 pixel at x ~ 2000; ProgramCU.cu:1044-1062).
    // Measured from the keypoint instead, the weights differ from the reference's by ~1e-5
    // (descriptor L2 up to 1.2e-5); so the 4 cells' weights use the reference's rounded centres:
    // nx = dnx - ox', ox' = crspt (ptx - x_key) + srspt (pty - y_key) (both differences exact),
    // and for the dual cell's left / right cells |nx| = nx / -nx, so that 1 - |nx| is one
    // subtraction (at the dual cell's edges the weights cross 0 by a rounding, continuously).
    float oxl[4], oyl[4];   // 1 -/+ ox', 1 -/+ oy' of cells (a-1,b-1), (a,b-1), (a-1,b), (a,b)
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const float ox = (float)(a - 1 + (k & 1)) - 1.5f, oy = (float)(b - 1 + (k >> 1)) - 1.5f;
        const float ptx = fma_(cspt, ox, -(sspt * oy)) + key.x;
        const float pty = fma_(cspt, oy, sspt * ox) + key.y;
        const float ex = ptx - key.x, ey = pty - key.y;
        const float oxp = fma_(crspt, ex, srspt * ey), oyp = fma_(crspt, ey, -(srspt * ex));
        oxl[k] = (k & 1) ? 1.0f - oxp : 1.0f + oxp;
        oyl[k] = (k >> 1) ? 1.0f - oyp : 1.0f + oyp;
    }
#endif
    // the lane's 4 cells x 8 bins, cells in pairs: acc[h][k] = bin k of cell slots 2h, 2h + 1
    // (slot 0: cell (a-1, b-1), 1: (a, b-1), 2: (a-1, b), 3: (a, b)), so that each packed fma
    // takes one scalar tent weight and a pair of cell weights
    f2v acc[2][8];
#pragma unroll
    for (int h = 0; h < 2; h++)
#pragma unroll
        for (int k = 0; k < 8; k++) acc[h][k] = f2v{0.0f, 0.0f};
    // a pixel's angle: the relaxed atan2, and within 1e-5 rad of the reference's one binning
    // discontinuity (theta rounding to 8.0 is dropped) the oracle's atan2 (descriptor_fast's
    // rule); the exact form is evaluated in one shared loop for the strip's flagged pixels (rare)
    auto pixel = [&](float dxk, float sdy, float cdy, float gx, float gy, bool valid) {
        const float m2 = fma_(gx, gx, gy * gy);
        // the relaxed atan2, and within 1e-5 rad of the reference's one binning discontinuity
        // (theta rounding to 8.0 is dropped) the oracle's atan2 (descriptor_fast's rule; rare)
        float rot = atan2_relaxed(gy, gx);
        const float dd = fabs_(anglef - rot);
        if (dd < 1e-5f || dd > 6.2831753f) rot = atan2_(gy, gx);
        rot = m2 == 0.0f ? 0.0f : rot;
        const float dnx = fma_(crspt, dxk, sdy);          // sdy = srspt dyk
        const float dny = fma_(-srspt, dxk, cdy);         // cdy = crspt dyk
        const float t = dnx + 2.5f, tv = dny + 2.5f;
        const float ft = floor_(t), fv = floor_(tv);
        const float u = t - ft, v = tv - fv;
        const float m = 0.5f * __builtin_amdgcn_sqrtf(m2);
        const float w = m * __builtin_amdgcn_exp2f(kexp * fma_(dnx, dnx, dny * dny));
        float theta = (anglef - rot) * rpi;
        if (theta < 0) theta += 8.0f;
        // theta outside [0, 8) (a caller orientation far outside (-pi, pi]) adds to no bin, as the
        // reference's k == fidx test; it would also index outside the histogram
        const bool take = valid && ft == fa && fv == fb && theta >= 0.0f && theta < 8.0f;
        // branch-free: a pixel not taken adds fma(tent, 0, acc) = acc (its theta replaced by 0 so
        // that no tent is NaN)
        const float wt = take ? w : 0.0f;
        const float th = take ? theta : 0.0f;
#if SGK_DUAL_REF
        (void)u; (void)v;
        const f2v cpa = wt * (f2v{oxl[0], oxl[1]} + f2v{-dnx, dnx}) * (f2v{oyl[0], oyl[1]} - dny);
        const f2v cpb = wt * (f2v{oxl[2], oxl[3]} + f2v{-dnx, dnx}) * (f2v{oyl[2], oyl[3]} + dny);
#else
        const f2v xu = f2v{1.0f - u, u};
        const float wv1 = wt * v, wv0 = wt - wv1;                    // w (1 - v), w v
        const f2v cpa = wv0 * xu, cpb = wv1 * xu;
#endif
        // tent weights max(0, 1 - |theta - k|), bin 0 also taking the wrap of bin 8
        // (ProgramCU.cu:1094), as descriptor_fast; then the outer product with the cell weights
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const float tk = k == 0 ? __builtin_amdgcn_fmed3f(fmax_(1.0f - th, th - 7.0f), 0.0f, 1.0f)
                                    : __builtin_amdgcn_fmed3f(1.0f - fabs_(th - (float)k), 0.0f, 1.0f);
            acc[0][k] = pk_fma(cpa, tk, acc[0][k]);
            acc[1][k] = pk_fma(cpb, tk, acc[1][k]);
        }
    };
    // walk: rows y0 + cp, y0 + cp + 2, ...; each row's span in strips of 4 pixels whose gradient
    // neighbours come from 4 vector loads (as descriptor_fast), the next strip's loads issued
    // before the current strip's pixels
    const char* gb = reinterpret_cast<const char*>(g);
    typedef float f4v __attribute__((ext_vector_type(4)));
    auto ld4 = [&](uint32_t byte) { return *reinterpret_cast<const f4v*>(gb + byte); };
    constexpr int RSTEP = 2;   // lane cp walks rows y0 + cp, y0 + cp + 2, ...
    int r = 0, lo = 0, len = 0, cx = 0;
    auto next_row = [&]() {   // advance r (by RSTEP) to the next row with a nonempty span
#pragma clang loop vectorize(disable) interleave(disable) unroll(disable)
        for (; r <= y1; r += RSTEP) {
            row_span(r, lo, len);
            if (len > 0) break;
        }
        cx = lo;
    };
    f4v na, nb, nu, nd;
    uint32_t npo = 4u * (uint32_t)(W + 1);   // row 1, column 1 when nothing is left (in-plane)
    auto fetch = [&]() {
        if (r <= y1) npo = 4u * (uint32_t)(r * W + cx);
        na = ld4(npo - 4u);            // x-1 .. x+2
        nb = ld4(npo + 4u);            // x+1 .. x+4
        nu = ld4(npo - 4u * W);        // row y-1, x .. x+3
        nd = ld4(npo + 4u * W);        // row y+1, x .. x+3
    };
    auto walk = [&](int r0) {
        r = r0;
        next_row();
        fetch();
        while (r <= y1) {
            const f4v gx = nb - na, gy = nd - nu;   // the strip's gradients (dx, dy per pixel)
            const float dyk = ((float)r + 0.5f) - key.y;
            const float sdy = srspt * dyk, cdy = crspt * dyk;
            const int nv = lo + len - cx;
            const float xc = (float)cx + 0.5f;   // (xc + i) - x_key: the same value in every lane
            cx += 4;
            if (cx >= lo + len) {
                r += RSTEP;
                next_row();
            }
            fetch();
            // one pixel at a time (sched_barrier): four interleaved took ~150 VGPRs
            pixel((xc) - key.x, sdy, cdy, gx.x, gy.x, true);
            __builtin_amdgcn_sched_barrier(0);
            pixel((xc + 1.0f) - key.x, sdy, cdy, gx.y, gy.y, nv > 1);
            __builtin_amdgcn_sched_barrier(0);
            pixel((xc + 2.0f) - key.x, sdy, cdy, gx.z, gy.z, nv > 2);
            __builtin_amdgcn_sched_barrier(0);
            pixel((xc + 3.0f) - key.x, sdy, cdy, gx.w, gy.w, nv > 3);
        }
    };
    // reduction: lanes 0..49 store their 32 bins ([lane][slot][bin], stride 33 floats against
    // bank conflicts); lane L then sums bins 2 sub, 2 sub + 1 of cell L >> 2 (descriptor_fast's
    // output layout) over the 4 dual cells x 2 lanes that hold that cell
    auto store_bins = [&]() {
        if (q < 25) {
            float* my = hist + lane * 33;
#pragma unroll
            for (int h = 0; h < 2; h++)
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    my[8 * (2 * h) + k] = acc[h][k].x;
                    my[8 * (2 * h + 1) + k] = acc[h][k].y;
                }
        }
        asm volatile("" ::: "memory");
    };
    const int cell = lane >> 2, sub = lane & 3;
    const int ix = cell & 3, iy = cell >> 2;
    float b0 = 0.0f, b1 = 0.0f;
    auto add_region = [&](const float* reg) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            // slot k of dual cell (ix + 1 - (k & 1), iy + 1 - (k >> 1)) is this cell
            const int dq = (iy + 1 - (k >> 1)) * 5 + ix + 1 - (k & 1);
#pragma unroll
            for (int c2 = 0; c2 < 2; c2++) {
                const float* src = reg + (2 * dq + c2) * 33 + 8 * k + 2 * sub;
                b0 += src[0];
                b1 += src[1];
            }
        }
        asm volatile("" ::: "memory");
    };
    walk(y0 + cp);
    store_bins();
    add_region(hist);
    if (fp.normalize) {
        float sn = fma_(b0, b0, b1 * b1);
#pragma unroll
        for (int k = 32; k >= 1; k >>= 1) sn += __shfl_xor(sn, k, 64);
        const float n1 = __builtin_amdgcn_rsqf(sn);
        b0 = fmin_(0.2f, b0 * n1);
        b1 = fmin_(0.2f, b1 * n1);
        sn = fma_(b0, b0, b1 * b1);
#pragma unroll
        for (int k = 32; k >= 1; k >>= 1) sn += __shfl_xor(sn, k, 64);
        const float n2 = __builtin_amdgcn_rsqf(sn);
        b0 *= n2;
        b1 *= n2;
    }
    *reinterpret_cast<float2*>(desc + (size_t)out * 128 + cell * 8 + sub * 2) = make_float2(b0, b1);
}

// One wave per feature (grid-stride), each wave with its own LDS histogram.
__global__ __launch_bounds__(256) SGK_DUAL_ATTR void k_descriptor_dual(const float* __restrict__ pyr,
                                                         const float4* __restrict__ feat,
                                                         const int2* __restrict__ feat_info,
                                                         const uint32_t* __restrict__ n_feat_dev,
                                                         const FeatureParams fp,
                                                         float* __restrict__ desc,
                                                         const int* __restrict__ out_index) {
    __shared__ float s_hist[4][kDualWords];
    const int lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float* hist = s_hist[wave];
    const uint32_t n = *n_feat_dev;
    for (uint32_t e = blockIdx.x * 4 + wave; e < n; e += gridDim.x * 4)
        descriptor_dual(e, lane, pyr, feat, feat_info, fp, desc,
                           out_index ? (uint32_t)out_index[e] : e, hist);
}

// ------------------------------------------------------------------------------------------
// Flat pixel-parallel descriptor (round 5, the shipped default for detected features).  The
// dual-cell kernel above gives every lane one dual cell and its own register histogram: 50 of 64
// lanes walk (lanes 50..63 idle), each lane's 4-pixel strips run past its row spans (masked
// pixels evaluated), and its gradient loads are 16-B gathers scattered over 25 cells.  Here the
// window's pixels are enumerated row-major over the rotated 5 x 5-cell square's row spans and
// dealt to the 64 lanes in turn (pixel p -> lane p mod 64): every lane busy, no masked tails,
// neighbouring lanes on neighbouring pixels (coalesced loads).  A pixel's dual cell (a, b) and
// its weights are those of descriptor_dual (the same dnx, dny, the reference's rounded cell
// centres, ProgramCU.cu:1044-1094, from a 6 x 6 per-feature table), its 4 cells x 2 orientation
// bins are 8 no-return 64-bit integer LDS adds (ds_add_u64 of a fixed-point word, to_fix32) into
// the wave's histogram, kept in kFlatCopies copies (lane mod kFlatCopies) against same-address
// serialisation and summed at the end.  Integer sums do not depend on their order, so a
// feature's descriptor does not depend on the batch around it or on how its pixels are split
// over waves (k_descriptor_wide); against the exact kernel the sums differ by the float order
// (L2 ~1e-6, tests/test_gpu_parity.py::test_shipped_descriptor_vs_exact).
#ifndef SGK_FLAT_COPIES
#define SGK_FLAT_COPIES 4
#endif
constexpr int kFlatCopies = SGK_FLAT_COPIES;
static_assert(kFlatCopies >= 1 && kFlatCopies <= 32 && (kFlatCopies & (kFlatCopies - 1)) == 0,
              "histogram copies");
// [4 x 4 cells][8 bins][copies] 64-bit words, a (cell, bin)'s copies kFlatStride words apart from
// the next's.  Measured per 128 x 1080p step (tests/diag/r05m.sh): 4 copies 1.51 ms, 1 / 2 / 8 /
// 16 copies 2.83 / 1.91 / 2.07 / 3.79 ms; a padded stride (copies + 1) 1.68 ms
#ifndef SGK_FLAT_PAD
#define SGK_FLAT_PAD 0
#endif
constexpr int kFlatStride = kFlatCopies + SGK_FLAT_PAD;
constexpr int kFlatHist = 16 * 8 * kFlatStride;
constexpr int kFlatRows = 64;                      // window rows per chunk (one per lane)
constexpr int kFlatWords = 2 * kFlatHist + 144;

// A contribution as a 64-bit fixed-point word, 32 fraction bits (two's complement; |v| < 2^31):
// the integer part by floor, the fraction (exact in float) scaled by 2^32 and truncated (error <
// 2^-32).  LDS integer adds are full rate where float adds (ds_add_f32) serialise their lanes
// (~4 cycles per lane, 7.8 ms per 128 x 1080p step against 1.37 with integer adds,
// tests/diag/r05l.sh), and integer sums do not depend on their order.
typedef __attribute__((address_space(3))) unsigned long long lds_u64;
typedef __attribute__((address_space(3))) uint32_t lds_u32;

// 1: features whose window cannot overflow it (unit-range input, <= kNarrowPix window pixels)
// sum their contributions as 32-bit fixed point (20 fraction bits, ds_add_u32: half the LDS
// traffic, 2 VALU per conversion instead of ~6) -- A/B build switch; 0: 64-bit for all
#ifndef SGK_FLAT_U32
#define SGK_FLAT_U32 0
#endif
// a contribution is <= 0.75 on unit-range images (m <= 0.5 sqrt(2), every weight <= 1 + rounding)
// and each pixel adds at most its own contribution to a bin: window pixels * 0.75 < 2^12
constexpr float kNarrowPix = 5000.0f;
__device__ __forceinline__ uint32_t to_fix20(float v) {   // v >= 0
    return (uint32_t)fma_(v, 1048576.0f, 0.5f);
}

// 1: the gradient's left / right neighbours from the neighbouring lanes' centre pixels by DPP
// (3 gathers per pixel; build variant); 0 (shipped): the 4 gathers -- the DPP form measured
// 1.492-1.493 against 1.425-1.430 ms per 128 x 1080p step (three alternating pairs, r06f): the
// shifts wait for the centre load, and the row-end lanes' loads are exec-masked instructions of
// their own
#ifndef SGK_DESC_DPP_NB
#define SGK_DESC_DPP_NB 0
#endif

__device__ __forceinline__ unsigned long long to_fix32(float v) {
    const float fl = floor_(v);
    const uint32_t lo = (uint32_t)((v - fl) * 4294967296.0f);
    return ((unsigned long long)(uint32_t)(int)fl << 32) | lo;
}

// Inclusive wave scan by DPP (row_shr 1 / 2 / 4 / 8 within each row of 16 lanes, then
// row_bcast:15 and row_bcast:31 carry the row totals into the rows above): 6 VALU with DPP
// operands instead of 6 ds_bpermute round trips through the LDS crossbar.
__device__ __forceinline__ int wave_incl_scan_dpp(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15 (rows 1, 3)
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31 (rows 2, 3)
    return v;
}

// Sum over the wave, in every lane: DPP within each row of 16 (quad_perm swaps, row_ror 4 / 8),
// then the four row sums read as scalars (v_readlane) and added in row order.
__device__ __forceinline__ float wave_sum_dpp(float v) {
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xb1, 0xf, 0xf, false));  // quad_perm [1,0,3,2]
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4e, 0xf, 0xf, false));  // quad_perm [2,3,0,1]
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xf, 0xf, false)); // row_ror:4
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, false)); // row_ror:8
    const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
    const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
    const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
    return (r0 + r1) + (r2 + r3);
}

__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) {
        const int u = __shfl_up(v, k, 64);
        if (lane >= k) v += u;
    }
    return v;
}

// the window's half side hb (feature frame: the rotated 5 x 5-cell square) -- flat_accumulate's
__device__ __forceinline__ float flat_half_box(const float4 key, const FeatureParams& fp) {
    const float spt = fabs_(key.z * fp.window_factor);
    float s, c;
    sincos_(key.w, &s, &c);
    return 2.5f * (fabs_(c * spt) + fabs_(s * spt)) + 0.01f;
}
// 32-bit sums for this feature (SGK_FLAT_U32, unit-range input, a window that cannot overflow)
__device__ __forceinline__ bool flat_narrow(const FeatureParams& fp, float hb) {
    return SGK_FLAT_U32 && fp.unit_input && (2.0f * hb + 2.0f) * (2.0f * hb + 2.0f) <= kNarrowPix;
}

// The accumulation of feature e's window into the histogram at sh (kFlatWords floats): wave wv
// of nwv takes the window's 64-pixel steps wv, wv + nwv, ... (every step when nwv = 1).
__device__ __forceinline__ void flat_accumulate(uint32_t e, int lane, const float* __restrict__ pyr,
                                                const float4* __restrict__ feat,
                                                const int2* __restrict__ feat_info,
                                                const FeatureParams& fp, float* __restrict__ sh,
                                                int wv, int nwv) {
    // the histogram as an LDS-space pointer, stated: its adds can only be ds_add_u64 (an LDS
    // offset outside the allocation is dropped by the LDS), never flat atomics through a generic
    // address, which the compiler would have to fall back to if the LDS origin of `sh` were lost
    // (round 5's fi64 variant faulted with an aperture violation)
    lds_u64* hist = (lds_u64*)sh;   // kFlatHist
    // 36: (1 + ox', 1 - ox', 1 + oy', 1 - oy') of cell (i, j)
    float4* ctab = reinterpret_cast<float4*>(sh + 2 * kFlatHist);
    const float4 key = feat[e];
    const int2 in = feat_info[e];
    const int o = in.y / fp.d, j = in.y - o * fp.d;
    const OctaveDesc& od = fp.oct[o];
    const int W = od.wa, H = od.h;
    const float* g = pyr + od.gauss_off + (long long)(1 + j) * od.level_stride +
                     (long long)in.x * W * H;
    const float rpi = (float)(4.0 / 3.14159265358979323846);
    const float spt = fabs_(key.z * fp.window_factor);
    float s, c;
    sincos_(key.w, &s, &c);
    const float anglef = (double)key.w > 3.14159265358979323846
                             ? (float)((double)key.w - (2.0 * 3.14159265358979323846))
                             : key.w;
    const float cspt = c * spt, sspt = s * spt, crspt = c / spt, srspt = s / spt;
    // the histogram (every copy) to zero; the cell centre table: cell (i, j), i, j = -1 .. 4 at
    // (j + 1) * 6 + i + 1 -- the reference's rounded centre, measured in the feature frame
    // (descriptor_dual's oxl / oyl)
#pragma unroll
    for (int i = lane; i < kFlatHist / 2; i += 64)
        reinterpret_cast<float4*>(sh)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (lane < 36) {
        const float ox = (float)(lane % 6 - 1) - 1.5f, oy = (float)(lane / 6 - 1) - 1.5f;
        const float ptx = fma_(cspt, ox, -(sspt * oy)) + key.x;
        const float pty = fma_(cspt, oy, sspt * ox) + key.y;
        const float ex = ptx - key.x, ey = pty - key.y;
        const float oxp = fma_(crspt, ex, srspt * ey), oyp = fma_(crspt, ey, -(srspt * ex));
        ctab[lane] = make_float4(1.0f + oxp, 1.0f - oxp, 1.0f + oyp, 1.0f - oyp);
    }
    // the window's bounding rows and columns: the 5 x 5-cell square (side 5 spt, rotated) around
    // the keypoint, clamped to rows / columns 1 .. H-2 / W-2 (the reference's [1.5, W - 1.5] box)
    const float hb = 2.5f * (fabs_(cspt) + fabs_(sspt)) + 0.01f;
    const float fH = (float)H, fW = (float)W;
    const int y0 = (int)fmax_(1.0f, fmin_(fH, ceilf(key.y - hb - 0.5f)));
    int y1 = (int)fmin_(fH - 2.0f, fmax_(-1.0f, floor_(key.y + hb - 0.5f)));
    const int bx0 = (int)fmax_(1.0f, fmin_(fW, ceilf(key.x - hb - 0.5f)));
    const int bx1 = (int)fmin_(fW - 2.0f, fmax_(-1.0f, floor_(key.x + hb - 0.5f)));
    const bool narrow = flat_narrow(fp, hb);
    lds_u32* hist32 = (lds_u32*)sh;
    if (!(spt > 0.0f)) y1 = y0 - 1;
    // a row's span: the columns whose dnx, dny can lie in [-2.5, 2.5) (0.05-pixel margin; the
    // per-pixel test decides)
    const bool use_c = fabs_(crspt) > 1e-4f / spt, use_s = fabs_(srspt) > 1e-4f / spt;
    const float icr = use_c ? 1.0f / crspt : 0.0f, isr = use_s ? 1.0f / srspt : 0.0f;
    const float kexp = -0.125f * 1.44269504f;   // e^(-x/8) = 2^(kexp x)
    const int copy = lane & (kFlatCopies - 1);
    asm volatile("" ::: "memory");
    for (int rb = y0; rb <= y1; rb += kFlatRows) {
        // this chunk's rows: lane L holds row rb + L's first column and first pixel index
        int lo = 0, len = 0;
        {
            const int py = rb + lane;
            if (py <= y1) {
                const float dyk = ((float)py + 0.5f) - key.y;
                float l = -1e30f, h = 1e30f;
                if (use_c) {   // crspt dxk in [-2.5 - srspt dyk, 2.5 - srspt dyk]
                    const float sd = srspt * dyk;
                    const float p0 = (-2.5f - sd) * icr, p1 = (2.5f - sd) * icr;
                    l = fmax_(l, fmin_(p0, p1));
                    h = fmin_(h, fmax_(p0, p1));
                }
                if (use_s) {   // -srspt dxk in [-2.5 - crspt dyk, 2.5 - crspt dyk]
                    const float cd = crspt * dyk;
                    const float p0 = (2.5f + cd) * isr, p1 = -(2.5f - cd) * isr;
                    l = fmax_(l, fmin_(p0, p1));
                    h = fmin_(h, fmax_(p0, p1));
                }
                const float xl = ceilf(l + key.x - 0.5f - 0.05f), xh = floor_(h + key.x - 0.5f + 0.05f);
                const int il = max(bx0, (int)fmax_(xl, -1.0f)), ih = min(bx1, (int)fmin_(xh, fW));
                lo = il;
                len = ih >= il ? ih - il + 1 : 0;
            }
        }
        const int incl = wave_incl_scan_dpp(len);
        const int rs = incl - len;                                   // row L's first pixel index
        const int total = __builtin_amdgcn_readlane(incl, kFlatRows - 1);
        int rcur = 0;   // a row at or before pixel `base`'s (uniform)
        for (int base = 64 * wv; base < total; base += 64 * nwv) {
            const int p = base + lane;
            const bool valid = p < total;
            // pixel p's row: rcur + the rows after it starting at or before p (their starts read
            // as uniform values; the loop stops at the first row past this step's pixels)
            int r = rcur;
            for (int k = rcur + 1; k < kFlatRows; k++) {
                const int sk = __builtin_amdgcn_readlane(rs, k);
                if (sk > base + 63 || sk >= total) break;
                r += p >= sk ? 1 : 0;
            }
            rcur = __builtin_amdgcn_readlane(r, 63);
            const int y = rb + r;
            // (the shuffles with every lane active: a lane outside the valid ones may be the
            // source; the asm keeps the compiler from moving them under the valid test)
            const int rsr = __shfl(rs, r, 64);        // row r's first pixel
            const int rnx = __shfl(incl, r, 64);      // the next row's first pixel
            int xr = __shfl(lo, r, 64) + (p - rsr);
            asm volatile("" : "+v"(xr));
            const int x = valid ? xr : bx0;
            const int yc = valid ? y : y0;
            // 32-bit byte offsets from the level image's base (an image plane is < 4 GB)
            const char* gp = reinterpret_cast<const char*>(g) + 4u * (uint32_t)(yc * W + x);
            const uint32_t W4 = 4u * (uint32_t)W;
#if SGK_DESC_DPP_NB
            // the gradient's 4 neighbours: the row above and below are gathered, the left and right
            // ones are the neighbouring lanes' centre pixels (lanes hold consecutive pixels of a
            // row: p - 1 and p + 1) taken by DPP wave shifts; only the lanes at a row's or the
            // step's ends load them -- 3 gathers per pixel instead of 4, the same values
            // (every load is issued before the shifts wait for the centre: one round trip)
            const bool from_r = valid && lane < 63 && p + 1 < rnx;   // lane + 1 holds x + 1
            const bool from_l = valid && lane > 0 && p > rsr;        // lane - 1 holds x - 1
            const float cen = *reinterpret_cast<const float*>(gp);
            const float gup = *reinterpret_cast<const float*>(gp - W4);
            const float gdn = *reinterpret_cast<const float*>(gp + W4);
            float lrt = 0.0f, llt = 0.0f;
            if (!from_r) lrt = *reinterpret_cast<const float*>(gp + 4);
            if (!from_l) llt = *reinterpret_cast<const float*>(gp - 4);
            const float srt = __int_as_float(__builtin_amdgcn_update_dpp(
                0, __float_as_int(cen), 0x130, 0xf, 0xf, false));   // wave_shl:1: lane + 1
            const float slt = __int_as_float(__builtin_amdgcn_update_dpp(
                0, __float_as_int(cen), 0x138, 0xf, 0xf, false));   // wave_shr:1: lane - 1
            const float gx = (from_r ? srt : lrt) - (from_l ? slt : llt);
            const float gy = gdn - gup;
#else
            (void)rnx;
            const float gx = *reinterpret_cast<const float*>(gp + 4) - *reinterpret_cast<const float*>(gp - 4);
            const float gy = *reinterpret_cast<const float*>(gp + W4) - *reinterpret_cast<const float*>(gp - W4);
#endif
            const float m2 = fma_(gx, gx, gy * gy);
            float rot = atan2_relaxed(gy, gx);
            const float dd = fabs_(anglef - rot);
            if (dd < 1e-5f || dd > 6.2831753f) rot = atan2_(gy, gx);
            rot = m2 == 0.0f ? 0.0f : rot;
            const float dxk = ((float)x + 0.5f) - key.x;
            const float dyk = ((float)yc + 0.5f) - key.y;
            const float dnx = fma_(crspt, dxk, srspt * dyk);
            const float dny = fma_(-srspt, dxk, crspt * dyk);
            const float ft = floor_(dnx + 2.5f), fv = floor_(dny + 2.5f);
            const float m = 0.5f * __builtin_amdgcn_sqrtf(m2);
            const float w = m * __builtin_amdgcn_exp2f(kexp * fma_(dnx, dnx, dny * dny));
            float theta = (anglef - rot) * rpi;
            if (theta < 0) theta += 8.0f;
            const bool take = valid && ft >= 0.0f && ft <= 4.0f && fv >= 0.0f && fv <= 4.0f &&
                              theta >= 0.0f && theta < 8.0f;
            if (take) {
                const int a = (int)ft, b = (int)fv;
                const int c00 = b * 6 + a;                 // cell (a - 1, b - 1) in the 6 x 6 table
                const float4 t0 = ctab[c00], t1 = ctab[c00 + 1], t2 = ctab[c00 + 6], t3 = ctab[c00 + 7];
                const float w0 = (w * (t0.x - dnx)) * (t0.z - dny);
                const float w1 = (w * (t1.y + dnx)) * (t1.z - dny);
                const float w2 = (w * (t2.x - dnx)) * (t2.w + dny);
                const float w3 = (w * (t3.y + dnx)) * (t3.w + dny);
                // orientation bins: floor(theta) and the next (8 -> 0), tent weights as
                // descriptor_dual's max(0, 1 - |theta - k|)
                const int b0 = min((int)theta, 7), b1 = (b0 + 1) & 7;
                const float tk0 = 1.0f - (theta - (float)b0);
                const float tk1 = b0 == 7 ? theta - 7.0f : 1.0f - ((float)(b0 + 1) - theta);
                // the 4 cells (a - 1 + dx, b - 1 + dy); cells outside 0 .. 3 (the dual cells on the
                // window's border) are not descriptor cells and take nothing
                const bool x0in = a >= 1, x1in = a <= 3, y0in = b >= 1, y1in = b <= 3;
                lds_u64* hp = hist + (((b - 1) * 4 + (a - 1)) * 8) * kFlatStride + copy;
                const int o0 = b0 * kFlatStride, o1 = b1 * kFlatStride;
                constexpr int CX = 8 * kFlatStride, CY = 4 * 8 * kFlatStride;
                const int hoff = (((b - 1) * 4 + (a - 1)) * 8) * kFlatStride + copy;
                auto add2 = [&](bool in, int off, float wc) {
                    if (in && narrow) {
                        __hip_atomic_fetch_add(hist32 + hoff + off + o0, to_fix20(wc * tk0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        __hip_atomic_fetch_add(hist32 + hoff + off + o1, to_fix20(wc * tk1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    } else if (in) {
                        __hip_atomic_fetch_add(hp + off + o0, to_fix32(wc * tk0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        __hip_atomic_fetch_add(hp + off + o1, to_fix32(wc * tk1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                };
                add2(x0in && y0in, 0, w0);
                add2(x1in && y0in, CX, w1);
                add2(x0in && y1in, CY, w2);
                add2(x1in && y1in, CY + CX, w3);
            }
        }
        asm volatile("" ::: "memory");
    }
}

// The descriptor from nh histograms (kFlatWords floats apart from sh on): cell (ix, iy) =
// lane >> 2, bins 2 sub, 2 sub + 1, every copy of every histogram summed as 64-bit integers --
// the same totals however the window's pixels were split over waves and copies -- then
// normalised (NormalizeDescriptor, ProgramCU.cu:1173-1208) and stored as row `out`.
__device__ __forceinline__ void flat_finish(int lane, const FeatureParams& fp,
                                            float* __restrict__ desc, uint32_t out,
                                            const float* __restrict__ sh, int nh, bool narrow,
                                            float* __restrict__ hdesc = nullptr) {
    const int cell = lane >> 2, sub = lane & 3;
    const int ix = cell & 3, iy = cell >> 2;
    unsigned long long s0 = 0, s1 = 0;
    const int hi = ((iy * 4 + ix) * 8 + 2 * sub) * kFlatStride;
    for (int w = 0; w < nh; w++) {
        if (narrow) {
            const lds_u32* hc = (const lds_u32*)(sh + w * kFlatWords) + hi;
#pragma unroll
            for (int k = 0; k < kFlatCopies; k++) {
                s0 += hc[k];
                s1 += hc[kFlatStride + k];
            }
        } else {
            const lds_u64* hc = (const lds_u64*)(sh + w * kFlatWords) + hi;
#pragma unroll
            for (int k = 0; k < kFlatCopies; k++) {
                s0 += hc[k];
                s1 += hc[kFlatStride + k];
            }
        }
    }
    const double scale = narrow ? 0x1p-20 : 0x1p-32;
    float b0 = (float)((double)(long long)s0 * scale), b1 = (float)((double)(long long)s1 * scale);
    asm volatile("" ::: "memory");
    if (fp.normalize) {
        float sn = wave_sum_dpp(fma_(b0, b0, b1 * b1));
        const float n1 = __builtin_amdgcn_rsqf(sn);
        b0 = fmin_(0.2f, b0 * n1);
        b1 = fmin_(0.2f, b1 * n1);
        sn = wave_sum_dpp(fma_(b0, b0, b1 * b1));
        const float n2 = __builtin_amdgcn_rsqf(sn);
        b0 *= n2;
        b1 *= n2;
    }
    *reinterpret_cast<float2*>(desc + (size_t)out * 128 + cell * 8 + sub * 2) = make_float2(b0, b1);
    if (hdesc)   // the row also to page-locked host memory (sgpu_set_host_output)
        *reinterpret_cast<float2*>(hdesc + (size_t)out * 128 + cell * 8 + sub * 2) = make_float2(b0, b1);
}

__device__ __forceinline__ void descriptor_flat(uint32_t e, int lane, const float* __restrict__ pyr,
                                                const float4* __restrict__ feat,
                                                const int2* __restrict__ feat_info,
                                                const FeatureParams& fp, float* __restrict__ desc,
                                                uint32_t out, float* __restrict__ sh) {
    flat_accumulate(e, lane, pyr, feat, feat_info, fp, sh, 0, 1);
    flat_finish(lane, fp, desc, out, sh, 1, flat_narrow(fp, flat_half_box(feat[e], fp)));
}

// waves per SIMD the allocation must allow: 8 (64 VGPRs, no spills): 1.448-1.451 ms per
// 128 x 1080p step against 1.520-1.524 at the compiler's 70 VGPRs / 7 waves (alternating
// processes, tests/diag/r05r.sh); 0 leaves it to the compiler
#ifndef SGK_FLAT_WPE
#define SGK_FLAT_WPE 8
#endif
#if SGK_FLAT_WPE
#define SGK_FLAT_ATTR __attribute__((amdgpu_waves_per_eu(SGK_FLAT_WPE)))
#else
#define SGK_FLAT_ATTR
#endif
__global__ __launch_bounds__(256) SGK_FLAT_ATTR void k_descriptor_flat(const float* __restrict__ pyr,
                                                         const float4* __restrict__ feat,
                                                         const int2* __restrict__ feat_info,
                                                         const uint32_t* __restrict__ n_feat_dev,
                                                         const FeatureParams fp,
                                                         float* __restrict__ desc,
                                                         const int* __restrict__ out_index) {
    __shared__ __attribute__((aligned(16))) float s_flat[4][kFlatWords];
    const int lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t n = *n_feat_dev;
    for (uint32_t e = blockIdx.x * 4 + wave; e < n; e += gridDim.x * 4)
        descriptor_flat(e, lane, pyr, feat, feat_info, fp, desc,
                        out_index ? (uint32_t)out_index[e] : e, s_flat[wave]);
}

// A workgroup of NWV (4) waves per feature, for few features (one image: ~1,500 features are ~1.5
// waves per SIMD under one wave each, and each wave walks its window alone).  The waves take every
// NWV-th 64-pixel step of the window into histograms of their own; wave 0 sums all of them.  The
// sums are integers, so the descriptor is k_descriptor_flat's bit for bit, in any batch.
template <int NWV>
__global__ __launch_bounds__(64 * NWV) SGK_FLAT_ATTR void k_descriptor_wide(const float* __restrict__ pyr,
                                                         const float4* __restrict__ feat,
                                                         const int2* __restrict__ feat_info,
                                                         const uint32_t* __restrict__ n_feat_dev,
                                                         const FeatureParams fp,
                                                         float* __restrict__ desc,
                                                         const int* __restrict__ out_index,
                                                         const HostCopy hc) {
    __shared__ __attribute__((aligned(16))) float s_flat[NWV][kFlatWords];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t n = *n_feat_dev;
    // host output (one image, sgpu_set_host_output): the count record, the first cap keys and
    // descriptors also go to page-locked host memory from here -- written over the host link
    // while the descriptors are computed, instead of by a k_copy_out launch after them
    if (hc.hrec && blockIdx.x == 0 && threadIdx.x < (unsigned)hc.rec_n) hc.hrec[threadIdx.x] = hc.rec[threadIdx.x];
    for (uint32_t e = blockIdx.x; e < n; e += gridDim.x) {   // uniform per workgroup
        flat_accumulate(e, lane, pyr, feat, feat_info, fp, s_flat[wave], wave, NWV);
        __syncthreads();
        const uint32_t out = out_index ? (uint32_t)out_index[e] : e;
        const bool to_host = hc.hkeys && out < hc.cap;
        if (wave == 0)
            flat_finish(lane, fp, desc, out, &s_flat[0][0], NWV,
                        flat_narrow(fp, flat_half_box(feat[e], fp)), to_host ? hc.hdesc : nullptr);
        else if (wave == 1 && lane == 0 && to_host)
            hc.hkeys[out] = hc.keys[e];
        __syncthreads();   // wave 0 has read every histogram before the next feature zeroes them
    }
}

// One wave per feature, grid-stride over the features (count read on the device).
// SGK_DESC_WPE: waves per SIMD the register allocation must allow (0: the compiler's choice, 91
// VGPRs = 5 waves; A/B knob)
#ifndef SGK_DESC_WPE
#define SGK_DESC_WPE 0
#endif
#if SGK_DESC_WPE
#define SGK_DESC_ATTR __attribute__((amdgpu_waves_per_eu(SGK_DESC_WPE)))
#else
#define SGK_DESC_ATTR
#endif
template <bool RECT>
__global__ __launch_bounds__(256) SGK_DESC_ATTR void k_descriptor_fast(const float* __restrict__ pyr,
                                                         const float4* __restrict__ feat,
                                                         const int2* __restrict__ feat_info,
                                                         const uint32_t* __restrict__ n_feat_dev,
                                                         const FeatureParams fp,
                                                         float* __restrict__ desc,
                                                         const int* __restrict__ out_index) {
    const int lane = threadIdx.x & 63;
    const uint32_t n = *n_feat_dev;
    // the feature index is wave-uniform: say so, so that the feature's record, level pointer and
    // geometry live in SGPRs and the gathers use the SGPR-base + 32-bit-offset form
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint32_t e = blockIdx.x * 4 + wave; e < n; e += gridDim.x * 4)
        descriptor_fast<RECT>(e, lane, pyr, feat, feat_info, fp, desc,
                              out_index ? (uint32_t)out_index[e] : e);
}

// One wave per feature, grid-stride over the features (count read on the device).
template <bool RECT>
__global__ __launch_bounds__(256) void k_descriptor(const float* __restrict__ pyr,
                                                    const float4* __restrict__ feat,
                                                    const int2* __restrict__ feat_info,
                                                    const uint32_t* __restrict__ n_feat_dev,
                                                    const FeatureParams fp,
                                                    float* __restrict__ desc,
                                                    const int* __restrict__ out_index) {
    const int lane = threadIdx.x & 63;
    const uint32_t n = *n_feat_dev;
    for (uint32_t e = blockIdx.x * 4 + (threadIdx.x >> 6); e < n; e += gridDim.x * 4)   // uniform per wave
        descriptor_one<RECT>(e, lane, pyr, feat, feat_info, fp, desc,
                             out_index ? (uint32_t)out_index[e] : e);
}

// Caller-supplied keypoints (SiftGPU::RunSIFT(num, keys, keys_have_orientation),
// SiftPyramid.cpp:83-89, 129-147, 167-177): feat holds the keypoint list in octave coordinates,
// grouped by level as GenerateFeatureListTex (PyramidCU.cpp:454-504) builds it.  The strongest
// orientation (ComputeOrientation_Kernel with existing_keypoint, ProgramCU.cu:830-833, 904)
// replaces feat.w, and the keys are rewritten in image coordinates at keys_out[index[e]]
// (DownloadKeypoints, PyramidCU.cpp:701-751).
__global__ __launch_bounds__(256) void k_orient_keys(const float* __restrict__ pyr,
                                                     float4* __restrict__ feat,
                                                     const int2* __restrict__ feat_info,
                                                     const int* __restrict__ index, int n,
                                                     const FeatureParams fp,
                                                     float4* __restrict__ keys_out) {
    __shared__ float s_vote[64 * 37];
    const int sub = threadIdx.x & 3, slot = threadIdx.x >> 2;
    float* vote_l = s_vote + slot * 37;
    const double twopi = 2.0 * 3.14159265358979323846;
    for (int e = blockIdx.x * 64 + slot; e < n; e += gridDim.x * 64) {   // uniform per quad
        const float4 k = feat[e];
        const int2 in = feat_info[e];
        const int o = in.y / fp.d, j = in.y - o * fp.d;
        const OctaveDesc& od = fp.oct[o];
        float angle = 0.0f;
        if (fp.num_orientation != 0) {
            const float* g = pyr + od.gauss_off + (long long)(1 + j) * od.level_stride +
                             (long long)in.x * od.wa * od.h;
            float vote[37];
            orientation_hist(g, od.wa, od.h, k.x, k.y, k.z, fp, sub, vote_l, vote);
            angle = strongest_orientation(vote);
        }
        if (sub == 0) {
            feat[e].w = angle;
            const float os = ldexpf(1.0f, o + fp.octave_min);
            keys_out[index[e]] = make_float4(os * (k.x - 0.5f) + fp.origin_offset,
                                             os * (k.y - 0.5f) + fp.origin_offset, os * k.z,
                                             (float)fmod(twopi - (double)angle, twopi));
        }
    }
}

// ------------------------------------------------------------------------------------------
// Feature-count limiting (-tc / -tc2 / -tc3), per image, on the level counts in octave-major
// order: the level skip of PyramidCU::GenerateFeatureList (PyramidCU.cpp:829-853; levels are
// visited coarsest first for -tc2, and a level is skipped once the running count exceeds the
// threshold) when list_stage, then SiftPyramid::LimitFeatureCount (SiftPyramid.cpp:219-260):
// -tc3 keeps the first levels until the threshold is reached, -tc / -tc2 drop the finest levels
// while the rest still exceeds it.
constexpr int kMaxLimitLevels = kMaxOctaves * 8;

__device__ void limit_levels(int* cnt, int nl, int T, int method, bool list_stage) {
    if (list_stage && method != 0) {
        int total = 0;
        for (int q = 0; q < nl; q++) {
            const int l = method == 1 ? nl - 1 - q : q;
            if (total > T) cnt[l] = 0;
            else total += cnt[l];
        }
    }
    int num = 0;
    for (int l = 0; l < nl; l++) num += cnt[l];
    if (method == 2) {
        int i = 0, kept = 0;
        for (; kept < T && i < nl; ++i) kept += cnt[i];
        for (; i < nl; ++i) cnt[i] = 0;
    } else {
        for (int i = 0; i < nl && num - cnt[i] > T; ++i) {
            num -= cnt[i];
            cnt[i] = 0;
        }
    }
}

__device__ __forceinline__ int level_of_row(const FeatureParams& fp, int r) {
    int o = 0;
    while (o + 1 < fp.n_octaves && fp.row_off[o + 1] <= r) o++;
    return o * fp.d + (r - fp.row_off[o]) / fp.oct[o].h;
}

// Stages 1-2 on the detected keypoints: the row counts of dropped levels are zeroed before the
// row scan, so their keypoints never enter the list.  One workgroup per image.
__global__ __launch_bounds__(256) void k_limit_rows(uint32_t* __restrict__ row_count,
                                                    const FeatureParams fp, int T, int method) {
    __shared__ int s_cnt[kMaxLimitLevels];
    const int nl = fp.n_octaves * fp.d;
    uint32_t* rc = row_count + (size_t)blockIdx.x * fp.rows_per_image;
    for (int l = threadIdx.x; l < nl; l += 256) s_cnt[l] = 0;
    __syncthreads();
    for (int r = threadIdx.x; r < fp.rows_per_image; r += 256) {
        const uint32_t v = rc[r];
        if (v) atomicAdd(&s_cnt[level_of_row(fp, r)], (int)v);
    }
    __syncthreads();
    if (threadIdx.x == 0) limit_levels(s_cnt, nl, T, method, true);
    __syncthreads();
    for (int r = threadIdx.x; r < fp.rows_per_image; r += 256)
        if (s_cnt[level_of_row(fp, r)] == 0) rc[r] = 0;
}

// Stage 3 (LimitFeatureCount(1) after ReshapeFeatureListCPU, SiftPyramid.cpp:152-160) on the
// oriented feature counts: the counts of dropped levels' keypoints are zeroed before the
// feature scan.  One workgroup per image.
__global__ __launch_bounds__(256) void k_limit_oriented(uint32_t* __restrict__ ocount,
                                                        const uint32_t* __restrict__ row_base,
                                                        const FeatureParams fp, int T, int method,
                                                        uint32_t cap) {
    __shared__ int s_cnt[kMaxLimitLevels];
    const int nl = fp.n_octaves * fp.d;
    const size_t r0 = (size_t)blockIdx.x * fp.rows_per_image;
    auto range = [&](int l, uint32_t& lo, uint32_t& hi) {
        const int o = l / fp.d, j = l - o * fp.d;
        const size_t first = r0 + fp.row_off[o] + (size_t)j * fp.oct[o].h;
        lo = min(row_base[first], cap);
        hi = min(row_base[first + fp.oct[o].h], cap);
    };
    for (int l = threadIdx.x; l < nl; l += 256) s_cnt[l] = 0;
    __syncthreads();
    for (int l = 0; l < nl; l++) {
        uint32_t lo, hi;
        range(l, lo, hi);
        int sum = 0;
        for (uint32_t f = lo + threadIdx.x; f < hi; f += 256) sum += (int)ocount[f];
        if (sum) atomicAdd(&s_cnt[l], sum);
    }
    __syncthreads();
    if (threadIdx.x == 0) limit_levels(s_cnt, nl, T, method, false);
    __syncthreads();
    for (int l = 0; l < nl; l++) {
        if (s_cnt[l] != 0) continue;
        uint32_t lo, hi;
        range(l, lo, hi);
        for (uint32_t f = lo + threadIdx.x; f < hi; f += 256) ocount[f] = 0;
    }
}


}  // namespace

// ------------------------------------------------------------------------------------------
hipError_t launch_gauss(const float* src, const uint8_t* src_u8, int src_stride,
                        long long src_img_stride, float* dst, long long dst_img_stride, int w,
                        int h, int fw, const Taps& taps, int batch, float* ds_dst, int ds_w,
                        int ds_h, long long ds_img_stride, hipStream_t stream, int wave_rows,
                        bool long_bands, const ZeroJob& zero) {
#define SGK_GAUSS(FW)                                                                       \
    case FW:                                                                                  \
        return gauss_dispatch<FW>(src, src_u8, src_stride, src_img_stride, dst, dst_img_stride, \
                                  w, h, taps, batch, ds_dst, ds_w, ds_h, ds_img_stride, stream, \
                                  wave_rows, long_bands, zero);
    switch (fw) {
        SGK_GAUSS(5) SGK_GAUSS(7) SGK_GAUSS(9) SGK_GAUSS(11) SGK_GAUSS(13) SGK_GAUSS(15)
        SGK_GAUSS(17) SGK_GAUSS(19) SGK_GAUSS(21) SGK_GAUSS(23) SGK_GAUSS(25) SGK_GAUSS(27)
        SGK_GAUSS(29) SGK_GAUSS(31) SGK_GAUSS(33)
        default: return hipErrorInvalidValue;
    }
#undef SGK_GAUSS
}

hipError_t launch_gauss_op(const LevelOp& op, hipStream_t stream, int wave_rows, bool long_bands) {
    return launch_gauss(op.src, op.src_u8, op.src_stride, op.src_img_stride, op.dst,
                        op.dst_img_stride, op.w, op.h, op.fw, op.taps, op.batch, op.ds_dst,
                        op.ds_w, op.ds_h, op.ds_img_stride, stream, wave_rows, long_bands, op.zero);
}

static bool diag_ok(const LevelOp& op) {
    return !op.src_u8 && !op.ds_dst && op.src && (op.src_stride % 4) == 0 &&
           (op.src_img_stride % 4) == 0 && (op.w % 4) == 0 && op.w >= 4 &&
           ((uintptr_t)op.src % 16) == 0 && !(op.zero.n[0] | op.zero.n[1] | op.zero.n[2]);
}

template <int FWA, int FWB>
static hipError_t gauss_diag_launch(const LevelOp& a, const LevelOp& b, hipStream_t stream,
                                    int wave_rows, bool long_bands) {
    const GaussWaveGrid ga = gauss_wave_grid(a.w, a.h, a.batch, wave_rows, 1, long_bands);
    const GaussWaveGrid gb = gauss_wave_grid(b.w, b.h, b.batch, wave_rows, 1, long_bands);
    const int nbA = (ga.total_waves + kGwWaves - 1) / kGwWaves;
    const int nbB = (gb.total_waves + kGwWaves - 1) / kGwWaves;
    const int nbBp = (nbB + 7) / 8 * 8;   // job A starts on XCD 0 (blocks are dealt round-robin)
    const GaussJob A{a.src, nullptr, a.src_stride, a.src_img_stride, a.dst, a.dst_img_stride, a.w,
                     a.h, a.taps, nullptr, 0, 0, 0, ga, ZeroJob{}};
    GaussJob B{b.src, nullptr, b.src_stride, b.src_img_stride, b.dst, b.dst_img_stride, b.w,
               b.h, b.taps, nullptr, 0, 0, 0, gb, ZeroJob{}};
    // the padding blocks of job B map to waves past its grid (gauss_lean_wave returns)
    B.gg.total_waves = gb.total_waves;
    hipLaunchKernelGGL((k_gauss_diag<FWA, FWB>), dim3((unsigned)(nbBp + nbA)), dim3(64 * kGwWaves),
                       0, stream, A, B, nbBp);
    return hipGetLastError();
}

hipError_t launch_gauss_two(const LevelOp& a, const LevelOp& b, hipStream_t stream, int wave_rows,
                            bool long_bands, int* launches) {
    if (launches) *launches = 1;
    if (wave_rows >= 0 && diag_ok(a) && diag_ok(b)) {
        // the default schedule's pairs (-d 3: levels 4 / 5 of octave o beside levels 1 / 2 of
        // octave o + 1); the larger job is A
        const bool swap = (long long)a.w * a.h * a.batch < (long long)b.w * b.h * b.batch;
        const LevelOp& big = swap ? b : a;
        const LevelOp& small = swap ? a : b;
#define SGK_DIAG(A, B) \
        if (big.fw == A && small.fw == B) return gauss_diag_launch<A, B>(big, small, stream, wave_rows, long_bands);
        SGK_DIAG(21, 11) SGK_DIAG(25, 13)
#undef SGK_DIAG
    }
    if (launches) *launches = 2;
    hipError_t e = launch_gauss_op(a, stream, wave_rows, long_bands);
    if (e != hipSuccess) return e;
    return launch_gauss_op(b, stream, wave_rows, long_bands);
}

hipError_t launch_color_to_gray(const uint8_t* src, int n, int w, int h, int stride,
                                int channels, bool bgr, float* dst, hipStream_t stream) {
    const int tw = w & ~3;
    if (n <= 0 || tw <= 0 || (channels != 3 && channels != 4) || stride < w * channels)
        return hipErrorInvalidValue;
    const dim3 grid((tw + 255) / 256, h, n);
#define SGK_COLOR(CH, B) \
    hipLaunchKernelGGL((k_color_gray<CH, B>), grid, dim3(256), 0, stream, src, tw, h, stride, dst)
    if (channels == 3 && !bgr) SGK_COLOR(3, false);
    else if (channels == 3) SGK_COLOR(3, true);
    else if (!bgr) SGK_COLOR(4, false);
    else SGK_COLOR(4, true);
#undef SGK_COLOR
    return hipGetLastError();
}

hipError_t launch_first_octave_input(const float* src, const uint8_t* src_u8, int stride,
                                     long long src_img_stride, int tw, int h, int fo, float* dst,
                                     int dw, int dh, long long dst_img_stride, int batch,
                                     hipStream_t stream) {
    if (fo > 0) {
        if (dw > (tw >> fo) + 3 || dh > (h >> fo)) return hipErrorInvalidValue;
        const dim3 grid((dw + 255) / 256, dh, batch);
        if (src_u8)
            hipLaunchKernelGGL(k_input_down<true>, grid, dim3(256), 0, stream, src, src_u8, stride,
                               src_img_stride, tw, h, fo, dst, dw, dh, dst_img_stride);
        else
            hipLaunchKernelGGL(k_input_down<false>, grid, dim3(256), 0, stream, src, src_u8,
                               stride, src_img_stride, tw, h, fo, dst, dw, dh, dst_img_stride);
    } else if (fo < 0) {
        const int s = -fo;
        if (s > 3 || dw != (tw << s) || dh != (h << s)) return hipErrorInvalidValue;
        const dim3 grid((tw + 255) / 256, h << s, batch);
        if (src_u8)
            hipLaunchKernelGGL(k_input_up<true>, grid, dim3(256), 0, stream, src, src_u8, stride,
                               src_img_stride, tw, h, s, dst, dst_img_stride);
        else
            hipLaunchKernelGGL(k_input_up<false>, grid, dim3(256), 0, stream, src, src_u8, stride,
                               src_img_stride, tw, h, s, dst, dst_img_stride);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_extrema(const float* pyr, uint32_t* mask, uint32_t* row_count,
                          const FeatureParams& fp, hipStream_t stream, bool tiles) {
    bool tile_ok = tiles && ((uintptr_t)pyr % 16) == 0;
    for (int o = 0; o < fp.n_octaves; o++)
        tile_ok = tile_ok && fp.oct[o].wa % 4 == 0 && fp.oct[o].wa >= 4 && fp.oct[o].gauss_off % 4 == 0 &&
                  fp.oct[o].level_stride % 4 == 0;
    if (tile_ok) {
        ExtremaTileGrid tg{};
        long long nb = 0;
        for (int o = 0; o < fp.n_octaves; o++) {
            tg.tile0[o] = (int)nb;
            tg.tx[o] = (fp.oct[o].wa + kEtW - 1) / kEtW;
            tg.ty[o] = (fp.oct[o].h + kEtH - 1) / kEtH;
            nb += (long long)tg.tx[o] * tg.ty[o] * fp.batch;
        }
        tg.tile0[fp.n_octaves] = (int)nb;
        if (nb <= 0 || nb >= (1ll << 31)) return hipErrorInvalidValue;
        switch (fp.d + 2) {
#define SGK_EXTT(ND) \
    case ND: hipLaunchKernelGGL((k_extrema_tile<ND>), dim3((unsigned)nb), dim3(256), 0, stream, pyr, mask, \
                                row_count, fp, tg); return hipGetLastError();
            SGK_EXTT(3) SGK_EXTT(4) SGK_EXTT(5) SGK_EXTT(6) SGK_EXTT(7) SGK_EXTT(8)
#undef SGK_EXTT
            default: return hipErrorInvalidValue;
        }
    }
    // one wave per (image, strip of tested columns, row segment); ~32k waves in all.  Two
    // columns per lane when every plane is 8-byte aligned (always, for pyramid levels: widths
    // are multiples of 4)
#ifndef SGK_EXT_CPL
#define SGK_EXT_CPL 2
#endif
#ifndef SGK_EXT_SEG_MIN
#define SGK_EXT_SEG_MIN 32
#endif
    bool pairs = SGK_EXT_CPL == 2 && ((uintptr_t)pyr % 8) == 0;
    for (int o = 0; o < fp.n_octaves; o++)
        pairs = pairs && fp.oct[o].wa % 2 == 0 && fp.oct[o].gauss_off % 2 == 0 &&
                fp.oct[o].level_stride % 2 == 0 && ((long long)fp.oct[o].wa * fp.oct[o].h) % 2 == 0;
    const int sw = pairs ? 126 : 62;
    ExtremaWaveGrid eg{};
    int nw = 0;
    for (int o = 0; o < fp.n_octaves; o++) {
        const OctaveDesc& od = fp.oct[o];
        const int strips_x = (od.wa + sw - 1) / sw;
        const long long per_col = (long long)strips_x * fp.batch;
#ifndef SGK_EXT_WAVES
#define SGK_EXT_WAVES 32768
#endif
        // segments of >= 16 rows; a single image >= 8 (C2: its ~1,100 octave-0 waves are
        // latency-bound walks, detection 35.6 vs 44.0 us, C2 0.371-0.377 vs 0.380-0.387 ms per
        // image, tests/diag/r04u.sh; batches keep 16: their halo rows are HBM bytes)
#ifndef SGK_EXT_MINROWS
#define SGK_EXT_MINROWS 16
#endif
        const int minrows = fp.batch == 1 ? 8 : SGK_EXT_MINROWS;
        int nseg = (int)std::min<long long>(std::max<long long>(1, (SGK_EXT_WAVES + per_col - 1) / per_col),
                                            std::max(1, od.h / minrows));
        // a segment reads one halo row above and below it: 2/17 = 12 % extra bytes on the 17-row
        // segments of the batch's upper octaves, so there segments get >= SGK_EXT_SEG_MIN rows
        // while the octave keeps >= 8192 waves (a single image keeps its short segments: there
        // the latency of the longest wave is the kernel's time)
        if (o > 0 && per_col * (od.h / SGK_EXT_SEG_MIN) >= 8192)
            nseg = std::min(nseg, std::max(1, od.h / SGK_EXT_SEG_MIN));
        const int rows = (od.h + nseg - 1) / nseg;
        nseg = (od.h + rows - 1) / rows;
        eg.wave0[o] = nw;
        eg.seg_rows[o] = rows;
        eg.nseg[o] = nseg;
        nw += strips_x * nseg * fp.batch;
    }
    eg.wave0[fp.n_octaves] = nw;
    const unsigned nb = (unsigned)((nw + 3) / 4);
    switch ((fp.d + 2) * 2 + (pairs ? 1 : 0)) {
#define SGK_EXTW(ND)                                                                             \
    case 2 * ND: hipLaunchKernelGGL((k_extrema_wave2<ND, 1>), dim3(nb), dim3(256), 0, stream, pyr, \
                                    mask, row_count, fp, eg); break;                             \
    case 2 * ND + 1: hipLaunchKernelGGL((k_extrema_wave2<ND, 2>), dim3(nb), dim3(256), 0, stream,  \
                                        pyr, mask, row_count, fp, eg); break;
        SGK_EXTW(3) SGK_EXTW(4) SGK_EXTW(5) SGK_EXTW(6) SGK_EXTW(7) SGK_EXTW(8)
        default: return hipErrorInvalidValue;
#undef SGK_EXTW
    }
    return hipGetLastError();
}

static size_t scan_blocks(size_t n) { return (n + 1023) / 1024; }

size_t scan_tmp_words(size_t n) {
    size_t words = 0;
    while (n > 1024) {
        size_t nb = scan_blocks(n);
        words += nb + nb + 1;   // block sums + their scan
        n = nb;
    }
    return words + 16;
}

__global__ __launch_bounds__(256) void k_zero(uint32_t* __restrict__ a, size_t na,
                                              uint32_t* __restrict__ b, size_t nb,
                                              uint32_t* __restrict__ c, size_t nc) {
    const size_t step = (size_t)gridDim.x * 256;
    for (size_t q = (size_t)blockIdx.x * 256 + threadIdx.x; q * 4 < na; q += step) zero_words(a, na, q);
    for (size_t q = (size_t)blockIdx.x * 256 + threadIdx.x; q * 4 < nb; q += step) zero_words(b, nb, q);
    for (size_t q = (size_t)blockIdx.x * 256 + threadIdx.x; q * 4 < nc; q += step) zero_words(c, nc, q);
}

hipError_t launch_zero(uint32_t* a, size_t na, uint32_t* b, size_t nb, uint32_t* c, size_t nc,
                       hipStream_t stream) {
    // the uint4 stores need 16-byte aligned buffers (hipMalloc's are)
    for (const uint32_t* p : {(const uint32_t*)a, (const uint32_t*)b, (const uint32_t*)c})
        if ((uintptr_t)p % 16) return hipErrorInvalidValue;
    if (!a) na = 0;
    if (!b) nb = 0;
    if (!c) nc = 0;
    const size_t quads = (std::max(na, std::max(nb, nc)) + 3) / 4;
    if (quads == 0) return hipSuccess;
    const unsigned grid = (unsigned)std::min<size_t>((quads + 255) / 256, 4096);
    hipLaunchKernelGGL(k_zero, dim3(grid), dim3(256), 0, stream, a, na, b, nb, c, nc);
    return hipGetLastError();
}

hipError_t launch_scan(const uint32_t* in, uint32_t* out, size_t n, uint32_t* tmp,
                       hipStream_t stream) {
    if (n <= 1024) {
        hipLaunchKernelGGL(k_scan_block, dim3(1), dim3(256), 0, stream, in, out, n,
                           (uint32_t*)nullptr);
        return hipGetLastError();
    }
    if (n <= 32768) {   // one workgroup, <= 32 elements per thread
        hipLaunchKernelGGL(k_scan_single, dim3(1), dim3(1024), 0, stream, in, out, n);
        return hipGetLastError();
    }
    const size_t nb = scan_blocks(n);
    uint32_t* sums = tmp;
    uint32_t* sums_scan = tmp + nb;
    hipLaunchKernelGGL(k_scan_block, dim3((unsigned)nb), dim3(256), 0, stream, in, out, n, sums);
    hipError_t e = launch_scan(sums, sums_scan, nb, tmp + nb + nb + 1, stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_scan_add, dim3((unsigned)nb), dim3(256), 0, stream, out, n, sums_scan);
    return hipGetLastError();
}

hipError_t launch_orientation(const float* pyr, const uint32_t* mask, const uint32_t* row_base,
                              int total_rows, const uint32_t* n_cand_dev, int n_cand_cap,
                              int grid_hint, const FeatureParams& fp, float4* out4, int2* info,
                              uint32_t* ocount, hipStream_t stream, bool wave_per_candidate) {
    if (n_cand_cap <= 0) return hipSuccess;
    if (wave_per_candidate) {
        const unsigned grid = (unsigned)std::max(1LL, std::min(((long long)grid_hint + 3) / 4, 8192LL));
        hipLaunchKernelGGL(k_orientation_wave, dim3(grid), dim3(256), 0, stream, pyr, mask,
                           row_base, total_rows, n_cand_dev, (uint32_t)n_cand_cap, fp, out4, info,
                           ocount);
        return hipGetLastError();
    }
    const unsigned grid = (unsigned)std::max(1LL, std::min(((long long)grid_hint + 63) / 64, 4096LL));
    hipLaunchKernelGGL(k_orientation, dim3(grid), dim3(256), 0, stream, pyr, mask, row_base,
                       total_rows, n_cand_dev, (uint32_t)n_cand_cap, fp, out4, info, ocount);
    return hipGetLastError();
}

// One image's keys and descriptors (up to cap features) and its count record straight into
// page-locked host memory (sgpu_set_host_output): one launch in the extract's stream in place of
// the record's copy and the two downloads of sgpu_copy_features -- on one 1080p image each of
// those copies costs ~20 us of DMA start-up and host round trip beside 5 + 19 us of transfer
// (tests/diag/c2_ab.sh timeline).  16-B stores; the host reads them after the stream's
// synchronisation.
__global__ __launch_bounds__(256) void k_copy_out(const float4* __restrict__ keys,
                                                  const float4* __restrict__ desc,
                                                  const uint32_t* __restrict__ n_dev, uint32_t cap,
                                                  const int64_t* __restrict__ rec, int rec_n,
                                                  float4* __restrict__ hkeys, float4* __restrict__ hdesc,
                                                  int64_t* __restrict__ hrec) {
    const uint32_t n = min(*n_dev, cap);
    const size_t t0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t step = (size_t)gridDim.x * blockDim.x;
    if (t0 < (size_t)rec_n) hrec[t0] = rec[t0];
    for (size_t i = t0; i < n; i += step) hkeys[i] = keys[i];
    if (hdesc)
        for (size_t i = t0; i < (size_t)n * 32; i += step) hdesc[i] = desc[i];
}

hipError_t launch_copy_out(const float4* keys, const float* desc, const uint32_t* n_dev, int cap,
                           const int64_t* rec, int rec_n, float* hkeys, float* hdesc,
                           int64_t* hrec, hipStream_t stream) {
    if (cap < 0 || rec_n < 0 || rec_n > 256 || !hkeys || !hrec) return hipErrorInvalidValue;
    const long long work = std::max<long long>(1, (long long)cap * (hdesc ? 32 : 1));
    const unsigned nb = (unsigned)std::min<long long>(256, std::max<long long>(1, (work + 1023) / 1024));
    hipLaunchKernelGGL(k_copy_out, dim3(nb), dim3(256), 0, stream, keys,
                       reinterpret_cast<const float4*>(desc), n_dev, (uint32_t)cap, rec, rec_n,
                       reinterpret_cast<float4*>(hkeys), reinterpret_cast<float4*>(hdesc), hrec);
    return hipGetLastError();
}

hipError_t launch_expand(const float4* cand, const int2* info, const uint32_t* eoff,
                         const uint32_t* n_cand_dev, int n_cand_cap, const FeatureParams& fp,
                         float4* feat, int2* feat_info, float4* keys, hipStream_t stream,
                         const ImageOffsetsArgs* io) {
    if (n_cand_cap <= 0) return hipSuccess;
    const ImageOffsetsArgs none{};
    const unsigned grid = (unsigned)std::min(((long long)n_cand_cap + 255) / 256, 1024LL) +
                          (io && io->off ? 1u : 0u);
    hipLaunchKernelGGL(k_expand, dim3(grid), dim3(256), 0, stream, cand, info, eoff, n_cand_dev,
                       fp, feat, feat_info, keys, (uint32_t)n_cand_cap, io ? *io : none);
    return hipGetLastError();
}

hipError_t launch_orient_keys(const float* pyr, float4* feat, const int2* feat_info,
                              const int* index, int n, const FeatureParams& fp, float4* keys_out,
                              hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    const unsigned grid = (unsigned)std::min((n + 63) / 64, 4096);
    hipLaunchKernelGGL(k_orient_keys, dim3(grid), dim3(256), 0, stream, pyr, feat, feat_info,
                       index, n, fp, keys_out);
    return hipGetLastError();
}

hipError_t launch_descriptor(const float* pyr, const float4* feat, const int2* feat_info,
                             const uint32_t* n_feat_dev, int n_feat_cap, const FeatureParams& fp,
                             float* desc, hipStream_t stream, const int* out_index,
                             bool rect, bool exact, bool dual, bool wide, const HostCopy* host) {
    if (n_feat_cap <= 0) return hipSuccess;
    if (host && (!wide || exact || rect || dual || host->rec_n < 0 || host->rec_n > 256 ||
                 !host->hkeys || !host->hrec || !host->keys || !host->rec))
        return hipErrorInvalidValue;   // only the workgroup-per-feature kernel writes the host
    const unsigned grid = (unsigned)std::min(((long long)n_feat_cap + 3) / 4, 65536LL);
#ifndef SGK_DESC_DUAL
#define SGK_DESC_DUAL 1
#endif
#ifndef SGK_DESC_FLAT
#define SGK_DESC_FLAT 1
#endif
    if (!exact && !rect && SGK_DESC_FLAT && !dual && wide) {
        // A/B knobs: SGPU_WIDE_DESC_WAVES (4 or 8 waves per feature), SGPU_WIDE_DESC_GRID (at most
        // this many workgroups, each taking every grid-th feature)
        static const int nwv = [] {
            const char* e = getenv("SGPU_WIDE_DESC_WAVES");
            return e && atoi(e) == 8 ? 8 : 4;
        }();
        static const long long gmax = [] {
            const char* e = getenv("SGPU_WIDE_DESC_GRID");
            return e && atoll(e) > 0 ? atoll(e) : 65536LL;
        }();
        const unsigned wgrid = (unsigned)std::min((long long)n_feat_cap, gmax);
        const HostCopy hc = host ? *host : HostCopy{};
        if (nwv == 8)
            hipLaunchKernelGGL(k_descriptor_wide<8>, dim3(wgrid), dim3(512), 0, stream, pyr, feat,
                               feat_info, n_feat_dev, fp, desc, out_index, hc);
        else
            hipLaunchKernelGGL(k_descriptor_wide<4>, dim3(wgrid), dim3(256), 0, stream, pyr, feat,
                               feat_info, n_feat_dev, fp, desc, out_index, hc);
        return hipGetLastError();
    }
    if (!exact && !rect && SGK_DESC_FLAT && !dual) {
        hipLaunchKernelGGL(k_descriptor_flat, dim3(grid), dim3(256), 0, stream, pyr, feat,
                           feat_info, n_feat_dev, fp, desc, out_index);
        return hipGetLastError();
    }
    if (!exact && !rect && SGK_DESC_DUAL) {
        hipLaunchKernelGGL(k_descriptor_dual, dim3(grid), dim3(256), 0, stream, pyr, feat,
                           feat_info, n_feat_dev, fp, desc, out_index);
        return hipGetLastError();
    }
    if (!exact) {
        if (rect)
            hipLaunchKernelGGL(k_descriptor_fast<true>, dim3(grid), dim3(256), 0, stream, pyr,
                               feat, feat_info, n_feat_dev, fp, desc, out_index);
        else
            hipLaunchKernelGGL(k_descriptor_fast<false>, dim3(grid), dim3(256), 0, stream, pyr,
                               feat, feat_info, n_feat_dev, fp, desc, out_index);
        return hipGetLastError();
    }
    if (rect)
        hipLaunchKernelGGL(k_descriptor<true>, dim3(grid), dim3(256), 0, stream, pyr, feat,
                           feat_info, n_feat_dev, fp, desc, out_index);
    else
        hipLaunchKernelGGL(k_descriptor<false>, dim3(grid), dim3(256), 0, stream, pyr, feat,
                           feat_info, n_feat_dev, fp, desc, out_index);
    return hipGetLastError();
}

hipError_t launch_limit_rows(uint32_t* row_count, const FeatureParams& fp, int threshold,
                             int method, hipStream_t stream) {
    if (fp.n_octaves * fp.d > kMaxLimitLevels) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_limit_rows, dim3(fp.batch), dim3(256), 0, stream, row_count, fp,
                       threshold, method);
    return hipGetLastError();
}

hipError_t launch_limit_oriented(uint32_t* ocount, const uint32_t* row_base,
                                 const FeatureParams& fp, int threshold, int method,
                                 uint32_t cand_cap, hipStream_t stream) {
    if (fp.n_octaves * fp.d > kMaxLimitLevels) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_limit_oriented, dim3(fp.batch), dim3(256), 0, stream, ocount, row_base,
                       fp, threshold, method, cand_cap);
    return hipGetLastError();
}


}  // namespace sgk
