// sift_gauss_pair.hip -- two consecutive Gaussian levels per launch (gfx950).
//
// Reference semantics: FilterH<FW> then FilterV<FW> (ProgramCU.cu:115-222, driven by
// ProgramCU::FilterImage, ProgramCU.cu:406-446) applied to level k and then to level k+1 by
// PyramidCU::BuildPyramid (PyramidCU.cpp:979-1044), with the level-0 ingest of octave 0
// (u8 -> p/255, GLTexImage.cpp:818) and DownsampleKernel<1> (ProgramCU.cu:287-298) of level d
// into the next octave's level 0 fused into the level that feeds it.
//
// The per-level kernel (k_gauss_pk2, sift_kernels.hip) reads level k from HBM and writes level
// k+1: 8 B per pixel and level.  Here one workgroup reads level k once and writes levels k+1
// AND k+2: 12 B per pixel for two levels (9 B when level k is the u8 input).  The middle level
// never makes a round trip through HBM; it lives in LDS between the two filters:
//
//   HBM level k -> regs (2 chunks ahead) -> s_in -> H1 -> ring1 -> V1 -> HBM level k+1
//                                                                   -> s_mid -> H2 -> ring2 -> V2
//                                                                                 -> HBM level k+2
//
// A workgroup owns a 64-column strip of one image and a band of rows, and walks down it in
// 32-row chunks.  Level k+1 is computed on the strip plus the H2 halo the second filter needs on
// either side (rounded up to 4 columns, so every output quad stays aligned) and on the band plus
// H2 rows above and below.  The extra columns and rows cost 19-38 % more arithmetic on the first
// filter.
//
// Exactness.  Each output is the reference's ordered fma chain from 0, taps 0..FW-1, exactly as
// in k_gauss_pk2 (bit-identical outputs, tests/test_gpu_parity.py).  Clamp-to-edge needs care
// in the fused form: outside the image the second filter must see the EDGE VALUE of level k+1,
// not level k+1 evaluated at a position outside the image.  So
//   * V1 reads ring1 at the clamped column: a middle-level column left of 0 (right of W-1) is
//     computed as column 0 (W-1) -- s_mid holds exactly the clamped row the reference filters;
//   * V2 reads ring2 at the clamped middle-level row (only in the chunks whose window crosses
//     the first or last image row; the others use the unclamped index).
// Middle rows outside the image are computed but never read.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <type_traits>

#include "sift_kernels.h"
#include "sift_math.h"

using namespace sgm;

namespace sgk {
namespace {

typedef float f2v __attribute__((ext_vector_type(2)));
template <int N>
using IC = std::integral_constant<int, N>;

// Filter FMAs are v_pk_fma_f32 on two independent outputs with the tap in a VGPR pair.  A
// packed FMA does 128 lane-FMAs per issue, twice a v_fma_f32, and a wave that is alone on its
// SIMD (two workgroups per CU here) issues one VALU instruction per 4 cycles either way.  The
// taps are moved to VGPRs once (vtap): as SGPR operands a packed FMA needs an aligned SGPR pair
// per tap, and two filters' worth of pairs spilled.
__device__ __forceinline__ f2v pfma(f2v a, f2v k, f2v c) { return __builtin_elementwise_fma(a, k, c); }

__device__ __forceinline__ f2v vtap(float t) {
    float v;
    asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "s"(t));
    return f2v{v, v};
}

__device__ __forceinline__ int clampi(int v, int lo, int hi) {
    return v < lo ? lo : (v > hi ? hi : v);
}

// p / 255.0f, exact for p in [0, 255] (same formula as sift_kernels.hip u8_to_unit)
__device__ __forceinline__ float u8_unit(uint32_t p) {
    const float x = (float)p, c = 1.0f / 255.0f;
    const float q = x * c;
    return fma_(fma_(-q, 255.0f, x), c, q);
}

// Workgroup barrier ordering LDS only.  __syncthreads() is a release fence on every address
// space, i.e. s_waitcnt vmcnt(0): each wave would wait for its HBM stores AND for the row
// prefetch of chunk c+2 at every barrier.  Global stores of this kernel are never read back
// inside the workgroup.
__device__ __forceinline__ void lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Gaussian taps are symmetric bit for bit (make_filter: exp(-i^2/2s^2) for i = -sz..sz, one
// normalisation), so tap m is read as tap min(m, FW-1-m) and only the H+1 distinct values
// occupy registers; the host checks the symmetry before launching.
struct HalfTaps { float k[17]; };
template <int FW>
__host__ __device__ constexpr int sym(int m) { return m < FW - 1 - m ? m : FW - 1 - m; }

constexpr int NT = 256;   // threads per workgroup (384, so that H1 / V1 take one round: slower)
constexpr int PG = 64;    // output columns per strip
constexpr int PC = 32;    // rows per chunk
constexpr int PRS = 64;   // ring rows: chunk k lives at rows (k & 1) * PC .. + PC - 1

// DownsampleKernel<1> into the next octave's level 0: ds(r, c) = src(2r, min(2c, W-1)), for
// the pair (x, x+1), x even, of output row y.  W is even.
__device__ __forceinline__ void write_ds(float* dd, int dsw, int dsh, int W, int y, int x, f2v a) {
    if (!(y & 1) && (y >> 1) < dsh) {
        float* drow = dd + (long long)(y >> 1) * dsw;
        if ((x >> 1) < dsw) drow[x >> 1] = a.x;
        if (x + 1 == W - 1)
            for (int cc = W >> 1; cc < dsw; cc++) drow[cc] = a.y;
    }
}

// H pass of one row pair x 4 columns: a[i] = (row 2p, row 2p+1) at column i, taps 0..FW-1 in
// order from 0.  `rowp` points at the first input column of the window (O = its parity).
template <int FW, int O>
__device__ __forceinline__ void hpass(const f2v* rowp, const f2v* tp, f2v (&a)[4]) {
    constexpr int NRD = (FW + 3) / 2;
#pragma unroll
    for (int i = 0; i < 4; i++) a[i] = f2v{0.f, 0.f};
#pragma unroll
    for (int q = 0; q < NRD; q++) {
        f2v e[2];
        if (O % 2 == 0) {
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
                if (m - i >= 0 && m - i < FW) a[i] = pfma(e[u], tp[sym<FW>(m - i)], a[i]);
        }
    }
}

// V pass of one task, 4 rows x 2 columns, on a ring whose chunk of parity KP holds the task's
// first row at KP * PC + 4 vq: acc[j] = sum over m of ring[row + j + m] * k[m - j], in tap
// order.  Rows KP * PC + 4 vq + m (m < FW + 3 <= 36) never wrap for KP = 0; for KP = 1 they
// wrap once 4 vq + m reaches 32, i.e. from a multiple of 4 of m on.  So every read is one
// ds_read with an immediate offset from one of two per-thread bases.  SPLIT: the two columns
// c0, c1 are read separately (clamped columns of a boundary strip); otherwise c1 = c0 + 1 and
// one ds_read_b64 serves both.
template <int FW, int HS, int KP, bool SPLIT>
__device__ __forceinline__ void vpass(const float* ring, const f2v* tp, int vq, int c0, int c1,
                                      f2v (&acc)[4]) {
    const float* h0 = ring + (KP * PC + 4 * vq) * HS + c0;
    const float* h1 = ring + (KP * PC + 4 * vq) * HS + c1;
#pragma unroll
    for (int j = 0; j < 4; j++) acc[j] = f2v{0.f, 0.f};
#pragma unroll
    for (int m = 0; m < FW + 3; m++) {
        const bool wrap = KP && vq + (m >> 2) >= (PRS - PC) / 4;
        const float* q0 = wrap ? h0 - PRS * HS : h0;
        f2v v;
        if (SPLIT) {
            const float* q1 = wrap ? h1 - PRS * HS : h1;
            v = f2v{q0[m * HS], q1[m * HS]};
        } else {
            v = *reinterpret_cast<const f2v*>(q0 + m * HS);
        }
#pragma unroll
        for (int j = 0; j < 4; j++)
            if (m - j >= 0 && m - j < FW) acc[j] = pfma(v, tp[sym<FW>(m - j)], acc[j]);
    }
}

template <int FW1, int FW2, bool U8>
__global__ __launch_bounds__(NT) void k_gauss_pair(
    const float* __restrict__ src, const uint8_t* __restrict__ src8, int src_stride,
    long long src_img_stride, float* __restrict__ dst1, float* __restrict__ dst2,
    long long dst_img_stride, int W, int H, HalfTaps t1, HalfTaps t2, float* __restrict__ ds,
    int ds_level, int dsw, int dsh, long long ds_img_stride, int rows_per_band) {
    constexpr int H1 = FW1 >> 1, H2 = FW2 >> 1;
    constexpr int H2A = (H2 + 3) & ~3;                 // middle-level halo, quad aligned
    constexpr int W1P = PG + 2 * H2A;                  // middle-level columns per strip
    constexpr int OFF2 = H2A - H2;                     // s_mid column of the H2 window start
    constexpr int OFF = (-(H1 + H2A)) & 3;             // s_in column of the first input column
    constexpr int IN_W = W1P + FW1 - 1 + OFF;          // input columns held per row
    constexpr int NQ = (IN_W + 3) / 4;                 // aligned input quads per row
    constexpr int IN_S = 4 * NQ + 2;                   // s_in row-pair stride (float2; 16 mod 32 B)
    constexpr int HS1 = W1P + 4;                       // ring1 row stride (floats)
    constexpr int MS = W1P + 2;                        // s_mid row-pair stride (float2; 16 mod 32 B)
    constexpr int HS2 = PG + 4;                        // ring2 row stride (floats)
    constexpr int NLD = ((PC / 2) * NQ + NT - 1) / NT;  // quads per thread per chunk
    constexpr int Q1 = W1P / 4, T1 = (PC / 2) * Q1;    // H1 tasks: row pair x 4 columns
    constexpr int P1 = W1P / 2, TV1 = (PC / 4) * P1;   // V1 tasks: 4 rows x 2 columns
    static_assert(FW1 + 3 <= 36 && FW2 + 3 <= 36, "V reads stay inside two ring chunks");
    static_assert(2 * H2 + FW1 - 1 <= 2 * PC, "input chunks stay two ahead of the output");
    __shared__ __attribute__((aligned(16))) f2v s_in[(PC / 2) * IN_S];
    __shared__ __attribute__((aligned(16))) float s_r1[PRS * HS1];
    __shared__ __attribute__((aligned(16))) f2v s_mid[(PC / 2) * MS];
    __shared__ __attribute__((aligned(16))) float s_r2[PRS * HS2];

    const int tid = threadIdx.x;
    const int strips_x = (W + PG - 1) / PG;
    const int bands = (H + rows_per_band - 1) / rows_per_band;
    const int id = blockIdx.x;
    const int sx = id % strips_x, rest = id / strips_x;
    const int sy = rest % bands, b = rest / bands;
    const int x0 = sx * PG;
    const int yb = sy * rows_per_band;
    const int ye = min(H, yb + rows_per_band);
    const int n = ye - yb;
    const int nmid = n + 2 * H2;
    const int nin = nmid + FW1 - 1;
    const int nchunk_in = (nin + PC - 1) / PC;
    const int nchunk_mid = (nmid + PC - 1) / PC;
    const int nchunk_out = (n + PC - 1) / PC;
    const int xm0 = x0 - H2A;                          // image column of middle column 0
    const int a0 = xm0 - H1 - OFF;                     // image column of input column 0 (aligned)
    const int iy0 = yb - H2 - H1;                      // image row of input row 0 (unclamped)
    const bool col_edge = xm0 < 0 || x0 + PG + H2A > W;

    f2v k1[H1 + 1], k2[H2 + 1];
#pragma unroll
    for (int i = 0; i <= H1; i++) k1[i] = vtap(t1.k[i]);
#pragma unroll
    for (int i = 0; i <= H2; i++) k2[i] = vtap(t2.k[i]);

    const float* sf = U8 ? nullptr : src + (long long)b * src_img_stride;
    const uint8_t* s8 = U8 ? src8 + (long long)b * src_img_stride : nullptr;
    float* d1 = dst1 + (long long)b * dst_img_stride;
    float* d2 = dst2 + (long long)b * dst_img_stride;
    float* dd = ds ? ds + (long long)b * ds_img_stride : nullptr;

    // ---- input rows: aligned quads, clamp-to-edge rows and columns (as k_gauss_pk2 VEC).
    // The prefetch keeps the RAW quads (f32, or the u8 words in .x); edge replication and the
    // u8 conversion happen when the chunk is stored to LDS.  Consuming the loaded registers right
    // after the load would make the compiler wait for each prefetch as soon as it is issued,
    // and with two workgroups per CU nothing else hides that latency.
    struct Elem { float4 v0, v1; };
    Elem stA[NLD], stB[NLD];
    // Chunk loads keep the RAW quads; edge replication and the u8 conversion happen when the
    // chunk is stored to LDS, so the compiler does not wait for a load right after issuing it.
    // (Issuing them from inline asm with explicit vmcnt waits saved 2 %, but the compiler then
    // copies and reuses the destination registers before the data lands: unsafe.)
    auto load_chunk = [&](Elem (&stage)[NLD], int c) {
#pragma unroll
        for (int m = 0; m < NLD; m++) {
            const int e = min(tid + NT * m, (PC / 2) * NQ - 1);
            const int p = e / NQ, j = e - p * NQ;
            const int gy0 = clampi(iy0 + c * PC + 2 * p, 0, H - 1);
            const int gy1 = clampi(iy0 + c * PC + 2 * p + 1, 0, H - 1);
            const int lq = clampi(a0 + 4 * j, 0, W - 4);
            if (U8) {
                stage[m].v0.x = __uint_as_float(*reinterpret_cast<const uint32_t*>(s8 + (long long)gy0 * src_stride + lq));
                stage[m].v1.x = __uint_as_float(*reinterpret_cast<const uint32_t*>(s8 + (long long)gy1 * src_stride + lq));
            } else {
                stage[m].v0 = *reinterpret_cast<const float4*>(sf + (long long)gy0 * src_stride + lq);
                stage[m].v1 = *reinterpret_cast<const float4*>(sf + (long long)gy1 * src_stride + lq);
            }
        }
    };
    auto store_chunk = [&](const Elem (&stage)[NLD]) {
#pragma unroll
        for (int m = 0; m < NLD; m++) {
            const int e = tid + NT * m;
            if (e < (PC / 2) * NQ) {
                const int p = e / NQ, j = e - p * NQ;
                const int gq = a0 + 4 * j;
                float r0[4], r1[4];
                if (U8) {
                    const uint32_t w0 = __float_as_uint(stage[m].v0.x), w1 = __float_as_uint(stage[m].v1.x);
#pragma unroll
                    for (int t = 0; t < 4; t++) {
                        r0[t] = u8_unit((w0 >> (8 * t)) & 255u);
                        r1[t] = u8_unit((w1 >> (8 * t)) & 255u);
                    }
                } else {
                    r0[0] = stage[m].v0.x; r0[1] = stage[m].v0.y; r0[2] = stage[m].v0.z; r0[3] = stage[m].v0.w;
                    r1[0] = stage[m].v1.x; r1[1] = stage[m].v1.y; r1[2] = stage[m].v1.z; r1[3] = stage[m].v1.w;
                }
                // a quad left of column 0 repeats column 0, right of W-1 repeats W-1
                const bool left = gq < 0, right = gq > W - 4;
                f2v q[4];
#pragma unroll
                for (int t = 0; t < 4; t++)
                    q[t] = f2v{left ? r0[0] : (right ? r0[3] : r0[t]),
                               left ? r1[0] : (right ? r1[3] : r1[t])};
                float4* dq = reinterpret_cast<float4*>(&s_in[p * IN_S + 4 * j]);
                dq[0] = make_float4(q[0].x, q[0].y, q[1].x, q[1].y);
                dq[1] = make_float4(q[2].x, q[2].y, q[3].x, q[3].y);
            }
        }
    };

    load_chunk(stA, 0);
    store_chunk(stA);
    load_chunk(stA, 1);
    load_chunk(stB, 2);
    lds_sync();

    // Step c (parity P, a template argument so that ring rows are compile-time offsets):
    // H1 of input chunk c, V1 + H2 of middle chunk c-1, V2 of output chunk c-2.  `cur` holds
    // chunk c+1 (loaded at the end of step c-2) and `nxt` chunk c+2 (end of step c-1); cur is
    // stored to s_in after H1 and reloaded with chunk c+3 before the V2 stores.
    auto step = [&](int c, auto pc, Elem (&cur)[NLD], Elem (&nxt)[NLD]) {
        constexpr int P = decltype(pc)::value;
        (void)nxt;
        const bool has_next = c + 1 < nchunk_in;
        // ---- H1 of input chunk c -> ring1 rows P*PC .. P*PC+31
        if (c < nchunk_in) {
#pragma unroll 1
            for (int r = 0; r < (T1 + NT - 1) / NT; r++) {
                const int e = tid + NT * r;
                if (e < T1) {
                    const int hp = e / Q1, hc = (e - hp * Q1) * 4;
                    f2v a[4];
                    hpass<FW1, OFF>(&s_in[hp * IN_S + hc + OFF], k1, a);
                    float* w = &s_r1[(P * PC + 2 * hp) * HS1 + hc];
                    *reinterpret_cast<float4*>(w) = make_float4(a[0].x, a[1].x, a[2].x, a[3].x);
                    *reinterpret_cast<float4*>(w + HS1) = make_float4(a[0].y, a[1].y, a[2].y, a[3].y);
                }
            }
        }
        lds_sync();
        // chunk c+1 -> s_in (H1 has finished with it)
        if (has_next) store_chunk(cur);
        const int km = c - 1;   // middle chunk of this step (parity 1 - P)
        if (km >= 0 && km < nchunk_mid) {
            // ---- V1 of middle chunk km: rows km*PC + 4vq + j, columns vc, vc+1
#pragma unroll 1
            for (int r = 0; r < (TV1 + NT - 1) / NT; r++) {
                const int e = tid + NT * r;
                if (e < TV1) {
                    const int vq = e / P1, vc = (e - vq * P1) * 2;
                    f2v acc[4];
                    if (!col_edge)
                        vpass<FW1, HS1, 1 - P, false>(s_r1, k1, vq, vc, vc + 1, acc);
                    else
                        vpass<FW1, HS1, 1 - P, true>(s_r1, k1, vq, clampi(xm0 + vc, 0, W - 1) - xm0,
                                                     clampi(xm0 + vc + 1, 0, W - 1) - xm0, acc);
                    // middle rows -> s_mid pairs (2vq, 2vq+1), columns vc, vc+1
                    *reinterpret_cast<float4*>(&s_mid[(2 * vq) * MS + vc]) =
                        make_float4(acc[0].x, acc[1].x, acc[0].y, acc[1].y);
                    *reinterpret_cast<float4*>(&s_mid[(2 * vq + 1) * MS + vc]) =
                        make_float4(acc[2].x, acc[3].x, acc[2].y, acc[3].y);
                    // level k+1 output: the strip's own columns and the band's own rows
                    const int x = xm0 + vc;
                    if (vc >= H2A && vc < H2A + PG && x < W) {
                        const int t0 = km * PC + 4 * vq - H2;
#pragma unroll
                        for (int j = 0; j < 4; j++) {
                            const int t = t0 + j;
                            if (t >= 0 && t < n) {
                                const int y = yb + t;
                                *reinterpret_cast<f2v*>(&d1[(long long)y * W + x]) = acc[j];
                                if (dd && ds_level == 1) write_ds(dd, dsw, dsh, W, y, x, acc[j]);
                            }
                        }
                    }
                }
            }
        }
        lds_sync();
        if (km >= 0 && km < nchunk_mid) {
            // ---- H2 of middle chunk km -> ring2 rows (1-P)*PC .. +31
            const int hp = tid >> 4, hc = (tid & 15) * 4;
            f2v a[4];
            hpass<FW2, OFF2>(&s_mid[hp * MS + hc + OFF2], k2, a);
            float* w = &s_r2[((1 - P) * PC + 2 * hp) * HS2 + hc];
            *reinterpret_cast<float4*>(w) = make_float4(a[0].x, a[1].x, a[2].x, a[3].x);
            *reinterpret_cast<float4*>(w + HS2) = make_float4(a[0].y, a[1].y, a[2].y, a[3].y);
        }
        lds_sync();
        const int ko = c - 2;   // output chunk of this step (parity P)
        const bool do_v2 = ko >= 0 && ko < nchunk_out;
        // ---- V2 of output chunk ko: rows ko*PC + 4vq + j.  The middle virtual row of output row
        // t and tap m is t + m (image row yb - H2 + t + m); chunks whose window crosses the first
        // or last image row read the clamped row instead.
        const int vq = tid >> 5, vc = (tid & 31) * 2;
        const int t0 = ko * PC + 4 * vq;
        f2v acc[4];
        if (do_v2) {
            const int lo = yb - H2 + ko * PC, hi = lo + PC + FW2 - 2;
            if (lo >= 0 && hi <= H - 1) {
                vpass<FW2, HS2, P, false>(s_r2, k2, vq, vc, vc + 1, acc);
            } else {
                const int base = yb - H2;   // image row of middle virtual row 0
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    acc[j] = f2v{0.f, 0.f};
#pragma unroll
                    for (int m = 0; m < FW2; m++) {
                        const int mr = clampi(base + t0 + j + m, 0, H - 1) - base;
                        const f2v v = *reinterpret_cast<const f2v*>(&s_r2[(mr & (PRS - 1)) * HS2 + vc]);
                        acc[j] = pfma(v, k2[sym<FW2>(m)], acc[j]);
                    }
                }
            }
        }
        // chunk c+3 (rows clamped, so always a valid address)
        load_chunk(cur, c + 3);
        if (do_v2) {
            const int x = x0 + vc;
            if (x < W) {
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int y = yb + t0 + j;
                    if (y < ye) {
                        *reinterpret_cast<f2v*>(&d2[(long long)y * W + x]) = acc[j];
                        if (dd && ds_level == 2) write_ds(dd, dsw, dsh, W, y, x, acc[j]);
                    }
                }
            }
        }
    };
    const int nsteps = nchunk_out + 2;
    for (int c = 0; c < nsteps; c += 2) {
        step(c, IC<0>(), stA, stB);
        if (c + 1 < nsteps) step(c + 1, IC<1>(), stB, stA);
    }
}

template <int FW1, int FW2>
hipError_t pair_dispatch(const GaussPairLaunch& L, hipStream_t stream) {
    const int strips_x = (L.w + PG - 1) / PG;
    const long long per_col = (long long)strips_x * L.batch;
    // bands: enough workgroups for ~4 per CU, band height a multiple of the chunk
    int nb = (int)std::min<long long>((1024 + per_col - 1) / per_col, (L.h + PC - 1) / PC);
    nb = std::max(nb, 1);
    int rows = (L.h + nb - 1) / nb;
    rows = (rows + PC - 1) / PC * PC;
    nb = (L.h + rows - 1) / rows;
    const dim3 grid((unsigned)(strips_x * nb * L.batch));
    HalfTaps a{}, c{};
    for (int i = 0; i < FW1; i++) {   // bitwise symmetric taps only
        if (__builtin_memcmp(&L.taps1[i], &L.taps1[FW1 - 1 - i], 4)) return hipErrorNotSupported;
        if (i <= FW1 / 2) a.k[i] = L.taps1[i];
    }
    for (int i = 0; i < FW2; i++) {
        if (__builtin_memcmp(&L.taps2[i], &L.taps2[FW2 - 1 - i], 4)) return hipErrorNotSupported;
        if (i <= FW2 / 2) c.k[i] = L.taps2[i];
    }
    if (L.src8)
        hipLaunchKernelGGL((k_gauss_pair<FW1, FW2, true>), grid, dim3(NT), 0, stream, nullptr,
                           L.src8, L.src_stride, L.src_img_stride, L.dst1, L.dst2, L.dst_img_stride,
                           L.w, L.h, a, c, L.ds, L.ds_level, L.dsw, L.dsh, L.ds_img_stride, rows);
    else
        hipLaunchKernelGGL((k_gauss_pair<FW1, FW2, false>), grid, dim3(NT), 0, stream, L.src,
                           nullptr, L.src_stride, L.src_img_stride, L.dst1, L.dst2,
                           L.dst_img_stride, L.w, L.h, a, c, L.ds, L.ds_level, L.dsw, L.dsh,
                           L.ds_img_stride, rows);
    return hipGetLastError();
}

}  // namespace

bool gauss_pair_supported(int fw1, int fw2) {
    return (fw1 == 13 && fw2 == 11) || (fw1 == 11 && fw2 == 13) || (fw1 == 13 && fw2 == 17) ||
           (fw1 == 17 && fw2 == 21) || (fw1 == 21 && fw2 == 25);
}

hipError_t launch_gauss_pair(const GaussPairLaunch& L, hipStream_t stream) {
    // aligned quads: 4-element row / image strides, 16-B (f32) or 4-B (u8) aligned base, and a
    // width that is a multiple of 4 (always true for pyramid levels)
    const void* base = L.src8 ? (const void*)L.src8 : (const void*)L.src;
    if (L.batch <= 0 || L.w < 4 || (L.w % 4) || (L.src_stride % 4) || (L.src_img_stride % 4) ||
        ((uintptr_t)base % (L.src8 ? 4 : 16)) || L.h < 1)
        return hipErrorNotSupported;
    if (L.fw1 == 13 && L.fw2 == 11) return pair_dispatch<13, 11>(L, stream);
    if (L.fw1 == 11 && L.fw2 == 13) return pair_dispatch<11, 13>(L, stream);
    if (L.fw1 == 13 && L.fw2 == 17) return pair_dispatch<13, 17>(L, stream);
    if (L.fw1 == 17 && L.fw2 == 21) return pair_dispatch<17, 21>(L, stream);
    if (L.fw1 == 21 && L.fw2 == 25) return pair_dispatch<21, 25>(L, stream);
    return hipErrorNotSupported;
}

}  // namespace sgk
