// sift_octave.hip -- one launch per octave builds all d+3 Gaussian levels (gfx950).
//
// Reference semantics: FilterImage / FilterH<FW> / FilterV<FW> (ProgramCU.cu:115-222,406-446)
// applied level after level by PyramidCU::BuildPyramid (PyramidCU.cpp:979-1044), the level-0
// ingest of octave 0 (GLTexImage.cpp:818, u8 -> p/255) and DownsampleKernel<1>
// (ProgramCU.cu:287-298) of level d into the next octave's level 0.
//
// The per-level path (k_gauss_pk2, sift_kernels.hip) reads every level back from HBM to filter
// the next one: 48 B per octave pixel.  Here one workgroup owns a vertical strip of one image
// and streams it from top to bottom through a pipeline of wavefronts, one per level:
//
//   loader wave -> [L0 filter wave] -> L1 wave -> L2 wave -> ... -> L5 wave
//
// Every step each wave consumes one ROW PAIR of the previous level from LDS, runs the
// horizontal filter on it (packed over the two rows: v_pk_fma_f32), pushes the two filtered
// rows into vertical accumulators that live in VGPRs, and emits one finished row pair of its own
// level: to LDS for the next wave and to HBM.  One barrier per step.  HBM traffic per octave
// pixel is the input read (1 B for u8 ingest, 4 B for an octave's level 0) plus the 6 (5) level
// writes and the 1/4-size downsample: 25-26 B instead of 48 B.
//
// Exactness: each output is the reference's ordered fma chain.
//   * H pass: h = fma(in[c-sz+i], k[i], h) for i = 0..FW-1 from h = 0, with clamp-to-edge
//     columns: the LDS row window holds the edge value at positions outside the image.
//   * V pass (push form): the accumulator of output row Y receives row j's contribution
//     fma(h_j, k[j-Y+sz], acc) when row j arrives; rows arrive in increasing order, so every
//     accumulator sees taps 0..FW-1 in order, starting from 0.  Out-of-range taps are skipped at
//     compile time (no fma with a zero weight).  Rows above 0 / below H-1 are the edge rows
//     pushed again (clamp-to-edge).
// A strip's columns are extended by the halo the remaining levels need (the sum of their
// half-widths, rounded up to 4), and a band of rows by the same vertical halo, so a workgroup
// never needs another workgroup's results.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <type_traits>

#include "sift_kernels.h"
#include "sift_math.h"

#pragma clang diagnostic ignored "-Winline-asm"   // m0 clobber of the LDS-DMA asm

using namespace sgm;

namespace sgk {
namespace {

typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));

// Two scalar v_fma_f32 (this file is built with -fno-slp-vectorize): the tap stays one SGPR.
// v_pk_fma_f32 has the same FLOP rate but needs its scalar operand as an aligned SGPR pair,
// which doubled the SGPRs the taps occupy and spilled them.
__device__ __forceinline__ f2v pk(f2v a, float b, f2v c) {
    return f2v{__builtin_fmaf(a.x, b, c.x), __builtin_fmaf(a.y, b, c.y)};
}

// p / 255.0f, exact (same as sift_kernels.hip)
__device__ __forceinline__ float u8_unit(uint32_t p) {
    const float x = (float)p, c = 1.0f / 255.0f;
    const float q = x * c;
    return fma_(fma_(-q, 255.0f, x), c, q);
}

// Workgroup barrier that orders LDS only.  __syncthreads() is a workgroup-scope release fence
// on ALL address spaces, i.e. an s_waitcnt vmcnt(0): every wave would wait for its own global
// stores (and the loader for its prefetches) at every step.
__device__ __forceinline__ void block_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// ---- stage-to-stage handoff: LDS rings of kSlots row pairs with produced / consumed counts --
// Each stage buffer s has one producer wave and one consumer wave.  The producer writes slot
// n % kSlots, then (LDS release: lgkmcnt(0)) publishes prod[s] = n + 1; the consumer waits for
// prod[s] > n, reads the slot and publishes cons[s] = n + 1 once its reads are done; the producer
// reuses a slot only when cons[s] allows it.  No workgroup barriers: every wave runs at its own
// pace and the SIMD loads, not the slowest wave of each step, set the throughput.
constexpr int kSlots = 4;

__device__ __forceinline__ int lds_load(const int* p) {
    return __builtin_amdgcn_readfirstlane(__atomic_load_n(p, __ATOMIC_RELAXED));
}
__device__ __forceinline__ void lds_publish(int* p, int v) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __atomic_store_n(p, v, __ATOMIC_RELAXED);
}
__device__ __forceinline__ void lds_wait_ge(const int* p, int v) {
    while (lds_load(p) < v) __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

constexpr int kWt = 240;        // widest core strip (columns stored by one workgroup)
constexpr int kSB = 448;        // f2v (row pairs) per LDS slot; every window + read halo fits
constexpr int kNPF = 8;         // loader prefetch depth in steps
constexpr int kMaxStages = 7;   // loader, L0 filter, L1..L5

// level filter widths of the default schedule (d = 3, filter factor 4): level k from k-1
constexpr int kFW[6] = {0, 11, 13, 17, 21, 25};
constexpr int r4(int x) { return (x + 3) & ~3; }
constexpr int halfw(int fw) { return fw >> 1; }
// column halo of level k's window: what levels k+1..5 still need (rounded up to 4 so every
// window starts on an aligned quad)
constexpr int kRP5 = 0;
constexpr int kRP4 = r4(kRP5 + halfw(kFW[5]));
constexpr int kRP3 = r4(kRP4 + halfw(kFW[4]));
constexpr int kRP2 = r4(kRP3 + halfw(kFW[3]));
constexpr int kRP1 = r4(kRP2 + halfw(kFW[2]));
constexpr int kRP0 = r4(kRP1 + halfw(kFW[1]));
constexpr int kRP[6] = {kRP0, kRP1, kRP2, kRP3, kRP4, kRP5};
constexpr int rp_in(int fw0) { return r4(kRP0 + halfw(fw0)); }
// columns per lane of each level's wave: 64 * CPT covers the window kWt + 2 * RP
constexpr int cpt_of(int rp) { return ((kWt + 2 * rp + 127) / 128) * 2; }

struct OctArgs {
    const uint8_t* src8;      // octave 0: u8 input (SRC 1)
    const float* srcf;        // octave 0: f32 input (SRC 2)
    int src_stride;           // elements between input rows
    long long src_img_stride; // elements between input images
    float* pyr;               // level 0 of image 0 of this octave
    long long level_stride;   // floats between levels
    int W, H;                 // level geometry (W = padded width = row stride)
    int wt, nstrips, nbands, band_rows;
    float* ds;                // next octave's level 0 of image 0 (nullptr: last octave)
    int dsw, dsh;
    long long ds_img_stride;
    float k[kMaxStages][33];  // taps per stage (stage 0 = loader: unused)
    int probe;                // timing probes (variant bits 18, 19): 1 no HBM stores, 2 no filter
};

struct Sched { int ys, js, jf, S, np; };

// Row schedule of the stage chain for rows [yb, ye) of the last level (see the file comment).
// Stage s > 0 pushes virtual row pairs j = jf, jf+2, ... one per step from step S; its
// emission at push j is the row pair j - D (D = sze).  Stage 0 (loader) delivers pairs
// ys, ys+2, ... one per step from step 0.
template <int NC>
__device__ __forceinline__ int make_schedule(const int (&sze)[NC], int yb, int ye, int He,
                                             Sched (&s)[NC]) {
    int ysv[NC], yev[NC];
    ysv[NC - 1] = yb;
    yev[NC - 1] = min(He, (ye + 1) & ~1);
#pragma unroll
    for (int k = NC - 1; k >= 1; k--) {
        ysv[k - 1] = max(0, ysv[k] - sze[k]);
        yev[k - 1] = min(He, yev[k] + sze[k]);
    }
    s[0].ys = ysv[0];
    s[0].js = ysv[0];
    s[0].jf = ysv[0];
    s[0].S = 0;
    s[0].np = (yev[0] - ysv[0]) >> 1;
    int T = s[0].np;
#pragma unroll
    for (int k = 1; k < NC; k++) {
        s[k].ys = ysv[k];
        s[k].js = ysv[k] - sze[k];
        s[k].jf = max(s[k].js, 0);
        s[k].np = (yev[k] + sze[k] - s[k].jf) >> 1;
        s[k].S = s[k - 1].S + ((k == 1 ? 0 : sze[k - 1]) - s[k - 1].jf + s[k].jf) / 2 + 1;
        T = max(T, s[k].S + s[k].np);
    }
    return T;
}

// ---- loader wave: row pairs of the input (octave 0) or of level 0 (octave > 0) into LDS ----
// Window positions p of columns x0 - RPL + p, clamped to [0, W-1] (the quads are aligned: RPL,
// x0 and W are multiples of 4, so a quad is wholly inside or outside the image).
// The rows travel HBM -> LDS by LDS-DMA (global_load_lds_dword[x4]) into a ring of kNPF steps,
// with explicit vmcnt waits: every step issues exactly 4 DMA instructions (2 rows x 2 quads per
// lane, unpredicated, clamped addresses), so "step t has landed" is vmcnt <= 4 * (kNPF - 1).
// (Register prefetch rings lost their depth to the compiler's loop-carried register rotation.)
// The loader then converts the landed rows to the row-pair layout the filter waves read, with
// clamp-to-edge replication of quads outside the image.
template <bool U8>
struct LoaderRing {
    static constexpr int QB = U8 ? 4 : 16;          // bytes per lane per DMA
    static constexpr int ROW = 128 * QB;            // bytes per ring row (2 DMAs of 64 lanes)
    static constexpr int BYTES = kNPF * 2 * ROW;
};

template <int N>
__device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    // s_waitcnt: vmcnt[3:0] bits 3:0, vmcnt[5:4] bits 15:14; expcnt / lgkmcnt left at max
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x70 | 0xF00);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

template <int SRC, int RPL>
__device__ __forceinline__ void loader_role(const OctArgs& a, int b, int x0, int wt, const Sched sc,
                                            f2v* __restrict__ out, uint8_t* __restrict__ ring,
                                            int* prod, const int* cons) {
    constexpr bool U8 = SRC == 1;
    typedef LoaderRing<U8> R;
    const int lane = threadIdx.x & 63;
    const int W = a.W, H = a.H;
    const int nq = (wt + 2 * RPL) >> 2;            // quads per row (<= 128)
    const uint8_t* s8 = nullptr;
    const float* sf = nullptr;
    int stride;
    if (SRC == 1) { s8 = a.src8 + (long long)b * a.src_img_stride; stride = a.src_stride; }
    else if (SRC == 2) { sf = a.srcf + (long long)b * a.src_img_stride; stride = a.src_stride; }
    else { sf = a.pyr + (long long)b * W * H; stride = W; }
    int qc[2];
    bool qv[2], ql[2], qr[2];
#pragma unroll
    for (int m = 0; m < 2; m++) {
        const int q = lane + 64 * m;
        const int c = x0 - RPL + 4 * q;
        qv[m] = q < nq;
        ql[m] = c < 0;
        qr[m] = c > W - 4;
        qc[m] = qv[m] ? min(max(c, 0), W - 4) : 0;
    }
    // The DMA is issued from inline asm: the compiler then neither waits on it (its LDS-DMA
    // alias tracking put a vmcnt(0) in front of every ring read) nor moves LDS accesses across
    // it ("memory").  M0 = LDS destination of lane 0.
    auto issue = [&](int slot, int t) {
        const int y = sc.ys + 2 * t;
        const int y1 = min(y + 1, H - 1);
        const uint32_t base = (uint32_t)(uintptr_t)(ring + slot * 2 * R::ROW);
#pragma unroll
        for (int r = 0; r < 2; r++)
#pragma unroll
            for (int m = 0; m < 2; m++) {
                const long long row = (long long)(r ? y1 : y) * stride;
                const uint32_t la = base + r * R::ROW + m * 64 * R::QB;
                if (U8) {
                    const uint8_t* g = s8 + row + qc[m];
                    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dword %1, off"
                                 :: "s"(la), "v"(g) : "memory", "m0");
                } else {
                    const float* g = sf + row + qc[m];
                    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
                                 :: "s"(la), "v"(g) : "memory", "m0");
                }
            }
    };
    const bool edge_strip = (x0 - RPL < 0) || (x0 - RPL + 4 * nq > W);
    auto put = [&](int slot, int t) {
        const uint8_t* base = ring + slot * 2 * R::ROW;
        f2v* o = out + (t % kSlots) * kSB;
#pragma unroll
        for (int m = 0; m < 2; m++) {
            if (!qv[m]) continue;
            float v0[4], v1[4];
            const int off = (lane + 64 * m) * R::QB;
            if constexpr (U8) {
                const uint32_t w0 = *reinterpret_cast<const uint32_t*>(base + off);
                const uint32_t w1 = *reinterpret_cast<const uint32_t*>(base + R::ROW + off);
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    v0[e] = u8_unit((w0 >> (8 * e)) & 255u);
                    v1[e] = u8_unit((w1 >> (8 * e)) & 255u);
                }
            } else {
                const f4v r0 = *reinterpret_cast<const f4v*>(base + off);
                const f4v r1 = *reinterpret_cast<const f4v*>(base + R::ROW + off);
#pragma unroll
                for (int e = 0; e < 4; e++) { v0[e] = r0[e]; v1[e] = r1[e]; }
            }
            if (edge_strip) {   // clamp-to-edge: quads left of 0 / right of W-1 repeat the edge
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    v0[e] = ql[m] ? v0[0] : (qr[m] ? v0[3] : v0[e]);
                    v1[e] = ql[m] ? v1[0] : (qr[m] ? v1[3] : v1[e]);
                }
            }
            f2v p[4];
#pragma unroll
            for (int e = 0; e < 4; e++) p[e] = f2v{v0[e], v1[e]};
            f4v* d = reinterpret_cast<f4v*>(o + 4 * (lane + 64 * m));
            d[0] = f4v{p[0].x, p[0].y, p[1].x, p[1].y};
            d[1] = f4v{p[2].x, p[2].y, p[3].x, p[3].y};
        }
    };
    const int tlast = max(sc.np - 1, 0);
#pragma unroll
    for (int ph = 0; ph < kNPF; ph++) issue(ph, min(ph, tlast));
    for (int t0 = 0; t0 < sc.np; t0 += kNPF) {
#pragma unroll
        for (int ph = 0; ph < kNPF; ph++) {
            const int t = t0 + ph;
            if (t >= sc.np) break;
            wait_vm<4 * (kNPF - 1)>();   // step t's 4 DMAs have landed
            if (t >= kSlots) lds_wait_ge(cons, t - kSlots + 1);   // slot t % kSlots is free
            // (stage 1 is one wave in both kernels)
            put(ph, t);
            lds_publish(prod, t + 1);
            issue(ph, min(t + kNPF, tlast));
        }
    }
    wait_vm<0>();
}

// ---- level wave: filter FW from the previous stage's row pairs ----
// This wave computes window positions POS0 + [0, 64 * CPT) of its level (a level may be split
// over two waves).  OFF = RP(prev) - RPK: window offset between the two stages; NPW / NCW:
// waves of the producing / consuming stage (NCW = 0: last level).
// Positions whose column lies outside the image are never stored and never read as such: in a
// strip that touches an image edge, the H pass reads the producer's row at clamped columns.
template <int FW, int CPT, int POS0, int OFF, int RPK, int NPW, int NCW>
__device__ __forceinline__ void level_role(const float* __restrict__ k, const f2v* __restrict__ sin,
                                           f2v* __restrict__ sout, int* cnt_in, int* cnt_out,
                                           int widx, const Sched sc, int W, int H, int x0,
                                           int xe, int wt, int yb, int ye,
                                           float* __restrict__ gdst, float* __restrict__ gds,
                                           int dsw, int dsh, int probe) {
    constexpr int SZ = FW >> 1;
    constexpr int D = (SZ + 1) & ~1;                 // emission lag (= sze)
    constexpr int P = (D + SZ + 1) / 2 + 1;          // pending row pairs
    constexpr int NCP = CPT / 2;                     // column pairs per lane
    constexpr int B0 = OFF - SZ;                     // first source position (lane-relative)
    static_assert(B0 >= 0, "window halo");
    constexpr int SH = B0 & 1;                       // odd start: read one early
    constexpr int NRD = (CPT + FW - 1 + SH + 1) / 2; // ds_read_b128 per H pass
    constexpr int NIN = CPT + FW - 1;                // row pairs one lane reads
    static_assert(POS0 + 64 * CPT + B0 + 2 * NRD <= kSB, "LDS slot");
    const int lane = threadIdx.x & 63;
    const int lw = POS0 + lane * CPT;
    int* const prod_in = cnt_in;                     // [0..NPW): producers of sin
    int* const cons_in = cnt_in + 2 + widx;          // this wave's consumed count of sin
    int* const prod_out = cnt_out + widx;            // this wave's produced count of sout
    const int* const cons_out = cnt_out + 2;         // [0..NCW): consumers of sout
    f2v acc[P][2][NCP];
#pragma unroll
    for (int s = 0; s < P; s++)
#pragma unroll
        for (int r = 0; r < 2; r++)
#pragma unroll
            for (int cp = 0; cp < NCP; cp++) acc[s][r][cp] = f2v{0.f, 0.f};
    float hl[CPT];
#pragma unroll
    for (int c = 0; c < CPT; c++) hl[c] = 0.f;
    // does some lane read a column outside [0, W-1]?
    const bool edge_read = (x0 - RPK - SZ < 0) || (x0 + wt + RPK + SZ > W);
    const int rp_prev = OFF + RPK;

    // one push of the row pair (j, j+1) given as h[c] = {row j, row j+1}; e = emitted pair
    auto push = [&](const f2v (&h)[CPT], f2v (&e)[2][NCP]) {
        f2v hj[NCP], hj1[NCP];
#pragma unroll
        for (int cp = 0; cp < NCP; cp++) {
            hj[cp] = f2v{h[2 * cp].x, h[2 * cp + 1].x};
            hj1[cp] = f2v{h[2 * cp].y, h[2 * cp + 1].y};
        }
        // two sweeps (row j, then row j+1) so that consecutive FMAs are independent
#pragma unroll
        for (int s = 0; s < P; s++) {
            const int a = D + SZ - 2 * s;   // tap of row j for output row Y = j - D + 2s
#pragma unroll
            for (int r = 0; r < 2; r++)
#pragma unroll
                for (int cp = 0; cp < NCP; cp++)
                    if (a - r >= 0 && a - r < FW) acc[s][r][cp] = pk(hj[cp], k[a - r], acc[s][r][cp]);
        }
#pragma unroll
        for (int s = 0; s < P; s++) {
            const int a = D + SZ - 2 * s;
#pragma unroll
            for (int r = 0; r < 2; r++) {
#pragma unroll
                for (int cp = 0; cp < NCP; cp++) {
                    f2v v = acc[s][r][cp];
                    if (a + 1 - r >= 0 && a + 1 - r < FW) v = pk(hj1[cp], k[a + 1 - r], v);
                    if (s == 0) e[r][cp] = v;
                    else acc[s - 1][r][cp] = v;
                }
            }
        }
#pragma unroll
        for (int r = 0; r < 2; r++)
#pragma unroll
            for (int cp = 0; cp < NCP; cp++) acc[P - 1][r][cp] = f2v{0.f, 0.f};
    };

    int n_in = 0, n_out = 0;   // pairs consumed from sin / produced into sout
    for (int u = 0; u < sc.np; u++) {
        const int j = sc.jf + 2 * u;
        f2v h[CPT];
        f2v e[2][NCP];
        if (j < H) {
#pragma unroll
            for (int w = 0; w < NPW; w++) lds_wait_ge(prod_in + w, n_in + 1);
            const f2v* slot = sin + (n_in % kSlots) * kSB;
            f2v in[NIN + 1];
            if (!edge_read) {
                const f2v* src = slot + lw + B0 - SH;
                f2v raw[2 * NRD];
#pragma unroll
                for (int q = 0; q < NRD; q++) {
                    const f4v v = *reinterpret_cast<const f4v*>(src + 2 * q);
                    raw[2 * q] = f2v{v.x, v.y};
                    raw[2 * q + 1] = f2v{v.z, v.w};
                }
#pragma unroll
                for (int m = 0; m < NIN; m++) in[m] = raw[SH + m];
            } else {   // clamp-to-edge columns
                const int c0 = x0 - RPK + lw - SZ;
#pragma unroll
                for (int m = 0; m < NIN; m++)
                    in[m] = slot[min(max(c0 + m, 0), W - 1) - x0 + rp_prev];
            }
            n_in++;
            lds_publish(cons_in, n_in);   // the reads above have completed (lgkmcnt(0))
            // tap-major: the CPT chains interleave (consecutive FMAs are independent)
#pragma unroll
            for (int c = 0; c < CPT; c++) h[c] = f2v{0.f, 0.f};
            if (probe & 2) {
#pragma unroll
                for (int c = 0; c < CPT; c++) h[c] = in[c + SZ];
            } else {
#pragma unroll
                for (int i = 0; i < FW; i++)
#pragma unroll
                    for (int c = 0; c < CPT; c++) h[c] = pk(in[c + i], k[i], h[c]);
            }
            if (j + 1 >= H)
#pragma unroll
                for (int c = 0; c < CPT; c++) h[c].y = h[c].x;
            if (j + 2 >= H)
#pragma unroll
                for (int c = 0; c < CPT; c++) hl[c] = h[c].y;
            if (u == 0 && sc.js < 0) {   // rows above the image = row 0 (clamp-to-edge)
                f2v h0[CPT];
#pragma unroll
                for (int c = 0; c < CPT; c++) h0[c] = f2v{h[c].x, h[c].x};
                for (int v = 0; v < (-sc.js) >> 1; v++) push(h0, e);
            }
        } else {   // rows below the image = row H-1
#pragma unroll
            for (int c = 0; c < CPT; c++) h[c] = f2v{hl[c], hl[c]};
        }
        if (probe & 2) {   // timing probe only: no vertical filter
#pragma unroll
            for (int cp = 0; cp < NCP; cp++) {
                e[0][cp] = f2v{h[2 * cp].x, h[2 * cp + 1].x};
                e[1][cp] = f2v{h[2 * cp].y, h[2 * cp + 1].y};
            }
        } else {
            push(h, e);
        }
        const int y0 = j - D;
        if (y0 < sc.ys) continue;
        if (NCW && n_out >= kSlots)   // the consumers have released slot n_out % kSlots
#pragma unroll
            for (int w = 0; w < NCW; w++) lds_wait_ge(cons_out + w, n_out - kSlots + 1);
        f2v* o = sout + (n_out % kSlots) * kSB;
#pragma unroll
        for (int cp = 0; cp < NCP; cp++)
            *reinterpret_cast<f4v*>(o + lw + 2 * cp) =
                f4v{e[0][cp].x, e[1][cp].x, e[0][cp].y, e[1][cp].y};
        n_out++;
        if (NCW) lds_publish(prod_out, n_out);
        // HBM: the core columns among this wave's positions, 4 per lane, read back transposed
        // (only this wave writes these positions, so the slot may be read after publishing)
        constexpr int G0 = POS0 > RPK ? (POS0 - RPK) / 4 : 0;
        constexpr int GE = (POS0 + 64 * CPT - RPK) / 4;   // groups [G0, GE) lie in this wave
        const int g = G0 + lane;
        if (gdst && !(probe & 1) && y0 >= yb && y0 < ye && g < GE && 4 * g < xe - x0) {
            wave_sync();
            const f4v* q = reinterpret_cast<const f4v*>(o + RPK + 4 * g);
            const f4v va = q[0], vb = q[1];
            const int c = x0 + 4 * g;
            *reinterpret_cast<f4v*>(gdst + (long long)y0 * W + c) = f4v{va.x, va.z, vb.x, vb.z};
            if (y0 + 1 < ye)
                *reinterpret_cast<f4v*>(gdst + (long long)(y0 + 1) * W + c) =
                    f4v{va.y, va.w, vb.y, vb.w};
            // DownsampleKernel<1>: next level 0 (r, cc) = this (2r, min(2cc, W-1))
            if (gds && (y0 >> 1) < dsh) {
                float* drow = gds + (long long)(y0 >> 1) * dsw;
                const int cc = c >> 1;
                if (cc + 1 < dsw) *reinterpret_cast<f2v*>(drow + cc) = f2v{va.x, vb.x};
                else if (cc < dsw) drow[cc] = va.x;
                if (c + 3 == W - 1)
                    for (int z = W >> 1; z < dsw; z++) drow[z] = vb.z;
            }
        }
    }
}

// SRC 0: octave > 0 (level 0 is in the pyramid); 1: u8 input; 2: f32 input (octave 0).
// Waves: one loader, one per level for L0..L4 (6 columns per lane), two for L5 (2 + 2), so
// that the SIMDs (waves w and w + 4 share one; a lone wave issues VALU at half rate) carry
// similar filter work: octave 0 {loader, L5b} {L4, L5a} {L3, L1} {L0, L2};
// octave > 0 {loader, L5b} {L4, L5a} {L3, L1} {L2}.
template <int FW0, int SRC>
__global__ __launch_bounds__(SRC ? 512 : 448) void k_octave(const OctArgs a) {
    constexpr bool IN = SRC != 0;
    constexpr int NC = IN ? 7 : 6;
    __shared__ __attribute__((aligned(16))) f2v lds[NC][kSlots * kSB];
    __shared__ __attribute__((aligned(16))) uint8_t ring[LoaderRing<SRC == 1>::BYTES];
    __shared__ int cnt[kMaxStages][4];   // per stage: produced by its waves [0,1], consumed [2,3]
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int id = blockIdx.x;
    const int sx = id % a.nstrips, rest = id / a.nstrips;
    const int sb = rest % a.nbands, b = rest / a.nbands;
    const int W = a.W, H = a.H, wt = a.wt;
    const int x0 = sx * wt, xe = min(W, x0 + wt);
    const int yb = sb * a.band_rows, ye = min(H, yb + a.band_rows);
    const int He = (H + 1) & ~1;
    int sze[NC];
    sze[0] = 0;
    if (IN) sze[1] = (halfw(FW0) + 1) & ~1;
#pragma unroll
    for (int l = 1; l <= 5; l++) sze[NC - 6 + l] = (halfw(kFW[l]) + 1) & ~1;
    Sched sc[NC];
    make_schedule<NC>(sze, yb, ye, He, sc);
    if (threadIdx.x < 4 * kMaxStages) (&cnt[0][0])[threadIdx.x] = 0;
    __syncthreads();
    const long long img = (long long)b * W * H;
    float* lev = a.pyr + img;
    float* gds = a.ds ? a.ds + (long long)b * a.ds_img_stride : nullptr;
    const int dsw = a.dsw, dsh = a.dsh;
    constexpr int o = NC - 6;   // stage of level L is o + L
    if (wave == 0) {
        loader_role<SRC, IN ? rp_in(FW0) : kRP0>(a, b, x0, wt, sc[0], lds[0], ring, &cnt[0][0],
                                                 &cnt[0][2]);
        return;
    }
    // stage of level L, its filter width, CPT, first position, previous halo, #producer and
    // #consumer waves, wave index within the level
#define SGK_LEVEL(WAVE, L, FWL, CPTL, POS, RPPREV, NPW, NCW, WIDX)                              \
    if (wave == WAVE) {                                                                        \
        level_role<FWL, CPTL, POS, (RPPREV) - kRP[L], kRP[L], NPW, NCW>(                       \
            a.k[o + (L)], lds[o + (L) - 1], lds[o + (L)], &cnt[o + (L) - 1][0],                 \
            &cnt[o + (L)][0], WIDX, sc[o + (L)], W, H, x0, xe, wt, yb, ye,                     \
            lev + (long long)(L) * a.level_stride, (L) == 3 ? gds : nullptr, dsw, dsh,         \
            a.probe);                                                                          \
        return;                                                                                \
    }
    if constexpr (IN) {
        SGK_LEVEL(3, 0, FW0, 6, 0, rp_in(FW0), 1, 1, 0)
        SGK_LEVEL(6, 1, kFW[1], 6, 0, kRP0, 1, 1, 0)
        SGK_LEVEL(7, 2, kFW[2], 6, 0, kRP1, 1, 1, 0)
        SGK_LEVEL(2, 3, kFW[3], 6, 0, kRP2, 1, 1, 0)
        SGK_LEVEL(1, 4, kFW[4], 6, 0, kRP3, 1, 2, 0)
        SGK_LEVEL(5, 5, kFW[5], 2, 0, kRP4, 1, 0, 0)
        SGK_LEVEL(4, 5, kFW[5], 2, 128, kRP4, 1, 0, 1)
    } else {
        SGK_LEVEL(6, 1, kFW[1], 6, 0, kRP0, 1, 1, 0)
        SGK_LEVEL(3, 2, kFW[2], 6, 0, kRP1, 1, 1, 0)
        SGK_LEVEL(2, 3, kFW[3], 6, 0, kRP2, 1, 1, 0)
        SGK_LEVEL(1, 4, kFW[4], 6, 0, kRP3, 1, 2, 0)
        SGK_LEVEL(5, 5, kFW[5], 2, 0, kRP4, 1, 0, 0)
        SGK_LEVEL(4, 5, kFW[5], 2, 128, kRP4, 1, 0, 1)
    }
#undef SGK_LEVEL
}

}  // namespace

bool octave_fused_supported(int nlev, const int* fw, int level_ds) {
    if (nlev != 6 || level_ds != 3) return false;
    for (int l = 1; l < 6; l++)
        if (fw[l] != kFW[l]) return false;
    return true;
}

hipError_t launch_octave(const OctaveLaunch& L, hipStream_t stream) {
    const int W = L.w, H = L.h;
    if (W < 4 || (W & 3) || H < 1 || L.batch < 1) return hipErrorInvalidValue;
    const int src = L.src8 ? 1 : (L.srcf ? 2 : 0);
    if (src) {
        if (L.fw0 != 11 && L.fw0 != 13) return hipErrorNotSupported;
        if ((L.src_stride & 3) || (L.src_img_stride & 3) ||
            ((uintptr_t)(L.src8 ? (const void*)L.src8 : (const void*)L.srcf) & 15))
            return hipErrorNotSupported;
    }
    OctArgs a;
    a.src8 = L.src8;
    a.srcf = L.srcf;
    a.src_stride = L.src_stride;
    a.src_img_stride = L.src_img_stride;
    a.pyr = L.pyr;
    a.level_stride = L.level_stride;
    a.W = W;
    a.H = H;
    const int ns = (W + kWt - 1) / kWt;
    a.wt = ((W + ns - 1) / ns + 3) & ~3;
    a.nstrips = (W + a.wt - 1) / a.wt;
    // bands: enough workgroups for ~2 per CU, bands of at least 64 rows
    const long long per_band = (long long)a.nstrips * L.batch;
    int nb = (int)std::min<long long>((512 + per_band - 1) / per_band, std::max(1, H / 64));
    nb = std::max(nb, 1);
    int rows = ((H + nb - 1) / nb + 1) & ~1;
    a.nbands = (H + rows - 1) / rows;
    a.band_rows = rows;
    a.ds = L.ds;
    a.dsw = L.dsw;
    a.dsh = L.dsh;
    a.ds_img_stride = L.ds_img_stride;
    a.probe = (get_variant() >> 18) & 3;
    for (int s = 0; s < kMaxStages; s++)
        for (int i = 0; i < 33; i++) a.k[s][i] = 0.f;
    const int o = src ? 1 : 0;
    if (src)
        for (int i = 0; i < L.fw0; i++) a.k[1][i] = L.taps0[i];
    for (int l = 1; l < 6; l++)
        for (int i = 0; i < kFW[l]; i++) a.k[o + l][i] = L.taps[l][i];
    const dim3 grid((unsigned)(a.nstrips * a.nbands * L.batch));
    if (src == 0) hipLaunchKernelGGL((k_octave<0, 0>), grid, dim3(448), 0, stream, a);
    else if (src == 1 && L.fw0 == 13) hipLaunchKernelGGL((k_octave<13, 1>), grid, dim3(512), 0, stream, a);
    else if (src == 1) hipLaunchKernelGGL((k_octave<11, 1>), grid, dim3(512), 0, stream, a);
    else if (L.fw0 == 13) hipLaunchKernelGGL((k_octave<13, 2>), grid, dim3(512), 0, stream, a);
    else hipLaunchKernelGGL((k_octave<11, 2>), grid, dim3(512), 0, stream, a);
    return hipGetLastError();
}

}  // namespace sgk
