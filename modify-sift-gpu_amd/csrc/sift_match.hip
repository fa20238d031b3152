// sift_match.hip -- SiftMatch on gfx950 MFMA with the best/second-best selection fused into
// the GEMM epilogue.
//
// Reference: MultiplyDescriptor_Kernel (SiftGPU/ProgramCU.cu:1466-1564) materialises the full
// num1 x num2 int32 dot matrix, RowMatch_Kernel / ColMatch_Kernel (:1785-1900) scan it again and
// SiftMatchCU::GetBestMatch (SiftMatchCU.cpp:149-179) does the mutual check.  Here no dot matrix
// exists: each workgroup keeps a 128-row panel of set A in registers as i8 MFMA fragments,
// streams set B through LDS in 128-column tiles, and folds every 16x16 accumulator tile into
// per-row running (max, argmax, second) state.  The column side is the same kernel with the sets
// swapped.
//
// Exactness: u8 descriptors are mapped to s8 by s = u - 128 (xor 0x80) so the signed i8 MFMA
// (v_mfma_i32_16x16x64_i8) applies; dot(u1, u2) = dot(s1, s2) + 128*sum(u1) + 128*sum(u2) -
// 2^21, all in int32.  The column term is the accumulator's initial value, the row term is added
// once per row at the end (it does not change a row's ordering).  Results equal the reference's
// integer dot products exactly.
#include "sift_kernels.h"

namespace sgk {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));

constexpr int kPanel = 128;      // A rows per workgroup (4 waves x 32)
constexpr int kTile = 128;       // B columns per LDS tile
constexpr int kLdsRow = 128 + 16;// bytes per staged B row (padding against bank conflicts)
constexpr int kNeg = -(1 << 29); // "minus infinity" for running maxima (no overflow with offsets)
constexpr int kNegCol = -(1 << 26);  // column term of a missing column: its dot stays far below
                                     // every real one (|dot| < 2^23) and (dot << 3) fits in int32

// v_med3_i32: the median of three.  With s <= m, med3(s, m, v) is the new second maximum after
// seeing v (v > m -> m; s < v <= m -> v; v <= s -> s).
__device__ __forceinline__ int med3i(int a, int b, int c) {
    int r;
    asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

__global__ __launch_bounds__(256) void k_rowsum(const uint8_t* __restrict__ d, int n,
                                                int* __restrict__ s, int scale, int bias) {
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (i >= n) return;
    const uint16_t v = reinterpret_cast<const uint16_t*>(d + (size_t)i * 128)[lane];
    int t = (v & 0xff) + (v >> 8);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
    if (lane == 0) s[i] = scale * t + bias;
}

__device__ __forceinline__ v4i load16_s8(const uint8_t* p) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    v4i r;
    r[0] = (int)(u.x ^ 0x80808080u);
    r[1] = (int)(u.y ^ 0x80808080u);
    r[2] = (int)(u.z ^ 0x80808080u);
    r[3] = (int)(u.w ^ 0x80808080u);
    return r;
}

// One row panel of A against columns [c_begin, c_end) of B.
// part[chunk * nA + row] = running top-2 of row over those columns (dot without the row term).
//
// Guided matching (MODE 1: A = set 1, the row decision; MODE 2: A = set 2, the column
// decision) folds the guided value of MultiplyDescriptorG_Kernel (ProgramCU.cu:1683-1733)
// instead of the dot: the accumulators then start at row term + column term (the exact dot, the
// masking below is not monotone in it), and `mask` (k_guided_mask) holds one byte per (4-row
// group of A, column): bit i = pair (4g+i, col) passes the geometric test, bit 4+i = some row of
// that pair's 8-row block of set 1 passes at that column (good_count > 0).
//   MODE 1: pass ? dot : good ? max(dot - 2^18, 0) : 0      (d_result = max(results, 0))
//   MODE 2: pass ? dot : good ? dot - 2^18 : -2^18          (the raw results of d_temp)
template <int MODE>
__global__ __launch_bounds__(256) void k_match_rows(const uint8_t* __restrict__ A, int nA,
                                                    const uint8_t* __restrict__ B, int nB,
                                                    const int* __restrict__ col_term,
                                                    int cols_per_chunk, Top2* __restrict__ part,
                                                    const int* __restrict__ row_term,
                                                    const uint8_t* __restrict__ mask,
                                                    int mask_pitch) {
    __shared__ __attribute__((aligned(16))) uint8_t s_b[2][kTile * kLdsRow];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int panel = blockIdx.x, chunk = blockIdx.y;
    const int c_begin = chunk * cols_per_chunk;
    const int c_end = min(nB, c_begin + cols_per_chunk);
    const int quad = lane >> 4, l16 = lane & 15;

    // A fragments: rows wave*32 + rb*16 + l16, bytes kh*64 + quad*16 .. +16
    v4i afrag[2][2];
#pragma unroll
    for (int rb = 0; rb < 2; rb++) {
        const int row = panel * kPanel + wave * 32 + rb * 16 + l16;
#pragma unroll
        for (int kh = 0; kh < 2; kh++) {
            if (row < nA) afrag[rb][kh] = load16_s8(A + (size_t)row * 128 + kh * 64 + quad * 16);
            else afrag[rb][kh] = v4i{0, 0, 0, 0};
        }
    }
    // guided: the row terms of this lane's rows and their 4-row mask groups
    int rterm[2][4] = {};
    int mgroup[2] = {};
    if constexpr (MODE != 0) {
#pragma unroll
        for (int rb = 0; rb < 2; rb++) {
            const int r0 = panel * kPanel + wave * 32 + rb * 16 + quad * 4;
            mgroup[rb] = r0 < nA ? r0 >> 2 : -1;
#pragma unroll
            for (int i = 0; i < 4; i++) rterm[rb][i] = r0 + i < nA ? row_term[r0 + i] : 0;
        }
    }
    // running state for this lane's 8 output rows: (rb, i) -> row wave*32 + rb*16 + quad*4 + i
    int M[2][4], S[2][4], I[2][4];
#pragma unroll
    for (int rb = 0; rb < 2; rb++)
#pragma unroll
        for (int i = 0; i < 4; i++) { M[rb][i] = kNeg; S[rb][i] = kNeg; I[rb][i] = -1; }

    // staging: thread t copies 64 bytes: column t>>1, half (t&1)
    auto stage_load = [&](int tbase, uint4* r) {
        const int col = tbase + (tid >> 1);
        const uint8_t* src = B + (size_t)col * 128 + (tid & 1) * 64;
#pragma unroll
        for (int q = 0; q < 4; q++)
            r[q] = col < c_end ? reinterpret_cast<const uint4*>(src)[q] : make_uint4(0, 0, 0, 0);
    };
    auto stage_store = [&](int buf, const uint4* r) {
        uint8_t* dst = &s_b[buf][(tid >> 1) * kLdsRow + (tid & 1) * 64];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            uint4 v = r[q];
            v.x ^= 0x80808080u; v.y ^= 0x80808080u; v.z ^= 0x80808080u; v.w ^= 0x80808080u;
            reinterpret_cast<uint4*>(dst)[q] = v;
        }
    };

    uint4 stg[4];
    int buf = 0;
    if (c_begin < c_end) {
        stage_load(c_begin, stg);
        stage_store(0, stg);
    }
    __syncthreads();
    for (int tb = c_begin; tb < c_end; tb += kTile) {
        const bool has_next = tb + kTile < c_end;
        if (has_next) stage_load(tb + kTile, stg);
        // accumulators start at the column term (invalid columns: -inf)
        v4i acc[2][8];
        uint32_t mb[2][8];
#pragma unroll
        for (int cb = 0; cb < 8; cb++) {
            const int col = tb + cb * 16 + l16;
            const int ct = col < c_end ? col_term[col] : kNegCol;
            if constexpr (MODE == 0) {
                acc[0][cb] = v4i{ct, ct, ct, ct};
                acc[1][cb] = acc[0][cb];
            } else {
#pragma unroll
                for (int rb = 0; rb < 2; rb++) {
                    acc[rb][cb] = v4i{ct + rterm[rb][0], ct + rterm[rb][1], ct + rterm[rb][2],
                                      ct + rterm[rb][3]};
                    mb[rb][cb] = (col < c_end && mgroup[rb] >= 0)
                                     ? mask[(size_t)mgroup[rb] * mask_pitch + col] : 0u;
                }
            }
        }
        const uint8_t* sb = s_b[buf];
#pragma unroll
        for (int cb = 0; cb < 8; cb++) {
#pragma unroll
            for (int kh = 0; kh < 2; kh++) {
                const v4i bfrag = *reinterpret_cast<const v4i*>(
                    sb + (cb * 16 + l16) * kLdsRow + kh * 64 + quad * 16);
                acc[0][cb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(afrag[0][kh], bfrag, acc[0][cb], 0, 0, 0);
                acc[1][cb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(afrag[1][kh], bfrag, acc[1][cb], 0, 0, 0);
            }
        }
        // epilogue: fold the 2x8 tiles into the running top-2 (C layout: col = l16,
        // row = quad*4 + i within the 16-row block).  Values are folded as keys
        // (dot << 3) | (7 - cb): one v_lshl_or, one v_max and one v_med3 per value; the key's
        // low bits name the column block and the tile is recorded once per tile when the
        // maximum moved.  Equal dots order by lower column first (the reference's strict '>'
        // scan); the second key of an equal pair carries the same dot, so ties still reject.
#pragma unroll
        for (int rb = 0; rb < 2; rb++)
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int m0 = M[rb][i];
                int m = m0, sv = S[rb][i];
#pragma unroll
                for (int cb = 0; cb < 8; cb++) {
                    int v = acc[rb][cb][i];
                    if constexpr (MODE != 0) {
                        const bool pass = (mb[rb][cb] >> i) & 1u;
                        const bool good = (mb[rb][cb] >> (4 + i)) & 1u;
                        const int off = MODE == 1 ? max(v - 262144, 0) : v - 262144;
                        v = pass ? v : (good ? off : (MODE == 1 ? 0 : -262144));
                    }
                    const int key = (v << 3) | (7 - cb);
                    sv = med3i(sv, m, key);
                    m = max(m, key);
                }
                I[rb][i] = m != m0 ? tb : I[rb][i];
                M[rb][i] = m;
                S[rb][i] = sv;
            }
        __syncthreads();
        if (has_next) {
            buf ^= 1;
            stage_store(buf, stg);
        }
        __syncthreads();
    }
    // keys -> (dot, column): column = tile + 16 * (7 - low bits) + l16
#pragma unroll
    for (int rb = 0; rb < 2; rb++)
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int k = M[rb][i];
            I[rb][i] = I[rb][i] < 0 ? -1 : I[rb][i] + 16 * (7 - (k & 7)) + l16;
            M[rb][i] = k >> 3;
            S[rb][i] = S[rb][i] >> 3;
        }
    // merge the 16 lanes that share a row (same quad): xor 1, 2, 4, 8
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) {
#pragma unroll
        for (int rb = 0; rb < 2; rb++)
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int m2 = __shfl_xor(M[rb][i], off, 64);
                const int s2 = __shfl_xor(S[rb][i], off, 64);
                const int i2 = __shfl_xor(I[rb][i], off, 64);
                const int m1 = M[rb][i], s1 = S[rb][i], i1 = I[rb][i];
                M[rb][i] = max(m1, m2);
                S[rb][i] = max(min(m1, m2), max(s1, s2));
                I[rb][i] = m2 > m1 ? i2 : (m1 > m2 ? i1 : min((unsigned)i1, (unsigned)i2));
            }
    }
    if (l16 == 0) {
#pragma unroll
        for (int rb = 0; rb < 2; rb++)
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int row = panel * kPanel + wave * 32 + rb * 16 + quad * 4 + i;
                if (row < nA) part[(size_t)chunk * nA + row] = Top2{M[rb][i], I[rb][i], S[rb][i]};
            }
    }
}

// Merge the column chunks of one side, add the row term, apply the distance/ratio test
// (RowMatch_Kernel / ColMatch_Kernel decision, ProgramCU.cu:1838-1841, 1884-1887).
__global__ __launch_bounds__(256) void k_match_finish(const Top2* __restrict__ part, int n,
                                                      int chunks, const int* __restrict__ row_term,
                                                      const float* __restrict__ dist,
                                                      float distmax, float ratiomax,
                                                      int* __restrict__ out,
                                                      Top2* __restrict__ best) {
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= n) return;
    Top2 t = part[r];
    for (int c = 1; c < chunks; c++) {
        const Top2 u = part[(size_t)c * n + r];
        const int m = max(t.max, u.max);
        const int s = max(min(t.max, u.max), max(t.second, u.second));
        const int id = u.max > t.max ? u.idx : (t.max > u.max ? t.idx : min((unsigned)t.idx, (unsigned)u.idx));
        t = Top2{m, id, s};
    }
    const int rt = row_term ? row_term[r] : 0;   // guided: folded in the accumulators
    // the reference's running maxima start at 0 with index -1 (ProgramCU.cu:1803)
    int mx = t.max + rt, sc = t.second + rt;
    int idx = t.idx;
    if (mx <= 0) { mx = 0; idx = -1; }
    if (sc < 0) sc = 0;
    if (best) best[r] = Top2{mx, idx, sc};
    const float d1 = dist[min(mx, 262144)], d2 = dist[min(sc, 262144)];
    out[r] = (d1 < distmax) && (d1 < d2 * ratiomax) ? idx : -1;
}

// Geometric test of MultiplyDescriptorG_Kernel (ProgramCU.cu:1648-1681), once per pair, in
// the operation order of oracle::guided_pass (row-only and column-only terms are hoisted, which
// does not change any value; FDIV(a, b) = a * (1 / b)).  One thread per (8-row block of set 1,
// 4 columns of set 2); it writes both masks k_match_rows<1/2> read:
//   rmask[g][j] (4-row groups g of set 1, pitch pitch_r): bit i = pass(4g+i, j), bits 4-7 = good
//   cmask[q][r] (4-row groups q of set 2, pitch pitch_c): bit c = pass(r, 4q+c), bit 4+c = good
// where good(r, j) = some row of r's 8-row block passes at j (good_count > 0, :1682).
__global__ __launch_bounds__(256) void k_guided_mask(const float2* __restrict__ loc1, int n1,
                                                     const float2* __restrict__ loc2, int n2,
                                                     GuidedParams gp, uint8_t* __restrict__ rmask,
                                                     int pitch_r, uint8_t* __restrict__ cmask,
                                                     int pitch_c) {
    const int nq = (n2 + 3) >> 2, nblk = (n1 + 7) >> 3;
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (int64_t)nq * nblk) return;
    const int q = (int)(t % nq), blk = (int)(t / nq);
    const float* H = gp.H;
    const float* F = gp.F;
    float x2[4], y2[4], t0[4], t1[4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const int j = q * 4 + c;
        const float2 l = j < n2 ? loc2[j] : make_float2(0.f, 0.f);
        x2[c] = l.x;
        y2[c] = l.y;
        t0[c] = __builtin_fmaf(F[0], l.x, __builtin_fmaf(F[3], l.y, F[6]));
        t1[c] = __builtin_fmaf(F[1], l.x, __builtin_fmaf(F[4], l.y, F[7]));
    }
    uint32_t pass = 0;   // bit k * 4 + c
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const int r = blk * 8 + k;
        if (r >= n1) break;
        const float2 l = loc1[r];
        const float h0 = __builtin_fmaf(H[0], l.x, __builtin_fmaf(H[1], l.y, H[2]));
        const float h1 = __builtin_fmaf(H[3], l.x, __builtin_fmaf(H[4], l.y, H[5]));
        const float h2 = __builtin_fmaf(H[6], l.x, __builtin_fmaf(H[7], l.y, H[8]));
        const float rh = 1.0f / h2;
        const float u = h0 * rh, v = h1 * rh;
        const float f0 = __builtin_fmaf(F[0], l.x, __builtin_fmaf(F[1], l.y, F[2]));
        const float f1 = __builtin_fmaf(F[3], l.x, __builtin_fmaf(F[4], l.y, F[5]));
        const float f2 = __builtin_fmaf(F[6], l.x, __builtin_fmaf(F[7], l.y, F[8]));
        const float d0 = __builtin_fmaf(f1, f1, f0 * f0);
#pragma unroll
        for (int c = 0; c < 4; c++) {
            if (q * 4 + c >= n2) break;
            if (!(__builtin_fabsf(u - x2[c]) < gp.hdistmax && __builtin_fabsf(v - y2[c]) < gp.hdistmax))
                continue;
            const float x2fx1 = __builtin_fmaf(x2[c], f0, __builtin_fmaf(y2[c], f1, f2));
            const float den = __builtin_fmaf(t1[c], t1[c], __builtin_fmaf(t0[c], t0[c], d0));
            const float se = (x2fx1 * x2fx1) * (1.0f / den);
            if (se < gp.fdistmax) pass |= 1u << (k * 4 + c);
        }
    }
    uint32_t good = 0;   // bit c
#pragma unroll
    for (int c = 0; c < 4; c++) good |= ((pass & (0x11111111u << c)) != 0) << c;
    // rmask: groups 2 blk + h, bytes for columns 4q .. 4q+3
#pragma unroll
    for (int h = 0; h < 2; h++) {
        uint32_t w = 0;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            uint32_t b = ((good >> c) & 1u) ? 0xf0u : 0u;
#pragma unroll
            for (int i = 0; i < 4; i++) b |= ((pass >> ((4 * h + i) * 4 + c)) & 1u) << i;
            w |= b << (8 * c);
        }
        *reinterpret_cast<uint32_t*>(rmask + (size_t)(2 * blk + h) * pitch_r + q * 4) = w;
    }
    // cmask: group q, bytes for rows 8 blk .. 8 blk + 7
    if (cmask) {
        uint32_t w[2] = {0, 0};
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint32_t b = ((pass >> (k * 4)) & 0xfu) | (good << 4);
            w[k >> 2] |= b << (8 * (k & 3));
        }
        *reinterpret_cast<uint2*>(cmask + (size_t)q * pitch_c + blk * 8) = make_uint2(w[0], w[1]);
    }
}

}  // namespace

hipError_t launch_guided_mask(const float* loc1, int n1, const float* loc2, int n2,
                              const GuidedParams& gp, uint8_t* rmask, int pitch_r,
                              uint8_t* cmask, int pitch_c, hipStream_t stream) {
    if (n1 <= 0 || n2 <= 0) return hipSuccess;
    if ((pitch_r & 3) || pitch_r < n2 || (cmask && ((pitch_c & 7) || pitch_c < n1)))
        return hipErrorInvalidValue;
    const int64_t threads = (int64_t)((n2 + 3) / 4) * ((n1 + 7) / 8);
    hipLaunchKernelGGL(k_guided_mask, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, stream,
                       reinterpret_cast<const float2*>(loc1), n1,
                       reinterpret_cast<const float2*>(loc2), n2, gp, rmask, pitch_r, cmask,
                       pitch_c);
    return hipGetLastError();
}

hipError_t launch_rowsums(const uint8_t* d, int n, int* out, int scale, int bias,
                          hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_rowsum, dim3((n + 3) / 4), dim3(256), 0, stream, d, n, out, scale, bias);
    return hipGetLastError();
}

int match_chunks(int nA, int nB) {
    // enough workgroups to fill 256 CUs ~4 deep; each chunk at least two tiles wide
    const int panels = (nA + kPanel - 1) / kPanel;
    int chunks = (1024 + panels - 1) / panels;
    const int max_chunks = max(1, (nB + 2 * kTile - 1) / (2 * kTile));
    return max(1, min(chunks, max_chunks));
}

hipError_t launch_match_rows(const uint8_t* A, int nA, const uint8_t* B, int nB,
                             const int* col_term, int chunks, Top2* part, hipStream_t stream,
                             int guided_mode, const int* row_term, const uint8_t* mask,
                             int mask_pitch) {
    if (nA <= 0 || nB <= 0) return hipSuccess;
    int per = (nB + chunks - 1) / chunks;
    per = (per + kTile - 1) / kTile * kTile;
    dim3 grid((nA + kPanel - 1) / kPanel, chunks);
    if (guided_mode != 0 && (!row_term || !mask || mask_pitch < nB)) return hipErrorInvalidValue;
    if (guided_mode == 0)
        hipLaunchKernelGGL(k_match_rows<0>, grid, dim3(256), 0, stream, A, nA, B, nB, col_term,
                           per, part, row_term, mask, mask_pitch);
    else if (guided_mode == 1)
        hipLaunchKernelGGL(k_match_rows<1>, grid, dim3(256), 0, stream, A, nA, B, nB, col_term,
                           per, part, row_term, mask, mask_pitch);
    else
        hipLaunchKernelGGL(k_match_rows<2>, grid, dim3(256), 0, stream, A, nA, B, nB, col_term,
                           per, part, row_term, mask, mask_pitch);
    return hipGetLastError();
}

hipError_t launch_match_finish(const Top2* part, int n, int chunks, const int* row_term,
                               const float* dist, float distmax, float ratiomax, int* out,
                               Top2* best, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_match_finish, dim3((n + 255) / 256), dim3(256), 0, stream, part, n,
                       chunks, row_term, dist, distmax, ratiomax, out, best);
    return hipGetLastError();
}

}  // namespace sgk
