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
__global__ __launch_bounds__(256) void k_match_rows(const uint8_t* __restrict__ A, int nA,
                                                    const uint8_t* __restrict__ B, int nB,
                                                    const int* __restrict__ col_term,
                                                    int cols_per_chunk, Top2* __restrict__ part) {
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
#pragma unroll
        for (int cb = 0; cb < 8; cb++) {
            const int col = tb + cb * 16 + l16;
            const int ct = col < c_end ? col_term[col] : kNegCol;
            acc[0][cb] = v4i{ct, ct, ct, ct};
            acc[1][cb] = acc[0][cb];
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
                    const int key = (acc[rb][cb][i] << 3) | (7 - cb);
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
    const int rt = row_term[r];
    // the reference's running maxima start at 0 with index -1 (ProgramCU.cu:1803)
    int mx = t.max + rt, sc = t.second + rt;
    int idx = t.idx;
    if (mx <= 0) { mx = 0; idx = -1; }
    if (sc < 0) sc = 0;
    if (best) best[r] = Top2{mx, idx, sc};
    const float d1 = dist[min(mx, 262144)], d2 = dist[min(sc, 262144)];
    out[r] = (d1 < distmax) && (d1 < d2 * ratiomax) ? idx : -1;
}

}  // namespace

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
                             const int* col_term, int chunks, Top2* part, hipStream_t stream) {
    if (nA <= 0 || nB <= 0) return hipSuccess;
    int per = (nB + chunks - 1) / chunks;
    per = (per + kTile - 1) / kTile * kTile;
    dim3 grid((nA + kPanel - 1) / kPanel, chunks);
    hipLaunchKernelGGL(k_match_rows, grid, dim3(256), 0, stream, A, nA, B, nB, col_term, per, part);
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
