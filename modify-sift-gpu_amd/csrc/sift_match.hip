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
#include <algorithm>
#include <type_traits>

#include "sift_kernels.h"

namespace sgk {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));

constexpr int kPanel = 128;      // A rows per workgroup (4 waves x 32)
constexpr int kTile = 128;       // B columns per LDS tile
constexpr int kCtPad = kTile;    // k_match_raw: zero column terms past nB (launch_prep_set)
constexpr int kCtMissing = -6291456;   // k_match_raw's column term of a column past nB (-2^22 - 2^21)
#ifndef SGK_MATCH_LDSROW
#define SGK_MATCH_LDSROW 144
#endif
constexpr int kLdsRow = SGK_MATCH_LDSROW;   // bytes per staged B row (padding against bank conflicts)
#ifndef SGK_MATCH_PF
#define SGK_MATCH_PF 1     // RAW kernel: tiles of staging loads in flight (1 or 2)
#endif
#ifndef SGK_MATCH_PIPE
#define SGK_MATCH_PIPE 1   // RAW kernel: column groups software-pipelined across tiles (0: tile by tile)
#endif
#ifndef SGK_MATCH_PKEY
#define SGK_MATCH_PKEY 1   // RAW fold: the tile index packed below the tile maximum (see k_match_rows)
#endif
constexpr int kMaxChunkTiles = 256;   // RAW packed keys: tiles per column chunk fit 8 bits
// Running maxima hold keys (acc << 7) | low, acc = dot - row term (- guided bias) in
// [-2^23 - 2^22, 2^23]: every key fits in int32 and INT_MIN is below all of them.
constexpr int kNeg = INT_MIN;
// Column term of a missing column: its acc stays <= 0 (a staged zero column adds at most 2^21),
// so with the row term >= 0 added in the finish it can neither win nor raise a second maximum,
// and (acc << 7) does not overflow.
constexpr int kNegCol = -(1 << 22);
#ifdef SGK_MATCH_SPLIT
constexpr int kMatchSplit = SGK_MATCH_SPLIT;   // column groups per tile of the keyless kernel
#else
constexpr int kMatchSplit = 2;   // 126 VGPRs: 4 waves per SIMD (one group of 8: 160, 3 waves)
#endif
static_assert(kMatchSplit == 1 || kMatchSplit == 2, "1 or 2 column groups");

// v_med3_i32: the median of three.  With s <= m, med3(s, m, v) is the new second maximum after
// seeing v (v > m -> m; s < v <= m -> v; v <= s -> s).  Written as min / max, which LLVM selects
// as one v_med3_i32 -- compiler-visible, so the hazard recognizer inserts the wait states an
// MFMA result needs before it is read (an inline-asm v_med3 hid that read from it and lost
// matches in rows 4q+1, 4q+2; round 2).
__device__ __forceinline__ int med3i(int a, int b, int c) {
    return max(min(a, b), min(max(a, b), c));
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

// Column chunks of one launch: ~4096 workgroups (about 5 per resident slot at 3 per CU) so
// that the last wave of workgroups is a small tail; each chunk at least two tiles wide.  Also
// evaluated on the device for a row count that only the device knows (compacted rows).
#ifndef SGK_MATCH_WG
#define SGK_MATCH_WG 4096
#endif
constexpr int kMatchWg = SGK_MATCH_WG;   // workgroups aimed at per launch (tuning knob)

// k_match_raw (LDS-DMA keyless kernel): 256-row panels, and 2 workgroups resident per CU (55 KB
// of LDS and 128 VGPRs each), 512 on the chip.  Its split is picked by a cost model instead of a
// workgroup target: for r = 1 .. kRawMaxRounds rounds of resident workgroups, the most chunks
// that fit r rounds; cost = rounds x (tiles per chunk + a chunk's fixed cost in tiles: its A
// fragments, the first two tiles in flight and the partials); the cheapest wins (ties: fewer
// chunks).  C5 rows: 5 chunks (2 rounds of 79 tiles) instead of 11 (5 rounds of 36).
#ifndef SGK_MATCH_RAW_WAVES
#define SGK_MATCH_RAW_WAVES 8
#endif
constexpr int kRawWaves = SGK_MATCH_RAW_WAVES;
constexpr int kRawRows = 32 * kRawWaves;
#ifndef SGK_MATCH_SLOTS
#define SGK_MATCH_SLOTS 512
#endif
#ifndef SGK_MATCH_OVT
#define SGK_MATCH_OVT 2
#endif
constexpr int kRawSlots = SGK_MATCH_SLOTS;
constexpr int kRawOvt = SGK_MATCH_OVT;
constexpr int kRawMaxRounds = 8;

// dma: the split of a k_match_raw launch (above); otherwise ~kMatchWg workgroups of 128 rows
__host__ __device__ inline int chunks_for(int nA, int nB, bool dma = false) {
    const int max_chunks = max(1, (nB + 2 * kTile - 1) / (2 * kTile));
    const int min_chunks = max(1, (nB + kMaxChunkTiles * kTile - 1) / (kMaxChunkTiles * kTile));
    if (!dma) {
        const int panels = (nA + kPanel - 1) / kPanel;
        const int chunks = (kMatchWg + panels - 1) / panels;
        return max(min_chunks, min(chunks, max_chunks));
    }
    const int panels = max(1, (nA + kRawRows - 1) / kRawRows);
    int best = min_chunks, best_cost = INT_MAX;
    for (int r = 1; r <= kRawMaxRounds; r++) {
        const int c = max(min_chunks, min(max_chunks, r * kRawSlots / panels));
        const int rounds = (panels * c + kRawSlots - 1) / kRawSlots;
        const int tiles = ((nB + c - 1) / c + kTile - 1) / kTile;
        const int cost = rounds * (tiles + kRawOvt);
        if (cost < best_cost) { best_cost = cost; best = c; }
    }
    return best;
}

// u8 descriptors -> s8 (s = u - 128, xor 0x80), once per match call for both sets
__global__ __launch_bounds__(256) void k_to_s8(const uint4* __restrict__ src, size_t n16,
                                               uint4* __restrict__ dst) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        uint4 v = src[i];
        v.x ^= 0x80808080u; v.y ^= 0x80808080u; v.z ^= 0x80808080u; v.w ^= 0x80808080u;
        dst[i] = v;
    }
}

// One pass over a descriptor set: the s8 form (xor 0x80), the row sums scale * sum(u8) + bias,
// and `nzero` ints of `zero` cleared (the matched-column flags).  A thread per 16 bytes, a
// descriptor per 8 consecutive lanes (the grid stride keeps the groups whole).
__global__ __launch_bounds__(256) void k_prep_set(const uint4* __restrict__ src, size_t n16,
                                                  uint4* __restrict__ dst, int* __restrict__ sums,
                                                  int scale, int bias, int* __restrict__ zero,
                                                  int nzero, int* __restrict__ ctp, int n,
                                                  int* __restrict__ ctfill) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) {
        uint4 v = src[i];
        int t = __builtin_amdgcn_udot4(v.x, 0x01010101u, 0, false);
        t = __builtin_amdgcn_udot4(v.y, 0x01010101u, t, false);
        t = __builtin_amdgcn_udot4(v.z, 0x01010101u, t, false);
        t = __builtin_amdgcn_udot4(v.w, 0x01010101u, t, false);
        v.x ^= 0x80808080u; v.y ^= 0x80808080u; v.z ^= 0x80808080u; v.w ^= 0x80808080u;
        dst[i] = v;
        t += __shfl_xor(t, 1, 64);
        t += __shfl_xor(t, 2, 64);
        t += __shfl_xor(t, 4, 64);
        if ((i & 7) == 0) {
            if (sums) sums[i >> 3] = scale * t + bias;
            if (ctp) ctp[i >> 3] = 128 * t - 2097152;   // k_match_raw's biased column term
            if (ctfill) ctfill[i >> 3] = kCtMissing;
        }
    }
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < (size_t)nzero; i += stride) zero[i] = 0;
    if (ctp)
        for (int i = blockIdx.x * 256 + threadIdx.x; i < kCtPad; i += (int)stride) ctp[n + i] = kCtMissing;
    if (ctfill)
        for (int i = blockIdx.x * 256 + threadIdx.x; i < kCtPad; i += (int)stride) ctfill[n + i] = kCtMissing;
}

// Equal-dot order of the two decisions: does column a come before column b (-1 = none)?
template <bool TIE32>
__device__ __forceinline__ bool tie_before(int a, int b) {
    if (a < 0) return false;
    if (b < 0) return true;
    if (TIE32 && (a & 31) != (b & 31)) return (a & 31) < (b & 31);
    return a < b;
}

// One row panel of A against columns [c_begin, c_end) of B.
// part[chunk * nA + row] = running top-2 of row over those columns (dot without the row term).
//
// Guided matching (GUIDED: the guided values of MultiplyDescriptorG_Kernel, ProgramCU.cu:
// 1683-1733, for the row decision with A = set 1 or the column decision with A = set 2).  The
// reference's value of a pair is dot (pass), dot - 2^18 (fail, but its 8-row block of set 1 has
// a passing row: good_count > 0) or -2^18 (no passing row); rows see max(v, 0).  Both decisions
// only ask which values are > 0 and how they order (running top-2 from (0, -1, 0); the finish
// clamps at 0), so dot - bias with bias = 2^18 * fail + 2^23 * !good decides identically
// (dot < 2^23 for u8 descriptors).  The bias goes into the accumulator's initial value, the row
// term stays in the finish as in the plain matcher: two VALU per value more than plain.
// `mask` (k_guided_mask) holds, per (32-row block of A, 128-column tile of B, lane), the lane's
// 16-byte record: byte rb * 8 + cb covers rows 32 R + 16 rb + 4 quad + i and column
// 128 T + 16 cb + l16 of this lane's accumulators; bit i = that pair fails the geometric test,
// bit 4+i = no row of its 8-row block of set 1 passes.  One dwordx4 load per lane and tile.
//
// Equal dots: the column side (A = set 2) takes the lowest column (ColMatch's row order); the
// row side (A = set 1, TIE32) takes the column lowest mod 32, then the lowest, as RowMatch_Kernel's
// 32 strided threads and tree reduction do (ProgramCU.cu:1803-1835).  Inside a tile the key's 7
// low bits order equal dots that way, so the tile's maximum key is its winner.  Across tiles a
// later tile may only take over when the key's tie-relevant prefix grows (the dot; TIE32: the dot
// and col % 32), and the key is recorded with its tile at that moment.
//
// COLS (mutual matching, one GEMM for both decisions): every tile also yields the column side
// (ColMatch_Kernel's decision over set-1 rows, ProgramCU.cu:1844-1900, fed by
// MultiplyDescriptor_Kernel's per-block partials, :1540-1552).  A column's value over the rows
// is acc + row term (= dot - column term; guided: = the guided value, the column term is already
// in acc); per column the panel's (max, argmax row, second) comes from keys ((acc + rt) << 7) |
// (127 - row in panel) -- equal values keep the lowest row -- merged over the 16 lanes and 4
// waves that hold the column and written to colpart[panel][column].  k_match_cols merges the
// panels in row order.  The row side is the plain kernel's.
// RAW (plain matching with ratiomax <= 1): the values are folded as they are, no key -- the
// accumulators start at the column term, a lane takes each row's maximum over its 8 columns of
// the tile (v_max3 chains, half a VALU per value) and folds only that into its running (max,
// second), recording the tile in which the maximum last grew (as the low 8 bits of the folded
// key: (tile maximum << 8) | tile index in the chunk).  The second is then the second
// largest (tile, lane) maximum -- a lower bound of the row's second, exact unless the row's two
// largest values share the winning lane's tile.  k_match_finish recomputes the dot products of
// those 8 columns for every row that passes the ratio test with the lower bound (a row that
// fails it fails with the exact second too): they give the column of the maximum and the
// second within them, and the test is repeated with the larger second.  A row that passes has
// second < max, so its maximum is unique and no tie order is needed (an equal second maximum
// fails the test for ratiomax <= 1, whichever column the reference would have named).
// amap / an (compacted rows): row r of A is A[amap[r]], and the row count is *an, known only on
// the device; the grid is then 1-D and each workgroup derives its (panel, chunk) from the count,
// with the split chunks_for(*an, nB) (k_match_finish derives the same one).
#ifndef SGK_MATCH_RAW_WPE
#define SGK_MATCH_RAW_WPE 1   // minimum waves per SIMD asked of the RAW kernel (1: no cap)
#endif
template <bool GUIDED, bool TIE32, bool COLS, bool RAW = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RAW ? SGK_MATCH_RAW_WPE : 1))) void k_match_rows(const uint8_t* __restrict__ A, int nA,
                                                    const uint8_t* __restrict__ B, int nB,
                                                    int cols_per_chunk, Top2* __restrict__ part,
                                                    const uint4* __restrict__ mask,
                                                    int mask_tiles,
                                                    const int* __restrict__ row_term,
                                                    Top2* __restrict__ colpart,
                                                    const int* __restrict__ amap,
                                                    const int* __restrict__ an) {
    __shared__ __attribute__((aligned(16))) uint8_t s_b[2][kTile * kLdsRow];
    __shared__ int s_ct[2][kTile];   // column terms of the staged tile (from its bytes)
    __shared__ int s_cm[COLS ? 4 : 1][COLS ? kTile : 1], s_cs[COLS ? 4 : 1][COLS ? kTile : 1];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int panel = blockIdx.x, chunk = blockIdx.y;
    if (an) {
        nA = *an;
        if (nA <= 0) return;
        const int panels = (nA + kPanel - 1) / kPanel, chunks = chunks_for(nA, nB);
        if ((int)blockIdx.x >= panels * chunks) return;
        panel = blockIdx.x % panels;
        chunk = blockIdx.x / panels;
        cols_per_chunk = ((nB + chunks - 1) / chunks + kTile - 1) / kTile * kTile;
    }
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
            if (row < nA) {
                const int src = amap ? amap[row] : row;
                afrag[rb][kh] = *reinterpret_cast<const v4i*>(A + (size_t)src * 128 + kh * 64 + quad * 16);
            }
            else afrag[rb][kh] = v4i{0, 0, 0, 0};
        }
    }
    // COLS: per row of this lane, the column keys' addend (row term << 7) | (127 - row in
    // panel); rows past nA get a row term of -2^22, so their values stay <= 0 and can only win
    // a column whose result the finish clamps to "no match" anyway
    int rtlow[2][4];
#pragma unroll
    for (int rb = 0; rb < 2; rb++)
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int rp = wave * 32 + rb * 16 + quad * 4 + i, row = panel * kPanel + rp;
            rtlow[rb][i] = COLS ? (((row < nA ? row_term[row] : -(1 << 22)) << 7) | (127 - rp)) : 0;
        }
    // guided: this lane's mask records (rows past nA read none)
    const bool rec_ok = GUIDED && panel * kPanel + wave * 32 < nA;
    const uint4* rec_p = rec_ok ? mask + (size_t)(panel * 4 + wave) * mask_tiles * 64 + lane : nullptr;
    uint4 rec = make_uint4(0, 0, 0, 0);
    if (rec_ok && c_begin < c_end) rec = rec_p[(c_begin / kTile) * 64];
    // running state for this lane's 8 output rows: (rb, i) -> row wave*32 + rb*16 + quad*4 + i:
    // max key, second key, tile of the winner and the winner's key when it was taken
    int M[2][4], S[2][4], I[2][4], W[2][4];
#pragma unroll
    for (int rb = 0; rb < 2; rb++)
#pragma unroll
        for (int i = 0; i < 4; i++) { M[rb][i] = kNeg; S[rb][i] = kNeg; I[rb][i] = -1; W[rb][i] = 0; }
    constexpr uint32_t kPrefix = TIE32 ? 4u : 128u;   // keys differing below this bit tie

    // staging: thread t copies 64 bytes: column t>>1, half (t&1).  The loads are unconditional
    // (columns past the set clamped to its last one; stage_store zeroes columns past the chunk),
    // so the compiler's wait before a store counts only the loads older than it.
    auto stage_load = [&](int tbase, uint4* r) {
        const int col = min(tbase + (tid >> 1), nB - 1);
        const uint8_t* src = B + (size_t)col * 128 + (tid & 1) * 64;
#pragma unroll
        for (int q = 0; q < 4; q++) r[q] = reinterpret_cast<const uint4*>(src)[q];
    };
    // The column term 128 * sum(u8 B[col]) - 2^21 is formed here from the staged s8 bytes
    // (sum(u) = sum(s) + 128 * 128; byte sums by v_dot4_i32_i8, the two half-columns joined by
    // one shuffle) instead of being loaded from global memory per tile: those loads sat between
    // the next tile's staging loads and the MFMAs, and waiting for them waited for the whole
    // prefetch.
    auto stage_store = [&](int buf, const uint4* r, int tbase) {
        uint8_t* dst = &s_b[buf][(tid >> 1) * kLdsRow + (tid & 1) * 64];
        const bool in_chunk = tbase + (tid >> 1) < c_end;
        int sum = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint4 v = in_chunk ? r[q] : make_uint4(0, 0, 0, 0);
            sum = __builtin_amdgcn_sdot4((int)v.x, 0x01010101, sum, false);
            sum = __builtin_amdgcn_sdot4((int)v.y, 0x01010101, sum, false);
            sum = __builtin_amdgcn_sdot4((int)v.z, 0x01010101, sum, false);
            sum = __builtin_amdgcn_sdot4((int)v.w, 0x01010101, sum, false);
            reinterpret_cast<uint4*>(dst)[q] = v;
        }
        sum += __shfl_xor(sum, 1, 64);
        if (!(tid & 1)) {
            const int col = tbase + (tid >> 1);
            s_ct[buf][tid >> 1] = col < c_end ? 128 * (sum + 16384) - 2097152 : kNegCol;
        }
    };

    // the key's low 7 bits per column block: a larger value = an earlier column in the
    // reference's tie order (TIE32: (31 - col % 32) << 2 | (3 - col / 32 in the tile); else
    // 127 - col in the tile)
    int low[8];
#pragma unroll
    for (int cb = 0; cb < 8; cb++)
        low[cb] = TIE32 ? ((31 - ((cb & 1) * 16 + l16)) << 2) | (3 - (cb >> 1))
                        : 127 - (cb * 16 + l16);

    // Tile j is computed from LDS buffer j & 1.  kPf = 2 (RAW): tile j + 2's loads are issued
    // at the start of tile j into register set j & 1 (free: tile j was stored before), and tile
    // j + 1 (register set (j + 1) & 1, loaded during tile j - 1) is stored at its end -- two
    // tiles of latency for every load.  kPf = 1: tile j + 1 is loaded and stored within tile j.
    // The loop is unrolled by two so that the register sets are static.
    constexpr int kPf = RAW ? SGK_MATCH_PF : 1;
    uint4 stg[2][4];
    if (c_begin < c_end) {
        stage_load(c_begin, stg[0]);
        stage_store(0, stg[0], c_begin);
        if constexpr (kPf == 2) stage_load(c_begin + kTile, stg[1]);
    }
    __syncthreads();
    auto tile = [&](auto par, int tb) {
        constexpr int buf = decltype(par)::value;
        const bool has_next = tb + kTile < c_end;
        if constexpr (kPf == 2) {
            stage_load(tb + 2 * kTile, stg[buf]);
            __builtin_amdgcn_sched_barrier(0);   // issue the loads here, before the MFMAs
        } else {
            stage_load(tb + kTile, stg[buf ^ 1]);
        }
        uint4 rec_next = rec;
        if (rec_ok && has_next) rec_next = rec_p[(tb / kTile + 1) * 64];
        int mt[2][4], st[2][4];
        if constexpr (!RAW) {
#pragma unroll
            for (int rb = 0; rb < 2; rb++)
#pragma unroll
                for (int i = 0; i < 4; i++) { mt[rb][i] = M[rb][i]; st[rb][i] = S[rb][i]; }
        }
        if constexpr (RAW) {
            // the tile in kMatchSplit column groups (accumulators start at the column term;
            // MFMAs, then the tile maxima, per group)
            constexpr int CB = 8 / kMatchSplit;
            int tmx[2][4];
#pragma unroll
            for (int h = 0; h < kMatchSplit; h++) {
                v4i acc[2][CB];
#pragma unroll
                for (int c = 0; c < CB; c++) {
                    const int ct = s_ct[buf][(h * CB + c) * 16 + l16];
                    acc[0][c] = v4i{ct, ct, ct, ct};
                    acc[1][c] = acc[0][c];
                }
#pragma unroll
                for (int c = 0; c < CB; c++) {
#pragma unroll
                    for (int kh = 0; kh < 2; kh++) {
                        const v4i bfrag = *reinterpret_cast<const v4i*>(
                            s_b[buf] + ((h * CB + c) * 16 + l16) * kLdsRow + kh * 64 + quad * 16);
                        acc[0][c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(afrag[0][kh], bfrag, acc[0][c], 0, 0, 0);
                        acc[1][c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(afrag[1][kh], bfrag, acc[1][c], 0, 0, 0);
                    }
                }
                // the tile's maximum per row over this lane's 8 columns (v_max3 chains: half a
                // VALU per value); folded into the running top-2 once per tile below
#pragma unroll
                for (int rb = 0; rb < 2; rb++)
#pragma unroll
                    for (int i = 0; i < 4; i++)
#pragma unroll
                        for (int c = 0; c < CB; c += 2) {
                            const int a = acc[rb][c][i], b2 = acc[rb][c + 1][i];
                            tmx[rb][i] = (h == 0 && c == 0) ? max(a, b2) : max(max(tmx[rb][i], a), b2);
                        }
            }
            // one fold per row and tile: the running (max, second) over the lane's tile maxima,
            // and the tile where the maximum last grew.  The exact second of the row is the
            // larger of that second and the second within the winning (tile, lane) set of 8
            // columns, which k_match_finish recomputes for every row that can still pass.
#if SGK_MATCH_PKEY
            // keys (tile maximum << 8) | tile index in the chunk: |maximum| <= 2^22, at most
            // kMaxChunkTiles tiles per chunk (chunks_for); one v_lshl_or instead of the
            // compare + select that recorded the tile
            const int tl = (tb - c_begin) / kTile;
#pragma unroll
            for (int rb = 0; rb < 2; rb++)
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int key = (tmx[rb][i] << 8) | tl;
                    S[rb][i] = med3i(S[rb][i], M[rb][i], key);
                    M[rb][i] = max(M[rb][i], key);
                }
#else
#pragma unroll
            for (int rb = 0; rb < 2; rb++)
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int v = tmx[rb][i], mo = M[rb][i];
                    S[rb][i] = med3i(S[rb][i], mo, v);
                    I[rb][i] = v > mo ? tb : I[rb][i];
                    M[rb][i] = max(mo, v);
                }
#endif
        } else {
        // plain: the accumulators start at 0 and the column term enters the key,
        // key = (acc << 7) + ((ct << 7) | low) = ((acc + ct) << 7) | low;
        // guided: they start at the column term minus the geometric bias (invalid columns: -inf)
        v4i acc[2][8];
        int ctlow[8];
#pragma unroll
        for (int cb = 0; cb < 8; cb++) {
            const int ct = s_ct[buf][cb * 16 + l16];
            if constexpr (!GUIDED) {
                ctlow[cb] = (ct << 7) | low[cb];
                acc[0][cb] = v4i{0, 0, 0, 0};
                acc[1][cb] = acc[0][cb];
            } else {
                ctlow[cb] = low[cb];
#pragma unroll
                for (int rb = 0; rb < 2; rb++) {
                    const uint32_t w = rb == 0 ? (cb < 4 ? rec.x : rec.y) : (cb < 4 ? rec.z : rec.w);
                    const int mb = (int)(w >> ((cb & 3) * 8));
#pragma unroll
                    for (int i = 0; i < 4; i++)
                        acc[rb][cb][i] = ct - (((mb >> i) & 1) << 18) - (((mb >> (4 + i)) & 1) << 23);
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
        // (acc << 7) | low[cb]: one v_lshl_or, one v_max and one v_med3 per value; the tile is
        // recorded once per tile when the maximum moved.  The second key of an equal pair
        // carries the same dot, so exact ties still reach the ratio test as the reference's do.
        // Column blocks 0..3 of every row first (their MFMAs finished earliest), then 4..7:
        // each row still folds its keys in column order, and the first half's reads do not
        // wait on the last MFMAs.
        if constexpr (!COLS) {
#pragma unroll
            for (int half = 0; half < 2; half++)
#pragma unroll
                for (int rb = 0; rb < 2; rb++)
#pragma unroll
                    for (int i = 0; i < 4; i++)
#pragma unroll
                        for (int cb = 4 * half; cb < 4 * half + 4; cb++) {
                            const int key = (acc[rb][cb][i] << 7) + ctlow[cb];
                            st[rb][i] = med3i(st[rb][i], mt[rb][i], key);
                            mt[rb][i] = max(mt[rb][i], key);
                        }
        } else {
            // both sides per column block, so that each accumulator block dies after its
            // folds: the row keys into the running row state, the column keys ((acc << 7) |
            // (127 - row in panel)) over this lane's 8 rows, then over the 4 lanes of the column
            // in this wave (xor 16, 32); the 4 waves meet in LDS
#pragma unroll
            for (int cb = 0; cb < 8; cb++) {
                int cm = kNeg, cs = kNeg;
#pragma unroll
                for (int rb = 0; rb < 2; rb++)
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        const int a = acc[rb][cb][i];
                        const int key = (a << 7) + ctlow[cb];
                        st[rb][i] = med3i(st[rb][i], mt[rb][i], key);
                        mt[rb][i] = max(mt[rb][i], key);
                        const int ck = (a << 7) + rtlow[rb][i];
                        cs = med3i(cs, cm, ck);
                        cm = max(cm, ck);
                    }
                // lanes l, l ^ 16 and l ^ 32 by v_permlane16/32_swap (VALU, no LDS): after a
                // swap of a value with itself the two results hold the pair's two values
                {
                    const auto a = __builtin_amdgcn_permlane16_swap(cm, cm, false, false);
                    const auto b2 = __builtin_amdgcn_permlane16_swap(cs, cs, false, false);
                    const int a0 = (int)a[0], a1 = (int)a[1];
                    cs = max(min(a0, a1), max((int)b2[0], (int)b2[1]));
                    cm = max(a0, a1);
                }
                {
                    const auto a = __builtin_amdgcn_permlane32_swap(cm, cm, false, false);
                    const auto b2 = __builtin_amdgcn_permlane32_swap(cs, cs, false, false);
                    const int a0 = (int)a[0], a1 = (int)a[1];
                    cs = max(min(a0, a1), max((int)b2[0], (int)b2[1]));
                    cm = max(a0, a1);
                }
                if (quad == 0) {
                    s_cm[wave][cb * 16 + l16] = cm;
                    s_cs[wave][cb * 16 + l16] = cs;
                }
            }
        }
        }   // !RAW
        if constexpr (!RAW) {
#pragma unroll
            for (int rb = 0; rb < 2; rb++)
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int m = mt[rb][i];
                    const bool took = (uint32_t)(m ^ M[rb][i]) >= kPrefix;
                    I[rb][i] = took ? tb : I[rb][i];
                    W[rb][i] = took ? m : W[rb][i];
                    M[rb][i] = m;
                    S[rb][i] = st[rb][i];
                }
        }
        // One barrier per tile suffices without COLS: the stores below go to the buffer of tile
        // t - 1, which every wave finished reading before the barrier that ended iteration t - 1
        // (COLS: the panel merge reads the other waves' s_cm / s_cs first).
        if constexpr (COLS) __syncthreads();
        if constexpr (COLS) {
            if (tid < kTile && tb + tid < c_end) {
                int cm = s_cm[0][tid], cs = s_cs[0][tid];
#pragma unroll
                for (int w = 1; w < 4; w++) {
                    const int m2 = s_cm[w][tid], s2 = s_cs[w][tid];
                    cs = max(min(cm, m2), max(cs, s2));
                    cm = max(cm, m2);
                }
                colpart[(size_t)panel * nB + tb + tid] =
                    Top2{cm >> 7, panel * kPanel + 127 - (cm & 127), cs >> 7};
            }
        }
        if (has_next) stage_store(buf ^ 1, stg[buf ^ 1], tb + kTile);
        rec = rec_next;
        __syncthreads();
    };
    for (int tb = c_begin; tb < c_end; tb += 2 * kTile) {
        tile(std::integral_constant<int, 0>{}, tb);
        if (tb + kTile < c_end) tile(std::integral_constant<int, 1>{}, tb + kTile);
    }
    // keys -> (acc, column); RAW: (tile, lane) -> tile + l16, the lane's columns in the tile
#pragma unroll
    for (int rb = 0; rb < 2; rb++)
#pragma unroll
        for (int i = 0; i < 4; i++) {
            if constexpr (RAW) {
#if SGK_MATCH_PKEY
                const int m = M[rb][i], sk = S[rb][i];
                I[rb][i] = m == kNeg ? -1 : c_begin + (m & 255) * kTile + l16;
                M[rb][i] = m == kNeg ? kNeg : m >> 8;
                S[rb][i] = sk == kNeg ? kNeg : sk >> 8;
#else
                I[rb][i] = I[rb][i] < 0 ? -1 : I[rb][i] + l16;
#endif
            } else {
                const int k = W[rb][i] & 127;
                const int in_tile = TIE32 ? (3 - (k & 3)) * 32 + (31 - (k >> 2)) : 127 - k;
                I[rb][i] = I[rb][i] < 0 ? -1 : I[rb][i] + in_tile;
                M[rb][i] >>= 7;
                S[rb][i] >>= 7;
            }
        }
    // merge the 16 lanes that share a row (same quad): xor 1, 2, 4, 8; equal dots resolve in the
    // side's tie order
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
                I[rb][i] = (m2 > m1 || (!RAW && m2 == m1 && tie_before<TIE32>(i2, i1))) ? i2 : i1;
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

// k_match_raw: the RAW row kernel (plain matching, ratiomax <= 1) with the B tiles staged by
// LDS-DMA (global_load_lds_dwordx4): no staging registers, so three LDS buffers keep two tiles of
// loads in flight across each tile's barrier (counted vmcnt, raw s_barrier), where the register
// staging of k_match_rows holds one (or two with copies the compiler adds).  Values, folds and
// partials are k_match_rows<.., RAW>'s:
//   * the column terms come precomputed (ctp[j] = 128 * sum(u8 B_j) - 2^21, launch_prep_set),
//     staged beside the tile four times over (a column's term fills one 16-B slot, read as the
//     v4i that starts the column's accumulators: no register moves); ctp is -2^22 - 2^21 for j
//     in [nB, nB + kTile) and columns past nB stage the last column's bytes, so their values
//     are acc - 2^22 - 2^21 < -128 * sum(u8 A_i) <= every real value of the row (no zeroing
//     select, which a DMA cannot apply);
//   * the tile image is XOR-swizzled by 16-B slots (slot j of column c at j ^ ((c >> 1) & 7)) so
//     the B-fragment ds_read_b128 are conflict-free; the DMA writes lane-linear 1-KB runs, so
//     the swizzle is applied to the per-lane global source address instead.
// NW waves per workgroup share each staged tile: a panel of 32 * NW rows of A.
constexpr int kRawBufs = 3;
typedef __attribute__((address_space(3))) void* lds_void_ptr;

#if SGK_MATCH_PIPE
#define SGK_RAW_ATTR __attribute__((amdgpu_waves_per_eu(4)))   // 128 VGPRs: 2 workgroups per CU
#else
#define SGK_RAW_ATTR
#endif
__global__ __launch_bounds__(64 * kRawWaves) SGK_RAW_ATTR void k_match_raw(const uint8_t* __restrict__ A, int nA,
                                                   const uint8_t* __restrict__ B, int nB,
                                                   const int* __restrict__ ctp, int cols_per_chunk,
                                                   Top2* __restrict__ part,
                                                   const int* __restrict__ amap,
                                                   const int* __restrict__ an,
                                                   const int* __restrict__ bn) {
    constexpr int NW = kRawWaves;
    constexpr int kRows = 32 * NW;        // panel rows
    constexpr int kDmaB = 16 / NW;        // 1-KB image runs per wave and tile
    constexpr int kCtW = kTile / NW;      // column terms staged per wave (lanes repeat them)
    static_assert(kTile * 128 == NW * kDmaB * 1024, "the image is NW x kDmaB runs");
    static_assert(kCtW * 4 == 64, "a wave stages its column terms as 16-B slots of 4 copies");
    __shared__ __attribute__((aligned(16))) uint8_t s_lds[kRawBufs * (kTile * 128 + NW * 256)];
    constexpr int kBuf = kTile * 128 + NW * 256;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int panel = blockIdx.x, chunk = blockIdx.y;
    if (bn) nB = *bn;   // a pruned B (launch_prune_set): its count on the device, B's bound at most
    if (an) {
        nA = *an;
        if (nA <= 0) return;
        const int panels = (nA + kRows - 1) / kRows, chunks = chunks_for(nA, nB, true);
        if ((int)blockIdx.x >= panels * chunks) return;
        panel = blockIdx.x % panels;
        chunk = blockIdx.x / panels;
        cols_per_chunk = ((nB + chunks - 1) / chunks + kTile - 1) / kTile * kTile;
    }
    const int c_begin = chunk * cols_per_chunk;
    const int c_end = min(nB, c_begin + cols_per_chunk);
    if (c_begin >= c_end) {
        // a chunk past the set (the split rounds up): empty partials, which k_match_finish reads
        if (tid < kRows && panel * kRows + tid < nA)
            part[(size_t)chunk * nA + panel * kRows + tid] = Top2{kNeg, -1, kNeg};
        return;
    }
    const int quad = lane >> 4, l16 = lane & 15;

    v4i afrag[2][2];
#pragma unroll
    for (int rb = 0; rb < 2; rb++) {
        const int row = panel * kRows + wave * 32 + rb * 16 + l16;
#pragma unroll
        for (int kh = 0; kh < 2; kh++) {
            if (row < nA) {
                const int src = amap ? amap[row] : row;
                afrag[rb][kh] = *reinterpret_cast<const v4i*>(A + (size_t)src * 128 + kh * 64 + quad * 16);
            } else {
                afrag[rb][kh] = v4i{0, 0, 0, 0};
            }
        }
    }
    // the A loads retire before any DMA is in flight (the compiler would otherwise wait for the
    // DMAs too at the first use of a fragment)
    __builtin_amdgcn_s_waitcnt(0xc07f & ~0xc00f);   // vmcnt(0)
    int M[2][4], S[2][4];
#pragma unroll
    for (int rb = 0; rb < 2; rb++)
#pragma unroll
        for (int i = 0; i < 4; i++) { M[rb][i] = kNeg; S[rb][i] = kNeg; }

    // this lane's DMA sources: instruction q fills 16-B slot (wave * kDmaB + q) * 64 + lane of
    // the image, i.e. column c = slot >> 3, position slot & 7, which holds the column's 16-B
    // piece (slot & 7) ^ ((c >> 1) & 7)
    int src_col[kDmaB], src_off[kDmaB];
#pragma unroll
    for (int q = 0; q < kDmaB; q++) {
        const int slot = (wave * kDmaB + q) * 64 + lane, c = slot >> 3;
        src_col[q] = c;
        src_off[q] = (((slot & 7) ^ ((c >> 1) & 7)) << 4);
    }
    auto issue = [&](int tb, int bi) {
        uint8_t* base = s_lds + bi * kBuf;
#pragma unroll
        for (int q = 0; q < kDmaB; q++) {
            const int col = min(tb + src_col[q], nB - 1);
            __builtin_amdgcn_global_load_lds(B + (size_t)col * 128 + src_off[q],
                                             (lds_void_ptr)(base + (wave * kDmaB + q) * 1024), 16, 0, 0);
        }
        const int ci = min(tb + wave * kCtW + lane / (64 / kCtW), nB + kCtPad - 1);
        __builtin_amdgcn_global_load_lds(ctp + ci, (lds_void_ptr)(base + kTile * 128 + wave * 256),
                                         4, 0, 0);
    };
    // this lane's LDS offsets in a tile buffer: column l16 of a 16-column block, its 16-B piece
    // j = 4 kh + quad at slot j ^ ((col >> 1) & 7) (the block's 16 columns do not change the
    // swizzle), and the column's term slot; the block adds a constant
    const int lane_b[2] = {l16 * 128 + ((quad ^ (l16 >> 1)) << 4), l16 * 128 + (((4 + quad) ^ (l16 >> 1)) << 4)};
    const int lane_ct = kTile * 128 + l16 * 16;
    // kDmaB + 1 DMA instructions per wave and tile: vmcnt(kDmaB + 1) retires all but the
    // newest tile (the immediate: vmcnt low bits, expcnt 7, lgkmcnt 0)
    constexpr int kWaitTile = 0x0070 | (kDmaB + 1);
    issue(c_begin, 0);
    issue(c_begin + kTile, 1);
    __builtin_amdgcn_s_waitcnt(kWaitTile);
    __builtin_amdgcn_s_barrier();
    // compiler memory barrier: the s_barrier intrinsic does not order memory operations for the
    // compiler, and no LDS read of a tile buffer may move above the barrier that publishes its DMA
    asm volatile("" ::: "memory");
#if SGK_MATCH_PIPE
    // software-pipelined by column group: group 1 of tile t is issued before group 0's fold, and
    // group 0 of tile t + 1 (after the barrier) before group 1's, so every fold's VALU work runs
    // beside MFMAs it does not depend on (the two groups' 64 accumulator registers, as before)
    static_assert(kMatchSplit == 2, "two column groups");
    constexpr int CB = 4;
    v4i g0[2][CB], g1[2][CB];
    int tmx[2][4];
    auto group = [&](int bi_, int h, v4i (&acc)[2][CB]) __attribute__((always_inline)) {
        const uint8_t* sb = s_lds + bi_ * kBuf;
#pragma unroll
        for (int c = 0; c < CB; c++) {
            const int cb = (h * CB + c) * 16;   // the column block: immediate offsets below
            const v4i ctv = *reinterpret_cast<const v4i*>(sb + lane_ct + cb * 16);
#pragma unroll
            for (int kh = 0; kh < 2; kh++) {
                const v4i bfrag = *reinterpret_cast<const v4i*>(sb + lane_b[kh] + cb * 128);
                acc[0][c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(afrag[0][kh], bfrag, kh ? acc[0][c] : ctv, 0, 0, 0);
                acc[1][c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(afrag[1][kh], bfrag, kh ? acc[1][c] : ctv, 0, 0, 0);
            }
        }
    };
    auto fold = [&](const v4i (&acc)[2][CB], bool first) __attribute__((always_inline)) {
#pragma unroll
        for (int rb = 0; rb < 2; rb++)
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int c = 0; c < CB; c += 2) {
                    const int a = acc[rb][c][i], b2 = acc[rb][c + 1][i];
                    tmx[rb][i] = (first && c == 0) ? max(a, b2) : max(max(tmx[rb][i], a), b2);
                }
    };
    int bi = 0;
    group(0, 0, g0);
    for (int tb = c_begin; tb < c_end; tb += kTile) {
        issue(tb + 2 * kTile, bi == 0 ? 2 : bi - 1);
        group(bi, 1, g1);
        fold(g0, true);
        // tile t + 1's DMAs retired (t + 2's stay in flight), this tile's reads done; the
        // compiler barrier keeps this tile's LDS reads above the wait and the s_barrier (after
        // which other waves issue the DMA into this buffer), as the one below keeps the next
        // tile's reads below them
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_waitcnt(kWaitTile);
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");   // (as above: the next tile's reads stay below it)
        bi = bi == 2 ? 0 : bi + 1;
        group(bi, 0, g0);   // (past the last tile: a staged tile of clamped columns, unused)
        fold(g1, false);
        const int tl = (tb - c_begin) / kTile;
#pragma unroll
        for (int rb = 0; rb < 2; rb++)
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int key = (tmx[rb][i] << 8) | tl;
                S[rb][i] = med3i(S[rb][i], M[rb][i], key);
                M[rb][i] = max(M[rb][i], key);
            }
    }
#else
    int bi = 0;
    for (int tb = c_begin; tb < c_end; tb += kTile) {
        issue(tb + 2 * kTile, bi == 0 ? 2 : bi - 1);
        const uint8_t* sb = s_lds + bi * kBuf;
        constexpr int CB = 8 / kMatchSplit;
        int tmx[2][4];
#pragma unroll
        for (int h = 0; h < kMatchSplit; h++) {
            v4i acc[2][CB];
#pragma unroll
            for (int c = 0; c < CB; c++) {
                const int cb = (h * CB + c) * 16;   // the column block: immediate offsets below
                const v4i ctv = *reinterpret_cast<const v4i*>(sb + lane_ct + cb * 16);
#pragma unroll
                for (int kh = 0; kh < 2; kh++) {
                    const v4i bfrag = *reinterpret_cast<const v4i*>(sb + lane_b[kh] + cb * 128);
                    acc[0][c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(afrag[0][kh], bfrag,
                                                                      kh ? acc[0][c] : ctv, 0, 0, 0);
                    acc[1][c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(afrag[1][kh], bfrag,
                                                                      kh ? acc[1][c] : ctv, 0, 0, 0);
                }
            }
#pragma unroll
            for (int rb = 0; rb < 2; rb++)
#pragma unroll
                for (int i = 0; i < 4; i++)
#pragma unroll
                    for (int c = 0; c < CB; c += 2) {
                        const int a = acc[rb][c][i], b2 = acc[rb][c + 1][i];
                        tmx[rb][i] = (h == 0 && c == 0) ? max(a, b2) : max(max(tmx[rb][i], a), b2);
                    }
        }
        const int tl = (tb - c_begin) / kTile;
#pragma unroll
        for (int rb = 0; rb < 2; rb++)
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int key = (tmx[rb][i] << 8) | tl;
                S[rb][i] = med3i(S[rb][i], M[rb][i], key);
                M[rb][i] = max(M[rb][i], key);
            }
        // tile t + 1's DMAs retired (t + 2's stay in flight), this tile's reads done (fenced
        // for the compiler on both sides, as in the pipelined loop)
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_waitcnt(kWaitTile);
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");   // (as above: the next tile's reads stay below it)
        bi = bi == 2 ? 0 : bi + 1;
    }
#endif
    // no DMA may land after the workgroup's LDS is handed to another one
    __builtin_amdgcn_s_waitcnt(0xc07f & ~0xc00f);   // vmcnt(0)
    int I[2][4];
#pragma unroll
    for (int rb = 0; rb < 2; rb++)
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int m = M[rb][i], sk = S[rb][i];
            I[rb][i] = m == kNeg ? -1 : c_begin + (m & 255) * kTile + l16;
            M[rb][i] = m == kNeg ? kNeg : m >> 8;
            S[rb][i] = sk == kNeg ? kNeg : sk >> 8;
        }
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
                I[rb][i] = m2 > m1 ? i2 : i1;
            }
    }
    if (l16 == 0) {
#pragma unroll
        for (int rb = 0; rb < 2; rb++)
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int row = panel * kRows + wave * 32 + rb * 16 + quad * 4 + i;
                if (row < nA) part[(size_t)chunk * nA + row] = Top2{M[rb][i], I[rb][i], S[rb][i]};
            }
    }
}

// Merge the column chunks of one side, add the row term, apply the distance/ratio test
// (RowMatch_Kernel / ColMatch_Kernel decision, ProgramCU.cu:1838-1841, 1884-1887).
// Equal maxima of two chunks resolve in the side's tie order (tie32: RowMatch_Kernel's, see
// k_match_rows); that choice is associative, so the chunks are merged in any grouping.
// raw_A / raw_B (u8, 128 bytes per descriptor; RAW partials): part.idx is (tile + lane) of the
// maximum and part.second the second largest (tile, lane) maximum; for a row that passes the
// ratio test with it, the dot products of the lane's 8 columns of that tile are recomputed: they
// give the column of the maximum and the second within those 8 columns, and the test is repeated
// with the larger second.  (best then holds the exact state only for the rows recomputed.)
// cl.map / cl.count (a launch over compacted rows): row r is row cl.map[r] of this side (its row
// term, u8 descriptor and output slot), n = *cl.count and the chunks are chunks_for(n, nB).
// cl.flag (row side of a mutual match): every column that a row matched is appended once to
// cl.list (count in *cl.count; the order is not deterministic and does not need to be).
// 8 lanes per row (a chain of dependent loads per row otherwise: partials, distance table,
// candidate descriptors): lane k merges chunks k, k + 8, ... and recomputes candidate k.
// The list slots are taken with one atomic add per workgroup: same-address atomics serialise,
// and one per wave cost ~25 us at 50k rows.
constexpr int kFinishThreads = 1024;
constexpr int kFinishRows = kFinishThreads / 8;

__global__ __launch_bounds__(kFinishThreads) void k_match_finish(const Top2* __restrict__ part, int n,
                                                      int chunks, const int* __restrict__ row_term,
                                                      const float* __restrict__ dist,
                                                      float distmax, float ratiomax,
                                                      int* __restrict__ out,
                                                      Top2* __restrict__ best, int tie32,
                                                      const uint8_t* __restrict__ raw_A,
                                                      const uint8_t* __restrict__ raw_B,
                                                      int nB, ColumnList cl) {
    if (cl.bn) nB = *cl.bn;   // the column side over a pruned set 1 (launch_prune_set)
    if (cl.map) {
        n = *cl.count;
        chunks = chunks_for(n, nB, cl.dma != 0);
    }
    __shared__ int s_cnt[kFinishThreads / 64], s_base;
    if ((int)blockIdx.x * kFinishRows >= n) return;   // whole workgroups only (barriers below)
    const int sub = threadIdx.x & 7, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r0 = blockIdx.x * kFinishRows + (threadIdx.x >> 3);
    const bool valid = r0 < n;   // whole 8-lane groups
    const int r = valid ? r0 : n - 1;
    const int g = cl.map ? cl.map[r] : r;
    auto merge = [&](Top2& t, const Top2& u) {
        const int s = max(min(t.max, u.max), max(t.second, u.second));
        const bool later = u.max > t.max ||
                           (u.max == t.max && (tie32 ? tie_before<true>(u.idx, t.idx)
                                                     : tie_before<false>(u.idx, t.idx)));
        t = Top2{max(t.max, u.max), later ? u.idx : t.idx, s};
    };
    Top2 t{INT_MIN, -1, INT_MIN};
    for (int c = sub; c < chunks; c += 8) merge(t, part[(size_t)c * n + r]);
#pragma unroll
    for (int off = 1; off < 8; off <<= 1)
        merge(t, Top2{__shfl_xor(t.max, off, 64), __shfl_xor(t.idx, off, 64),
                      __shfl_xor(t.second, off, 64)});
    const int rt = row_term ? row_term[g] : 0;   // COLS: already in the accumulators
    // the reference's running maxima start at 0 with index -1 (ProgramCU.cu:1803)
    int mx = t.max + rt, sc = t.second + rt;
    int idx = t.idx;
    if (mx <= 0) { mx = 0; idx = -1; }
    if (sc < 0) sc = 0;
    const float d1 = dist[min(mx, 262144)], d2 = dist[min(sc, 262144)];
    // raw partials: sc is a lower bound of the second (see below), so a row that fails here
    // fails with the exact second too
    bool ok = (d1 < distmax) && (d1 < d2 * ratiomax);
    if (raw_A && ok) {
        // lane k: candidate column (tile) + 16 k + (lane in tile); the lowest equal one wins
        // (there is one: a passing maximum is unique)
        const int c = (idx & ~127) + 16 * sub + (idx & 15);
        const uint4* a = reinterpret_cast<const uint4*>(raw_A + (size_t)g * 128);
        const int cb = max(min(c, nB - 1), 0);
        const uint4* b = reinterpret_cast<const uint4*>(raw_B + (size_t)(cl.bmap ? cl.bmap[cb] : cb) * 128);
        uint4 av[8], bv[8];
#pragma unroll
        for (int q = 0; q < 8; q++) { av[q] = a[q]; bv[q] = b[q]; }
        int d = 0;
#pragma unroll
        for (int q = 0; q < 8; q++) {
            d = __builtin_amdgcn_udot4(av[q].x, bv[q].x, d, false);
            d = __builtin_amdgcn_udot4(av[q].y, bv[q].y, d, false);
            d = __builtin_amdgcn_udot4(av[q].z, bv[q].z, d, false);
            d = __builtin_amdgcn_udot4(av[q].w, bv[q].w, d, false);
        }
        const unsigned long long bal = __ballot(c < nB && d == mx);
        const uint32_t mine = (uint32_t)(bal >> (lane & ~7)) & 0xffu;
        idx = mine ? (idx & ~127) + 16 * (__ffs(mine) - 1) + (idx & 15) : -1;
        // the partials carry the second largest tile maximum; the row's second is the larger of
        // that and the second within the winning lane's 8 columns (an equal pair counts twice)
        int m8 = c < nB ? d : INT_MIN, s8 = INT_MIN;
#pragma unroll
        for (int off = 1; off < 8; off <<= 1) {
            const int m2 = __shfl_xor(m8, off, 64), s2 = __shfl_xor(s8, off, 64);
            s8 = max(min(m8, m2), max(s8, s2));
            m8 = max(m8, m2);
        }
        sc = max(sc, s8);
        ok = ok && d1 < dist[min(sc, 262144)] * ratiomax;
    }
    // pruned column side: B's index -> the row of set 1 (a passing maximum has idx >= 0)
    const int res = ok && idx >= 0 ? (cl.bmap ? cl.bmap[idx] : idx) : -1;
    if (valid && sub == 0) {
        out[g] = res;
        if (best) best[g] = Top2{mx, idx, sc};
        if (cl.rmax) cl.rmax[g] = mx;   // >= every dot of the row (mx is its largest, clamped at 0)
    }
    if (cl.ntau && valid && sub == 0 && res >= 0) {
        // Column j = res will be decided with a maximum M >= mx (row g's dot with it) and fails
        // the ratio test exactly when its second s satisfies dist[M] >= dist[s] * ratiomax; that
        // predicate is monotone in s (dist does not increase), so every s below the smallest
        // failing value tau(mx) <= tau(M) passes, whichever row it comes from.  A row whose dots
        // are all below min tau can neither be a listed column's maximum (tau <= mx <= M) nor
        // decide its test: the column side skips it (launch_prune_set).  Any lower bound of tau
        // keeps that true (it only keeps more rows): tau ~ cos(dist[mx] / ratiomax) * 2^18 less
        // a margin of 64 (far above the float error of cos and of the table), checked with the
        // test's own comparison at the value below it -- if that one already fails, the bound
        // falls back to 0 (nothing pruned).  An 18-step bisection of the table measured 42 vs
        // 12 us for this finish at C5 (dependent loads per row); the check is one load.
        const float dm = dist[min(mx, 262144)];
        int lo = (int)floorf(cosf(dm / ratiomax) * 262144.f) - 64;
        lo = min(max(lo, 0), 262144);
        if (lo > 0 && dm >= dist[lo - 1] * ratiomax) lo = 0;
        atomicMax(cl.ntau, INT_MAX - lo);
    }
    if (cl.flag) {
        // the first claim of a column appends it: slots per wave (ballot), per workgroup
        // (LDS prefix), one atomic add
        const bool first = valid && sub == 0 && res >= 0 && atomicExch(&cl.flag[res], 1) == 0;
        const unsigned long long bal = __ballot(first);
        if (lane == 0) s_cnt[wave] = __popcll(bal);
        __syncthreads();
        if (threadIdx.x == 0) {
            int tot = 0;
            for (int w = 0; w < kFinishThreads / 64; w++) {
                const int c = s_cnt[w];
                s_cnt[w] = tot;
                tot += c;
            }
            s_base = tot ? atomicAdd(cl.count, tot) : 0;
        }
        __syncthreads();
        if (first) cl.list[s_base + s_cnt[wave] + __popcll(bal & ((1ull << lane) - 1))] = res;
    }
}

// The rows of set 1 that the column side of a plain mutual match still needs (ColumnList rmax /
// ntau): 8 lanes per row copy its s8 descriptor (16 B each) to the next free slot; slots per wave
// by ballot, per workgroup by an LDS prefix and one atomic add.
__global__ __launch_bounds__(256) void k_prune_set(const int* __restrict__ rmax,
                                                   const int* __restrict__ ntau, int n,
                                                   const uint4* __restrict__ s8,
                                                   const int* __restrict__ ct,
                                                   uint4* __restrict__ s8c, int* __restrict__ ctc,
                                                   int* __restrict__ mapc, int* __restrict__ countc) {
    __shared__ int s_cnt[4], s_base;
    const int tau = INT_MAX - *ntau;   // no passing row: INT_MAX, nothing kept (no listed column)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, sub = lane & 7;
    const int r = blockIdx.x * 32 + (threadIdx.x >> 3);
    const bool keep = r < n && rmax[r] >= tau;
    const unsigned long long bal = __ballot(keep && sub == 0);
    if (lane == 0) s_cnt[wave] = __popcll(bal);
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
        for (int w = 0; w < 4; w++) {
            const int c = s_cnt[w];
            s_cnt[w] = tot;
            tot += c;
        }
        s_base = tot ? atomicAdd(countc, tot) : 0;
    }
    __syncthreads();
    if (keep) {
        const int slot = s_base + s_cnt[wave] + __popcll(bal & ((1ull << (lane & ~7)) - 1));
        s8c[(size_t)slot * 8 + sub] = s8[(size_t)r * 8 + sub];
        if (sub == 0) {
            ctc[slot] = ct[r];
            mapc[slot] = r;
        }
    }
}

// Column decision of the fused GEMM (COLS): merge the panels' partials of column j in row
// order (equal maxima keep the earlier panel: ColMatch_Kernel, ProgramCU.cu:1874-1882), add the
// column term (acc = dot - column term), clamp as the reference's running state from (0, -1, 0)
// and apply the distance / ratio test.
constexpr int kColGroups = 16;   // panel groups per column in k_match_cols

__device__ __forceinline__ void top2_merge(Top2& t, const Top2& u) {
    // equal maxima keep the lower row: the order of the merges does not matter
    const int s = max(min(t.max, u.max), max(t.second, u.second));
    if (u.max > t.max || (u.max == t.max && u.idx < t.idx)) t.idx = u.idx;
    t.max = max(t.max, u.max);
    t.second = s;
}

__global__ __launch_bounds__(256) void k_match_cols(const Top2* __restrict__ colpart, int n,
                                                    int panels, const int* __restrict__ col_term,
                                                    const float* __restrict__ dist,
                                                    float distmax, float ratiomax,
                                                    int* __restrict__ out,
                                                    Top2* __restrict__ best) {
    // 16 columns x 16 panel groups per workgroup: group g merges panels g, g + 16, ...
    __shared__ Top2 s_t[kColGroups][256 / kColGroups];
    const int cl = threadIdx.x % (256 / kColGroups), g = threadIdx.x / (256 / kColGroups);
    const int j = blockIdx.x * (256 / kColGroups) + cl;
    Top2 t{INT_MIN, INT_MAX, INT_MIN};
    if (j < n)
        for (int p = g; p < panels; p += kColGroups) top2_merge(t, colpart[(size_t)p * n + j]);
    s_t[g][cl] = t;
    __syncthreads();
    if (g != 0 || j >= n) return;
    for (int q = 1; q < kColGroups; q++) top2_merge(t, s_t[q][cl]);
    const int ct = col_term[j];
    int mx = t.max + ct, sc = t.second + ct, idx = t.idx;
    if (mx <= 0) { mx = 0; idx = -1; }
    if (sc < 0) sc = 0;
    if (best) best[j] = Top2{mx, idx, sc};
    const float d1 = dist[min(mx, 262144)], d2 = dist[min(sc, 262144)];
    out[j] = (d1 < distmax) && (d1 < d2 * ratiomax) ? idx : -1;
}

// Geometric test of MultiplyDescriptorG_Kernel (ProgramCU.cu:1648-1681), once per pair, in
// the operation order of oracle::guided_pass (row-only and column-only terms are hoisted, which
// does not change any value; FDIV(a, b) = a * (1 / b)).  One workgroup per 128 x 128 block of
// pairs at a time (set-1 tile a = blockIdx.y; kMaskTiles set-2 tiles b in turn from
// blockIdx.x * kMaskTiles): each thread tests one set-1 row
// against 64 columns (the homography branch-free, the Sampson error only for the pairs that
// passed it) into an LDS bit matrix, which is then read out as both sides' 16-byte lane records
// (k_match_rows): rec1 for the row decision (A = set 1, tiles of set 2), rec2 for the column
// decision (A = set 2, tiles of set 1), both written coalesced.
// good(r, j) = some row of r's 8-row block of set 1 passes at j (good_count > 0, :1682).
constexpr int kPassPitch = 5;   // words per LDS bit row (4 + 1 against bank conflicts)

constexpr int kMaskTiles = 8;   // set-2 tiles per workgroup (amortises the row set-up)

__global__ __launch_bounds__(256) void k_guided_mask(const float2* __restrict__ loc1, int n1,
                                                     const float2* __restrict__ loc2, int n2,
                                                     GuidedParams gp, uint4* __restrict__ rec1,
                                                     int tiles2, uint4* __restrict__ rec2,
                                                     int tiles1) {
    __shared__ uint32_t s_pass[128 * kPassPitch];   // [set-1 row][set-2 column word]
    __shared__ uint32_t s_good[16 * kPassPitch];    // [8-row block of set 1][column word]
    __shared__ __attribute__((aligned(16))) float2 s_loc2[128];
    const int tid = threadIdx.x;
    const int a = blockIdx.y;
    const float* H = gp.H;
    const float* F = gp.F;
    const int il = tid >> 1, h = tid & 1;
    const int r = a * 128 + il;
    const float2 l = loc1[min(r, n1 - 1)];
    const float h0 = __builtin_fmaf(H[0], l.x, __builtin_fmaf(H[1], l.y, H[2]));
    const float h1 = __builtin_fmaf(H[3], l.x, __builtin_fmaf(H[4], l.y, H[5]));
    const float h2 = __builtin_fmaf(H[6], l.x, __builtin_fmaf(H[7], l.y, H[8]));
    const float rh = 1.0f / h2;
    const float u = h0 * rh, v = h1 * rh;
    const int rr = tid >> 6, lane = tid & 63, quad = lane >> 4, l16 = lane & 15;
    const int b_end = min(tiles2, (int)(blockIdx.x + 1) * kMaskTiles);
    float2 next = make_float2(0.f, 0.f);
    int b = blockIdx.x * kMaskTiles;
    if (tid < 128 && b * 128 + tid < n2) next = loc2[b * 128 + tid];
    for (; b < b_end; b++) {
        if (tid < 128) s_loc2[tid] = next;
        __syncthreads();
        if (tid < 128 && b + 1 < b_end && (b + 1) * 128 + tid < n2) next = loc2[(b + 1) * 128 + tid];
        uint32_t w[2];
#pragma unroll
        for (int q = 0; q < 2; q++) {
            // 32 columns' (x, y) as 16 ds_read_b128, then a branch-free test per pair (bitwise
            // '&': a short-circuit '&&' compiles to a branch per pair)
            const float4* c4 = reinterpret_cast<const float4*>(s_loc2 + h * 64 + q * 32);
            float4 cc[16];
#pragma unroll
            for (int k = 0; k < 16; k++) cc[k] = c4[k];
            uint32_t bits = 0;
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const bool ok0 = (__builtin_fabsf(u - cc[k].x) < gp.hdistmax) &
                                 (__builtin_fabsf(v - cc[k].y) < gp.hdistmax);
                const bool ok1 = (__builtin_fabsf(u - cc[k].z) < gp.hdistmax) &
                                 (__builtin_fabsf(v - cc[k].w) < gp.hdistmax);
                bits |= ((uint32_t)ok0 << (2 * k)) | ((uint32_t)ok1 << (2 * k + 1));
            }
            const int c0 = b * 128 + h * 64 + q * 32;   // first column of this word
            const int nvalid = min(max(n2 - c0, 0), 32);
            w[q] = r < n1 ? bits & (nvalid == 32 ? 0xffffffffu : ((1u << nvalid) - 1u)) : 0u;
        }
        if (w[0] | w[1]) {
            const float f0 = __builtin_fmaf(F[0], l.x, __builtin_fmaf(F[1], l.y, F[2]));
            const float f1 = __builtin_fmaf(F[3], l.x, __builtin_fmaf(F[4], l.y, F[5]));
            const float f2 = __builtin_fmaf(F[6], l.x, __builtin_fmaf(F[7], l.y, F[8]));
            const float d0 = __builtin_fmaf(f1, f1, f0 * f0);
#pragma unroll
            for (int q = 0; q < 2; q++) {
                for (uint32_t rest = w[q]; rest; rest &= rest - 1) {
                    const int jj = __builtin_ctz(rest);
                    const float2 p2 = s_loc2[h * 64 + q * 32 + jj];
                    const float t0 = __builtin_fmaf(F[0], p2.x, __builtin_fmaf(F[3], p2.y, F[6]));
                    const float t1 = __builtin_fmaf(F[1], p2.x, __builtin_fmaf(F[4], p2.y, F[7]));
                    const float x2fx1 = __builtin_fmaf(p2.x, f0, __builtin_fmaf(p2.y, f1, f2));
                    const float den = __builtin_fmaf(t1, t1, __builtin_fmaf(t0, t0, d0));
                    const float se = (x2fx1 * x2fx1) * (1.0f / den);
                    if (!(se < gp.fdistmax)) w[q] &= ~(1u << jj);
                }
            }
        }
        s_pass[il * kPassPitch + h * 2] = w[0];
        s_pass[il * kPassPitch + h * 2 + 1] = w[1];
        __syncthreads();
        if (tid < 64) {
            const int blk = tid >> 2, wd = tid & 3;
            uint32_t g = 0;
#pragma unroll
            for (int k = 0; k < 8; k++) g |= s_pass[(blk * 8 + k) * kPassPitch + wd];
            s_good[blk * kPassPitch + wd] = g;
        }
        __syncthreads();
        // rec1: rows 32 (4a + rr) + 16 rb + 4 quad + i of set 1, columns 128 b + 16 cb + l16
        if ((a * 4 + rr) * 32 < n1) {
            uint32_t o[4] = {0, 0, 0, 0};
#pragma unroll
            for (int rb = 0; rb < 2; rb++) {
                const int row0 = rr * 32 + rb * 16 + quad * 4;
                const int blk = row0 >> 3;
#pragma unroll
                for (int cb = 0; cb < 8; cb++) {
                    const int col = cb * 16 + l16, wd = col >> 5, bit = col & 31;
                    uint32_t byte = ((s_good[blk * kPassPitch + wd] >> bit) & 1u) ? 0u : 0xf0u;
#pragma unroll
                    for (int i = 0; i < 4; i++)
                        byte |= (((s_pass[(row0 + i) * kPassPitch + wd] >> bit) & 1u) ^ 1u) << i;
                    o[rb * 2 + (cb >> 2)] |= byte << ((cb & 3) * 8);
                }
            }
            rec1[((size_t)(a * 4 + rr) * tiles2 + b) * 64 + lane] = make_uint4(o[0], o[1], o[2], o[3]);
        }
        // rec2: rows 32 (4b + rr) + 16 rb + 4 quad + c of set 2, columns 128 a + 16 cb + l16 of
        // set 1
        if (rec2 && (b * 4 + rr) * 32 < n2) {
            uint32_t o[4] = {0, 0, 0, 0};
#pragma unroll
            for (int cb = 0; cb < 8; cb++) {
                const int rl = cb * 16 + l16;
                const uint32_t pw = s_pass[rl * kPassPitch + rr];
                const uint32_t gw = s_good[(rl >> 3) * kPassPitch + rr];
#pragma unroll
                for (int rb = 0; rb < 2; rb++) {
                    const int sh = rb * 16 + quad * 4;
                    const uint32_t byte = (~(pw >> sh) & 0xfu) | ((~(gw >> sh) & 0xfu) << 4);
                    o[rb * 2 + (cb >> 2)] |= byte << ((cb & 3) * 8);
                }
            }
            rec2[((size_t)(b * 4 + rr) * tiles1 + a) * 64 + lane] = make_uint4(o[0], o[1], o[2], o[3]);
        }
        // the next tile's s_loc2 / s_pass writes wait for every read of this one
        __syncthreads();
    }
}

}  // namespace

size_t guided_mask_bytes(int nA, int nB) {
    return (size_t)((nA + 31) / 32) * ((nB + kTile - 1) / kTile) * 64 * 16;
}

hipError_t launch_guided_mask(const float* loc1, int n1, const float* loc2, int n2,
                              const GuidedParams& gp, uint8_t* rec1, uint8_t* rec2,
                              hipStream_t stream) {
    if (n1 <= 0 || n2 <= 0) return hipSuccess;
    const int t1 = (n1 + kTile - 1) / kTile, t2 = (n2 + kTile - 1) / kTile;
    hipLaunchKernelGGL(k_guided_mask, dim3((t2 + kMaskTiles - 1) / kMaskTiles, t1), dim3(256), 0, stream,
                       reinterpret_cast<const float2*>(loc1), n1,
                       reinterpret_cast<const float2*>(loc2), n2, gp,
                       reinterpret_cast<uint4*>(rec1), t2, reinterpret_cast<uint4*>(rec2), t1);
    return hipGetLastError();
}

hipError_t launch_to_s8(const uint8_t* src, int n, uint8_t* dst, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    const size_t n16 = (size_t)n * 8;   // 128 bytes = 8 uint4 per descriptor
    const unsigned grid = (unsigned)std::min<size_t>((n16 + 255) / 256, 4096);
    hipLaunchKernelGGL(k_to_s8, dim3(grid), dim3(256), 0, stream,
                       reinterpret_cast<const uint4*>(src), n16, reinterpret_cast<uint4*>(dst));
    return hipGetLastError();
}

hipError_t launch_prep_set(const uint8_t* src, int n, uint8_t* dst, int* sums, int scale,
                           int bias, int* zero, int nzero, hipStream_t stream, int* ctp,
                           int* ctfill) {
    if (n <= 0 && nzero <= 0) return hipSuccess;
    const size_t n16 = (size_t)std::max(n, 0) * 8;
    const size_t work = std::max(n16, (size_t)std::max(nzero, 0));
    const unsigned grid = (unsigned)std::min<size_t>((work + 255) / 256, 4096);
    hipLaunchKernelGGL(k_prep_set, dim3(grid), dim3(256), 0, stream,
                       reinterpret_cast<const uint4*>(src), n16, reinterpret_cast<uint4*>(dst),
                       sums, scale, bias, zero, nzero, ctp, std::max(n, 0), ctfill);
    return hipGetLastError();
}

hipError_t launch_rowsums(const uint8_t* d, int n, int* out, int scale, int bias,
                          hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_rowsum, dim3((n + 3) / 4), dim3(256), 0, stream, d, n, out, scale, bias);
    return hipGetLastError();
}

int match_chunks(int nA, int nB, bool dma) { return chunks_for(nA, nB, dma); }
int match_ct_pad() { return kCtPad; }

// bounds over every row count m <= nA of chunks_for(m, nB, dma) * m (partials) and of
// panels(m) * chunks_for(m, nB, dma) (workgroups).  Register kernels: chunks <= max_chunks,
// and chunks * panels < kMatchWg + panels (128-row panels).  k_match_raw: chunks is min_chunks
// or at most kRawMaxRounds * kRawSlots / panels (256-row panels), so chunks * m is at most
// kRawMaxRounds * kRawSlots * 256 and chunks * panels at most kRawMaxRounds * kRawSlots.
size_t match_part_bound(int nA, int nB, bool dma) {
    const size_t panels = (nA + kPanel - 1) / kPanel;
    const size_t max_chunks = std::max(1, (nB + 2 * kTile - 1) / (2 * kTile));
    const size_t min_chunks = std::max(1, (nB + kMaxChunkTiles * kTile - 1) / (kMaxChunkTiles * kTile));
    const size_t cap = dma ? (size_t)kRawMaxRounds * kRawSlots * kRawRows : (kMatchWg + panels) * kPanel;
    return std::max(std::min(cap, max_chunks * (size_t)nA), min_chunks * (size_t)nA);
}
static unsigned match_grid_bound(int nA, int nB, bool dma) {
    const size_t min_chunks = std::max(1, (nB + kMaxChunkTiles * kTile - 1) / (kMaxChunkTiles * kTile));
    if (dma) {
        const size_t panels = (nA + kRawRows - 1) / kRawRows;
        return (unsigned)std::max((size_t)kRawMaxRounds * kRawSlots, min_chunks * panels);
    }
    const size_t panels = (nA + kPanel - 1) / kPanel;
    const size_t max_chunks = std::max(1, (nB + 2 * kTile - 1) / (2 * kTile));
    return (unsigned)std::max(std::min(kMatchWg + panels, max_chunks * panels),
                              min_chunks * panels);
}

int match_panels(int nA) { return (nA + kPanel - 1) / kPanel; }

hipError_t launch_match_rows(const uint8_t* A, int nA, const uint8_t* B, int nB,
                             int chunks, Top2* part, hipStream_t stream,
                             const uint8_t* mask, bool row_side, const int* row_term,
                             Top2* colpart, bool raw, const int* amap, const int* an,
                             const int* ctp, const int* bn) {
    if (raw && (mask || colpart)) return hipErrorInvalidValue;
    if (nA <= 0 || nB <= 0) return hipSuccess;
    if (colpart && (!row_term || !row_side)) return hipErrorInvalidValue;
    if ((amap != nullptr) != (an != nullptr) || (an && (mask || colpart))) return hipErrorInvalidValue;
    if (bn && !(raw && ctp && an)) return hipErrorInvalidValue;   // a device-side B count: k_match_raw, 1-D grid
    int per = (nB + chunks - 1) / chunks;
    per = (per + kTile - 1) / kTile * kTile;
    // compacted rows (at most nA of them): a 1-D grid large enough for any count
    const bool dma = raw && ctp;
    const dim3 grid = an ? dim3(match_grid_bound(nA, nB, dma))
                         : dim3((nA + kPanel - 1) / kPanel, chunks);
    const int tiles = (nB + kTile - 1) / kTile;
    const uint4* rec = reinterpret_cast<const uint4*>(mask);
#define SGK_MR(G, T, C)                                                                       \
    hipLaunchKernelGGL((k_match_rows<G, T, C>), grid, dim3(256), 0, stream, A, nA, B, nB, per, \
                       part, rec, tiles, row_term, colpart, amap, an)
#define SGK_MRR(T)                                                                            \
    hipLaunchKernelGGL((k_match_rows<false, T, false, true>), grid, dim3(256), 0, stream, A, nA, \
                       B, nB, per, part, rec, tiles, row_term, colpart, amap, an)
    if (dma) {
        constexpr int rows = kRawRows;
        const dim3 rgrid = an ? grid : dim3((nA + rows - 1) / rows, chunks);
        hipLaunchKernelGGL(k_match_raw, rgrid, dim3(64 * kRawWaves), 0, stream, A, nA,
                           B, nB, ctp, per, part, amap, an, bn);
    } else if (raw) {
        if (row_side) SGK_MRR(true); else SGK_MRR(false);
    } else if (an) {
        if (row_side) SGK_MR(false, true, false); else SGK_MR(false, false, false);
    } else if (colpart) {
        if (mask) SGK_MR(true, true, true); else SGK_MR(false, true, true);
    } else if (!mask) {
        if (row_side) SGK_MR(false, true, false); else SGK_MR(false, false, false);
    } else {
        if (row_side) SGK_MR(true, true, false); else SGK_MR(true, false, false);
    }
#undef SGK_MR
#undef SGK_MRR
    return hipGetLastError();
}

hipError_t launch_prune_set(const int* rmax, const int* ntau, int n, const uint8_t* s8,
                            const int* ct, uint8_t* s8c, int* ctc, int* mapc, int* countc,
                            hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_prune_set, dim3((n + 31) / 32), dim3(256), 0, stream, rmax, ntau, n,
                       reinterpret_cast<const uint4*>(s8), ct, reinterpret_cast<uint4*>(s8c), ctc,
                       mapc, countc);
    return hipGetLastError();
}

hipError_t launch_match_cols(const Top2* colpart, int n, int panels, const int* col_term,
                             const float* dist, float distmax, float ratiomax, int* out,
                             Top2* best, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    const int per = 256 / kColGroups;
    hipLaunchKernelGGL(k_match_cols, dim3((n + per - 1) / per), dim3(256), 0, stream, colpart, n,
                       panels, col_term, dist, distmax, ratiomax, out, best);
    return hipGetLastError();
}

hipError_t launch_match_finish(const Top2* part, int n, int chunks, const int* row_term,
                               const float* dist, float distmax, float ratiomax, int* out,
                               Top2* best, hipStream_t stream, bool row_side,
                               const uint8_t* raw_A, const uint8_t* raw_B, int nB,
                               ColumnList cl) {
    if (n <= 0) return hipSuccess;
    if ((cl.map && !cl.count) || (cl.flag && (!cl.list || !cl.count || cl.map))) return hipErrorInvalidValue;
    if ((cl.rmax != nullptr) != (cl.ntau != nullptr) || (cl.ntau && (!cl.flag || !raw_A)) ||
        (cl.bmap != nullptr) != (cl.bn != nullptr) || (cl.bn && (!cl.map || !raw_A)))
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_match_finish, dim3((n + kFinishRows - 1) / kFinishRows), dim3(kFinishThreads), 0,
                       stream, part, n,
                       chunks, row_term, dist, distmax, ratiomax, out, best, row_side ? 1 : 0,
                       raw_A, raw_B, nB, cl);
    return hipGetLastError();
}

}  // namespace sgk
