// sift_kernels.h -- launch interface of the gfx950 SIFT kernels (sift_kernels.hip).
//
// All launchers are asynchronous on `stream` and take device pointers.  Images of one batch
// share one geometry; every kernel covers the whole batch in one launch (grid.z / flat index).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sgk {

constexpr int kMaxLevels = 16;     // d + 3 Gaussian levels per octave (d <= 10 in the CLI)
constexpr int kMaxOctaves = 16;

struct Taps { float k[33]; };

// Per-octave geometry and buffer offsets used by the feature kernels.
struct OctaveDesc {
    int w, h, wa;          // wa = padded width = row stride of every level image
    int nwords;            // bitmask words per row = ceil(wa / 32)
    long long gauss_off;   // float offset of (octave, level 0, image 0) in the pyramid buffer
    long long level_stride;// floats between levels of one octave = batch * wa * h
    long long mask_off;    // uint32 offset of (octave, dog level 0, image 0) in the bitmask buffer
    long long mask_level_stride; // words between dog levels = batch * h * nwords
};

struct FeatureParams {
    int batch, n_octaves, d;             // d = dog_level_num
    int rows_per_image;                  // sum over octaves of d * h
    int row_off[kMaxOctaves];            // first row id of (octave o, level 0) inside an image
    float level_sigma[kMaxLevels];       // GetLevelSigma(j), j = 0..d-1
    float sigma_step;                    // 2^(1/d)
    float t0, t, edge;                   // dog threshold * 0.8 (subpixel), dog threshold, (r+1)^2/r
    float gaussian_factor, sample_factor;// orientation window (1.5, 3.0)
    float window_factor;                 // descriptor (3.0)
    int subpixel, num_orientation, keep_sign, circular, normalize;
    float origin_offset;                 // 0.5 (or 0 with -loweo)
    int octave_min;                      // -fo: octave o of the pyramid is octave o + octave_min
    int unit_input;                      // the image's values lie in [0, 1] (u8 / 255, colour, -prep)
    OctaveDesc oct[kMaxOctaves];
};

// Up to three u32 buffers to zero (null / 0 words: none).
struct ZeroJob {
    uint32_t* p[3] = {nullptr, nullptr, nullptr};
    size_t n[3] = {0, 0, 0};
};

// Gaussian level filter: dst = V(H(src)) with the reference's clamp-to-edge semantics.
// src_u8 != nullptr selects the ingest variant (src value = u8 / 255.0f).  src_stride is the
// row stride in elements of whichever source is used.
// ds_dst != nullptr additionally writes the 2x point-downsampled output (next octave level 0).
// wave_rows < 0: the workgroup strip kernel (k_gauss_pk2); >= 0: the wave-streaming level
// kernel k_gauss_lean (FW <= 33) with bands of wave_rows rows (0: chosen from the grid size).
// Both give bit-identical levels; unaligned sources always take k_gauss_pk2.
hipError_t launch_gauss(const float* src, const uint8_t* src_u8, int src_stride,
                        long long src_img_stride, float* dst, long long dst_img_stride,
                        int w, int h, int fw, const Taps& taps, int batch,
                        float* ds_dst, int ds_w, int ds_h, long long ds_img_stride,
                        hipStream_t stream, int wave_rows = -1, bool long_bands = false,
                        const ZeroJob& zero = ZeroJob{});

// One level filter of a pyramid stage (the arguments of launch_gauss).  zero (optional): the
// launch also zeroes these buffers (the extremum kernel's mask and row counts, the orientation
// counts) -- one launch fewer per extract than launch_zero, which a single image pays per launch.
struct LevelOp {
    const float* src;
    const uint8_t* src_u8;
    int src_stride;
    long long src_img_stride;
    float* dst;
    long long dst_img_stride;
    int w, h, fw;
    Taps taps;
    int batch;
    float* ds_dst;
    int ds_w, ds_h;
    long long ds_img_stride;
    ZeroJob zero;
};
// long_bands: bands of >= 4 chunks on every level (the A/B hook SGPU_DEBUG_GAUSS_LONG_BANDS)
hipError_t launch_gauss_op(const LevelOp& op, hipStream_t stream, int wave_rows,
                           bool long_bands = false);
// Two independent level filters (no data dependence between them) in one launch of the
// wave-streaming kernel when their widths have a compiled pair, f32 sources and no decimation
// (the "diagonal" schedule of the pyramid: octave o+1's level k beside octave o's level k + kds);
// otherwise two launches.  Bit-identical to two launch_gauss calls.
// *launches (optional): how many kernel launches it took (1 or 2).
hipError_t launch_gauss_two(const LevelOp& a, const LevelOp& b, hipStream_t stream, int wave_rows,
                            bool long_bands = false, int* launches = nullptr);

// Two consecutive levels in one launch (sift_gauss_duo.hip): a = level k -> k+1, b = level
// k+1 -> k+2 (b.src == a.dst); f32 widths (11, 13) or (21, 25): 12 B of HBM
// traffic per pixel for the two levels instead of 16 (and (17, 21) with level k+1 decimated into
// the next octave's level 0, (13, 17) with level k+2 decimated); or the u8 ingest pair (13, 11),
// level 0 from the image and level 1 (with a's ZeroJob): 9 B instead of 13.  Bit-identical to two
// launch_gauss_op calls.  trash: kGaussDuoTrashBytes of device scratch.  rows_hint > 0 forces
// the band height.
constexpr size_t kGaussDuoTrashBytes = 1024 * 3072;
bool gauss_duo_supported(const LevelOp& a, const LevelOp& b);
hipError_t launch_gauss_duo(const LevelOp& a, const LevelOp& b, hipStream_t stream, int rows_hint,
                            float* trash);

// Three consecutive levels in one launch (sift_gauss_trio.hip): a = level k -> k+1, b = k+1 ->
// k+2, c = k+2 -> k+3 (b.src == a.dst, c.src == b.dst) with level k+3 decimated into the next
// octave's level 0 (c.ds_dst); f32 widths (11, 13, 17): 17 B of HBM traffic per pixel for the
// three levels instead of 25 for a paired-level launch plus one level.  Bit-identical to three
// launch_gauss_op calls.  trash: kGaussTrioTrashBytes of device scratch.
constexpr size_t kGaussTrioTrashBytes = 1024 * 4096;
bool gauss_trio_supported(const LevelOp& a, const LevelOp& b, const LevelOp& c);
hipError_t launch_gauss_trio(const LevelOp& a, const LevelOp& b, const LevelOp& c,
                             hipStream_t stream, int rows_hint, float* trash);

// One level in 2-D tiles (sift_gauss_tile.hip): a workgroup loads its 64 x 32 output tile's
// whole input window at once, H pass into LDS, V pass from LDS -- for cache-resident levels (one
// image: the wave walk of k_gauss_lean is a chain of load latencies there).  Bit-identical to
// launch_gauss_op.  launch_gauss_tile_two: two independent levels in one launch (the diagonal
// schedule's compiled width pairs), else two launches (*launches says which).
bool gauss_tile_supported(const LevelOp& op);
hipError_t launch_gauss_tile(const LevelOp& op, hipStream_t stream);
hipError_t launch_gauss_tile_two(const LevelOp& a, const LevelOp& b, hipStream_t stream,
                                 int* launches = nullptr);
// Two consecutive levels per tile (a = level k -> k+1, b = level k+1 -> k+2, b.src == a.dst): one
// load of level k's window, level k+1 filtered into LDS over the region b's filter needs, its
// tile stored, then level k+2 (and b's decimation) -- bit-identical to two launch_gauss_tile calls.
// launch_gauss_tile_duo_one: that duo beside an independent single level c in one launch (the
// compiled combination (21, 25) + 11: octave o's last levels with octave o+1's first), else two.
bool gauss_tile_duo_supported(const LevelOp& a, const LevelOp& b);
hipError_t launch_gauss_tile_duo(const LevelOp& a, const LevelOp& b, hipStream_t stream);
hipError_t launch_gauss_tile_duo_one(const LevelOp& a, const LevelOp& b, const LevelOp& c,
                                     hipStream_t stream, int* launches = nullptr);

// First octave of -fo != 0 (BuildPyramid, PyramidCU.cpp:1011-1016): the batch's input
// (u8 p/255 or f32; tw = w & ~3 columns used, rows `stride` apart) resampled into dst
// (dw x dh per image, dst_img_stride apart): SampleImageD by 2^fo for fo > 0, UpsampleKernel
// by 2^-fo for fo < 0 (then dw = tw << -fo).
hipError_t launch_first_octave_input(const float* src, const uint8_t* src_u8, int stride,
                                     long long src_img_stride, int tw, int h, int fo, float* dst,
                                     int dw, int dh, long long dst_img_stride, int batch,
                                     hipStream_t stream);

// Color ingest (DownSamplePixelDataI2F<u8>, GLTexImage.cpp:834-858): n images of w x h
// pixels with `channels` (3 or 4) bytes each, rows `stride` bytes apart; bgr swaps the red and
// blue weights.  dst gets tw = w & ~3 floats per row (the truncated width), images tw*h apart.
hipError_t launch_color_to_gray(const uint8_t* src, int n, int w, int h, int stride,
                                int channels, bool bgr, float* dst, hipStream_t stream);

// Extremum detection for all octaves, all d levels and all images (one launch): sets the
// keypoint bits in the zeroed mask and adds per-row keypoint counts into the zeroed row_count
// (rows ordered image, octave, level, row).  tiles: the 2-D tile kernel (k_extrema_tile: each
// workgroup loads its 64 x 16-pixel window of every plane at once; for cache-resident pyramids),
// else the wave-streaming k_extrema_wave2 -- the same bits and counts.
hipError_t launch_extrema(const float* pyr, uint32_t* mask, uint32_t* row_count,
                          const FeatureParams& fp, hipStream_t stream, bool tiles = false);

// Exclusive scan of n uint32 values into out[0..n]; out[n] = total.  tmp needs
// scan_tmp_words(n) words.
size_t scan_tmp_words(size_t n);
// Zero up to three u32 buffers (null / 0 words: skipped) in one launch: hipMemsetAsync is two
// fill dispatches per buffer, which a single-image extract pays three times.
hipError_t launch_zero(uint32_t* a, size_t na, uint32_t* b, size_t nb, uint32_t* c, size_t nc,
                       hipStream_t stream);
hipError_t launch_scan(const uint32_t* in, uint32_t* out, size_t n, uint32_t* tmp,
                       hipStream_t stream);

// Keypoint materialisation + orientation: a quad per detected keypoint (wave_per_candidate: a
// wave, for few candidates), grid-stride over min(*n_cand_dev, n_cand_cap) keypoints (the grid
// is sized from grid_hint).  Both forms give the same bits.
// out4: (x, y, s, packed orientations) in octave coordinates; info: (image, level id);
// ocount: number of oriented features the keypoint expands to.
hipError_t launch_orientation(const float* pyr, const uint32_t* mask, const uint32_t* row_base,
                              int total_rows, const uint32_t* n_cand_dev, int n_cand_cap,
                              int grid_hint, const FeatureParams& fp, float4* out4, int2* info,
                              uint32_t* ocount, hipStream_t stream,
                              bool wave_per_candidate = false);

// Expansion into oriented features (+ image-coordinate keypoints).  io (optional): the same
// launch also writes the extract's readback record (io.off[0] = candidate count, io.off[1 + b]
// = image b's first feature for b in [0, batch], the readback of an extract).
struct ImageOffsetsArgs {
    const uint32_t* row_base = nullptr;
    int batch = 0, rows_per_image = 0, total_rows = 0;
    int64_t* off = nullptr;
};
hipError_t launch_expand(const float4* cand, const int2* info, const uint32_t* eoff,
                         const uint32_t* n_cand_dev, int n_cand_cap, const FeatureParams& fp,
                         float4* feat, int2* feat_info, float4* keys, hipStream_t stream,
                         const ImageOffsetsArgs* io = nullptr);

// Copy *n_dev (at most cap) keys (float4) and descriptors (128 floats; desc may be null) and the
// rec_n (<= 256) int64 words of rec into page-locked host buffers, in one launch.
hipError_t launch_copy_out(const float4* keys, const float* desc, const uint32_t* n_dev, int cap,
                           const int64_t* rec, int rec_n, float* hkeys, float* hdesc,
                           int64_t* hrec, hipStream_t stream);

// Descriptors (+ normalisation) of the expanded features; n_feat_cap sizes the grid (one wave
// per feature), the kernel grid-strides over *n_feat_dev.  out_index (optional): feature e's
// descriptor goes to row out_index[e].  rect: the rectangle descriptor of keys given with
// keys_have_orientation == -1 (feat = (x, y, width, height) in octave coordinates).
// exact: the reference's per-bin fma order and the oracle's transcendentals (bit-identical to the
// oracle; the test mode); otherwise the relaxed-order pixel-parallel kernel k_descriptor_flat
// (L2 ~1e-6 from the oracle), or with dual the round-4 dual-cell kernel (A/B).  wide: the
// relaxed-order kernel with a workgroup of 4 waves per feature (k_descriptor_wide, for few
// features; the grid is then one workgroup per feature up to n_feat_cap) -- the same bits.
// host (wide only): keys[e], descriptor row e (e < cap) and the rec_n (<= 256) int64 words of rec
// also to page-locked host memory, in place of a launch_copy_out after the kernel.
struct HostCopy {
    const float4* keys = nullptr;
    const int64_t* rec = nullptr;
    int rec_n = 0;
    uint32_t cap = 0;
    float4* hkeys = nullptr;
    float* hdesc = nullptr;
    int64_t* hrec = nullptr;
};
hipError_t launch_descriptor(const float* pyr, const float4* feat, const int2* feat_info,
                             const uint32_t* n_feat_dev, int n_feat_cap, const FeatureParams& fp,
                             float* desc, hipStream_t stream, const int* out_index = nullptr,
                             bool rect = false, bool exact = false, bool dual = false,
                             bool wide = false, const HostCopy* host = nullptr);

// Caller-supplied keypoints: strongest orientation into feat[e].w (num_orientation != 0, else
// 0) and the image-coordinate key at keys_out[index[e]].
hipError_t launch_orient_keys(const float* pyr, float4* feat, const int2* feat_info,
                              const int* index, int n, const FeatureParams& fp, float4* keys_out,
                              hipStream_t stream);

// Feature-count limiting (-tc / -tc2 / -tc3, method 0 / 1 / 2), per image of the batch.
// launch_limit_rows: on the detected keypoints' row counts (before the row scan);
// launch_limit_oriented: on the oriented counts (after orientation, before the feature scan).
hipError_t launch_limit_rows(uint32_t* row_count, const FeatureParams& fp, int threshold,
                             int method, hipStream_t stream);
hipError_t launch_limit_oriented(uint32_t* ocount, const uint32_t* row_base,
                                 const FeatureParams& fp, int threshold, int method,
                                 uint32_t cand_cap, hipStream_t stream);


// Test hook, NOT in the product library: the candidates of the orientation stage back as
// (col, row, level id, image) + (dx, dy, ds, result), from lib/libsiftgpu_debug.so
// (csrc/sgpu_debug.hip), which sgpu_debug_candidates loads on first use.
typedef hipError_t (*DebugCandidatesFn)(const float* pyr, const uint32_t* mask,
                                        const uint32_t* row_base, int total_rows,
                                        const uint32_t* n_cand_dev, int n_cand_cap,
                                        const FeatureParams* fp, int4* ints, float4* floats,
                                        hipStream_t stream);

// ---- matcher (sift_match.hip) ----
// Distance table dist[v] = float(acos(min(v * 2^-18, 1.0))) for v in [0, 262144], built on the
// host with the same expression as the oracle and uploaded once.
constexpr int kDistTable = 262145;
struct Top2 { int max, idx, second; };
// dst = src xor 0x80 (u8 -> s8 descriptors, the operands of the i8 MFMA), n descriptors
hipError_t launch_to_s8(const uint8_t* src, int n, uint8_t* dst, hipStream_t stream);
// s[i] = scale * sum_k d[i][k] + bias
hipError_t launch_rowsums(const uint8_t* d, int n, int* s, int scale, int bias, hipStream_t stream);
// both at once, for one set: dst = s8 form, sums[i] = scale * sum_k src[i][k] + bias (sums may
// be null), zero[0 .. nzero) = 0, and ctp (optional, n + match_ct_pad() entries) the biased
// column terms of a raw launch_match_rows with this set as B
// ctfill (optional, n + match_ct_pad() entries): set to the column term of a missing column, so
// that a launch_prune_set output over it reads as padded past its device-side count
hipError_t launch_prep_set(const uint8_t* src, int n, uint8_t* dst, int* sums, int scale,
                           int bias, int* zero, int nzero, hipStream_t stream,
                           int* ctp = nullptr, int* ctfill = nullptr);
int match_ct_pad();
// column chunks of a row launch: dma = the launch runs k_match_raw (raw with ctp), whose split
// is its own cost model (sift_match.hip chunks_for)
int match_chunks(int nA, int nB, bool dma = false);
// part[chunk][nA]: per-row top-2 of (A_i . B_j + col_term[j]) over each column chunk, with
// col_term[j] = 128 * sum(B_j) - 2^21 formed in the kernel from the staged bytes.  A and B are
// the s8 forms of the descriptor sets (launch_to_s8).
// row_side: equal maxima resolve as RowMatch_Kernel does (A = set 1); else in column order.
// With a mask (launch_guided_mask, this side's lane records): the guided values
// (k_match_rows<true>).
// colpart != nullptr (row_side only; row_term = 128 * sum(A rows)): the fused mutual form --
// colpart[panel][nB] also receives every 128-row panel's column-side (max, row, second) of
// (dot - column term) (guided: of the guided value), for launch_match_cols.
// raw (plain matching with ratiomax <= 1 only): values folded without keys; part.idx is then
// (tile + lane) and k_match_finish recovers the column (pass raw_A / raw_B to it).
// ctp (raw only; launch_prep_set of B): the LDS-DMA kernel k_match_raw, same partials.
// amap / an (plain matching only): the rows are A[amap[r]] for r < *an (a count on the device,
// at most nA); the launch covers every count and the split is chunks_for(*an, nB, dma), which
// launch_match_finish with ColumnList{map, count, dma} derives again.  part needs
// match_part_bound(nA, nB, dma) entries.
hipError_t launch_match_rows(const uint8_t* A, int nA, const uint8_t* B, int nB,
                             int chunks, Top2* part, hipStream_t stream,
                             const uint8_t* mask, bool row_side, const int* row_term = nullptr,
                             Top2* colpart = nullptr, bool raw = false,
                             const int* amap = nullptr, const int* an = nullptr,
                             const int* ctp = nullptr, const int* bn = nullptr);
size_t match_part_bound(int nA, int nB, bool dma = false);
int match_panels(int nA);
// Column decisions from the panels' partials: col_term[j] = 128 * sum(B_j) - 2^21 (guided: 0).
hipError_t launch_match_cols(const Top2* colpart, int n, int panels, const int* col_term,
                             const float* dist, float distmax, float ratiomax, int* out,
                             Top2* best, hipStream_t stream);
// Guided matching geometry (SiftMatchGPU::GetGuidedSiftMatch): H, F row-major 3x3.
struct GuidedParams { float H[9]; float F[9]; float hdistmax, fdistmax; };
// bytes of one side's guided mask records (A rows, B columns)
size_t guided_mask_bytes(int nA, int nB);
// loc1 [n1][2], loc2 [n2][2]; rec1 = guided_mask_bytes(n1, n2) bytes (row decision), rec2
// (optional) = guided_mask_bytes(n2, n1) bytes (column decision).
hipError_t launch_guided_mask(const float* loc1, int n1, const float* loc2, int n2,
                              const GuidedParams& gp, uint8_t* rec1, uint8_t* rec2,
                              hipStream_t stream);
// merge chunks, add row_term (nullptr: none), apply distmax / ratiomax -> out[i] = matched
// index or -1
// raw_A / raw_B / nB: the u8 sets of a raw launch_match_rows (A = this side's rows; nB = the
// other side's count, also needed with cl.map)
// The column side of a mutual match only needs the columns some row matched (the host's check
// reads match2[j] only for j = match1[i] >= 0).  ColumnList, row side: flag (nB ints, zeroed)
// and count (zeroed) set -> each matched column is appended once to list.  Column side: map =
// that list and count -> the launch covers rows map[0 .. *count) (n = the upper bound).
// Pruning of the column side (row side: rmax, ntau set): rmax[i] = row i's largest dot over set 2
// (an upper bound of every dot of row i), ntau (zeroed) = INT_MAX - the smallest second value
// tau that would fail the ratio test of a column whose maximum is a passing row's maximum; rows
// with rmax < tau cannot change any listed column's decision (launch_prune_set).  Column side:
// bmap / bn = the kept rows of set 1 (original row of each, count on the device) that B holds.
struct ColumnList {
    int* flag = nullptr;
    int* list = nullptr;
    int* count = nullptr;
    const int* map = nullptr;
    int dma = 0;   // map launches: the rows ran through k_match_raw (its chunk split)
    int* rmax = nullptr;
    int* ntau = nullptr;
    const int* bmap = nullptr;
    const int* bn = nullptr;
};
// The rows of set 1 that a listed column's decision can depend on (rmax[i] >= INT_MAX - *ntau),
// compacted: s8c / ctc / mapc [slot] = s8 row, k_match_raw column term, original index, in
// workgroup order (the order changes no decision: a passing column maximum is unique), *countc =
// their number (zeroed before).  ctc must hold the missing-column term past the count
// (launch_prep_set's ctfill).
hipError_t launch_prune_set(const int* rmax, const int* ntau, int n, const uint8_t* s8,
                            const int* ct, uint8_t* s8c, int* ctc, int* mapc, int* countc,
                            hipStream_t stream);
hipError_t launch_match_finish(const Top2* part, int n, int chunks, const int* row_term,
                               const float* dist, float distmax, float ratiomax, int* out,
                               Top2* best, hipStream_t stream, bool row_side,
                               const uint8_t* raw_A = nullptr, const uint8_t* raw_B = nullptr,
                               int nB = 0, ColumnList cl = ColumnList{});

}  // namespace sgk
