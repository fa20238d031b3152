/* sgpu.h -- C ABI of the MI355X SIFT hot path (libsiftgpu.so).
 *
 * Plain C types only (no torch, no C++): this is the boundary a cgo/ctypes/JNI binding or the
 * C++ SiftGPU/SiftMatchGPU classes (include/SiftGPU.h) call.  Each entry point names the
 * reference interface it replaces (paths relative to the reference repo root).
 *
 * Errors: every function returns SGPU_OK (0) or a negative SGPU_E* code; sgpu_last_error()
 * returns a message.  There is no CPU fallback: when no gfx950 device is usable the context
 * cannot be created and every compute call fails with SGPU_ENODEV.
 */
#ifndef SGPU_H
#define SGPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SGPU_OK 0
#define SGPU_EINVAL (-1)   /* bad argument */
#define SGPU_ENODEV (-2)   /* no usable GPU / HIP runtime error */
#define SGPU_ENOMEM (-3)   /* device or host allocation failed */
#define SGPU_ERANGE (-4)   /* capacity exceeded (e.g. more matches than max_match) */

/* Extraction / matching options.  Field meaning and defaults follow the reference's global
 * parameters (SiftGPU/GlobalUtil.cpp:50-135) and ParseParam (SiftGPU/SiftGPU.cpp:801-1246). */
typedef struct sgpu_options {
    float filter_width_factor;         /* -f   (4.0)                                        */
    float descriptor_window_factor;    /* -dw  (3.0)                                        */
    float orientation_window_factor;   /* -w   (2.0)                                        */
    float orientation_gaussian_factor; /*      (1.5)                                        */
    float dog_threshold;               /* -t   (0 -> 0.02/dog_level_num)                    */
    float edge_threshold;              /* -e   (0 -> 10)                                    */
    int subpixel;                      /* -s   (1)                                          */
    int max_orientation;               /* -m   (2)                                          */
    int fixed_orientation;             /* -ofix (0)                                         */
    int octave_min;                    /* -fo  first octave, >= -2 (0)                       */
    int octave_num;                    /* -no  (-1 = floor(log2(min(w,h)))-3)                */
    int dog_level_num;                 /* -d   (3)                                          */
    int lowe_origin;                   /* -loweo (0)                                        */
    int normalized;                    /* -unn clears (1)                                   */
    int descriptors;                   /* -sd clears (1)                                    */
    int keep_extremum_sign;            /* -sign (0)                                         */
    int circular_window;               /* 0: square orientation window of the active
                                          ProgramCU.cu:869-884; 1: circular window of
                                          ProgramCU-0.cu:834 / the GLSL path                */
    int verbose;                       /* -v   (0 here; the library prints nothing at 0)     */
    int max_dimension;                 /* -maxd (13200, GlobalUtil.cpp:86; SiftGPU::SetMaxDimension):
                                          while the first octave is wider or taller, octave_min
                                          is raised by one (PyramidCU::InitPyramid,
                                          PyramidCU.cpp:129-135)                              */
    int preprocess_on_cpu;             /* -prep / -noprep (1, GlobalUtil.cpp:81): with -fo > 0
                                          the input is first sampled by 2^fo and its width
                                          truncated (GLTexInput::SetImageData,
                                          GLTexImage.cpp:928-1009), then run from octave 0;
                                          0: the first octave is SampleImageD of the full input  */
    int feature_count_threshold;       /* -tc[1|2|3] <n> (-1 = off, GlobalUtil.cpp:135)         */
    int truncate_method;               /* 0: -tc / -tc1, 1: -tc2, 2: -tc3 (SiftGPU.cpp:1185-1203;
                                          SiftPyramid::LimitFeatureCount, SiftPyramid.cpp:219-260,
                                          and the level skip of PyramidCU::GenerateFeatureList,
                                          PyramidCU.cpp:829-853)                              */
} sgpu_options;

/* Defaults of GlobalUtil.cpp:50-135. */
void sgpu_default_options(sgpu_options* opt);

/* Parse reference command-line options into *opt (SiftGPU::ParseParam, SiftGPU.cpp:801-1246:
 * first-4-character case-insensitive option hashing, same argument rules).  Options the MI355X
 * path has no use for (-cuda, -winpos, -display, -pack, ...) are accepted and ignored; -cuda <n>
 * sets *device when device != NULL.  Returns SGPU_OK. */
int sgpu_parse_args(sgpu_options* opt, int argc, const char* const* argv, int* device);

typedef struct sgpu_ctx sgpu_ctx;

/* Create a context bound to HIP device `device` (replaces ProgramCU::CheckCudaDevice,
 * ProgramCU.cu:1414-1448, + PyramidCU construction).  The context owns all device buffers. */
int sgpu_ctx_create(int device, const sgpu_options* opt, sgpu_ctx** out);
int sgpu_ctx_destroy(sgpu_ctx* ctx);
int sgpu_ctx_set_options(sgpu_ctx* ctx, const sgpu_options* opt);
const char* sgpu_last_error(const sgpu_ctx* ctx);
/* Number of visible HIP devices (0 when the runtime is unusable). */
int sgpu_device_count(void);

/* Input flags. */
#define SGPU_INPUT_HOST   0   /* `images` is a host pointer                                */
#define SGPU_INPUT_DEVICE 1   /* `images` is a device pointer on the context's device      */
#define SGPU_INPUT_STAGED 2   /* use the batch staged in HBM by sgpu_stage_input (images
                                 may be NULL); the input stays resident across calls       */

/* Copy a batch of u8 images (same layout as sgpu_extract) into the context's device input
 * buffer, so that later extract calls with SGPU_INPUT_STAGED start from HBM-resident input. */
int sgpu_stage_input(sgpu_ctx* ctx, const uint8_t* images, int n, int w, int h, int stride);

/* Allocate now every device and pinned buffer that an extract of n gray u8 images of w x h
 * pixels (rows `stride` bytes apart, staged or uploaded) needs, so that the next
 * sgpu_stage_input + sgpu_extract of that geometry allocates nothing unless its keypoints exceed
 * the first-guess capacity.  Replaces SiftGPU::AllocatePyramid (SiftGPU.h:193,
 * SiftGPU.cpp:1435-1460 -> PyramidCU::ResizePyramid, PyramidCU.cpp:178-271).  Like an extract
 * it replaces the batch: the previous results and the staged input are gone. */
int sgpu_reserve(sgpu_ctx* ctx, int n, int w, int h, int stride);
/* The last extract's Gaussian pyramid (part 0): returns the number of kernel launches that
 * filtered its levels and stores the number of level filters in *filters (the reference's
 * FilterImage calls, PyramidCU.cpp:979-1044; several run in one launch under the diagonal and
 * paired-level schedules).  bench.py divides the pyramid's bytes and time by it. */
int sgpu_last_pyramid_launches(const sgpu_ctx* ctx, int* filters);
/* Test hook: number of device and pinned-host allocations the library has made so far. */
long long sgpu_debug_alloc_count(void);

/* Extract SIFT features from n gray u8 images of w x h pixels, row stride `stride` bytes,
 * image i at images + i*stride*h.  Replaces SiftGPU::RunSIFT(w, h, data, GL_LUMINANCE,
 * GL_UNSIGNED_BYTE) (SiftGPU.h:176, SiftGPU.cpp:233-268 -> SiftPyramid::RunSIFT,
 * SiftPyramid.cpp:58-216), batched.  Results stay valid until the next extract call. */
int sgpu_extract(sgpu_ctx* ctx, const uint8_t* images, int n, int w, int h, int stride,
                 int flags);

/* Host-in / host-out extraction of a stream of batches: nbatches batches of `batch` u8 gray
 * images (batches[k] -> batch images of w x h, rows `stride` bytes apart, in host memory).  The
 * keys (x, y, scale, orientation) and descriptors of all images go to keys[cap][4] and
 * desc[cap][128] (either may be NULL) in image order, counts[nbatches * batch] the per-image
 * feature counts.  Replaces a loop of SiftGPU::RunSIFT(w, h, data, GL_LUMINANCE,
 * GL_UNSIGNED_BYTE) + GetFeatureVector (SiftGPU.cpp:233-268, SiftPyramid.cpp:287-291) with the
 * reference's upload (PyramidCU.cpp:949-976) and descriptor download (PyramidCU.cpp:434) in the
 * pipeline: the upload of batch k+1 and the download of batch k-1 overlap batch k's kernels.
 * The copies overlap only from page-locked memory (sgpu_host_alloc).  Returns SGPU_ERANGE when
 * the features exceed cap (counts are complete, the features stop at the last batch that fit).
 * Afterwards the context holds no "last batch" for the per-image queries. */
int sgpu_extract_stream(sgpu_ctx* ctx, const uint8_t* const* batches, int nbatches, int batch,
                        int w, int h, int stride, float* keys, float* desc, int64_t cap,
                        int32_t* counts);
/* Page-locked host memory for sgpu_extract_stream's input and output (hipHostMalloc). */
void* sgpu_host_alloc(size_t bytes);
void sgpu_host_free(void* p);

/* Same with float luminance input in [0, 1] (stride in floats): the GL_FLOAT / converted-RGB
 * input path of GLTexInput::SetImageData (GLTexImage.cpp:981-1006). */
int sgpu_extract_f32(sgpu_ctx* ctx, const float* images, int n, int w, int h, int stride,
                     int flags);

/* Color input, converted to luminance on the device with the reference's formula
 * (GLTexInput::SetImageData -> DownSamplePixelDataI2F<u8>, GLTexImage.cpp:834-858:
 * (19595 r + 38470 g + 7471 b) / (65535 * 255); BGR swaps r and b; alpha ignored).  `format`
 * is one of SGPU_RGB, SGPU_BGR, SGPU_RGBA, SGPU_BGRA; `stride` in bytes.  Replaces
 * RunSIFT(w, h, data, GL_RGB | GL_BGR | GL_RGBA | GL_BGRA, GL_UNSIGNED_BYTE), batched. */
#define SGPU_RGB  1
#define SGPU_BGR  2
#define SGPU_RGBA 3
#define SGPU_BGRA 4
int sgpu_extract_color(sgpu_ctx* ctx, const uint8_t* images, int n, int w, int h, int stride,
                       int format, int flags);

/* Feature count of image i of the last extract (SiftGPU::GetFeatureNum, SiftGPU.cpp:1411). */
int sgpu_feature_count(const sgpu_ctx* ctx, int image);
/* Total over the batch. */
int64_t sgpu_feature_total(const sgpu_ctx* ctx);

/* Copy image i's keypoints (x, y, scale, orientation: 4 floats each) and descriptors (128
 * floats each) to host memory; either pointer may be NULL (SiftGPU::GetFeatureVector,
 * SiftGPU.cpp:1416-1428, SiftPyramid::CopyFeatureVector, SiftPyramid.cpp:287-291). */
int sgpu_copy_features(sgpu_ctx* ctx, int image, float* keys, float* descriptors);

/* Device pointers to the whole batch's keypoints [total][4] / descriptors [total][128] and the
 * per-image start offsets [n+1] (host array).  Zero-copy access for batch consumers. */
int sgpu_device_features(sgpu_ctx* ctx, const float** keys, const float** descriptors,
                         const int64_t** image_offsets);

/* Descriptors of caller-supplied keypoints on image `image` of the last extract (its pyramid is
 * reused): SiftGPU::RunSIFT(num, keys, keys_have_orientation) (SiftGPU.cpp:287-291,
 * SiftPyramid::SetKeypointList SiftPyramid.cpp:293-310, GenerateFeatureListTex
 * PyramidCU.cpp:454-504).  keys: num x (x, y, scale, orientation) in image coordinates.  With
 * has_orientation == 0 the strongest orientation is computed (ComputeOrientation_Kernel with
 * existing_keypoint) and the keys are rewritten as DownloadKeypoints does.  has_orientation ==
 * -1 is the rectangle mode (SIFT_RECT_DESCRIPTION, SiftPyramid.cpp:308-309): keys are
 * (x, y, width, height) and ComputeDescriptorRECT_Kernel (ProgramCU.cu:1104-1171) describes the
 * rectangle; keys come back unchanged.  Results (input order)
 * replace the context's features: image `image` reports num features (sgpu_copy_features),
 * every other image none. */
int sgpu_extract_keypoints(sgpu_ctx* ctx, int image, const float* keys, int num,
                           int has_orientation);

/* Matcher.  d1 [n1][128], d2 [n2][128] u8 descriptors (the reference quantizes float
 * descriptors as (unsigned char)int(512*d+0.5), SiftMatchCU.cpp:87-101: see
 * sgpu_quantize_descriptors).  Replaces SiftMatchGPU::SetDescriptors + GetSiftMatch
 * (SiftGPU.h:300-311; SiftMatchCU.cpp:139-179; kernels ProgramCU.cu:1466-1900).
 * Writes pairs {i, j} in ascending i into out_pairs (max_match entries) and returns the match
 * count (>= 0) or an error. */
int sgpu_match(sgpu_ctx* ctx, const uint8_t* d1, int n1, const uint8_t* d2, int n2,
               float distmax, float ratiomax, int mutual_best_match, int max_match,
               int* out_pairs, int flags);

/* Guided matcher: SiftMatchGPU::SetFeautreLocation + GetGuidedSiftMatch (SiftGPU.h:313-321;
 * SiftMatch.cpp:663-677; SiftMatchCU.cpp:104-136; kernel MultiplyDescriptorG_Kernel
 * ProgramCU.cu:1607-1777).  loc1 [n1][2], loc2 [n2][2] feature (x, y) (packed: the reference's
 * `gap` is applied by the caller); H, F row-major 3x3.  A pair passes when
 * |H x1 - x2| < hdistmax in both coordinates and its Sampson error under F is < fdistmax; the
 * dot of every pair of an 8-row block with a passing row enters the row/column decisions as
 * MultiplyDescriptorG_Kernel defines them.  H == NULL and F == NULL: plain sgpu_match; one of
 * them NULL: the identity with threshold 1e20.  SGPU_INPUT_DEVICE covers the locations too. */
int sgpu_match_guided(sgpu_ctx* ctx, const uint8_t* d1, int n1, const uint8_t* d2, int n2,
                      const float* loc1, const float* loc2, const float* H, const float* F,
                      float distmax, float ratiomax, float hdistmax, float fdistmax,
                      int mutual_best_match, int max_match, int* out_pairs, int flags);

/* Sharded matcher (multi-GPU extension of SiftMatchGPU::GetSiftMatch):
 * this rank holds rows [row_begin, row_begin + ns) of set 1 (d1 = those rows) and all n2 rows
 * of set 2.  The result over all ranks equals sgpu_match on the whole of set 1.
 * sgpu_match_shard_begin: row_match[ns] = the row decision of each local row (matched set-2
 * row or -1; RowMatch_Kernel, ProgramCU.cu:1785-1841) and, with mutual_best_match, col_best
 * [n2][3] = this shard's clamped column state (max dot, global set-1 row, second dot) of
 * ColMatch_Kernel (ProgramCU.cu:1844-1900).
 * sgpu_match_shard_end (host only, no device): merges the nshards column states (rank order),
 * applies the column decision and the mutual check (SiftMatchCU.cpp:166-176) and writes this
 * shard's pairs {global i, j} in ascending i; returns their count.  Concatenated in rank order
 * the shards' pairs are sgpu_match's (max_match applies per call).
 * sgpu_match_sharded: both, with the exchange as an RCCL all-gather over the context's
 * communicator (sgpu_comm_init; without one it is a single shard). */
int sgpu_match_shard_begin(sgpu_ctx* ctx, const uint8_t* d1, int ns, int row_begin,
                           const uint8_t* d2, int n2, float distmax, float ratiomax,
                           int mutual_best_match, int* row_match, int* col_best, int flags);
int sgpu_match_shard_end(const int* col_best_all, int nshards, int n2, const int* row_match,
                         int ns, int row_begin, float distmax, float ratiomax,
                         int mutual_best_match, int max_match, int* out_pairs);
int sgpu_match_sharded(sgpu_ctx* ctx, const uint8_t* d1, int ns, int row_begin,
                       const uint8_t* d2, int n2, float distmax, float ratiomax,
                       int mutual_best_match, int max_match, int* out_pairs, int flags);

/* float -> u8 quantization of SiftMatchCU::SetDescriptors (SiftMatchCU.cpp:94-99), host side. */
void sgpu_quantize_descriptors(const float* d, size_t count, uint8_t* out);

/* Timing of the last call: stage times in milliseconds measured with HIP events
 * (SiftGPU::_timing, SiftPyramid.cpp:48-56).  times[0..7] =
 * {upload, pyramid, detect, orientation, expand, descriptor, download, total} of the last
 * extract; times[8] = the last sgpu_match call; times[9] = the feature-list (row scan) part of
 * detect; times[10], [11] = the key and descriptor copies of the last sgpu_copy_features.
 * SiftGPU::_timing[2..8] map them to the reference's slots (siftgpu_api.cpp).  Slots 0-7 and
 * 9-11 read 0 after a one-stream extract / copy made with the stage timing off. */
int sgpu_last_timing(const sgpu_ctx* ctx, float* times, int n);
/* Register page-locked host buffers (sgpu_host_alloc) for the NEXT extract of one image
 * (sgpu_extract / _f32 / _color with n == 1): it writes image 0's keys (4 floats each) and
 * descriptors (128 floats each; descriptors may be NULL) for up to `capacity` features into them
 * from the GPU, in its own stream before its one synchronisation, in place of the count copy and
 * the two downloads of sgpu_copy_features.  sgpu_copy_features(ctx, 0, keys, descriptors) with
 * the same pointers then returns at once when the image's features fit (otherwise it copies as
 * usual).  The registration is consumed by that extract.  No reference counterpart: the
 * reference's RunSIFT downloads keys and descriptors after the pyramid (PyramidCU.cpp:434). */
int sgpu_set_host_output(sgpu_ctx* ctx, float* keys, float* descriptors, int capacity);
/* Stage timing on (default) or off.  Replaces the reference's GlobalUtil::_timingS (GlobalUtil.cpp:51,
 * set by SiftGPU::SetVerbose, SiftGPU.cpp:401-429; 0 skips the per-stage finish calls,
 * PyramidCU.cpp:439,873,1041).  Off, a one-stream extract records none of its ~10 stage events
 * (each ~4.5 us of GPU time between two kernels); the multi-stream layouts and
 * sgpu_extract_stream keep the events they synchronise on. */
int sgpu_set_stage_timing(sgpu_ctx* ctx, int on);

/* ---- multi-GPU batch driver (no reference counterpart: the reference
 * runs one SiftGPU per device thread, TestWin/MultiThreadSIFT.cpp:141-155).  One process per
 * GPU, each with its own context; images are sharded and the only exchange is an RCCL
 * all-gather (over xGMI) of the per-image feature counts.  Rendezvous: rank 0 creates the id,
 * the launcher distributes it (bench.py uses torch.distributed on the host). */
#define SGPU_COMM_ID_BYTES 128
/* Create a communicator id (ncclGetUniqueId) into id[bytes], bytes >= SGPU_COMM_ID_BYTES. */
int sgpu_comm_unique_id(uint8_t* id, int bytes);
/* Join the communicator of nranks contexts (ncclCommInitRank, collective over the ranks). */
int sgpu_comm_init(sgpu_ctx* ctx, int nranks, int rank, const uint8_t* id, int bytes);
/* recv[r*n + i] = send of rank r, element i (host arrays; device staging + ncclAllGather). */
int sgpu_comm_allgather_i32(sgpu_ctx* ctx, const int32_t* send, int n, int32_t* recv);
/* In-place all-reduce of n doubles (op_max != 0: max, else sum). */
int sgpu_comm_allreduce_f64(sgpu_ctx* ctx, double* v, int n, int op_max);

/* ---- test hooks (parity tests read intermediate stages; not part of the drop-in surface) ---- */
/* Per-context debug flags (0 = shipped configuration). */
#define SGPU_DEBUG_PARTS2   1   /* split a batch into 2 parts on separate streams              */
#define SGPU_DEBUG_PARTS4   2   /* ... into 4 parts                                            */
#define SGPU_DEBUG_TINY_CAP 4   /* start the keypoint capacity at 64 per part, so that the
                                   capacity-overflow re-run of a part is exercised             */
#define SGPU_DEBUG_FUSED_MATCH 8 /* plain mutual matching through the fused one-GEMM kernel
                                   (the guided matcher always uses it)                         */
#define SGPU_DEBUG_EXACT_DESCRIPTOR 16 /* descriptors in the reference's per-bin fma order with the
                                   oracle's transcendentals: bit-identical to the oracle.  The
                                   shipped kernel sums in any order with hardware sqrt/rcp/exp
                                   (descriptor L2 ~1e-6 from the oracle).  Also set at context
                                   creation by the environment variable SGPU_EXACT_DESCRIPTOR=1 */
#define SGPU_DEBUG_GAUSS_BLOCK 32 /* Gaussian levels through the workgroup strip kernel
                                   (k_gauss_pk2) instead of the shipped wave-streaming one
                                   (k_gauss_lean); both are bit-identical.  Bits
                                   SGPU_DEBUG_BAND_SHIFT.. of the flags, when not 0, force the
                                   wave kernel's band height in rows (test / tuning hook) */
#define SGPU_DEBUG_BAND_SHIFT 20  /* band height field: (flags >> 20) & 0x7ff rows (< 2048); the flag bits
                                     below it never reach it (DESC_DUAL at 1 << 16
                                     used to share its bit with the band field) */
#define SGPU_DEBUG_KEYED_MATCH 64 /* plain matching through the keyed epilogue (every value
                                   folded with its column's tie-order bits) even when
                                   ratiomax <= 1, where the keyless one is exact and used     */
#define SGPU_DEBUG_FULL_COLUMNS 128 /* plain mutual matching decides every column of set 2, not
                                   only the columns some row of set 1 matched                 */
#define SGPU_DEBUG_DESC_DUAL 256 /* detected features' descriptors through the round-4 dual-cell
                                    kernel instead of the pixel-parallel k_descriptor_flat */
#define SGPU_DEBUG_ORIENT_WAVE 512 /* orientation one wave per candidate for any count (the shipped
                                     path picks it for few candidates only): same bits */
#define SGPU_DEBUG_GAUSS_TILE_ALWAYS 1024 /* every level through the 2-D tile kernel
                                             (k_gauss_tile) and the extremum detection through
                                             k_extrema_tile, whatever the size (the shipped path
                                             tiles levels of at most SGPU_GAUSS_TILE_MB, default
                                             16 MB: a single image's): same levels and keys */
#define SGPU_DEBUG_MATCH_REGSTAGE 2048 /* keyless plain matching through the register-staged
                                          k_match_rows<..., RAW> instead of the LDS-DMA
                                          k_match_raw: same pairs */
#define SGPU_DEBUG_PYR_SERIAL 4096 /* the pyramid octave by octave, one level per launch (the
                                      shipped path runs octave o+1's first levels in the same
                                      launches as octave o's last ones; the stream layout runs
                                      octaves >= 1 on a second stream): same levels */
#define SGPU_DEBUG_GAUSS_LONG_BANDS 8192 /* Gaussian bands of >= 4 chunks on every level (round
                                            2's band rule; the shipped rule lets cache-resident
                                            levels use 1-chunk bands): same levels.  Also set at
                                            context creation by SGPU_GAUSS_BANDS=long */
#define SGPU_DEBUG_DUO_ALWAYS 16384 /* paired-level Gaussian launches (k_gauss_duo) for every
                                        eligible level pair, whatever its size (the shipped path
                                        pairs only levels of >= 128 MB): same levels */
#define SGPU_DEBUG_DUO_OFF 32768 /* no paired-level launches (one level per launch, the round-4
                                    schedule): same levels */
#define SGPU_DEBUG_GAUSS_TILE_OFF 65536 /* no 2-D tile launches: every level through the
                                           wave-streaming kernels (round 5): same levels */
#define SGPU_DEBUG_DESC_WIDE_OFF 131072 /* descriptors one wave per feature for every count (the
                                           shipped path gives few features a workgroup each):
                                           same bits */
#define SGPU_DEBUG_DESC_WIDE_ALWAYS 262144 /* descriptors one workgroup per feature for every
                                              count: same bits */
#define SGPU_DEBUG_EXTREMA_TILE_OFF 524288 /* extremum detection always through the
                                              wave-streaming k_extrema_wave2 (the shipped path
                                              tiles cache-resident pyramids, k_extrema_tile;
                                              SGPU_DEBUG_GAUSS_TILE_ALWAYS tiles every one) */

int sgpu_debug_set_flags(sgpu_ctx* ctx, int flags);
/* The batch pyramid's launch plan, a test / A-B hook -- the levels are the same
 * bits in every plan.  trio: three-level launches (k_gauss_trio): none (shipped), on levels of
 * >= 512 MB, or wherever the widths and the decimation allow (SGPU_TRIO=off / on / always at
 * context creation).  pairs: the octave's paired-level launches taken from its end, (4, 5),
 * (2, 3) with the decimation, (0, 1) (shipped), or from its front (SGPU_DUO_PLAN=end / front). */
#define SGPU_TRIO_OFF 0
#define SGPU_TRIO_ON 1
#define SGPU_TRIO_ALWAYS 2
#define SGPU_PAIRS_FRONT 0
#define SGPU_PAIRS_END 1
int sgpu_debug_set_schedule(sgpu_ctx* ctx, int trio, int pairs);
/* Plain mutual matching (ratiomax <= 1) decides the listed columns over the rows of set 1 that can
 * change a decision -- those with some dot at or above the smallest second value that fails the
 * ratio test against the weakest passing row maximum -- instead of all of set 1 (on != 0, the
 * shipped default; SGPU_MATCH_PRUNE=off at context creation turns it off): the same pairs
 * (DESIGN.md 4.8), a test / A-B hook. */
int sgpu_debug_set_match_prune(sgpu_ctx* ctx, int on);
/* Octave geometry of the last extract: n_octaves, and (w, h, wa) per octave. */
int sgpu_debug_geometry(const sgpu_ctx* ctx, int* n_octaves, int* dims /* 3*max */, int max);
/* Gaussian level (image, octave, level 0..level_num-1) as wa*h floats. */
int sgpu_debug_gaussian(sgpu_ctx* ctx, int image, int octave, int level, float* out);
/* Detected (pre-orientation) keypoints of the batch in reference order: per entry
 * {col, row, level_id, image} ints and {dx, dy, ds, pad} floats.  Returns count via *n. */
int sgpu_debug_candidates(sgpu_ctx* ctx, int* ints, float* floats, int cap, int* n);

#ifdef __cplusplus
}
#endif
#endif /* SGPU_H */
