// sgpu_capi.cpp -- the C ABI (include/sgpu.h) over the gfx950 kernels.
//
// Host orchestration of one batch (replaces SiftPyramid::RunSIFT, SiftPyramid.cpp:58-216, and
// the PyramidCU stage methods).  A batch can be split into parts of consecutive images, each
// with its own HIP streams and buffers; part p+1 starts its pyramid when part p has finished
// detection, so that the HBM-bound pyramid/extremum kernels of one part can run beside the
// VALU-bound orientation/descriptor kernels of the previous one (one part by default, see
// extract_impl).  Inside a part everything is queued
// without host round trips (keypoint counts stay on the device; launch grids come from buffer
// capacities); the host waits once per batch, reads the per-image offsets and, if a part's
// candidates overflowed its capacity, grows the buffers and re-runs that part.  (The reference
// does four host round trips per DoG level, PyramidCU.cpp:783-813.)
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/sgpu.h"
#include "sift_kernels.h"
#include "sift_params.h"

namespace {

// paired-level Gaussian launches in the shipped schedule (1), or only when asked for by
// SGPU_DUO=on / the debug flags (0)
#ifndef SGK_DUO_DEFAULT
#define SGK_DUO_DEFAULT 1
#endif
// paired-level Gaussian launches only for levels of at least this many MB (smaller ones stay in
// the Infinity Cache between launches and are latency-bound: one level per launch, 1-chunk bands)
#ifndef SGK_DUO_MIN_MB
#define SGK_DUO_MIN_MB 128
#endif
// paired levels: (11, 13) from SGK_DUO_MIN_MB; (17, 21) with the decimation, whose arithmetic
// makes it latency-bound on smaller levels, from SGK_DUO_WIDE_MIN_MB (128 x 1080p: octave 0
// 903 us against 1,052 for two launches; octave 1 309 against ~270, tests/diag/r05i.sh); (21, 25)
// only by SGPU_DUO_WIDE=1 (1,016 us against ~1,050, and it would take level 4 from (17, 21))
#ifndef SGK_DUO_WIDE_MIN_MB
#define SGK_DUO_WIDE_MIN_MB 512
#endif
// three levels per launch (k_gauss_trio: widths (11, 13, 17), the third decimated into the next
// octave) for levels of at least this many MB; the octave's remaining (21, 25) pair then runs as a
// paired-level launch
// the octave's level pairs taken from its end ((4, 5), (2, 3) with the decimation, (0, 1)): 1,
// or from its front: 0 (sgpu_ctx::duo_plan); from the end only on levels of at most
// SGK_DUO_PLAN_MAXW columns (128 x 1080p: octave 0 2.575 vs 2.613 ms; 16 x 4096^2 (C4): 2.87 vs
// 2.80 ms -- every paired-level launch of the 4096-column levels runs ~10 % slower than on 1920
// columns)
#ifndef SGK_DUO_PLAN
#define SGK_DUO_PLAN 1
#endif
#ifndef SGK_DUO_PLAN_MAXW
#define SGK_DUO_PLAN_MAXW 2048
#endif
#ifndef SGK_TRIO_MIN_MB
#define SGK_TRIO_MIN_MB 512
#endif

// 2-D tile launches (k_gauss_tile, sift_gauss_tile.hip) for levels of at most this many MB (one
// 1080p image: 8.3 MB at octave 0), where the wave walk of k_gauss_lean is latency-bound
#ifndef SGK_TILE_MB
#define SGK_TILE_MB 16
#endif

// feature counts (of the previous call) up to which each descriptor gets a workgroup of 4 waves
// (k_descriptor_wide): ~1,500 features of one 1080p image are ~1.5 waves per SIMD under one wave
// each
#ifndef SGK_WIDE_DESC_MAX
#define SGK_WIDE_DESC_MAX 8192
#endif

// device and pinned-host allocations made by the library (sgpu_debug_alloc_count): a test hook
// for sgpu_reserve, whose point is that the extract after it allocates nothing
std::atomic<long long> g_allocs{0};

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    hipError_t ensure(size_t n) {
        if (n <= bytes) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        n = std::max<size_t>(n, 256);
        g_allocs++;
        hipError_t e = hipMalloc(&p, n);
        if (e == hipSuccess) bytes = n;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <class T> T* as() const { return reinterpret_cast<T*>(p); }
};

// stage timings (sgpu_last_timing): T_DETECT spans the extremum kernel and the row scan (the
// reference's "Detection" and "Feature List" stages, SiftPyramid.cpp:107,123); T_LIST is the
// row-scan part of it
enum { T_UPLOAD, T_PYRAMID, T_DETECT, T_ORIENT, T_EXPAND, T_DESC, T_DOWNLOAD, T_TOTAL, T_MATCH,
       T_LIST, T_COPY_KEYS, T_COPY_DESC, T_N };

// One part of a batch: consecutive images [img0, img0 + n) with their own stream and buffers.
struct Part {
    hipStream_t stream = nullptr;      // high priority: pyramid + detection
    hipStream_t stream_lo = nullptr;   // low priority: orientation, descriptors, readback
    // a small batch (one image through SiftGPU::RunSIFT) runs every stage on `stream`: the
    // cross-stream event waits cost more than the overlap gains there (extract_body)
    bool one_stream = false;
    hipStream_t stream_oct = nullptr;  // high priority: pyramid octaves >= 1 (enqueue_part)
    hipEvent_t ev_ds = nullptr;        // octave 0's decimating level done
    hipEvent_t ev_oct = nullptr;       // octaves >= 1 done
    size_t cand_hint = 0, feat_hint = 0;   // counts of the previous call (launch-grid sizing)
    int gauss_launches = 0, gauss_filters = 0;   // the last pyramid: launches, level filters
    bool events = true;                    // the last enqueue recorded its stage events
    bool copied_out = false;               // the last enqueue copied its results to host_out
    hipEvent_t ev[10] = {};  // start, pyramid, detect, orientation, expand, descriptor, end,
                             // extrema done (before the row scan), (spare), (spare)
    int img0 = 0, n = 0;
    sgk::FeatureParams fp{};
    int total_rows = 0;
    long long mask_words = 0;
    size_t cand_cap = 0;     // candidate capacity of cand/info/ocount (features: 2x)
    uint32_t n_cand = 0;
    std::vector<int64_t> img_off;          // local per-image offsets [n + 1]
    int64_t* h_read = nullptr;             // pinned readback: [0] = n_cand, [1..n+1] = offsets
    size_t h_read_n = 0;
    DevBuf pyr, mask, row_count, row_base, scan_tmp, cand, info, ocount, eoff, feat, feat_info,
        keys, desc, img_off_dev;
    float timing[T_N] = {};

    void release() {
        DevBuf* bufs[] = {&pyr, &mask, &row_count, &row_base, &scan_tmp, &cand, &info, &ocount,
                          &eoff, &feat, &feat_info, &keys, &desc, &img_off_dev};
        for (DevBuf* b : bufs) b->release();
        if (h_read) (void)hipHostFree(h_read);
        h_read = nullptr;
        for (hipEvent_t& e : ev)
            if (e) (void)hipEventDestroy(e);
        if (stream) (void)hipStreamDestroy(stream);
        if (stream_lo) (void)hipStreamDestroy(stream_lo);
        if (ev_ds) (void)hipEventDestroy(ev_ds);
        if (ev_oct) (void)hipEventDestroy(ev_oct);
        ev_ds = ev_oct = nullptr;
        if (stream_oct) (void)hipStreamDestroy(stream_oct);
        stream = stream_lo = stream_oct = nullptr;
    }
};

constexpr int kMaxParts = 4;
// candidate counts (of the previous call) up to which orientation runs one wave per candidate
#ifndef SGPU_WAVE_ORIENT_MAX
#define SGPU_WAVE_ORIENT_MAX 16384
#endif
constexpr size_t kWaveOrientationMax = SGPU_WAVE_ORIENT_MAX;

}  // namespace

struct sgpu_ctx {
    int device = 0;
    hipStream_t stream = nullptr;   // matcher, uploads, gathers
    sgpu_options opt{};
    sgp::Schedule sched{};
    sgp::InputPlan plan{};                 // first octave of the last extract (plan_input)
    int debug_flags = 0;                   // SGPU_DEBUG_* test hooks
    bool multi_stream = false;             // SGPU_STREAMS=multi: octave and feature streams
    bool duo_on = false;                   // SGPU_DUO=on: paired-level launches (size rule)
    bool duo_wide = false;                 // SGPU_DUO_WIDE=1: also the (21, 25) pairs
    bool duo_u8 = false;                   // SGPU_DUO_U8=1: the u8 ingest pair (13, 11)
    int trio_mode = SGPU_TRIO_OFF;         // three-level launches: SGPU_TRIO_* (SGPU_TRIO=off / on /
                                           // always; sgpu_debug_set_schedule)
    int duo_plan = SGK_DUO_PLAN;           // SGPU_PAIRS_END: pairs from the octave's end
                                           // (SGPU_DUO_PLAN=end), SGPU_PAIRS_FRONT: from its front
    size_t wide_desc_max = SGK_WIDE_DESC_MAX;   // feature counts (of the previous call) up to which
                                           // descriptors run a workgroup per feature
                                           // (SGPU_WIDE_DESC_MAX)
    bool unit_input = true;                // the last extract's input lies in [0, 1] (not a caller's f32)
    bool tile_duo = false;                 // tile duos when every level is tiled (SGPU_TILE_DUO=on;
                                           // measured slower)
    int tile_mb = SGK_TILE_MB;             // levels of at most this many MB: 2-D tile launches
                                           // (SGPU_GAUSS_TILE_MB; k_gauss_tile)
    int env_flags = 0;                     // debug flags set from the environment at creation
    // sgpu_set_host_output: page-locked host buffers the next one-image extract fills in its own
    // stream (armed until that extract); done = the last extract filled them
    struct HostOut {
        float* keys = nullptr;
        float* desc = nullptr;
        int cap = 0;
        bool armed = false, active = false, done = false;
    } host_out;
    // per-stage HIP events of an extract (sgpu_last_timing's stage slots).  Each event record
    // costs ~4.5 us of GPU time between the commands around it (tests/microbench/event_gap.hip),
    // ~40 us per single-image extract; sgpu_set_stage_timing(ctx, 0) drops them where they only
    // time (one-stream extracts; the multi-stream layouts need some to synchronise)
    bool stage_timing = true;
    bool streaming = false;                // inside sgpu_extract_stream (its waits use events)
    std::string err;
    // last extract
    int batch = 0, w = 0, h = 0, nparts = 0;
    std::vector<sgp::Octave> oct;
    size_t staged_bytes = 0;
    std::vector<int64_t> img_off;          // global per-image offsets [batch + 1]
    Part part[kMaxParts];
    DevBuf input, all_keys, all_desc, gray, pre;  // all_*: lazily gathered multi-part outputs;
                                                  // pre: the 2^ds-sampled input (-fo > 0)
    // sgpu_extract_stream: second input slot, copy-engine streams, slot events
    DevBuf input2;
    DevBuf duo_trash;                      // k_gauss_duo's / k_gauss_trio's scratch stores
    hipStream_t h2d = nullptr, d2h = nullptr;
    hipEvent_t up_ev[2] = {}, down_ev[2] = {};
    bool gathered = false;
    hipEvent_t ev[T_N + 1] = {};
    float timing[T_N] = {};
    // matcher
    DevBuf m_d1, m_d2, m_s1, m_s2, m_part, m_terms, m_match, m_dist, m_mask, m_loc, m_colpart, m_cols;
    DevBuf m_prune, m_s1c;                 // pruned column side: [rmax n1][map n1][ct n1 + pad], s8 rows
    bool match_prune = true;               // plain mutual matching prunes set 1 for the column side
                                           // (sgpu_debug_set_match_prune; SGPU_MATCH_PRUNE=off)
    std::vector<int> h_match;
    bool dist_ready = false;
    // multi-GPU: RCCL communicator of this context's device (sgpu_comm_*)
    ncclComm_t comm = nullptr;
    int comm_ranks = 0, comm_rank = 0;
    DevBuf c_buf;

    int fail(int code, const char* what, hipError_t e = hipSuccess) {
        err = what;
        if (e != hipSuccess) {
            err += ": ";
            err += hipGetErrorString(e);
        }
        return code;
    }
    // part holding image i of the last batch
    int part_of(int i) const {
        for (int p = 0; p < nparts; p++)
            if (i < part[p].img0 + part[p].n) return p;
        return nparts - 1;
    }
};

#define HIPCHK(ctx, call)                                                \
    do {                                                                 \
        hipError_t _e = (call);                                          \
        if (_e != hipSuccess) return (ctx)->fail(SGPU_ENODEV, #call, _e); \
    } while (0)
#define ALLOCCHK(ctx, call)                                              \
    do {                                                                 \
        hipError_t _e = (call);                                          \
        if (_e != hipSuccess) return (ctx)->fail(SGPU_ENOMEM, #call, _e); \
    } while (0)

extern "C" {

void sgpu_default_options(sgpu_options* o) {
    o->filter_width_factor = 4.0f;
    o->descriptor_window_factor = 3.0f;
    o->orientation_window_factor = 2.0f;
    o->orientation_gaussian_factor = 1.5f;
    o->dog_threshold = 0.0f;
    o->edge_threshold = 0.0f;
    o->subpixel = 1;
    o->max_orientation = 2;
    o->fixed_orientation = 0;
    o->octave_min = 0;
    o->octave_num = -1;
    o->dog_level_num = 3;
    o->lowe_origin = 0;
    o->normalized = 1;
    o->descriptors = 1;
    o->keep_extremum_sign = 0;
    o->circular_window = 0;
    o->verbose = 0;
    o->max_dimension = 13200;
    o->preprocess_on_cpu = 1;
    o->feature_count_threshold = -1;
    o->truncate_method = 0;
}

// SiftGPU::ParseParam (SiftGPU.cpp:801-1246): options are matched on their first four
// characters, case-insensitively; numeric arguments are consumed only when they parse and
// pass the same range checks as the reference.
int sgpu_parse_args(sgpu_options* o, int argc, const char* const* argv, int* device) {
    if (!o) return SGPU_EINVAL;
    auto key = [](const char* s) {
        std::string k;
        for (int i = 0; i < 4 && s[i]; i++) k += (char)((s[i] >= 'A' && s[i] <= 'Z') ? s[i] + 32 : s[i]);
        return k;
    };
    for (int i = 0; i < argc; i++) {
        const char* arg = argv[i];
        if (!arg || arg[0] != '-' || !arg[1]) continue;
        const std::string k = key(arg + 1);
        const char* param = (i + 1 < argc) ? argv[i + 1] : nullptr;
        float fv = 0.f;
        int iv = 0;
        if (k == "cuda") {
            int dev = -1;
            if (param && sscanf(param, "%d", &dev) == 1 && dev >= 0) {
                if (device) *device = dev;
                i++;
            }
        } else if (k == "sd") o->descriptors = 0;
        else if (k == "unn") o->normalized = 0;
        else if (k == "ndes") o->normalized = 1;
        else if (k == "m" || k == "mo") {
            int mo = 2;
            if (param) sscanf(param, "%d", &mo);
            o->max_orientation = std::min(std::max(1, mo), 4);
        } else if (k == "m2p") o->max_orientation = 2;
        else if (k == "s") {
            int sp = 1;
            if (param) sscanf(param, "%d", &sp);
            o->subpixel = std::min(std::max(0, sp), 5);
        } else if (k == "ofix") o->fixed_orientation = (strcmp(arg + 1, "ofix") == 0);
        else if (k == "lowe") o->lowe_origin = 1;
        else if (k == "sign") o->keep_extremum_sign = 1;
        else if (k == "prep") o->preprocess_on_cpu = 1;
        else if (k == "nopr") o->preprocess_on_cpu = 0;
        else if (!param) continue;
        else if (k == "tc" || k == "tc1" || k == "tc2" || k == "tc3") {
            // SiftGPU.cpp:1185-1203: the method is set even when no count follows
            o->truncate_method = k == "tc2" ? 1 : k == "tc3" ? 2 : 0;
            if (sscanf(param, "%d", &iv) == 1 && iv > 0) { o->feature_count_threshold = iv; i++; }
        } else if (k == "maxd") {   // SiftGPU.cpp:1213-1222
            if (sscanf(param, "%d", &iv) == 1 && iv > 0) { o->max_dimension = iv; i++; }
        }
        else if (k == "f") { if (sscanf(param, "%f", &fv) == 1 && fv > 0) { o->filter_width_factor = fv; i++; } }
        else if (k == "w") { if (sscanf(param, "%f", &fv) == 1 && fv > 0) { o->orientation_window_factor = fv; i++; } }
        else if (k == "dw") { if (sscanf(param, "%f", &fv) == 1 && fv > 0) { o->descriptor_window_factor = fv; i++; } }
        else if (k == "fo") { iv = -3; if (sscanf(param, "%d", &iv) == 1 && iv >= -2) { o->octave_min = iv; i++; } }
        else if (k == "no") {
            iv = -1;
            if (sscanf(param, "%d", &iv) == 1) {
                iv = std::max(-1, iv);
                if (iv == -1 || iv >= 1) { o->octave_num = iv; i++; }
            }
        } else if (k == "t") { if (sscanf(param, "%f", &fv) == 1 && fv > 0 && fv < 0.5f) { o->dog_threshold = fv; i++; } }
        else if (k == "e") { if (sscanf(param, "%f", &fv) == 1 && fv > 0) { o->edge_threshold = fv; i++; } }
        else if (k == "d") { if (sscanf(param, "%d", &iv) == 1 && iv >= 1 && iv <= 6) { o->dog_level_num = iv; i++; } }
        else if (k == "v") { if (sscanf(param, "%d", &iv) == 1 && iv >= 0 && iv <= 4) o->verbose = iv; }
    }
    return SGPU_OK;
}

int sgpu_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int sgpu_ctx_set_options(sgpu_ctx* ctx, const sgpu_options* opt) {
    if (!ctx) return SGPU_EINVAL;
    sgpu_options o;
    if (opt) o = *opt; else sgpu_default_options(&o);
    // -fo -2 runs as in the reference: its initial smoothing sigma is 0 (sqrt only when
    // 1.6 > 0.5 * 4 + 0.001, SiftGPU.cpp:446-452), CreateFilterKernel(0) yields NaN taps
    // (ProgramCU.cu:391-398) and the NaN pyramid has no keypoint with an orientation: the call
    // succeeds with 0 features.  -fo below -3 is clamped to -3
    // (PyramidCU.cpp:106-107).
    if (o.octave_min < -3) o.octave_min = -3;
    if (o.dog_level_num < 1 || o.dog_level_num > 6) return ctx->fail(SGPU_EINVAL, "dog_level_num must be 1..6");
    if (o.max_dimension < 8) return ctx->fail(SGPU_EINVAL, "max_dimension must be >= 8");
    ctx->opt = o;
    sgp::Options po;
    po.filter_width_factor = o.filter_width_factor;
    po.dog_level_num = o.dog_level_num;
    po.dog_threshold = o.dog_threshold;
    po.edge_threshold = o.edge_threshold;
    po.octave_min = o.octave_min;
    ctx->sched = sgp::make_schedule(po);
    return SGPU_OK;
}

// A part's streams and events, created when the part is first used: the pyramid/detection
// stream gets the dispatch priority over the orientation/descriptor stream (of the previous
// part, when a batch runs in parts); octaves >= 1 of the pyramid run on a third stream.
enum { PS_MAIN = 1, PS_LO = 2, PS_OCT = 4, PS_ALL = 7 };
static int part_streams(Part& pt, int which = PS_ALL) {
    int prio_lo = 0, prio_hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
    if ((which & PS_MAIN) && !pt.stream &&
        hipStreamCreateWithPriority(&pt.stream, hipStreamNonBlocking, prio_hi) != hipSuccess)
        return SGPU_ENODEV;
    if ((which & PS_LO) && !pt.stream_lo &&
        hipStreamCreateWithPriority(&pt.stream_lo, hipStreamNonBlocking, prio_lo) != hipSuccess)
        return SGPU_ENODEV;
    if ((which & PS_OCT) && !pt.stream_oct &&
        hipStreamCreateWithPriority(&pt.stream_oct, hipStreamNonBlocking, prio_hi) != hipSuccess)
        return SGPU_ENODEV;
    if (!pt.ev_ds) {
        // stage events.  Each record leaves the GPU idle ~4.5 us between the kernels around it
        // (C2 kernel trace; tests/microbench/event_gap.hip), whatever its flags: a device-scope
        // release or no timing at all measured the same
        for (hipEvent_t& e : pt.ev)
            if (hipEventCreate(&e) != hipSuccess) return SGPU_ENODEV;
        if (hipEventCreateWithFlags(&pt.ev_ds, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&pt.ev_oct, hipEventDisableTiming) != hipSuccess)
            return SGPU_ENODEV;
    }
    return SGPU_OK;
}

int sgpu_ctx_create(int device, const sgpu_options* opt, sgpu_ctx** out) {
    if (!out) return SGPU_EINVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return SGPU_ENODEV;
    if (device < 0 || device >= n) return SGPU_EINVAL;
    sgpu_ctx* ctx = new sgpu_ctx();
    ctx->device = device;
    if (hipSetDevice(device) != hipSuccess ||
        hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return SGPU_ENODEV;
    }
    for (int i = 0; i <= T_N; i++) (void)hipEventCreate(&ctx->ev[i]);
    // Streams in an order that puts the concurrently busy ones on distinct hardware queues: the
    // runtime hands a process's streams the hardware queues in turn (4 on the GPU box), so the
    // i-th stream created here shares a queue with the (i+4)-th.  Busy together: a part's
    // pyramid stream and its octave stream (extract), and in sgpu_extract_stream also the copy
    // streams h2d / d2h (a batch's orientation / descriptor stream runs beside the copies
    // only).  Order (queue = index mod 4): 0 context stream, 1 part 0 main, 2 part 0 octaves,
    // 3 h2d, 4 d2h, 5 part 0 low, 6 part 1 octaves, 7-8 part 2 main / low (idle unless
    // SGPU_DEBUG_PARTS4), 9 part 1 main, 10 part 1 low: the main and octave streams on queues
    // 1 and 2, the copies on 3 and 0.  Measured: the same streams created part by part put a
    // copy stream beside a pyramid stream and cost the host-in / host-out stream 13 % (DESIGN.md
    // 4.3).  The rest are created when first used (part_streams).
    {
        Part* p = ctx->part;
        bool ok = part_streams(p[0], PS_MAIN) == SGPU_OK && part_streams(p[0], PS_OCT) == SGPU_OK &&
                  hipStreamCreateWithFlags(&ctx->h2d, hipStreamNonBlocking) == hipSuccess &&
                  hipStreamCreateWithFlags(&ctx->d2h, hipStreamNonBlocking) == hipSuccess &&
                  part_streams(p[0], PS_LO) == SGPU_OK && part_streams(p[1], PS_OCT) == SGPU_OK &&
                  part_streams(p[2], PS_MAIN) == SGPU_OK && part_streams(p[2], PS_LO) == SGPU_OK &&
                  part_streams(p[1], PS_MAIN) == SGPU_OK && part_streams(p[1], PS_LO) == SGPU_OK;
        for (int i = 0; ok && i < 2; i++)
            ok = hipEventCreateWithFlags(&ctx->up_ev[i], hipEventDisableTiming) == hipSuccess &&
                 hipEventCreateWithFlags(&ctx->down_ev[i], hipEventDisableTiming) == hipSuccess;
        if (!ok) {
            sgpu_ctx_destroy(ctx);
            return SGPU_ENODEV;
        }
    }
    // test mode for the C++ replicas, which only see SiftGPU.h: the bit-exact descriptor
    if (const char* ev = getenv("SGPU_EXACT_DESCRIPTOR"))
        if (ev[0] == '1') ctx->debug_flags |= SGPU_DEBUG_EXACT_DESCRIPTOR;
    // A/B hook for the Gaussian kernels (bench / probe runs in one process tree)
    if (const char* ev = getenv("SGPU_GAUSS")) {
        if (!strcmp(ev, "block")) ctx->debug_flags |= SGPU_DEBUG_GAUSS_BLOCK;
    }
    if (const char* ev = getenv("SGPU_DUO")) {   // A/B hook of the paired-level kernel
        if (!strcmp(ev, "off")) ctx->debug_flags |= SGPU_DEBUG_DUO_OFF;
        if (!strcmp(ev, "always")) ctx->debug_flags |= SGPU_DEBUG_DUO_ALWAYS;
        if (!strcmp(ev, "on")) ctx->duo_on = true;
    }
    if (const char* ev = getenv("SGPU_DUO_WIDE")) {
        if (ev[0] == '1') ctx->duo_wide = true;
    }
    if (const char* ev = getenv("SGPU_DUO_U8")) {
        if (ev[0] == '1') ctx->duo_u8 = true;
    }
    if (const char* ev = getenv("SGPU_DUO_PLAN")) {   // A/B hook of the octave pairing
        if (!strcmp(ev, "end")) ctx->duo_plan = SGPU_PAIRS_END;
        if (!strcmp(ev, "front")) ctx->duo_plan = SGPU_PAIRS_FRONT;
    }
    if (const char* ev = getenv("SGPU_TRIO")) {   // A/B hook of the three-level kernel
        if (!strcmp(ev, "off")) ctx->trio_mode = SGPU_TRIO_OFF;
        if (!strcmp(ev, "always")) ctx->trio_mode = SGPU_TRIO_ALWAYS;
        if (!strcmp(ev, "on")) ctx->trio_mode = SGPU_TRIO_ON;
    }
    if (const char* ev = getenv("SGPU_GAUSS_BANDS"))
        if (!strcmp(ev, "long")) ctx->debug_flags |= SGPU_DEBUG_GAUSS_LONG_BANDS;
    if (const char* ev = getenv("SGPU_PYR")) {
        if (!strcmp(ev, "serial")) ctx->debug_flags |= SGPU_DEBUG_PYR_SERIAL;
    }
    if (const char* ev = getenv("SGPU_STREAMS")) ctx->multi_stream = !strcmp(ev, "multi");
    if (const char* ev = getenv("SGPU_MATCH"))
        if (!strcmp(ev, "reg")) ctx->debug_flags |= SGPU_DEBUG_MATCH_REGSTAGE;
    if (const char* ev = getenv("SGPU_DESC")) {
        if (!strcmp(ev, "dual")) ctx->debug_flags |= SGPU_DEBUG_DESC_DUAL;
        if (!strcmp(ev, "narrow")) ctx->debug_flags |= SGPU_DEBUG_DESC_WIDE_OFF;
        if (!strcmp(ev, "wide")) ctx->debug_flags |= SGPU_DEBUG_DESC_WIDE_ALWAYS;
    }
    if (const char* ev = getenv("SGPU_GAUSS_TILE")) {   // A/B hook of the tile kernel
        if (!strcmp(ev, "off")) ctx->debug_flags |= SGPU_DEBUG_GAUSS_TILE_OFF;
        if (!strcmp(ev, "always")) ctx->debug_flags |= SGPU_DEBUG_GAUSS_TILE_ALWAYS;
    }
    if (const char* ev = getenv("SGPU_WIDE_DESC_MAX"))
        if (atoll(ev) >= 0) ctx->wide_desc_max = (size_t)atoll(ev);
    if (const char* ev = getenv("SGPU_EXTREMA")) {   // A/B hook of the tile extremum kernel
        if (!strcmp(ev, "wave")) ctx->debug_flags |= SGPU_DEBUG_EXTREMA_TILE_OFF;
    }
    if (const char* ev = getenv("SGPU_TILE_DUO"))
        ctx->tile_duo = !strcmp(ev, "on");
    if (const char* ev = getenv("SGPU_MATCH_PRUNE"))   // A/B hook of the pruned column side
        ctx->match_prune = strcmp(ev, "off") != 0;
    if (const char* ev = getenv("SGPU_GAUSS_TILE_MB"))
        if (atoi(ev) >= 0) ctx->tile_mb = atoi(ev);
    ctx->env_flags = ctx->debug_flags;   // kept by sgpu_debug_set_flags (A/B runs of the probes)
    int rc = sgpu_ctx_set_options(ctx, opt);
    if (rc != SGPU_OK) {
        sgpu_ctx_destroy(ctx);
        return rc;
    }
    *out = ctx;
    return SGPU_OK;
}

int sgpu_ctx_destroy(sgpu_ctx* ctx) {
    if (!ctx) return SGPU_EINVAL;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (Part& pt : ctx->part) {
        if (pt.stream) (void)hipStreamSynchronize(pt.stream);
        if (pt.stream_lo) (void)hipStreamSynchronize(pt.stream_lo);
        if (pt.stream_oct) (void)hipStreamSynchronize(pt.stream_oct);
        pt.release();
    }
    if (ctx->comm) (void)ncclCommDestroy(ctx->comm);
    ctx->comm = nullptr;
    for (hipStream_t st : {ctx->h2d, ctx->d2h})
        if (st) (void)hipStreamSynchronize(st);
    for (int i = 0; i < 2; i++) {
        if (ctx->up_ev[i]) (void)hipEventDestroy(ctx->up_ev[i]);
        if (ctx->down_ev[i]) (void)hipEventDestroy(ctx->down_ev[i]);
    }
    if (ctx->h2d) (void)hipStreamDestroy(ctx->h2d);
    if (ctx->d2h) (void)hipStreamDestroy(ctx->d2h);
    DevBuf* bufs[] = {&ctx->input, &ctx->input2, &ctx->duo_trash, &ctx->all_keys, &ctx->all_desc, &ctx->gray, &ctx->pre, &ctx->m_d1, &ctx->m_d2, &ctx->m_s1, &ctx->m_s2,
                      &ctx->m_part, &ctx->m_terms, &ctx->m_match, &ctx->m_dist, &ctx->m_mask, &ctx->m_loc,
                      &ctx->m_colpart, &ctx->m_cols, &ctx->m_prune, &ctx->m_s1c,
                      &ctx->c_buf};
    for (DevBuf* b : bufs) b->release();
    for (int i = 0; i <= T_N; i++)
        if (ctx->ev[i]) (void)hipEventDestroy(ctx->ev[i]);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return SGPU_OK;
}

const char* sgpu_last_error(const sgpu_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

// Layout of one part of the planned batch (plan_batch): feature parameters, buffer offsets,
// capacities, and every device and pinned buffer the part's pipeline needs, allocated (grow-only).
// enqueue_part runs it first; sgpu_reserve (SiftGPU::AllocatePyramid) runs it alone.
static int layout_part(sgpu_ctx* ctx, Part& pt) {
    const sgpu_options& O = ctx->opt;
    const sgp::Schedule& S = ctx->sched;
    const int d = S.dog_level_num, nlev = S.level_num;
    const int noct = (int)ctx->oct.size();
    const int n = pt.n;

    // ---- layout: pyramid [octave][level][image][h][wa]; mask [octave][dog level][image][h][words]
    sgk::FeatureParams& fp = pt.fp;
    fp = sgk::FeatureParams{};
    fp.batch = n;
    fp.n_octaves = noct;
    fp.d = d;
    long long goff = 0, moff = 0;
    int rows = 0;
    for (int o = 0; o < noct; o++) {
        const sgp::Octave& oc = ctx->oct[o];
        sgk::OctaveDesc& od = fp.oct[o];
        od.w = oc.w;
        od.h = oc.h;
        od.wa = oc.wa;
        od.nwords = (oc.wa + 31) / 32;
        od.gauss_off = goff;
        od.level_stride = (long long)n * oc.wa * oc.h;
        goff += od.level_stride * nlev;
        od.mask_off = moff;
        od.mask_level_stride = (long long)n * oc.h * od.nwords;
        moff += od.mask_level_stride * d;
        fp.row_off[o] = rows;
        rows += d * oc.h;
    }
    fp.rows_per_image = rows;
    pt.total_rows = rows * n;
    pt.mask_words = moff;
    for (int j = 0; j < d; j++) fp.level_sigma[j] = sgp::level_sigma(S, j + S.level_min + 1);
    fp.sigma_step = powf(2.0f, 1.0f / d);
    fp.t0 = (O.subpixel ? 0.8f : 1.0f) * S.dog_threshold;
    fp.t = S.dog_threshold;
    fp.edge = (S.edge_threshold + 1) * (S.edge_threshold + 1) / S.edge_threshold;
    fp.gaussian_factor = O.orientation_gaussian_factor;
    fp.sample_factor = O.orientation_gaussian_factor * O.orientation_window_factor;
    fp.window_factor = O.descriptor_window_factor;
    fp.subpixel = O.subpixel ? 1 : 0;
    fp.num_orientation = O.fixed_orientation ? 0 : std::min(O.max_orientation, 2);
    fp.keep_sign = O.keep_extremum_sign;
    fp.circular = O.circular_window;
    fp.normalize = O.normalized;
    fp.unit_input = ctx->unit_input ? 1 : 0;
    fp.origin_offset = O.lowe_origin ? 0.0f : 0.5f;
    fp.octave_min = ctx->plan.octave_min + ctx->plan.ds;   // coordinate scale 2^(om + ds)

    // candidate capacity: grow-only, first guess one per 256 octave pixels
    const size_t sum_px = (size_t)goff / (size_t)std::max(1, nlev) / (size_t)n;
    pt.cand_cap = (ctx->debug_flags & SGPU_DEBUG_TINY_CAP)
                      ? std::max<size_t>(pt.cand_cap, 64)
                      : std::max(pt.cand_cap, std::max<size_t>(1024, sum_px / 256 * n));
    const size_t nc = pt.cand_cap, ne_cap = 2 * nc;
    // + 256 B: the descriptor's 16-byte strip loads may read up to 4 floats past the end of a
    // row (k_descriptor_fast).  Invariant: every strip it loads starts at a sample of the
    // feature's box, which is clamped to columns 1 .. W-2 and rows 1 .. H-2 of the plane for any
    // keypoint (detected or caller-supplied), and an empty box loads at row 1, column 1; so the
    // overshoot past the last plane is at most 5 floats, whatever the keypoint.
    ALLOCCHK(ctx, pt.pyr.ensure((size_t)goff * sizeof(float) + 256));
    ALLOCCHK(ctx, pt.mask.ensure((size_t)moff * sizeof(uint32_t)));
    ALLOCCHK(ctx, pt.row_count.ensure((size_t)pt.total_rows * sizeof(uint32_t)));
    ALLOCCHK(ctx, pt.row_base.ensure(((size_t)pt.total_rows + 1) * sizeof(uint32_t)));
    ALLOCCHK(ctx, pt.img_off_dev.ensure((size_t)(n + 2) * sizeof(int64_t)));
    ALLOCCHK(ctx, pt.cand.ensure(nc * sizeof(float4)));
    ALLOCCHK(ctx, pt.info.ensure(nc * sizeof(int2)));
    ALLOCCHK(ctx, pt.ocount.ensure(nc * sizeof(uint32_t)));
    ALLOCCHK(ctx, pt.eoff.ensure((nc + 1) * sizeof(uint32_t)));
    ALLOCCHK(ctx, pt.feat.ensure(ne_cap * sizeof(float4)));
    ALLOCCHK(ctx, pt.feat_info.ensure(ne_cap * sizeof(int2)));
    ALLOCCHK(ctx, pt.keys.ensure(ne_cap * sizeof(float4)));
    if (O.descriptors) ALLOCCHK(ctx, pt.desc.ensure(ne_cap * 128 * sizeof(float)));
    ALLOCCHK(ctx, pt.scan_tmp.ensure((sgk::scan_tmp_words(std::max<size_t>(nc, pt.total_rows)) + 16) * 4));
    if (pt.h_read_n < (size_t)n + 2) {
        if (pt.h_read) (void)hipHostFree(pt.h_read);
        pt.h_read = nullptr;
        g_allocs++;
        ALLOCCHK(ctx, hipHostMalloc((void**)&pt.h_read, ((size_t)n + 2) * sizeof(int64_t)));
        pt.h_read_n = (size_t)n + 2;
    }
    return SGPU_OK;
}

// Queue the whole pipeline of one part on its stream.  `wait` (may be null) is an event the
// part's pyramid must wait for.  No host synchronisation.
static int enqueue_part(sgpu_ctx* ctx, Part& pt, const void* src_in, bool is_f32, int stride,
                        hipEvent_t wait, hipEvent_t wait_lo = nullptr) {
    hipStream_t st = pt.stream;   // reassigned per stage below
    const sgpu_options& O = ctx->opt;
    const sgp::Schedule& S = ctx->sched;
    const int nlev = S.level_num;
    const int noct = (int)ctx->oct.size();
    const int n = pt.n, h = ctx->h;
    const int rc_layout = layout_part(ctx, pt);
    if (rc_layout != SGPU_OK) return rc_layout;
    const sgk::FeatureParams& fp = pt.fp;
    const long long moff = pt.mask_words;
    const size_t nc = pt.cand_cap, ne_cap = 2 * nc;

    if (wait) HIPCHK(ctx, hipStreamWaitEvent(st, wait, 0));
    // stage events: always where a stream waits on them (the multi-stream layouts, the
    // host-in / host-out stream), else only when the context times its stages
    pt.events = ctx->stage_timing || !pt.one_stream || ctx->nparts > 1 || ctx->streaming;
    auto rec = [&](int i, hipStream_t s_) -> hipError_t {
        return pt.events ? hipEventRecord(pt.ev[i], s_) : hipSuccess;
    };
    HIPCHK(ctx, rec(0, st));
    const size_t img_elems = (size_t)stride * h;
    const uint8_t* src8 = is_f32 ? nullptr : (const uint8_t*)src_in + (size_t)pt.img0 * img_elems;
    const float* srcf = is_f32 ? (const float*)src_in + (size_t)pt.img0 * img_elems : nullptr;

    // ---- Gaussian pyramid (BuildPyramid, PyramidCU.cpp:979-1044): one launch per level
    // (k_gauss_wave) for the whole part.  Level kds = level_ds - level_min of octave o also writes
    // its 2x decimation as level 0 of octave o+1 (PyramidCU.cpp:1024).
    float* pyr = pt.pyr.as<float>();
    sgk::Taps ltaps[sgk::kMaxLevels], taps0;
    int lfw[sgk::kMaxLevels] = {0};
    for (int k = 1; k < nlev; k++)
        lfw[k] = sgp::make_filter(S.sigma[k - 1], O.filter_width_factor, ltaps[k].k);
    const int fw0 = sgp::make_filter(S.initial_smooth, O.filter_width_factor, taps0.k);
    const int kds = S.level_ds - S.level_min;
    // Stream layout (SGPU_STREAMS=multi, not the default: extract_body): octaves >= 1 run on a
    // second stream, which starts as soon as octave 0's level kds has written octave 1's base
    // (level 0), so their small launches run beside octave 0's last levels (pyramid 3.64 vs
    // 3.69-3.74 ms per 128 x 1080p), and the main stream waits for them before
    // the extremum kernel.  SGPU_DEBUG_PYR_SERIAL: one stream for the pyramid only.
    const bool side = noct > 1 && !pt.one_stream && !(ctx->debug_flags & SGPU_DEBUG_PYR_SERIAL);
    const int wave_rows = (ctx->debug_flags & SGPU_DEBUG_GAUSS_BLOCK)
                              ? -1 : ((ctx->debug_flags >> SGPU_DEBUG_BAND_SHIFT) & 0x7ff);
    const bool long_bands = (ctx->debug_flags & SGPU_DEBUG_GAUSS_LONG_BANDS) != 0;
    // 2-D tiles for the cache-resident levels (sift_gauss_tile.hip): not with a forced kernel or
    // band height (those test the wave kernels)
    const bool tiles_on = wave_rows == 0 && !long_bands &&
                          !(ctx->debug_flags & SGPU_DEBUG_GAUSS_TILE_OFF);
    const bool tiles_all = tiles_on && (ctx->debug_flags & SGPU_DEBUG_GAUSS_TILE_ALWAYS);
    auto tiled = [&](const sgk::LevelOp& op) {
        return tiles_on && sgk::gauss_tile_supported(op) &&
               (tiles_all || 4ll * op.w * op.h * op.batch <= ((long long)ctx->tile_mb << 20));
    };
    auto level = [&](const sgk::LevelOp& op, hipStream_t s_) {
        return tiled(op) ? sgk::launch_gauss_tile(op, s_)
                         : sgk::launch_gauss_op(op, s_, wave_rows, long_bands);
    };
    // the level filters of every octave: op (o, k) filters level k-1 into level k (op (0, 0)
    // smooths the input into level 0); level kds of octave o also writes its decimation, level 0
    // of octave o+1
    struct Op { sgk::LevelOp op; int o, k; };
    std::vector<Op> ops;
    pt.gauss_launches = 0;   // kernel launches of the level filters (sgpu_last_pyramid_launches)
    ops.reserve((size_t)noct * nlev);
    for (int o = 0; o < noct; o++) {
        const sgk::OctaveDesc& od = fp.oct[o];
        const long long npx = (long long)od.wa * od.h;
        float* lvl0 = pyr + od.gauss_off;
        float* ds = nullptr;
        int dsw = 0, dsh = 0;
        long long ds_stride = 0;
        if (o + 1 < noct) {
            const sgk::OctaveDesc& nd = fp.oct[o + 1];
            ds = pyr + nd.gauss_off;
            dsw = nd.wa;
            dsh = nd.h;
            ds_stride = (long long)nd.wa * nd.h;
        }
        const float* in_f = srcf;
        const uint8_t* in_8 = src8;
        int in_stride = stride;
        long long in_img = (long long)img_elems;
        if (o == 0 && ctx->plan.octave_min != 0) {
            // -fo != 0: resample the input into level 1's storage (free until level 1 is
            // filtered), then the initial smoothing as for a float input
            float* tmp = lvl0 + od.level_stride;
            HIPCHK(ctx, sgk::launch_first_octave_input(srcf, src8, stride, (long long)img_elems,
                                                       ctx->w & ~3, h, ctx->plan.octave_min, tmp,
                                                       od.wa, od.h, npx, n, st));
            in_f = tmp;
            in_8 = nullptr;
            in_stride = od.wa;
            in_img = npx;
        }
        for (int k = (o == 0 ? 0 : 1); k < nlev; k++) {
            Op e{};
            e.o = o;
            e.k = k;
            sgk::LevelOp& op = e.op;
            op.fw = k == 0 ? fw0 : lfw[k];
            const float* tk = k == 0 ? taps0.k : ltaps[k].k;
            for (int i = 0; i < op.fw; i++) op.taps.k[i] = tk[i];
            const bool dk = ds && kds == k;
            op.src = k == 0 ? in_f : lvl0 + (k - 1) * od.level_stride;
            op.src_u8 = k == 0 ? in_8 : nullptr;
            op.src_stride = k == 0 ? in_stride : od.wa;
            op.src_img_stride = k == 0 ? in_img : npx;
            op.dst = lvl0 + k * od.level_stride;
            op.dst_img_stride = npx;
            op.w = od.wa;
            op.h = od.h;
            op.batch = n;
            op.ds_dst = dk ? ds : nullptr;
            op.ds_w = dk ? dsw : 0;
            op.ds_h = dk ? dsh : 0;
            op.ds_img_stride = dk ? ds_stride : 0;
            if (o == 0 && k == 0 && pt.one_stream) {
                // the first level launch also zeroes the extremum kernel's mask and row counts
                // and the orientation counts (one launch fewer than launch_zero)
                op.zero.p[0] = pt.row_count.as<uint32_t>();
                op.zero.n[0] = (size_t)pt.total_rows;
                op.zero.p[1] = pt.mask.as<uint32_t>();
                op.zero.n[1] = (size_t)moff;
                op.zero.p[2] = pt.ocount.as<uint32_t>();
                op.zero.n[2] = nc;
            }
            ops.push_back(e);
        }
    }
    pt.gauss_filters = (int)ops.size();
    // every level tiled (a cache-resident pyramid: one image, C2) and tile duos asked for
    // (SGPU_TILE_DUO=on, or SGPU_DEBUG_DUO_ALWAYS with SGPU_DEBUG_GAUSS_TILE_ALWAYS): the tile-duo
    // schedule -- octave
    // 0 pairs levels (0, 1), (2, 3), (4, 5) into tile duos (two levels per launch from one load,
    // sift_gauss_tile.hip), octaves >= 1 run level 1 alone and pair the rest; a job launches right
    // after the job holding its input, and octave o+1's level 1 shares the launch of octave o's last
    // duo (-no 4 -d 3: 9 launches instead of 15).  Measured slower than the single-level tiles of
    // the diagonal schedule (C2 pyramid 115-119 vs 97-99 us: a duo tile's stage-1 halo region and
    // its five barrier phases cost more than the launch and the level's round trip it saves,
    // DESIGN.md 4.6), so not the default.
    const bool want_duo = ctx->tile_duo || ((ctx->debug_flags & SGPU_DEBUG_DUO_ALWAYS) &&
                                            (ctx->debug_flags & SGPU_DEBUG_GAUSS_TILE_ALWAYS));
    bool all_tiled = want_duo && !side && !(ctx->debug_flags & SGPU_DEBUG_PYR_SERIAL) &&
                     kds >= 1 && !ops.empty();
    for (const Op& e : ops) all_tiled = all_tiled && tiled(e.op);
    if (all_tiled) {
        struct Job { size_t i0; int n, launch; };
        std::vector<Job> jobs;
        std::vector<int> job_of(ops.size(), -1);
        auto op_index = [&](int o, int k) -> int {
            for (size_t i = 0; i < ops.size(); i++)
                if (ops[i].o == o && ops[i].k == k) return (int)i;
            return -1;
        };
        for (size_t i = 0; i < ops.size();) {
            const Op& e = ops[i];
            const bool pair = e.k % 2 == 0 && i + 1 < ops.size() && ops[i + 1].o == e.o &&
                              ops[i + 1].k == e.k + 1 &&
                              sgk::gauss_tile_duo_supported(e.op, ops[i + 1].op);
            jobs.push_back({i, pair ? 2 : 1, 0});
            job_of[i] = (int)jobs.size() - 1;
            if (pair) job_of[i + 1] = (int)jobs.size() - 1;
            i += pair ? 2 : 1;
        }
        int last_launch = 0;
        for (Job& jb : jobs) {
            const Op& e = ops[jb.i0];
            int dep = -1;   // the op writing this job's input level
            if (e.k >= 2 || (e.k == 1 && e.o == 0)) dep = op_index(e.o, e.k - 1);
            else if (e.k == 1) dep = op_index(e.o - 1, kds);
            jb.launch = dep < 0 ? 0 : jobs[job_of[dep]].launch + 1;
            last_launch = std::max(last_launch, jb.launch);
        }
        for (int L = 0; L <= last_launch; L++) {
            std::vector<const Job*> in;
            for (const Job& jb : jobs)
                if (jb.launch == L) in.push_back(&jb);
            size_t q = 0;
            if (in.size() == 2 && in[0]->n != in[1]->n) {   // a duo beside a single level
                const Job* d = in[0]->n == 2 ? in[0] : in[1];
                const Job* o1 = in[0]->n == 2 ? in[1] : in[0];
                int nl = 0;
                HIPCHK(ctx, sgk::launch_gauss_tile_duo_one(ops[d->i0].op, ops[d->i0 + 1].op,
                                                           ops[o1->i0].op, st, &nl));
                pt.gauss_launches += nl;
                q = 2;
            } else if (in.size() == 2 && in[0]->n == 1 && in[1]->n == 1) {
                int nl = 0;
                HIPCHK(ctx, sgk::launch_gauss_tile_two(ops[in[0]->i0].op, ops[in[1]->i0].op, st, &nl));
                pt.gauss_launches += nl;
                q = 2;
            }
            for (; q < in.size(); q++) {
                const Job& jb = *in[q];
                if (jb.n == 2) HIPCHK(ctx, sgk::launch_gauss_tile_duo(ops[jb.i0].op, ops[jb.i0 + 1].op, st));
                else HIPCHK(ctx, sgk::launch_gauss_tile(ops[jb.i0].op, st));
                pt.gauss_launches++;
            }
        }
    } else if (side || (ctx->debug_flags & SGPU_DEBUG_PYR_SERIAL) || kds < 1) {
        // octave by octave, one level per launch (octaves >= 1 on the side stream in the
        // stream layout)
        for (const Op& e : ops) {
            const hipStream_t so = side && e.o >= 1 ? pt.stream_oct : st;
            pt.gauss_launches++;
            if (side && e.o == 1 && e.k == 1) HIPCHK(ctx, hipStreamWaitEvent(so, pt.ev_ds, 0));
            HIPCHK(ctx, level(e.op, so));
            if (side && e.o == 0 && e.k == kds && e.op.ds_dst) HIPCHK(ctx, hipEventRecord(pt.ev_ds, st));
        }
    } else {
        // Diagonal schedule: op (o, k) in slot o * kds + k.  Its inputs come
        // from earlier slots -- (o, k-1), and for k = 1 octave o-1's level kds (slot o * kds)
        // -- so the ops of a slot are independent and share a launch: octave o+1's levels 1, 2
        // run beside octave o's levels kds+1, kds+2 (15 launches instead of 21 for -no 4 -d 3),
        // the small jobs' latency-bound waves filling the large ones' CU slots.
        // Paired levels: ops (o, k) and (o, k+1) of a streaming-size level
        // (>= SGK_DUO_MIN_MB: not left in the Infinity Cache by the previous launch) with a
        // compiled width pair run as one k_gauss_duo launch in slot o * kds + k + 1 -- level k
        // read once, levels k+1 and k+2 written (12 instead of 16 B per pixel).
        const bool duo_all = (ctx->debug_flags & SGPU_DEBUG_DUO_ALWAYS) != 0;
        const bool duo_off = (ctx->debug_flags & SGPU_DEBUG_DUO_OFF) != 0 ||
                             (!SGK_DUO_DEFAULT && !duo_all && !ctx->duo_on);
        // Three levels: ops (o, k), (o, k+1), (o, k+2) with the widths (11, 13,
        // 17) and the third decimated into octave o+1 run as one k_gauss_trio launch in slot
        // o * kds + k + 2 (level k read once, levels k+1 .. k+3 and the decimation written:
        // 17 instead of 25 B per pixel), on levels >= SGK_TRIO_MIN_MB (any size with
        // SGPU_TRIO_ALWAYS); the octave's (21, 25) pair after it then pairs too.
        std::vector<char> trio_third(ops.size(), 0), in_trio(ops.size(), 0);
        std::vector<char> trio_octave(sgk::kMaxOctaves, 0);
        if (!duo_off && wave_rows >= 0 && ctx->trio_mode != SGPU_TRIO_OFF) {
            for (size_t i = 0; i + 2 < ops.size(); i++) {
                const Op& a = ops[i];
                const Op& b = ops[i + 1];
                const Op& c = ops[i + 2];
                if (in_trio[i] || a.o != b.o || a.o != c.o || b.k != a.k + 1 || c.k != a.k + 2) continue;
                const long long bytes = 4ll * a.op.w * a.op.h * a.op.batch;
                if (ctx->trio_mode != SGPU_TRIO_ALWAYS && bytes < ((long long)SGK_TRIO_MIN_MB << 20))
                    continue;
                if (!sgk::gauss_trio_supported(a.op, b.op, c.op)) continue;
                in_trio[i] = in_trio[i + 1] = in_trio[i + 2] = 1;
                trio_third[i + 2] = 1;
                trio_octave[a.o] = 1;
            }
        }
        std::vector<int> duo_next(ops.size(), -1);   // op i pairs with op duo_next[i]
        std::vector<char> duo_second(ops.size(), 0);
        // Pairs from the octave's end: on a level of >= SGK_DUO_WIDE_MIN_MB (any
        // size with SGPU_DEBUG_DUO_ALWAYS), octave o's levels pair as (4, 5) = (21, 25), (2, 3) =
        // (13, 17) with level 3's decimation, (0, 1) = the u8 ingest pair (13, 11) -- three
        // launches for octave 0 instead of four (level 0, (1, 2), (3, 4), level 5), 34 instead of
        // 38 B per pixel -- when the (2, 3) pair is supported; otherwise the pairs from the front.
        if (!duo_off && wave_rows >= 0 && ctx->duo_plan == SGPU_PAIRS_END) {
            for (size_t j = ops.size(); j >= 2; j--) {
                const size_t i = j - 2;   // candidate pair (i, i + 1)
                const Op& a = ops[i];
                const Op& b = ops[i + 1];
                if (a.o != b.o || b.k != a.k + 1 || (b.k % 2) != 1) continue;
                if (in_trio[i] || in_trio[i + 1] || duo_second[i] || duo_next[i + 1] >= 0) continue;
                const long long bytes = 4ll * a.op.w * a.op.h * a.op.batch;
                if (!duo_all && (bytes < ((long long)SGK_DUO_WIDE_MIN_MB << 20) ||
                                 a.op.w > SGK_DUO_PLAN_MAXW))
                    continue;
                // the octave takes the plan only with its (2, 3) pair: look it up first
                bool mid_ok = false;
                for (size_t q = 0; q + 1 < ops.size(); q++)
                    if (ops[q].o == a.o && ops[q].k == 2 && ops[q + 1].k == 3 && ops[q + 1].o == a.o)
                        mid_ok = sgk::gauss_duo_supported(ops[q].op, ops[q + 1].op) &&
                                 ops[q + 1].op.ds_dst != nullptr;
                if (!mid_ok || !sgk::gauss_duo_supported(a.op, b.op)) continue;
                duo_next[i] = (int)(i + 1);
                duo_second[i + 1] = 1;
            }
        }
        if (!duo_off && wave_rows >= 0) {
            for (size_t i = 0; i + 1 < ops.size(); i++) {
                const Op& a = ops[i];
                const Op& b = ops[i + 1];
                if (in_trio[i] || in_trio[i + 1]) continue;
                if (duo_second[i] || duo_next[i] >= 0 || duo_second[i + 1] || duo_next[i + 1] >= 0) continue;
                if (a.o != b.o || b.k != a.k + 1) continue;
                const long long bytes = 4ll * a.op.w * a.op.h * a.op.batch;
                if (!duo_all && bytes < ((long long)SGK_DUO_MIN_MB << 20)) continue;
                if (!duo_all && a.op.fw + b.op.fw > 24) {
                    const bool ds_pair = a.op.ds_dst != nullptr;
                    if (!ds_pair && !ctx->duo_wide && !trio_octave[a.o]) continue;
                    if (bytes < ((long long)SGK_DUO_WIDE_MIN_MB << 20)) continue;
                }
                // the u8 ingest pair (levels 0, 1: 725 us) displaces the (11, 13) pair of levels
                // 1, 2 (750 us, level 0 alone 390): opt-in
                if (!duo_all && !ctx->duo_u8 && a.op.src_u8) continue;
                // (a pair that decimates its second level only in the plan from the octave's end)
                if (b.op.ds_dst || !sgk::gauss_duo_supported(a.op, b.op)) continue;
                duo_next[i] = (int)(i + 1);
                duo_second[i + 1] = 1;
            }
        }
        bool any_duo = false, any_trio = false;
        for (int v : duo_next) any_duo |= v >= 0;
        for (char v : trio_third) any_trio |= v != 0;
        if (any_duo || any_trio)
            ALLOCCHK(ctx, ctx->duo_trash.ensure(std::max(sgk::kGaussDuoTrashBytes,
                                                         sgk::kGaussTrioTrashBytes)));
        int last = 0;
        for (const Op& e : ops) last = std::max(last, e.o * kds + e.k);
        for (int slot = 0; slot <= last; slot++) {
            const sgk::LevelOp* in_slot[sgk::kMaxOctaves];
            int m = 0;
            for (size_t i = 0; i < ops.size(); i++) {
                const Op& e = ops[i];
                if (trio_third[i] && e.o * kds + e.k == slot) {   // the trio ends in this slot
                    HIPCHK(ctx, sgk::launch_gauss_trio(ops[i - 2].op, ops[i - 1].op, e.op, st,
                                                       wave_rows, ctx->duo_trash.as<float>()));
                    pt.gauss_launches++;
                } else if (duo_second[i] && e.o * kds + e.k == slot) {   // the pair ends in this slot
                    HIPCHK(ctx, sgk::launch_gauss_duo(ops[i - 1].op, e.op, st, wave_rows,
                                                      ctx->duo_trash.as<float>()));
                    pt.gauss_launches++;
                } else if (!in_trio[i] && duo_next[i] < 0 && !duo_second[i] && e.o * kds + e.k == slot) {
                    in_slot[m++] = &e.op;
                }
            }
            int i = 0;
            for (; i + 1 < m; i += 2) {
                int nl = 0;
                const bool ta = tiled(*in_slot[i]), tb = tiled(*in_slot[i + 1]);
                if (ta && tb) {
                    HIPCHK(ctx, sgk::launch_gauss_tile_two(*in_slot[i], *in_slot[i + 1], st, &nl));
                } else if (!ta && !tb) {
                    HIPCHK(ctx, sgk::launch_gauss_two(*in_slot[i], *in_slot[i + 1], st, wave_rows,
                                                      long_bands, &nl));
                } else {
                    HIPCHK(ctx, level(*in_slot[i], st));
                    HIPCHK(ctx, level(*in_slot[i + 1], st));
                    nl = 2;
                }
                pt.gauss_launches += nl;
            }
            if (i < m) {
                HIPCHK(ctx, level(*in_slot[i], st));
                pt.gauss_launches++;
            }
        }
    }
    if (side) {
        HIPCHK(ctx, hipEventRecord(pt.ev_oct, pt.stream_oct));
        HIPCHK(ctx, hipStreamWaitEvent(st, pt.ev_oct, 0));
    }
    HIPCHK(ctx, rec(1, st));

    // ---- extrema + row scan (the strip extremum kernel only sets the bits it accepts)
    // (the row counts and the mask start zeroed: on one stream the first level launch zeroed
    // them and the orientation counts; otherwise one launch here, and the orientation counts
    // are zeroed on the feature stream after its waits)
    if (!pt.one_stream)
        HIPCHK(ctx, sgk::launch_zero(pt.row_count.as<uint32_t>(), (size_t)pt.total_rows,
                                     pt.mask.as<uint32_t>(), (size_t)moff, nullptr, 0, st));
    // a cache-resident pyramid (the same size rule as the level tiles): the tile extremum kernel
    const bool ext_tiles = !(ctx->debug_flags & SGPU_DEBUG_EXTREMA_TILE_OFF) &&
                           ((ctx->debug_flags & SGPU_DEBUG_GAUSS_TILE_ALWAYS) ||
                            4ll * fp.oct[0].wa * fp.oct[0].h * n <= ((long long)ctx->tile_mb << 20));
    HIPCHK(ctx, sgk::launch_extrema(pyr, pt.mask.as<uint32_t>(), pt.row_count.as<uint32_t>(),
                                    fp, st, ext_tiles));
    if (O.feature_count_threshold > 0)   // -tc: GenerateFeatureList skip + LimitFeatureCount(0)
        HIPCHK(ctx, sgk::launch_limit_rows(pt.row_count.as<uint32_t>(), fp,
                                           O.feature_count_threshold, O.truncate_method, st));
    HIPCHK(ctx, rec(7, st));
    HIPCHK(ctx, sgk::launch_scan(pt.row_count.as<uint32_t>(), pt.row_base.as<uint32_t>(),
                                 pt.total_rows, pt.scan_tmp.as<uint32_t>(), st));
    HIPCHK(ctx, rec(2, st));

    // ---- orientation (+ keypoint refinement), expansion, descriptors on the low-priority
    // stream: counts stay on the device, grids come from the previous call's counts (the
    // kernels grid-stride over whatever the device count is)
    if (!pt.one_stream) {
        st = pt.stream_lo;
        HIPCHK(ctx, hipStreamWaitEvent(st, pt.ev[2], 0));
    }
    if (wait_lo) HIPCHK(ctx, hipStreamWaitEvent(st, wait_lo, 0));   // previous features read out
    const uint32_t* n_cand_dev = pt.row_base.as<uint32_t>() + pt.total_rows;
    if (!pt.one_stream)
        HIPCHK(ctx, sgk::launch_zero(pt.ocount.as<uint32_t>(), nc, nullptr, 0, nullptr, 0, st));
    const int cand_grid = (int)std::min(nc, pt.cand_hint ? pt.cand_hint : nc);
    // few candidates (a single image): one wave per candidate instead of a quad, so that the
    // SIMDs are filled and each window is walked 64 samples at a time (same bits)
    const bool ori_wave = (ctx->debug_flags & SGPU_DEBUG_ORIENT_WAVE) ||
                          (pt.cand_hint > 0 && pt.cand_hint <= kWaveOrientationMax);
    const int feat_grid = (int)std::min(ne_cap, pt.feat_hint ? pt.feat_hint : ne_cap);
    // few features (a single image): a workgroup of 4 waves per feature instead of one wave
    // (k_descriptor_wide, same bits)
    const bool desc_wide = !(ctx->debug_flags & SGPU_DEBUG_DESC_WIDE_OFF) &&
                           ((ctx->debug_flags & SGPU_DEBUG_DESC_WIDE_ALWAYS) ||
                            (pt.feat_hint > 0 && pt.feat_hint <= ctx->wide_desc_max));
    HIPCHK(ctx, sgk::launch_orientation(pyr, pt.mask.as<uint32_t>(), pt.row_base.as<uint32_t>(),
                                        pt.total_rows, n_cand_dev, (int)nc, cand_grid, fp,
                                        pt.cand.as<float4>(), pt.info.as<int2>(),
                                        pt.ocount.as<uint32_t>(), st, ori_wave));
    if (O.feature_count_threshold > 0 && fp.num_orientation >= 2)   // LimitFeatureCount(1)
        HIPCHK(ctx, sgk::launch_limit_oriented(pt.ocount.as<uint32_t>(), pt.row_base.as<uint32_t>(),
                                               fp, O.feature_count_threshold, O.truncate_method,
                                               (uint32_t)nc, st));
    HIPCHK(ctx, rec(3, st));
    const uint32_t* n_feat_dev = pt.eoff.as<uint32_t>() + nc;
    // (the expansion launch also writes the readback record: candidate count + per-image offsets)
    sgk::ImageOffsetsArgs io;
    io.row_base = pt.row_base.as<uint32_t>();
    io.batch = n;
    io.rows_per_image = fp.rows_per_image;
    io.total_rows = pt.total_rows;
    io.off = pt.img_off_dev.as<int64_t>();
    // (the scan and the expansion in one single-workgroup launch measured slower for one image:
    // 17.0-17.5 against ~13.5 us for the two launches)
    HIPCHK(ctx, sgk::launch_scan(pt.ocount.as<uint32_t>(), pt.eoff.as<uint32_t>(), nc,
                                 pt.scan_tmp.as<uint32_t>(), st));
    HIPCHK(ctx, sgk::launch_expand(pt.cand.as<float4>(), pt.info.as<int2>(),
                                   pt.eoff.as<uint32_t>(), n_cand_dev, (int)nc, fp,
                                   pt.feat.as<float4>(), pt.feat_info.as<int2>(),
                                   pt.keys.as<float4>(), st, &io));
    HIPCHK(ctx, rec(4, st));
    // one image with registered host buffers: its keys, descriptors and count record go straight
    // to the host (enqueue_readback then copies nothing) -- from the workgroup-per-feature
    // descriptor kernel itself when it runs (written over the host link while it computes), else
    // by k_copy_out after it
    pt.copied_out = ctx->host_out.active && pt.one_stream && n == 1 && ctx->nparts == 1;
    const bool exact_desc = ctx->debug_flags & SGPU_DEBUG_EXACT_DESCRIPTOR;
    const bool dual_desc = ctx->debug_flags & SGPU_DEBUG_DESC_DUAL;
    const bool host_in_desc = pt.copied_out && O.descriptors && desc_wide && !exact_desc && !dual_desc;
    sgk::HostCopy hcopy;
    if (host_in_desc) {
        hcopy.keys = pt.keys.as<float4>();
        hcopy.rec = pt.img_off_dev.as<int64_t>();
        hcopy.rec_n = n + 2;
        hcopy.cap = (uint32_t)ctx->host_out.cap;
        hcopy.hkeys = reinterpret_cast<float4*>(ctx->host_out.keys);
        hcopy.hdesc = ctx->host_out.desc;
        hcopy.hrec = pt.h_read;
    }
    if (O.descriptors)
        HIPCHK(ctx, sgk::launch_descriptor(pyr, pt.feat.as<float4>(), pt.feat_info.as<int2>(),
                                           n_feat_dev, feat_grid, fp, pt.desc.as<float>(), st,
                                           nullptr, false, exact_desc, dual_desc, desc_wide,
                                           host_in_desc ? &hcopy : nullptr));
    HIPCHK(ctx, rec(5, st));
    if (pt.copied_out && !host_in_desc)
        HIPCHK(ctx, sgk::launch_copy_out(pt.keys.as<float4>(), O.descriptors ? pt.desc.as<float>() : nullptr,
                                         n_feat_dev, ctx->host_out.cap, pt.img_off_dev.as<int64_t>(),
                                         n + 2, ctx->host_out.keys,
                                         O.descriptors ? ctx->host_out.desc : nullptr, pt.h_read, st));
    return SGPU_OK;
}

// Queue the (pinned) readback of a part's counts and offsets.
static int enqueue_readback(sgpu_ctx* ctx, Part& pt) {
    hipStream_t st = pt.one_stream ? pt.stream : pt.stream_lo;
    // one copy: [0] = the candidate count, [1 .. n + 1] = the per-image feature offsets (the
    // record k_expand writes); none when k_copy_out wrote it with the features
    if (!pt.copied_out)
        HIPCHK(ctx, hipMemcpyAsync(pt.h_read, pt.img_off_dev.p, (size_t)(pt.n + 2) * sizeof(int64_t),
                                   hipMemcpyDeviceToHost, st));
    if (pt.events) HIPCHK(ctx, hipEventRecord(pt.ev[6], st));
    return SGPU_OK;
}

// Geometry of a batch of n images of w x h (first octave: GLTexInput::SetImageData +
// PyramidCU::InitPyramid with -fo, -prep, -maxd; octaves; sigma schedule) into the context.
static int plan_batch(sgpu_ctx* ctx, int n, int w, int h) {
    const sgpu_options& O = ctx->opt;
    const sgp::InputPlan plan = sgp::plan_input(w, h, O.octave_min, O.max_dimension, O.preprocess_on_cpu);
    if (plan.w < 8 || plan.h < 8) return ctx->fail(SGPU_EINVAL, "image too small for the first octave");
    {
        sgp::Options po;
        po.filter_width_factor = O.filter_width_factor;
        po.dog_level_num = O.dog_level_num;
        po.dog_threshold = O.dog_threshold;
        po.edge_threshold = O.edge_threshold;
        po.octave_min = plan.octave_min + plan.ds;   // GetInitialSmoothSigma(_octave_min + ds)
        ctx->sched = sgp::make_schedule(po);
    }
    ctx->plan = plan;
    ctx->oct = sgp::make_octaves(plan.w, plan.h, O.octave_num, plan.octave_min);
    const int noct = (int)ctx->oct.size();
    if (noct > sgk::kMaxOctaves) return ctx->fail(SGPU_EINVAL, "too many octaves");
    for (const auto& oc : ctx->oct)
        if (oc.w < 4 || oc.h < 4) return ctx->fail(SGPU_EINVAL, "image too small for the octave count");
    ctx->batch = n;
    ctx->w = plan.ds ? plan.w : w;
    ctx->h = plan.h;
    ctx->gathered = false;
    return SGPU_OK;
}

// After a failed extract nothing may still be queued that reads the caller's input or writes
// the caller's outputs, and no per-image query may read the previous extract's offsets (the
// batch geometry was already replaced): wait for every stream of the context, then forget the
// batch.
static int abandon_batch(sgpu_ctx* ctx, int rc) {
    ctx->host_out.done = false;
    for (hipStream_t st : {ctx->stream, ctx->h2d, ctx->d2h})
        if (st) (void)hipStreamSynchronize(st);
    for (Part& pt : ctx->part) {
        if (pt.stream) (void)hipStreamSynchronize(pt.stream);
        if (pt.stream_lo) (void)hipStreamSynchronize(pt.stream_lo);
        if (pt.stream_oct) (void)hipStreamSynchronize(pt.stream_oct);
        pt.img_off.clear();
    }
    ctx->batch = 0;
    ctx->img_off.clear();
    ctx->gathered = false;
    return rc;
}

// Argument checks of sgpu_extract*: a rejected call queues nothing and leaves the previous
// extract's results readable.
static int check_extract_args(sgpu_ctx* ctx, const void* images, bool is_f32, int n, int w, int h,
                              int stride, int flags, int color) {
    const bool staged = (flags & SGPU_INPUT_STAGED) != 0;
    const int channels = color == SGPU_RGB || color == SGPU_BGR ? 3 : color ? 4 : 1;
    if ((!images && !staged) || n <= 0 || w < 8 || h < 8 || stride < w * channels)
        return ctx->fail(SGPU_EINVAL, "bad image arguments");
    if (color && (staged || is_f32 || color > SGPU_BGRA))
        return ctx->fail(SGPU_EINVAL, "bad color input");
    if (staged && (is_f32 || ctx->staged_bytes < (size_t)n * h * stride))
        return ctx->fail(SGPU_EINVAL, "staged input does not match the batch");
    return SGPU_OK;
}

static int extract_body(sgpu_ctx* ctx, const void* images, bool is_f32, int n, int w, int h,
                        int stride, int flags, int color) {
    // a caller's float image may hold any range; u8, colour and the library's own conversions of
    // them lie in [0, 1] (the descriptor's 32-bit sums rely on it, sift_kernels.hip flat_narrow)
    ctx->unit_input = !is_f32;
    const bool staged = (flags & SGPU_INPUT_STAGED) != 0;
    const int channels = color == SGPU_RGB || color == SGPU_BGR ? 3 : color ? 4 : 1;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    int rc0 = plan_batch(ctx, n, w, h);
    if (rc0 != SGPU_OK) return rc0;
    const sgp::InputPlan plan = ctx->plan;

    // parts: one by default.  Measured on MI355X (profiles/): a second
    // part's pyramid starves beside the previous part's descriptor kernel (the dispatcher keeps
    // filling the CUs with descriptor workgroups despite the stream priorities), so splitting
    // does not pay yet.  Test hook: SGPU_DEBUG_PARTS2 / SGPU_DEBUG_PARTS4.
    int np = 1;
    if ((ctx->debug_flags & SGPU_DEBUG_PARTS2) && n >= 2) np = 2;
    if ((ctx->debug_flags & SGPU_DEBUG_PARTS4) && n >= 4) np = 4;
    ctx->nparts = np;
    for (int p = 0; p < np; p++)
        if (part_streams(ctx->part[p]) != SGPU_OK)
            return ctx->fail(SGPU_ENODEV, "stream creation failed");
    for (int p = 0, i0 = 0; p < np; p++) {
        const int cnt = n / np + (p < n % np ? 1 : 0);
        ctx->part[p].img0 = i0;
        ctx->part[p].n = cnt;
        ctx->part[p].one_stream = false;
        i0 += cnt;
    }
    // A single-part batch runs upload, pyramid and feature stages on one stream.  Measured
    // (alternating processes): the octave stream and the feature stream, each
    // joined by a cross-stream event wait, cost more than their overlap gains -- C2 (one image
    // through SiftGPU::RunSIFT) 0.50 vs 0.56-0.61 ms per image, the 128 x 1080p batch 15.26-15.33k
    // vs 14.50-14.75k images/s (extrema 1.72 vs 1.92 ms, orientation 0.50 vs 0.55 ms after the
    // waits).  SGPU_STREAMS=multi keeps the stream layout (A/B hook).
    const bool one = np == 1 && !ctx->multi_stream;
    ctx->part[0].one_stream = one;
    const hipStream_t up = one ? ctx->part[0].stream : ctx->stream;

    // input: host batches are uploaded first on the context stream.  The upload's events are
    // recorded only when there is input work to time or a stream to join: every event record
    // in a stream costs ~4.5 us of GPU time between the commands around it, whatever its flags
    // (tests/microbench/event_gap.hip: 2.2 vs 6.7 us per short kernel), and a staged or device
    // batch on one stream has neither (C2, the bench's batches)
    const size_t in_bytes = (size_t)n * h * stride * (is_f32 ? sizeof(float) : 1);
    const bool up_events = !one || ((color || plan.ds > 0 ||
                                     !(flags & (SGPU_INPUT_DEVICE | SGPU_INPUT_STAGED))) &&
                                    ctx->stage_timing);
    if (up_events) HIPCHK(ctx, hipEventRecord(ctx->ev[0], up));
    const void* src_in = staged ? ctx->input.p : images;
    if (!(flags & (SGPU_INPUT_DEVICE | SGPU_INPUT_STAGED))) {
        ctx->staged_bytes = 0;
        ALLOCCHK(ctx, ctx->input.ensure(in_bytes));
        HIPCHK(ctx, hipMemcpyAsync(ctx->input.p, images, in_bytes, hipMemcpyHostToDevice, up));
        src_in = ctx->input.p;
    }
    if (color) {
        // luminance on the device; the pipeline then takes it as float input, tw floats a row
        const int tw = w & ~3;
        ALLOCCHK(ctx, ctx->gray.ensure((size_t)n * h * tw * sizeof(float)));
        HIPCHK(ctx, sgk::launch_color_to_gray((const uint8_t*)src_in, n, w, h, stride, channels,
                                              color == SGPU_BGR || color == SGPU_BGRA,
                                              ctx->gray.as<float>(), up));
        src_in = ctx->gray.p;
        is_f32 = true;
        stride = tw;
    }
    if (plan.ds > 0) {
        // -fo > 0 with -prep (GLTexInput::SetImageData -> DownSamplePixelDataI2F/F,
        // GLTexImage.cpp:928-1009): pixel (r << ds, c << ds) of the input, plan.w x plan.h
        // (the sampled columns never reach the truncated-away ones)
        const size_t px = (size_t)plan.w * plan.h;
        ALLOCCHK(ctx, ctx->pre.ensure((size_t)n * px * sizeof(float)));
        HIPCHK(ctx, sgk::launch_first_octave_input(is_f32 ? (const float*)src_in : nullptr,
                                                   is_f32 ? nullptr : (const uint8_t*)src_in,
                                                   stride, (long long)stride * h, w & ~3, h, plan.ds,
                                                   ctx->pre.as<float>(), plan.w, plan.h,
                                                   (long long)px, n, up));
        src_in = ctx->pre.p;
        is_f32 = true;
        stride = plan.w;
    }
    if (up_events) HIPCHK(ctx, hipEventRecord(ctx->ev[1], up));

    // part p's pyramid starts when part p-1 has finished detection
    for (int p = 0; p < np; p++) {
        hipEvent_t wait = p == 0 ? (one ? nullptr : ctx->ev[1]) : ctx->part[p - 1].ev[2];
        int rc = enqueue_part(ctx, ctx->part[p], src_in, is_f32, stride, wait);
        if (rc != SGPU_OK) return rc;
    }
    for (int p = 0; p < np; p++) {
        int rc = enqueue_readback(ctx, ctx->part[p]);
        if (rc != SGPU_OK) return rc;
    }
    for (int p = 0; p < np; p++) {
        HIPCHK(ctx, hipStreamSynchronize(ctx->part[p].stream));
        HIPCHK(ctx, hipStreamSynchronize(ctx->part[p].stream_lo));
    }

    // capacity check: a part whose candidates overflowed is re-run with larger buffers
    for (int p = 0; p < np; p++) {
        Part& pt = ctx->part[p];
        uint32_t nc = (uint32_t)pt.h_read[0];
        if (nc > pt.cand_cap) {
            pt.cand_cap = (size_t)nc + nc / 4 + 1024;
            int rc = enqueue_part(ctx, pt, src_in, is_f32, stride, nullptr);
            if (rc == SGPU_OK) rc = enqueue_readback(ctx, pt);
            if (rc != SGPU_OK) return rc;
            HIPCHK(ctx, hipStreamSynchronize(pt.one_stream ? pt.stream : pt.stream_lo));
            nc = (uint32_t)pt.h_read[0];
            if (nc > pt.cand_cap) return ctx->fail(SGPU_ERANGE, "keypoint capacity overflow");
        }
        pt.n_cand = nc;
        pt.img_off.assign(pt.h_read + 1, pt.h_read + 2 + pt.n);
        pt.cand_hint = (size_t)nc + nc / 16 + 64;
        pt.feat_hint = (size_t)pt.img_off[pt.n] + pt.img_off[pt.n] / 16 + 64;
    }
    ctx->img_off.assign(n + 1, 0);
    int64_t base = 0;
    for (int p = 0; p < np; p++) {
        const Part& pt = ctx->part[p];
        for (int i = 0; i <= pt.n; i++) ctx->img_off[pt.img0 + i] = base + pt.img_off[i];
        base += pt.img_off[pt.n];
    }

    // timings: stages of part 0 (its pyramid and detection run alone), total over all parts
    Part& p0 = ctx->part[0];
    ctx->timing[T_UPLOAD] = 0.0f;
    if (!p0.events) {   // sgpu_set_stage_timing(ctx, 0): no stage events were recorded
        for (int i = T_UPLOAD; i <= T_DOWNLOAD; i++) ctx->timing[i] = 0.0f;
        ctx->timing[T_TOTAL] = ctx->timing[T_LIST] = 0.0f;
        return SGPU_OK;
    }
    if (up_events) (void)hipEventElapsedTime(&ctx->timing[T_UPLOAD], ctx->ev[0], ctx->ev[1]);
    (void)hipEventElapsedTime(&ctx->timing[T_PYRAMID], p0.ev[0], p0.ev[1]);
    (void)hipEventElapsedTime(&ctx->timing[T_DETECT], p0.ev[1], p0.ev[2]);
    (void)hipEventElapsedTime(&ctx->timing[T_LIST], p0.ev[7], p0.ev[2]);
    (void)hipEventElapsedTime(&ctx->timing[T_ORIENT], p0.ev[2], p0.ev[3]);
    (void)hipEventElapsedTime(&ctx->timing[T_EXPAND], p0.ev[3], p0.ev[4]);
    (void)hipEventElapsedTime(&ctx->timing[T_DESC], p0.ev[4], p0.ev[5]);
    (void)hipEventElapsedTime(&ctx->timing[T_DOWNLOAD], p0.ev[5], p0.ev[6]);
    (void)hipEventElapsedTime(&ctx->timing[T_TOTAL], up_events ? ctx->ev[0] : p0.ev[0], ctx->part[np - 1].ev[6]);
    return SGPU_OK;
}

static int extract_impl(sgpu_ctx* ctx, const void* images, bool is_f32, int n, int w, int h,
                        int stride, int flags, int color = 0) {
    if (!ctx) return SGPU_EINVAL;
    // a registered host output serves this extract only (consumed even when the extract is
    // rejected: ADVICE r05), and only one image
    const bool armed = ctx->host_out.armed;
    ctx->host_out.armed = false;
    ctx->host_out.done = false;
    const int rc_args = check_extract_args(ctx, images, is_f32, n, w, h, stride, flags, color);
    if (rc_args != SGPU_OK) return rc_args;
    ctx->host_out.active = armed && n == 1;
    const int rc = extract_body(ctx, images, is_f32, n, w, h, stride, flags, color);
    ctx->host_out.done = rc == SGPU_OK && ctx->host_out.active && ctx->nparts == 1 &&
                         ctx->part[0].copied_out;
    ctx->host_out.active = false;
    ctx->part[0].copied_out = ctx->part[1].copied_out = false;
    return rc == SGPU_OK ? rc : abandon_batch(ctx, rc);
}

// Host-in / host-out extraction of a stream of batches: SiftGPU::RunSIFT(w, h, data) per image
// followed by GetFeatureVector, i.e. with the reference's input upload (PyramidCU.cpp:949-976)
// and descriptor download (PyramidCU.cpp:434) in the measured work.  Two slots -- parts 0 and 1
// with their own buffers, two device input buffers -- alternate between batches: the upload of
// batch k+1 (host-to-device copy engine) and the download of batch k-1's keys and descriptors
// (device-to-host copy engine) run while batch k computes.  Kernels of consecutive batches stay
// in order (batch k+1's pyramid waits for batch k's last kernel), so every batch sees the whole
// GPU as in sgpu_extract.  One host wait per batch: the small count readback of batch k-1, needed
// to size its download, happens after batch k is queued.
static int extract_stream_body(sgpu_ctx* ctx, const uint8_t* const* batches, int nbatches,
                               int batch, int w, int h, int stride, float* keys, float* desc,
                               int64_t cap, int32_t* counts) {
    if (!batches || nbatches <= 0 || batch <= 0 || w < 8 || h < 8 || stride < w || !counts ||
        cap < 0)
        return ctx->fail(SGPU_EINVAL, "bad stream arguments");
    for (int k = 0; k < nbatches; k++)
        if (!batches[k]) return ctx->fail(SGPU_EINVAL, "null batch pointer");
    if (desc && !ctx->opt.descriptors) return ctx->fail(SGPU_EINVAL, "descriptors disabled (-sd)");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    int rc = plan_batch(ctx, batch, w, h);
    if (rc != SGPU_OK) return rc;
    int64_t out_base = 0;
    int result = SGPU_OK;
    auto emit_counts = [&](int k, const std::vector<int64_t>& off, int n) {
        for (int i = 0; i < n; i++) counts[(size_t)k * batch + i] = (int32_t)(off[i + 1] - off[i]);
    };
    if (ctx->plan.ds > 0) {
        // -fo > 0 with -prep samples the input on the device first (extract_impl): no overlap,
        // batch by batch
        for (int k = 0; k < nbatches; k++) {
            rc = extract_impl(ctx, batches[k], false, batch, w, h, stride, SGPU_INPUT_HOST);
            if (rc != SGPU_OK) return rc;
            emit_counts(k, ctx->img_off, batch);
            const int64_t nf = ctx->img_off[batch];
            if (out_base + nf > cap) {
                result = ctx->fail(SGPU_ERANGE, "features exceed the output capacity");
            } else if (nf > 0) {
                const Part& pt = ctx->part[0];
                if (keys)
                    HIPCHK(ctx, hipMemcpy(keys + out_base * 4, pt.keys.p, nf * sizeof(float4),
                                          hipMemcpyDeviceToHost));
                if (desc)
                    HIPCHK(ctx, hipMemcpy(desc + out_base * 128, pt.desc.p,
                                          nf * 128 * sizeof(float), hipMemcpyDeviceToHost));
            }
            out_base += nf;
        }
        return result;
    }
    if (part_streams(ctx->part[1]) != SGPU_OK)
        return ctx->fail(SGPU_ENODEV, "stream creation failed");
    if (!ctx->h2d) {   // created with the context; kept for a context whose creation order changes
        HIPCHK(ctx, hipStreamCreateWithFlags(&ctx->h2d, hipStreamNonBlocking));
        HIPCHK(ctx, hipStreamCreateWithFlags(&ctx->d2h, hipStreamNonBlocking));
        for (int i = 0; i < 2; i++) {
            HIPCHK(ctx, hipEventCreateWithFlags(&ctx->up_ev[i], hipEventDisableTiming));
            HIPCHK(ctx, hipEventCreateWithFlags(&ctx->down_ev[i], hipEventDisableTiming));
        }
    }
    const size_t in_bytes = (size_t)batch * h * stride;
    // each slot's kernels on its own stream (extract_body's measurement); slots and copies overlap
    ctx->part[0].one_stream = ctx->part[1].one_stream = !ctx->multi_stream;
    ctx->staged_bytes = 0;
    ALLOCCHK(ctx, ctx->input.ensure(in_bytes));
    ALLOCCHK(ctx, ctx->input2.ensure(in_bytes));
    void* din[2] = {ctx->input.p, ctx->input2.p};
    ctx->nparts = 1;
    // batch k's results: wait for its counts, re-run it on overflow, queue its download
    auto finish = [&](int k) -> int {
        Part& pt = ctx->part[k & 1];
        HIPCHK(ctx, hipEventSynchronize(pt.ev[6]));
        uint32_t nc = (uint32_t)pt.h_read[0];
        if (nc > pt.cand_cap) {
            pt.cand_cap = (size_t)nc + nc / 4 + 1024;
            int r = enqueue_part(ctx, pt, din[k & 1], false, stride, nullptr, nullptr);
            if (r == SGPU_OK) r = enqueue_readback(ctx, pt);
            if (r != SGPU_OK) return r;
            HIPCHK(ctx, hipStreamSynchronize(pt.one_stream ? pt.stream : pt.stream_lo));
            nc = (uint32_t)pt.h_read[0];
            if (nc > pt.cand_cap) return ctx->fail(SGPU_ERANGE, "keypoint capacity overflow");
        }
        pt.n_cand = nc;
        pt.img_off.assign(pt.h_read + 1, pt.h_read + 2 + pt.n);
        pt.cand_hint = (size_t)nc + nc / 16 + 64;
        pt.feat_hint = (size_t)pt.img_off[pt.n] + pt.img_off[pt.n] / 16 + 64;
        emit_counts(k, pt.img_off, pt.n);
        const int64_t nf = pt.img_off[pt.n];
        if (out_base + nf > cap) {
            result = ctx->fail(SGPU_ERANGE, "features exceed the output capacity");
        } else if (nf > 0) {
            HIPCHK(ctx, hipStreamWaitEvent(ctx->d2h, pt.ev[6], 0));
            if (keys)
                HIPCHK(ctx, hipMemcpyAsync(keys + out_base * 4, pt.keys.p, nf * sizeof(float4),
                                           hipMemcpyDeviceToHost, ctx->d2h));
            if (desc)
                HIPCHK(ctx, hipMemcpyAsync(desc + out_base * 128, pt.desc.p,
                                           nf * 128 * sizeof(float), hipMemcpyDeviceToHost,
                                           ctx->d2h));
        }
        HIPCHK(ctx, hipEventRecord(ctx->down_ev[k & 1], ctx->d2h));
        out_base += nf;
        return SGPU_OK;
    };
    for (int k = 0; k < nbatches; k++) {
        const int slot = k & 1;
        Part& pt = ctx->part[slot];
        pt.img0 = 0;
        pt.n = batch;
        // upload k into its slot once batch k-2's pyramid (the slot's last reader) is done
        if (k >= 2) HIPCHK(ctx, hipStreamWaitEvent(ctx->h2d, pt.ev[1], 0));
        HIPCHK(ctx, hipMemcpyAsync(din[slot], batches[k], in_bytes, hipMemcpyHostToDevice,
                                   ctx->h2d));
        HIPCHK(ctx, hipEventRecord(ctx->up_ev[slot], ctx->h2d));
        // compute k after batch k-1's last kernel; its features overwrite the slot only after
        // batch k-2's download
        if (k >= 1) HIPCHK(ctx, hipStreamWaitEvent(pt.stream, ctx->part[slot ^ 1].ev[5], 0));
        rc = enqueue_part(ctx, pt, din[slot], false, stride, ctx->up_ev[slot],
                          k >= 2 ? ctx->down_ev[slot] : nullptr);
        if (rc == SGPU_OK) rc = enqueue_readback(ctx, pt);
        if (rc == SGPU_OK && k >= 1) rc = finish(k - 1);
        if (rc != SGPU_OK) return rc;
    }
    rc = finish(nbatches - 1);
    if (rc != SGPU_OK) return rc;
    HIPCHK(ctx, hipStreamSynchronize(ctx->d2h));
    return result;
}

int sgpu_extract_stream(sgpu_ctx* ctx, const uint8_t* const* batches, int nbatches, int batch,
                        int w, int h, int stride, float* keys, float* desc, int64_t cap,
                        int32_t* counts) {
    if (!ctx) return SGPU_EINVAL;
    ctx->streaming = true;   // its waits use the slots' stage events
    ctx->host_out.done = false;
    const int rc = extract_stream_body(ctx, batches, nbatches, batch, w, h, stride, keys, desc,
                                       cap, counts);
    ctx->streaming = false;
    // on success as on failure: every copy from the caller's batches and into the caller's
    // outputs has completed, and the per-image queries (sgpu_copy_features, ...) have no "last
    // batch" after a stream
    return abandon_batch(ctx, rc);
}

void* sgpu_host_alloc(size_t bytes) {
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) return nullptr;
    return p;
}

void sgpu_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

// SiftGPU::RunSIFT(num, keys, keys_have_orientation) on image `image` of the last extract
// (SiftPyramid::SetKeypointList with run_on_current, SiftPyramid.cpp:293-310): the keys are
// assigned to levels as GenerateFeatureListTex does (PyramidCU.cpp:454-504, host side: a few
// float ops per key), then the device computes the strongest orientation when the keys have
// none and the descriptors, both written back in input order.  The results replace the
// context's features: image `image` has `num` features, every other image none.
int sgpu_extract_keypoints(sgpu_ctx* ctx, int image, const float* keys, int num,
                           int has_orientation) {
    if (!ctx || !keys || num <= 0) return SGPU_EINVAL;
    ctx->host_out.done = false;   // the features it writes replace what k_copy_out delivered
    if (ctx->batch <= 0 || image < 0 || image >= ctx->batch)
        return ctx->fail(SGPU_EINVAL, "no extracted image to describe keypoints on");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    const int p = ctx->part_of(image);
    Part& pt = ctx->part[p];
    const int b = image - pt.img0;
    const sgpu_options& O = ctx->opt;
    const sgp::Schedule& S = ctx->sched;
    const int d = S.dog_level_num, noct = (int)ctx->oct.size();
    const double twopi = 2.0 * 3.14159265358979323846;
    const float sigma_half_step = powf(2.0f, 0.5f / d);
    const float offset = O.lowe_origin ? 0.0f : 0.5f;
    const bool rect = has_orientation == -1;
    std::vector<float4> lf;
    std::vector<int2> li;
    std::vector<int> lidx;
    float octave_sigma = ldexpf(1.0f, ctx->plan.octave_min + ctx->plan.ds);   // PyramidCU.cpp:461-463
    for (int i = 0; i < noct; i++, octave_sigma *= 2.0f)
        for (int j = 0; j < d; j++) {
            const float level_sigma = sgp::level_sigma(S, j + S.level_min + 1) * octave_sigma;
            const float sigma_min = level_sigma / sigma_half_step;
            const float sigma_max = level_sigma * sigma_half_step;
            for (int k = 0; k < num; k++) {
                const float* key = keys + 4 * (size_t)k;
                // RECT (keys_have_orientation == -1, SiftPyramid.cpp:308-309): (x, y, width,
                // height) rectangles, levelled by min(width, height) / 12 (PyramidCU.cpp:480)
                const float sigmak = rect ? std::min(key[2], key[3]) / 12.0f : key[2];
                if ((sigmak >= sigma_min && sigmak < sigma_max) ||
                    (sigmak < sigma_min && i == 0 && j == 0) ||
                    (sigmak > sigma_max && i == noct - 1 && j == d - 1)) {
                    lf.push_back(make_float4((key[0] - offset) / octave_sigma + 0.5f,
                                             (key[1] - offset) / octave_sigma + 0.5f,
                                             key[2] / octave_sigma,
                                             rect ? key[3] / octave_sigma
                                                  : (float)std::fmod(twopi - key[3], twopi)));
                    li.push_back(make_int2(b, i * d + j));
                    lidx.push_back(k);
                }
            }
        }
    // the reference re-orders list entries i < num (_featureNum) only
    const int m = std::min<int>(num, (int)lf.size());
    hipStream_t st = ctx->stream;
    const size_t cap = std::max<size_t>(lf.size(), (size_t)num);
    ALLOCCHK(ctx, pt.feat.ensure(cap * sizeof(float4)));
    ALLOCCHK(ctx, pt.feat_info.ensure(cap * sizeof(int2)));
    ALLOCCHK(ctx, pt.keys.ensure((size_t)num * sizeof(float4)));
    ALLOCCHK(ctx, pt.ocount.ensure((cap + 1) * sizeof(int)));   // list -> input index, count
    if (O.descriptors) ALLOCCHK(ctx, pt.desc.ensure((size_t)num * 128 * sizeof(float)));
    int* d_index = pt.ocount.as<int>();
    uint32_t* d_m = pt.ocount.as<uint32_t>() + cap;
    if (m > 0) {
        HIPCHK(ctx, hipMemcpyAsync(pt.feat.p, lf.data(), m * sizeof(float4), hipMemcpyHostToDevice, st));
        HIPCHK(ctx, hipMemcpyAsync(pt.feat_info.p, li.data(), m * sizeof(int2), hipMemcpyHostToDevice, st));
        HIPCHK(ctx, hipMemcpyAsync(d_index, lidx.data(), m * sizeof(int), hipMemcpyHostToDevice, st));
    }
    const uint32_t mm = (uint32_t)m;
    HIPCHK(ctx, hipMemcpyAsync(d_m, &mm, sizeof(uint32_t), hipMemcpyHostToDevice, st));
    // keys come back unchanged when they carry orientations (no DownloadKeypoints)
    HIPCHK(ctx, hipMemcpyAsync(pt.keys.p, keys, (size_t)num * sizeof(float4), hipMemcpyHostToDevice, st));
    if (!has_orientation)
        HIPCHK(ctx, sgk::launch_orient_keys(pt.pyr.as<float>(), pt.feat.as<float4>(),
                                            pt.feat_info.as<int2>(), d_index, m, pt.fp,
                                            pt.keys.as<float4>(), st));
    if (O.descriptors) {
        HIPCHK(ctx, hipMemsetAsync(pt.desc.p, 0, (size_t)num * 128 * sizeof(float), st));
        HIPCHK(ctx, sgk::launch_descriptor(pt.pyr.as<float>(), pt.feat.as<float4>(),
                                           pt.feat_info.as<int2>(), d_m, std::max(m, 1), pt.fp,
                                           pt.desc.as<float>(), st, d_index, rect,
                                           ctx->debug_flags & SGPU_DEBUG_EXACT_DESCRIPTOR,
                                           ctx->debug_flags & SGPU_DEBUG_DESC_DUAL));
    }
    HIPCHK(ctx, hipStreamSynchronize(st));
    // the described image now owns the context's feature list
    for (int q = 0; q < ctx->nparts; q++) {
        Part& pq = ctx->part[q];
        for (int i = 0; i <= pq.n; i++)
            pq.img_off[i] = (q == p && pq.img0 + i > image) ? num : 0;
    }
    for (int i = 0; i <= ctx->batch; i++) ctx->img_off[i] = i > image ? num : 0;
    ctx->gathered = false;
    return SGPU_OK;
}

// SiftMatchGPU::SetDescriptors + GetSiftMatch (SiftMatchCU.cpp:71-179) in one call; with
// `guided`, SetFeautreLocation + GetGuidedSiftMatch (SiftMatchCU.cpp:104-136).
static int match_impl(sgpu_ctx* ctx, const uint8_t* d1, int n1, const uint8_t* d2, int n2,
                      float distmax, float ratiomax, int mbm, int max_match, int* out_pairs,
                      int flags, const float* loc1, const float* loc2,
                      const sgk::GuidedParams* guided) {
    if (!ctx) return SGPU_EINVAL;
    if (n1 <= 0 || n2 <= 0) return 0;   // SiftMatchCU.cpp:142
    if (!d1 || !d2 || (max_match > 0 && !out_pairs)) return ctx->fail(SGPU_EINVAL, "bad match arguments");
    if (guided && (!loc1 || !loc2)) return ctx->fail(SGPU_EINVAL, "guided match needs locations");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    if (!ctx->dist_ready) {
        // the same expression as RowMatch_Kernel (ProgramCU.cu:1838), evaluated on the host
        std::vector<float> t(sgk::kDistTable);
        for (int v = 0; v < sgk::kDistTable; v++)
            t[v] = (float)std::acos(std::min((double)(v * 0.000003814697265625f), 1.0));
        ALLOCCHK(ctx, ctx->m_dist.ensure(t.size() * sizeof(float)));
        HIPCHK(ctx, hipMemcpy(ctx->m_dist.p, t.data(), t.size() * sizeof(float), hipMemcpyHostToDevice));
        ctx->dist_ready = true;
    }
    const uint8_t* a = d1;
    const uint8_t* b = d2;
    // (no event before the uploads: nothing reads it, and each record costs ~4.5 us of GPU time)
    if (!(flags & SGPU_INPUT_DEVICE)) {
        ALLOCCHK(ctx, ctx->m_d1.ensure((size_t)n1 * 128));
        ALLOCCHK(ctx, ctx->m_d2.ensure((size_t)n2 * 128));
        HIPCHK(ctx, hipMemcpyAsync(ctx->m_d1.p, d1, (size_t)n1 * 128, hipMemcpyHostToDevice, st));
        HIPCHK(ctx, hipMemcpyAsync(ctx->m_d2.p, d2, (size_t)n2 * 128, hipMemcpyHostToDevice, st));
        a = ctx->m_d1.as<uint8_t>();
        b = ctx->m_d2.as<uint8_t>();
    }
    // guided: locations (float2 per feature) and the two geometric masks
    const size_t rmask_bytes = sgk::guided_mask_bytes(n1, n2);
    const size_t cmask_bytes = 0;   // the fused GEMM derives the column side from the same values
    const float* l1 = loc1;
    const float* l2 = loc2;
    if (guided) {
        ALLOCCHK(ctx, ctx->m_mask.ensure(rmask_bytes + cmask_bytes));
        if (!(flags & SGPU_INPUT_DEVICE)) {
            ALLOCCHK(ctx, ctx->m_loc.ensure((size_t)(n1 + n2) * 2 * sizeof(float)));
            float* dl = ctx->m_loc.as<float>();
            HIPCHK(ctx, hipMemcpyAsync(dl, loc1, (size_t)n1 * 2 * sizeof(float), hipMemcpyHostToDevice, st));
            HIPCHK(ctx, hipMemcpyAsync(dl + 2 * n1, loc2, (size_t)n2 * 2 * sizeof(float),
                                       hipMemcpyHostToDevice, st));
            l1 = dl;
            l2 = dl + 2 * n1;
        }
    }
    HIPCHK(ctx, hipEventRecord(ctx->ev[1], st));
    // Mutual matching: guided (or SGPU_DEBUG_FUSED_MATCH) computes the dots once and derives
    // both decisions from them (k_match_rows<.., COLS>); plain matching runs the row kernel a
    // second time with the sets swapped, which measured faster (1.07 vs 1.15 ms at 50k x 50k,
    // DESIGN.md section 10) because the fused epilogue halves the kernel's occupancy.
    const bool fused = mbm && (guided || (ctx->debug_flags & SGPU_DEBUG_FUSED_MATCH));
    // keyless folding (k_match_raw / k_match_rows<..., RAW>): exact whenever a tied maximum
    // cannot pass the ratio test, i.e. ratiomax <= 1 (the reference's default 0.8);
    // SGPU_DEBUG_KEYED_MATCH keeps the keyed epilogue.  dma: through the LDS-DMA kernel
    // k_match_raw (its own chunk split), unless SGPU_DEBUG_MATCH_REGSTAGE
    const bool raw = !guided && !(ratiomax > 1.0f) && !(ctx->debug_flags & SGPU_DEBUG_KEYED_MATCH);
    const bool dma = raw && !(ctx->debug_flags & SGPU_DEBUG_MATCH_REGSTAGE);
    const int ca = sgk::match_chunks(n1, n2, dma && !fused), panels = sgk::match_panels(n1);
    const int cb = mbm && !fused ? sgk::match_chunks(n2, n1, dma) : 0;
    // plain mutual matching decides only the columns some row matched (see below); their
    // count is known on the device only, so the partials are sized for any count
    const bool compact = mbm && !fused && !(ctx->debug_flags & SGPU_DEBUG_FULL_COLUMNS);
    const size_t part_b = compact ? sgk::match_part_bound(n2, n1, dma) : (size_t)cb * n2;
    // ... over the rows of set 1 that can change a listed column's decision (the LDS-DMA kernel
    // only: its B count may live on the device)
    const bool prune = compact && dma && ctx->match_prune;
    ALLOCCHK(ctx, ctx->m_part.ensure(std::max((size_t)ca * n1, part_b) * sizeof(sgk::Top2)));
    if (fused) ALLOCCHK(ctx, ctx->m_colpart.ensure((size_t)panels * n2 * sizeof(sgk::Top2)));
    if (compact) ALLOCCHK(ctx, ctx->m_cols.ensure((size_t)(2 * n2 + 3) * sizeof(int)));
    if (prune) {
        ALLOCCHK(ctx, ctx->m_prune.ensure(((size_t)3 * n1 + sgk::match_ct_pad()) * sizeof(int)));
        ALLOCCHK(ctx, ctx->m_s1c.ensure((size_t)n1 * 128));
    }
    ALLOCCHK(ctx, ctx->m_terms.ensure(((size_t)2 * (n1 + n2) + 2 * sgk::match_ct_pad()) * sizeof(int)));
    ALLOCCHK(ctx, ctx->m_match.ensure((size_t)(n1 + n2) * sizeof(int)));
    int* row1 = ctx->m_terms.as<int>();          // row terms 128 * sum(d1), column terms
    int* col2 = row1 + n1;                       // 128 * sum(d2) - 2^21
    int* ct1 = col2 + n2;                        // k_match_raw's column terms of each set
    int* ct2 = ct1 + n1 + sgk::match_ct_pad();
    int* match1 = ctx->m_match.as<int>();
    int* match2 = match1 + n1;
    sgk::Top2* part = ctx->m_part.as<sgk::Top2>();
    sgk::Top2* colpart = fused ? ctx->m_colpart.as<sgk::Top2>() : nullptr;
    uint8_t* rmask = guided ? ctx->m_mask.as<uint8_t>() : nullptr;
    if (guided)
        HIPCHK(ctx, sgk::launch_guided_mask(l1, n1, l2, n2, *guided, rmask, nullptr, st));
    // s8 forms of both sets: the operands of the i8 MFMA
    ALLOCCHK(ctx, ctx->m_s1.ensure((size_t)n1 * 128));
    ALLOCCHK(ctx, ctx->m_s2.ensure((size_t)n2 * 128));
    const uint8_t* s1 = ctx->m_s1.as<uint8_t>();
    const uint8_t* s2 = ctx->m_s2.as<uint8_t>();
    // ... with the row terms 128 * sum(d1) and, for mutual matching, the column side's terms
    // (two GEMMs: 128 * sum(d2), the row terms of the swapped launch; fused: the column terms
    // 128 * sum(d2) - 2^21, guided: 0) and the matched-column flags cleared
    // [flag n2][count][ntau][pruned count][list n2]
    int* cw = compact ? ctx->m_cols.as<int>() : nullptr;
    int* rmax1 = prune ? ctx->m_prune.as<int>() : nullptr;   // pruning: row maxima of set 1,
    int* map1c = prune ? rmax1 + n1 : nullptr;                // the kept rows' indices,
    int* ct1c = prune ? map1c + n1 : nullptr;                 // their column terms
    HIPCHK(ctx, sgk::launch_prep_set(a, n1, ctx->m_s1.as<uint8_t>(), row1, 128, 0, nullptr, 0, st,
                                     dma && mbm && !fused ? ct1 : nullptr, ct1c));
    if (mbm || dma)
        HIPCHK(ctx, sgk::launch_prep_set(b, n2, ctx->m_s2.as<uint8_t>(), mbm ? col2 : nullptr,
                                         guided && fused ? 0 : 128,
                                         fused && !guided ? -2097152 : 0,
                                         cw, compact ? n2 + 3 : 0, st, dma ? ct2 : nullptr));
    else
        HIPCHK(ctx, sgk::launch_to_s8(b, n2, ctx->m_s2.as<uint8_t>(), st));
    if (mbm && !fused) {
        // The mutual check below reads the column decision match2[j] only for j = match1[i] >=
        // 0, so the column GEMM runs over those columns alone: the row finish appends each
        // matched column once to a list (flags and count zeroed here), and the column launches
        // take their rows from it, their count from the device.  Every listed column still
        // scans all of set 1, so its decision is the reference's (SGPU_DEBUG_FULL_COLUMNS:
        // every column, as ColMatch_Kernel does).  The flags and the count were cleared with
        // the s8 conversion.
        //
        // Pruning (plain mutual matching with ratiomax <= 1): a listed column's decision depends
        // only on rows of set 1 with some dot >= tau, the smallest second value that fails the
        // ratio test against the weakest passing row maximum (k_match_finish).
        // The row finish records every row's maximum and that bound, k_prune_set compacts the
        // rows at or above it, and the column GEMM runs over them (count on the device): the
        // same decisions, the same pairs.
        sgk::ColumnList claim, cols;
        if (compact) {
            claim.flag = cw;
            claim.count = cw + n2;
            claim.list = cw + n2 + 3;
            cols.count = claim.count;
            cols.map = claim.list;
            cols.dma = dma ? 1 : 0;
        }
        if (prune) {
            claim.rmax = rmax1;
            claim.ntau = cw + n2 + 1;
            cols.bmap = map1c;
            cols.bn = cw + n2 + 2;
        }
        HIPCHK(ctx, sgk::launch_match_rows(s1, n1, s2, n2, ca, part, st, nullptr, true, nullptr,
                                           nullptr, raw, nullptr, nullptr, dma ? ct2 : nullptr));
        HIPCHK(ctx, sgk::launch_match_finish(part, n1, ca, row1, ctx->m_dist.as<float>(), distmax,
                                             ratiomax, match1, nullptr, st, true,
                                             raw ? a : nullptr, raw ? b : nullptr, n2, claim));
        if (prune)
            HIPCHK(ctx, sgk::launch_prune_set(rmax1, claim.ntau, n1, s1, ct1,
                                              ctx->m_s1c.as<uint8_t>(), ct1c, map1c,
                                              cw + n2 + 2, st));
        HIPCHK(ctx, sgk::launch_match_rows(s2, n2, prune ? ctx->m_s1c.as<uint8_t>() : s1, n1, cb,
                                           part, st, nullptr, false, nullptr, nullptr, raw,
                                           cols.map, cols.count,
                                           prune ? ct1c : dma ? ct1 : nullptr, cols.bn));
        HIPCHK(ctx, sgk::launch_match_finish(part, n2, cb, col2, ctx->m_dist.as<float>(), distmax,
                                             ratiomax, match2, nullptr, st, false,
                                             raw ? b : nullptr, raw ? a : nullptr, n1, cols));
    } else if (mbm) {
        // one GEMM for both decisions (MultiplyDescriptor_Kernel's row results + column
        // partials, ProgramCU.cu:1466-1564)
        // guided: the column values already hold the column term (col_term 0)
        HIPCHK(ctx, sgk::launch_match_rows(s1, n1, s2, n2, ca, part, st, rmask, true, row1, colpart));
        HIPCHK(ctx, sgk::launch_match_finish(part, n1, ca, row1, ctx->m_dist.as<float>(),
                                             distmax, ratiomax, match1, nullptr, st, true));
        HIPCHK(ctx, sgk::launch_match_cols(colpart, n2, panels, col2, ctx->m_dist.as<float>(),
                                           distmax, ratiomax, match2, nullptr, st));
    } else {
        const bool r1 = raw && !rmask;
        HIPCHK(ctx, sgk::launch_match_rows(s1, n1, s2, n2, ca, part, st, rmask, true, nullptr,
                                           nullptr, r1, nullptr, nullptr,
                                           r1 && dma ? ct2 : nullptr));
        HIPCHK(ctx, sgk::launch_match_finish(part, n1, ca, row1, ctx->m_dist.as<float>(), distmax,
                                             ratiomax, match1, nullptr, st, true,
                                             r1 ? a : nullptr, r1 ? b : nullptr, n2));
    }
    HIPCHK(ctx, hipEventRecord(ctx->ev[2], st));
    ctx->h_match.resize((size_t)n1 + n2);
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_match.data(), match1, (size_t)(mbm ? n1 + n2 : n1) * sizeof(int),
                               hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipStreamSynchronize(st));
    (void)hipEventElapsedTime(&ctx->timing[T_MATCH], ctx->ev[1], ctx->ev[2]);
    // mutual check in ascending i (SiftMatchCU.cpp:166-176)
    const int* bufr = ctx->h_match.data();
    const int* bufc = bufr + n1;
    int nmatch = 0;
    for (int i = 0; i < n1 && nmatch < max_match; ++i) {
        const int j = bufr[i];
        if (j >= 0 && (!mbm || bufc[j] == i)) {
            out_pairs[2 * nmatch] = i;
            out_pairs[2 * nmatch + 1] = j;
            nmatch++;
        }
    }
    return nmatch;
}

int sgpu_match(sgpu_ctx* ctx, const uint8_t* d1, int n1, const uint8_t* d2, int n2,
               float distmax, float ratiomax, int mbm, int max_match, int* out_pairs,
               int flags) {
    return match_impl(ctx, d1, n1, d2, n2, distmax, ratiomax, mbm, max_match, out_pairs, flags,
                      nullptr, nullptr, nullptr);
}

// ---- sharded matcher: rows of set 1 split over ranks, set 2 replicated ----
// The row decision of a set-1 row needs only its own dots, so it stays local.  The column
// decision of a set-2 row j needs the best / second-best over ALL set-1 rows: every rank
// reduces its shard to the clamped running state (max, argmax, second) that
// RowMatch_Kernel / ColMatch_Kernel keep (ProgramCU.cu:1803, 1850: running maxima start at 0
// with index -1), the ranks exchange those n2 x 3 ints, and the merge -- max, the column
// side's tie order (lowest set-1 row first), second = max(min of the maxima, seconds) -- gives
// exactly the single-device state, because clamping at 0 commutes with max.

// float(acos(min(v * 2^-18, 1.0))) -- the expression of RowMatch_Kernel (ProgramCU.cu:1838)
// and of the device distance table
static float match_dist(int v) {
    v = std::min(std::max(v, 0), sgk::kDistTable - 1);
    return (float)std::acos(std::min((double)(v * 0.000003814697265625f), 1.0));
}

int sgpu_match_shard_begin(sgpu_ctx* ctx, const uint8_t* d1, int ns, int row_begin,
                           const uint8_t* d2, int n2, float distmax, float ratiomax, int mbm,
                           int* row_match, int* col_best, int flags) {
    if (!ctx) return SGPU_EINVAL;
    if (ns < 0 || n2 < 0 || row_begin < 0 || (ns > 0 && (!d1 || !row_match)) ||
        (n2 > 0 && !d2) || (mbm && n2 > 0 && !col_best))
        return ctx->fail(SGPU_EINVAL, "bad shard-match arguments");
    if (mbm)   // an empty shard contributes the initial state (0, -1, 0) to every column
        for (int j = 0; j < n2; j++) {
            col_best[3 * j] = 0;
            col_best[3 * j + 1] = -1;
            col_best[3 * j + 2] = 0;
        }
    if (ns == 0 || n2 == 0) {
        for (int i = 0; i < ns; i++) row_match[i] = -1;
        return SGPU_OK;
    }
    HIPCHK(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    if (!ctx->dist_ready) {
        std::vector<float> t(sgk::kDistTable);
        for (int v = 0; v < sgk::kDistTable; v++) t[v] = match_dist(v);
        ALLOCCHK(ctx, ctx->m_dist.ensure(t.size() * sizeof(float)));
        HIPCHK(ctx, hipMemcpy(ctx->m_dist.p, t.data(), t.size() * sizeof(float), hipMemcpyHostToDevice));
        ctx->dist_ready = true;
    }
    const uint8_t* a = d1;
    const uint8_t* b = d2;
    // (no event before the uploads: nothing reads it, and each record costs ~4.5 us of GPU time)
    if (!(flags & SGPU_INPUT_DEVICE)) {
        ALLOCCHK(ctx, ctx->m_d1.ensure((size_t)ns * 128));
        ALLOCCHK(ctx, ctx->m_d2.ensure((size_t)n2 * 128));
        HIPCHK(ctx, hipMemcpyAsync(ctx->m_d1.p, d1, (size_t)ns * 128, hipMemcpyHostToDevice, st));
        HIPCHK(ctx, hipMemcpyAsync(ctx->m_d2.p, d2, (size_t)n2 * 128, hipMemcpyHostToDevice, st));
        a = ctx->m_d1.as<uint8_t>();
        b = ctx->m_d2.as<uint8_t>();
    }
    HIPCHK(ctx, hipEventRecord(ctx->ev[1], st));
    const bool fused = mbm && (ctx->debug_flags & SGPU_DEBUG_FUSED_MATCH);   // see match_impl
    const int ca = sgk::match_chunks(ns, n2), panels = sgk::match_panels(ns);
    const int cb = mbm && !fused ? sgk::match_chunks(n2, ns) : 0;
    const size_t part_n = std::max((size_t)ca * ns, (size_t)cb * n2);
    ALLOCCHK(ctx, ctx->m_part.ensure(part_n * sizeof(sgk::Top2) + (size_t)n2 * sizeof(sgk::Top2)));
    if (fused) ALLOCCHK(ctx, ctx->m_colpart.ensure((size_t)panels * n2 * sizeof(sgk::Top2)));
    ALLOCCHK(ctx, ctx->m_terms.ensure((size_t)2 * (ns + n2) * sizeof(int)));
    ALLOCCHK(ctx, ctx->m_match.ensure((size_t)(ns + n2) * sizeof(int)));
    int* row1 = ctx->m_terms.as<int>();
    int* col2 = row1 + ns;
    int* match1 = ctx->m_match.as<int>();
    int* match2 = match1 + ns;
    sgk::Top2* part = ctx->m_part.as<sgk::Top2>();
    sgk::Top2* best2 = part + part_n;
    sgk::Top2* colpart = fused ? ctx->m_colpart.as<sgk::Top2>() : nullptr;
    const float* dist = ctx->m_dist.as<float>();
    ALLOCCHK(ctx, ctx->m_s1.ensure((size_t)ns * 128));
    ALLOCCHK(ctx, ctx->m_s2.ensure((size_t)n2 * 128));
    const uint8_t* s1 = ctx->m_s1.as<uint8_t>();
    const uint8_t* s2 = ctx->m_s2.as<uint8_t>();
    HIPCHK(ctx, sgk::launch_prep_set(a, ns, ctx->m_s1.as<uint8_t>(), row1, 128, 0, nullptr, 0, st));
    if (mbm && !fused)
        HIPCHK(ctx, sgk::launch_prep_set(b, n2, ctx->m_s2.as<uint8_t>(), col2, 128, 0, nullptr, 0, st));
    else
        HIPCHK(ctx, sgk::launch_to_s8(b, n2, ctx->m_s2.as<uint8_t>(), st));
    // the shard's row decisions through the keyless fold as in match_impl; the column side's
    // per-column (max, row, second) is merged over the ranks, so it needs every column's row
    // index and stays keyed
    const bool raw = !(ratiomax > 1.0f) && !(ctx->debug_flags & SGPU_DEBUG_KEYED_MATCH);
    if (mbm && !fused) {
        HIPCHK(ctx, sgk::launch_match_rows(s1, ns, s2, n2, ca, part, st, nullptr, true, nullptr,
                                           nullptr, raw));
        HIPCHK(ctx, sgk::launch_match_finish(part, ns, ca, row1, dist, distmax, ratiomax, match1,
                                             nullptr, st, true, raw ? a : nullptr,
                                             raw ? b : nullptr, n2));
        HIPCHK(ctx, sgk::launch_match_rows(s2, n2, s1, ns, cb, part, st, nullptr, false));
        HIPCHK(ctx, sgk::launch_match_finish(part, n2, cb, col2, dist, distmax, ratiomax, match2,
                                             best2, st, false));
    } else if (mbm) {
        HIPCHK(ctx, sgk::launch_rowsums(b, n2, col2, 128, -2097152, st));
        HIPCHK(ctx, sgk::launch_match_rows(s1, ns, s2, n2, ca, part, st, nullptr, true, row1, colpart));
        HIPCHK(ctx, sgk::launch_match_finish(part, ns, ca, row1, dist, distmax, ratiomax,
                                             match1, nullptr, st, true));
        HIPCHK(ctx, sgk::launch_match_cols(colpart, n2, panels, col2, dist, distmax, ratiomax,
                                           match2, best2, st));
    } else {
        HIPCHK(ctx, sgk::launch_match_rows(s1, ns, s2, n2, ca, part, st, nullptr, true, nullptr,
                                           nullptr, raw));
        HIPCHK(ctx, sgk::launch_match_finish(part, ns, ca, row1, dist, distmax, ratiomax, match1,
                                             nullptr, st, true, raw ? a : nullptr,
                                             raw ? b : nullptr, n2));
    }
    HIPCHK(ctx, hipEventRecord(ctx->ev[2], st));
    HIPCHK(ctx, hipMemcpyAsync(row_match, match1, (size_t)ns * sizeof(int), hipMemcpyDeviceToHost, st));
    if (mbm) {
        static_assert(sizeof(sgk::Top2) == 3 * sizeof(int), "Top2 = 3 ints");
        HIPCHK(ctx, hipMemcpyAsync(col_best, best2, (size_t)n2 * sizeof(sgk::Top2),
                                   hipMemcpyDeviceToHost, st));
    }
    HIPCHK(ctx, hipStreamSynchronize(st));
    (void)hipEventElapsedTime(&ctx->timing[T_MATCH], ctx->ev[1], ctx->ev[2]);
    if (mbm)   // Top2 is (max, idx, second); the shard's row index becomes the global one
        for (int j = 0; j < n2; j++)
            if (col_best[3 * j + 1] >= 0) col_best[3 * j + 1] += row_begin;
    return SGPU_OK;
}

int sgpu_match_shard_end(const int* col_best_all, int nshards, int n2, const int* row_match,
                         int ns, int row_begin, float distmax, float ratiomax, int mbm,
                         int max_match, int* out_pairs) {
    if (ns < 0 || n2 < 0 || (ns > 0 && !row_match) || (max_match > 0 && !out_pairs) ||
        (mbm && (nshards < 1 || (n2 > 0 && !col_best_all))))
        return SGPU_EINVAL;
    std::vector<int> col_match;
    if (mbm) {
        col_match.assign((size_t)n2, -1);
        for (int j = 0; j < n2; j++) {
            // shards in rank order: rank r's rows precede rank r+1's (lowest row wins ties)
            int m = col_best_all[3 * j], idx = col_best_all[3 * j + 1], sc = col_best_all[3 * j + 2];
            for (int r = 1; r < nshards; r++) {
                const int* u = col_best_all + ((size_t)r * n2 + j) * 3;
                const bool later = u[0] > m || (u[0] == m && u[1] >= 0 && (idx < 0 || u[1] < idx));
                sc = std::max(std::min(m, u[0]), std::max(sc, u[2]));
                if (later) idx = u[1];
                m = std::max(m, u[0]);
            }
            const float d1 = match_dist(m), d2 = match_dist(sc);
            col_match[j] = (d1 < distmax) && (d1 < d2 * ratiomax) ? idx : -1;
        }
    }
    int nmatch = 0;
    for (int i = 0; i < ns && nmatch < max_match; ++i) {
        const int j = row_match[i];
        if (j >= 0 && j < n2 && (!mbm || col_match[j] == row_begin + i)) {
            out_pairs[2 * nmatch] = row_begin + i;
            out_pairs[2 * nmatch + 1] = j;
            nmatch++;
        }
    }
    return nmatch;
}

int sgpu_match_sharded(sgpu_ctx* ctx, const uint8_t* d1, int ns, int row_begin,
                       const uint8_t* d2, int n2, float distmax, float ratiomax, int mbm,
                       int max_match, int* out_pairs, int flags) {
    if (!ctx) return SGPU_EINVAL;
    const int ranks = ctx->comm ? ctx->comm_ranks : 1;
    std::vector<int> rows((size_t)std::max(ns, 1)), mine((size_t)3 * std::max(n2, 1));
    int rc = sgpu_match_shard_begin(ctx, d1, ns, row_begin, d2, n2, distmax, ratiomax, mbm,
                                    rows.data(), mine.data(), flags);
    const bool collective = mbm && ctx->comm && n2 > 0;
    if (collective) {
        // every rank learns whether any rank failed locally before the data collective, so a
        // local failure never leaves the peers waiting inside ncclAllGather
        double failed = rc != SGPU_OK ? 1.0 : 0.0;
        const int rs = sgpu_comm_allreduce_f64(ctx, &failed, 1, 1);
        if (rs != SGPU_OK) return rs;
        if (failed != 0.0)
            return rc != SGPU_OK ? rc : ctx->fail(SGPU_ENODEV, "sgpu_match_sharded: a peer rank failed");
    } else if (rc != SGPU_OK) {
        return rc;
    }
    std::vector<int> all;
    if (collective) {   // RCCL all-gather of the n2 x 3 column states
        all.resize((size_t)3 * n2 * ranks);
        rc = sgpu_comm_allgather_i32(ctx, mine.data(), 3 * n2, all.data());
        if (rc != SGPU_OK) return rc;
    } else {
        all = mine;
    }
    return sgpu_match_shard_end(all.data(), ranks, n2, rows.data(), ns, row_begin, distmax,
                                ratiomax, mbm, max_match, out_pairs);
}

// SiftMatchGPU::GetGuidedSiftMatch (SiftMatch.cpp:663-677 defaults, SiftMatchCU.cpp:126-136).
int sgpu_match_guided(sgpu_ctx* ctx, const uint8_t* d1, int n1, const uint8_t* d2, int n2,
                      const float* loc1, const float* loc2, const float* H, const float* F,
                      float distmax, float ratiomax, float hdistmax, float fdistmax, int mbm,
                      int max_match, int* out_pairs, int flags) {
    if (!ctx) return SGPU_EINVAL;
    if (!H && !F)
        return match_impl(ctx, d1, n1, d2, n2, distmax, ratiomax, mbm, max_match, out_pairs,
                          flags, nullptr, nullptr, nullptr);
    // a missing matrix is the identity with its threshold at 1e20 (SiftMatch.cpp:667-675)
    static const float kIdentity[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    sgk::GuidedParams gp;
    memcpy(gp.H, H ? H : kIdentity, sizeof(gp.H));
    memcpy(gp.F, F ? F : kIdentity, sizeof(gp.F));
    gp.hdistmax = H ? hdistmax : 1.0e+20f;
    gp.fdistmax = F ? fdistmax : 1.0e+20f;
    return match_impl(ctx, d1, n1, d2, n2, distmax, ratiomax, mbm, max_match, out_pairs, flags,
                      loc1, loc2, &gp);
}

// ---- multi-GPU: one process per GPU, RCCL over xGMI ----
int sgpu_comm_unique_id(uint8_t* id, int bytes) {
    if (!id || bytes < (int)sizeof(ncclUniqueId)) return SGPU_EINVAL;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return SGPU_ENODEV;
    memcpy(id, &u, sizeof(u));
    return SGPU_OK;
}

int sgpu_comm_init(sgpu_ctx* ctx, int nranks, int rank, const uint8_t* id, int bytes) {
    if (!ctx || !id || nranks < 1 || rank < 0 || rank >= nranks || bytes < (int)sizeof(ncclUniqueId))
        return SGPU_EINVAL;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    if (ctx->comm) (void)ncclCommDestroy(ctx->comm);
    ctx->comm = nullptr;
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    const ncclResult_t r = ncclCommInitRank(&ctx->comm, nranks, u, rank);
    if (r != ncclSuccess) {
        ctx->comm = nullptr;
        return ctx->fail(SGPU_ENODEV, ncclGetErrorString(r));
    }
    ctx->comm_ranks = nranks;
    ctx->comm_rank = rank;
    return SGPU_OK;
}

int sgpu_comm_allgather_i32(sgpu_ctx* ctx, const int32_t* send, int n, int32_t* recv) {
    if (!ctx || !ctx->comm || n < 0 || (n && (!send || !recv))) return SGPU_EINVAL;
    if (n == 0) return SGPU_OK;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    const size_t total = (size_t)n * ctx->comm_ranks;
    ALLOCCHK(ctx, ctx->c_buf.ensure((total + n) * sizeof(int32_t)));
    int32_t* dsend = ctx->c_buf.as<int32_t>() + total;
    HIPCHK(ctx, hipMemcpyAsync(dsend, send, n * sizeof(int32_t), hipMemcpyHostToDevice, ctx->stream));
    const ncclResult_t r = ncclAllGather(dsend, ctx->c_buf.p, (size_t)n, ncclInt32, ctx->comm, ctx->stream);
    if (r != ncclSuccess) return ctx->fail(SGPU_ENODEV, ncclGetErrorString(r));
    HIPCHK(ctx, hipMemcpyAsync(recv, ctx->c_buf.p, total * sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    return SGPU_OK;
}

int sgpu_comm_allreduce_f64(sgpu_ctx* ctx, double* v, int n, int op_max) {
    if (!ctx || !ctx->comm || !v || n <= 0) return SGPU_EINVAL;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    ALLOCCHK(ctx, ctx->c_buf.ensure((size_t)n * sizeof(double)));
    HIPCHK(ctx, hipMemcpyAsync(ctx->c_buf.p, v, n * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    const ncclResult_t r = ncclAllReduce(ctx->c_buf.p, ctx->c_buf.p, (size_t)n, ncclFloat64,
                                         op_max ? ncclMax : ncclSum, ctx->comm, ctx->stream);
    if (r != ncclSuccess) return ctx->fail(SGPU_ENODEV, ncclGetErrorString(r));
    HIPCHK(ctx, hipMemcpyAsync(v, ctx->c_buf.p, n * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    return SGPU_OK;
}

int sgpu_stage_input(sgpu_ctx* ctx, const uint8_t* images, int n, int w, int h, int stride) {
    if (!ctx || !images || n <= 0 || stride < w) return SGPU_EINVAL;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    const size_t bytes = (size_t)n * h * stride;
    ALLOCCHK(ctx, ctx->input.ensure(bytes));
    HIPCHK(ctx, hipMemcpy(ctx->input.p, images, bytes, hipMemcpyHostToDevice));
    ctx->staged_bytes = bytes;
    return SGPU_OK;
}

// SiftGPU::AllocatePyramid (SiftGPU.cpp:1435-1460: PyramidCU::ResizePyramid for the first
// octave of a width x height input): every device and pinned buffer an extract of n images of
// w x h u8 pixels (rows `stride` bytes apart) needs -- the staged input, the pyramid, the mask,
// the row and candidate arrays at their first-guess capacity -- allocated now, so that the next
// sgpu_stage_input + sgpu_extract of that geometry allocates nothing (unless its keypoints
// exceed the first-guess capacity).  Like an extract it replaces the batch: the previous
// results are gone.
int sgpu_reserve(sgpu_ctx* ctx, int n, int w, int h, int stride) {
    if (!ctx) return SGPU_EINVAL;
    if (n <= 0 || w < 8 || h < 8 || stride < w) return ctx->fail(SGPU_EINVAL, "bad reserve arguments");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    int rc = abandon_batch(ctx, SGPU_OK);   // nothing queued may still use the buffers
    ctx->staged_bytes = 0;                  // the input buffer may be reallocated
    if (rc == SGPU_OK) rc = plan_batch(ctx, n, w, h);
    if (rc == SGPU_OK && part_streams(ctx->part[0]) != SGPU_OK)
        rc = ctx->fail(SGPU_ENODEV, "stream creation failed");
    if (rc == SGPU_OK) {
        ctx->nparts = 1;
        Part& pt = ctx->part[0];
        pt.img0 = 0;
        pt.n = n;
        rc = layout_part(ctx, pt);
    }
    if (rc == SGPU_OK && ctx->input.ensure((size_t)n * h * stride) != hipSuccess)
        rc = ctx->fail(SGPU_ENOMEM, "device allocation failed");
    return abandon_batch(ctx, rc);
}

long long sgpu_debug_alloc_count(void) { return g_allocs.load(); }

int sgpu_set_host_output(sgpu_ctx* ctx, float* keys, float* descriptors, int capacity) {
    if (!ctx || capacity < 0) return SGPU_EINVAL;
    ctx->host_out.keys = keys;
    ctx->host_out.desc = descriptors;
    ctx->host_out.cap = capacity;
    ctx->host_out.armed = keys != nullptr && capacity > 0;
    ctx->host_out.done = false;
    return SGPU_OK;
}

int sgpu_set_stage_timing(sgpu_ctx* ctx, int on) {
    if (!ctx) return SGPU_EINVAL;
    ctx->stage_timing = on != 0;
    return SGPU_OK;
}

int sgpu_last_pyramid_launches(const sgpu_ctx* ctx, int* filters) {
    if (!ctx || ctx->batch <= 0) return SGPU_EINVAL;
    if (filters) *filters = ctx->part[0].gauss_filters;
    return ctx->part[0].gauss_launches;
}

int sgpu_extract(sgpu_ctx* ctx, const uint8_t* images, int n, int w, int h, int stride,
                 int flags) {
    return extract_impl(ctx, images, false, n, w, h, stride, flags);
}

int sgpu_extract_f32(sgpu_ctx* ctx, const float* images, int n, int w, int h, int stride,
                     int flags) {
    return extract_impl(ctx, images, true, n, w, h, stride, flags);
}

int sgpu_extract_color(sgpu_ctx* ctx, const uint8_t* images, int n, int w, int h, int stride,
                       int format, int flags) {
    if (!ctx) return SGPU_EINVAL;
    if (format < SGPU_RGB || format > SGPU_BGRA) return ctx->fail(SGPU_EINVAL, "bad color format");
    return extract_impl(ctx, images, false, n, w, h, stride, flags, format);
}

int sgpu_feature_count(const sgpu_ctx* ctx, int image) {
    if (!ctx || image < 0 || image >= ctx->batch || ctx->img_off.empty()) return 0;
    return (int)(ctx->img_off[image + 1] - ctx->img_off[image]);
}

int64_t sgpu_feature_total(const sgpu_ctx* ctx) {
    if (!ctx || ctx->img_off.empty()) return 0;
    return ctx->img_off[ctx->batch];
}

int sgpu_copy_features(sgpu_ctx* ctx, int image, float* keys, float* descriptors) {
    if (!ctx || image < 0 || image >= ctx->batch || ctx->img_off.empty()) return SGPU_EINVAL;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    const Part& pt = ctx->part[ctx->part_of(image)];
    const int li = image - pt.img0;
    const int64_t a = pt.img_off[li], nf = pt.img_off[li + 1] - a;
    if (nf <= 0) {   // nothing copied: the copy slots read 0, not the previous call's times
        ctx->timing[T_COPY_KEYS] = 0.f;
        ctx->timing[T_COPY_DESC] = 0.f;
        return SGPU_OK;
    }
    if (descriptors && !ctx->opt.descriptors) return ctx->fail(SGPU_EINVAL, "descriptors disabled (-sd)");
    const auto& ho = ctx->host_out;
    if (ho.done && image == 0 && a == 0 && keys == ho.keys && (!descriptors || descriptors == ho.desc) &&
        nf <= ho.cap) {
        // the extract already wrote them there (sgpu_set_host_output)
        ctx->timing[T_COPY_KEYS] = ctx->timing[T_COPY_DESC] = 0.f;
        return SGPU_OK;
    }
    // both copies, then one synchronisation; events split the time between them
    // (sgpu_last_timing slots 10, 11) when the context times its stages
    const bool tm = ctx->stage_timing;
    if (tm) HIPCHK(ctx, hipEventRecord(ctx->ev[T_COPY_KEYS], ctx->stream));
    if (keys)
        HIPCHK(ctx, hipMemcpyAsync(keys, pt.keys.as<float4>() + a, nf * sizeof(float4),
                                   hipMemcpyDeviceToHost, ctx->stream));
    if (tm) HIPCHK(ctx, hipEventRecord(ctx->ev[T_COPY_DESC], ctx->stream));
    if (descriptors)
        HIPCHK(ctx, hipMemcpyAsync(descriptors, pt.desc.as<float>() + a * 128,
                                   nf * 128 * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
    if (tm) HIPCHK(ctx, hipEventRecord(ctx->ev[T_N], ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    ctx->timing[T_COPY_KEYS] = ctx->timing[T_COPY_DESC] = 0.f;
    if (tm) {
        (void)hipEventElapsedTime(&ctx->timing[T_COPY_KEYS], ctx->ev[T_COPY_KEYS], ctx->ev[T_COPY_DESC]);
        (void)hipEventElapsedTime(&ctx->timing[T_COPY_DESC], ctx->ev[T_COPY_DESC], ctx->ev[T_N]);
    }
    return SGPU_OK;
}

int sgpu_device_features(sgpu_ctx* ctx, const float** keys, const float** descriptors,
                         const int64_t** image_offsets) {
    if (!ctx) return SGPU_EINVAL;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    const float* k = nullptr;
    const float* dsc = nullptr;
    if (ctx->nparts == 1) {
        k = ctx->part[0].keys.as<float>();
        dsc = ctx->part[0].desc.as<float>();
    } else if (ctx->nparts > 1) {
        // one contiguous copy of the batch's features, gathered on first request
        const int64_t total = ctx->img_off.empty() ? 0 : ctx->img_off[ctx->batch];
        if (!ctx->gathered) {
            ALLOCCHK(ctx, ctx->all_keys.ensure((size_t)std::max<int64_t>(total, 1) * sizeof(float4)));
            if (ctx->opt.descriptors)
                ALLOCCHK(ctx, ctx->all_desc.ensure((size_t)std::max<int64_t>(total, 1) * 128 * sizeof(float)));
            for (int p = 0; p < ctx->nparts; p++) {
                const Part& pt = ctx->part[p];
                const int64_t base = ctx->img_off[pt.img0], nf = pt.img_off[pt.n];
                if (nf <= 0) continue;
                HIPCHK(ctx, hipMemcpyAsync(ctx->all_keys.as<float4>() + base, pt.keys.p,
                                           nf * sizeof(float4), hipMemcpyDeviceToDevice, ctx->stream));
                if (ctx->opt.descriptors)
                    HIPCHK(ctx, hipMemcpyAsync(ctx->all_desc.as<float>() + base * 128, pt.desc.p,
                                               nf * 128 * sizeof(float), hipMemcpyDeviceToDevice,
                                               ctx->stream));
            }
            HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
            ctx->gathered = true;
        }
        k = ctx->all_keys.as<float>();
        dsc = ctx->all_desc.as<float>();
    }
    if (keys) *keys = k;
    if (descriptors) *descriptors = ctx->opt.descriptors ? dsc : nullptr;
    if (image_offsets) *image_offsets = ctx->img_off.data();
    return SGPU_OK;
}

void sgpu_quantize_descriptors(const float* d, size_t count, uint8_t* out) {
    for (size_t i = 0; i < count; ++i) out[i] = (uint8_t)(int)(512 * d[i] + 0.5);
}

int sgpu_last_timing(const sgpu_ctx* ctx, float* times, int n) {
    if (!ctx || !times) return SGPU_EINVAL;
    for (int i = 0; i < n && i < T_N; i++) times[i] = ctx->timing[i];
    return SGPU_OK;
}

int sgpu_debug_set_flags(sgpu_ctx* ctx, int flags) {
    if (!ctx) return SGPU_EINVAL;
    ctx->debug_flags = flags | ctx->env_flags;
    return SGPU_OK;
}

int sgpu_debug_set_match_prune(sgpu_ctx* ctx, int on) {
    if (!ctx) return SGPU_EINVAL;
    ctx->match_prune = on != 0;
    return SGPU_OK;
}

int sgpu_debug_set_schedule(sgpu_ctx* ctx, int trio, int pairs) {
    if (!ctx || trio < SGPU_TRIO_OFF || trio > SGPU_TRIO_ALWAYS || pairs < SGPU_PAIRS_FRONT ||
        pairs > SGPU_PAIRS_END)
        return SGPU_EINVAL;
    ctx->trio_mode = trio;
    ctx->duo_plan = pairs;
    return SGPU_OK;
}

int sgpu_debug_geometry(const sgpu_ctx* ctx, int* n_octaves, int* dims, int max) {
    if (!ctx || !n_octaves) return SGPU_EINVAL;
    *n_octaves = (int)ctx->oct.size();
    for (int o = 0; o < (int)ctx->oct.size() && o < max; o++) {
        dims[3 * o] = ctx->oct[o].w;
        dims[3 * o + 1] = ctx->oct[o].h;
        dims[3 * o + 2] = ctx->oct[o].wa;
    }
    return SGPU_OK;
}

int sgpu_debug_gaussian(sgpu_ctx* ctx, int image, int octave, int level, float* out) {
    if (!ctx || image < 0 || image >= ctx->batch || octave < 0 ||
        octave >= (int)ctx->oct.size() || level < 0 || level >= ctx->sched.level_num)
        return SGPU_EINVAL;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    const Part& pt = ctx->part[ctx->part_of(image)];
    const sgk::OctaveDesc& od = pt.fp.oct[octave];
    const long long npx = (long long)od.wa * od.h;
    const float* src = pt.pyr.as<float>() + od.gauss_off + level * od.level_stride +
                       (image - pt.img0) * npx;
    HIPCHK(ctx, hipMemcpy(out, src, npx * sizeof(float), hipMemcpyDeviceToHost));
    return SGPU_OK;
}

// The test-hook library beside this one (lib/libsiftgpu_debug.so, csrc/sgpu_debug.hip), loaded on
// first use: the candidate dump's kernel is not part of the product library.
static sgk::DebugCandidatesFn debug_candidates_hook() {
    static sgk::DebugCandidatesFn fn = [] {
        Dl_info info{};
        if (!dladdr(reinterpret_cast<void*>(&sgpu_debug_candidates), &info) || !info.dli_fname)
            return (sgk::DebugCandidatesFn) nullptr;
        std::string path(info.dli_fname);
        const size_t slash = path.rfind('/');
        path = (slash == std::string::npos ? std::string(".") : path.substr(0, slash)) +
               "/libsiftgpu_debug.so";
        void* h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
        return h ? reinterpret_cast<sgk::DebugCandidatesFn>(dlsym(h, "sgpu_testhook_candidates"))
                 : (sgk::DebugCandidatesFn) nullptr;
    }();
    return fn;
}

int sgpu_debug_candidates(sgpu_ctx* ctx, int* ints, float* floats, int cap, int* n) {
    if (!ctx || !n) return SGPU_EINVAL;
    uint32_t total = 0;
    for (int p = 0; p < ctx->nparts; p++) total += ctx->part[p].n_cand;
    *n = (int)total;
    if (!ints || !floats || cap < (int)total) return total ? SGPU_ERANGE : SGPU_OK;
    if (total == 0) return SGPU_OK;
    const sgk::DebugCandidatesFn hook = debug_candidates_hook();
    if (!hook) return ctx->fail(SGPU_EINVAL, "test-hook library lib/libsiftgpu_debug.so not found");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    DevBuf a, b;
    ALLOCCHK(ctx, a.ensure(total * sizeof(int4)));
    ALLOCCHK(ctx, b.ensure(total * sizeof(float4)));
    uint32_t at = 0;
    for (int p = 0; p < ctx->nparts; p++) {
        const Part& pt = ctx->part[p];
        if (!pt.n_cand) continue;
        HIPCHK(ctx, hook(pt.pyr.as<float>(), pt.mask.as<uint32_t>(), pt.row_base.as<uint32_t>(),
                         pt.total_rows, pt.row_base.as<uint32_t>() + pt.total_rows,
                         (int)pt.n_cand, &pt.fp, a.as<int4>() + at, b.as<float4>() + at,
                         ctx->stream));
        at += pt.n_cand;
    }
    HIPCHK(ctx, hipMemcpyAsync(ints, a.p, total * sizeof(int4), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(floats, b.p, total * sizeof(float4), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    // the kernel reports part-local image indices
    at = 0;
    for (int p = 0; p < ctx->nparts; p++) {
        const Part& pt = ctx->part[p];
        for (uint32_t i = 0; i < pt.n_cand; i++) ints[4 * (at + i) + 3] += pt.img0;
        at += pt.n_cand;
    }
    a.release();
    b.release();
    return SGPU_OK;
}

}  // extern "C"
