// sgpu_capi.cpp -- the C ABI (include/sgpu.h) over the gfx950 kernels.
//
// Host orchestration of one batch (replaces SiftPyramid::RunSIFT, SiftPyramid.cpp:58-216, and
// the PyramidCU stage methods).  Per batch the host syncs twice: once to size the keypoint
// arrays after the row scan, once at the end to read the per-image offsets.  Everything else
// is queued on one HIP stream; no per-level host round trips (the reference does four per
// DoG level, PyramidCU.cpp:783-813).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/sgpu.h"
#include "sift_kernels.h"
#include "sift_params.h"

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    hipError_t ensure(size_t n) {
        if (n <= bytes) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        n = std::max<size_t>(n, 256);
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

enum { T_UPLOAD, T_PYRAMID, T_DETECT, T_ORIENT, T_EXPAND, T_DESC, T_DOWNLOAD, T_TOTAL, T_MATCH, T_N };

}  // namespace

struct sgpu_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    sgpu_options opt{};
    sgp::Schedule sched{};
    std::string err;
    // last extract
    int batch = 0, w = 0, h = 0;
    std::vector<sgp::Octave> oct;
    sgk::FeatureParams fp{};
    int total_rows = 0;
    uint32_t n_cand = 0;
    size_t staged_bytes = 0;
    std::vector<int64_t> img_off;
    DevBuf input, pyr, mask, row_count, row_base, scan_tmp, cand, info, ocount, eoff, feat,
        feat_info, keys, desc, img_off_dev, n_dev;
    hipEvent_t ev[T_N + 1] = {};
    float timing[T_N] = {};
    // matcher
    DevBuf m_d1, m_d2, m_part, m_terms, m_match, m_dist;
    std::vector<int> h_match;
    bool dist_ready = false;

    int fail(int code, const char* what, hipError_t e = hipSuccess) {
        err = what;
        if (e != hipSuccess) {
            err += ": ";
            err += hipGetErrorString(e);
        }
        return code;
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
        else if (!param) continue;
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
    if (o.octave_min != 0) return ctx->fail(SGPU_EINVAL, "only first octave 0 (-fo 0) is implemented");
    if (o.dog_level_num < 1 || o.dog_level_num > 6) return ctx->fail(SGPU_EINVAL, "dog_level_num must be 1..6");
    ctx->opt = o;
    sgp::Options po;
    po.filter_width_factor = o.filter_width_factor;
    po.dog_level_num = o.dog_level_num;
    po.dog_threshold = o.dog_threshold;
    po.edge_threshold = o.edge_threshold;
    ctx->sched = sgp::make_schedule(po);
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
    DevBuf* bufs[] = {&ctx->input, &ctx->pyr, &ctx->mask, &ctx->row_count, &ctx->row_base,
                      &ctx->scan_tmp, &ctx->cand, &ctx->info, &ctx->ocount, &ctx->eoff,
                      &ctx->feat, &ctx->feat_info, &ctx->keys, &ctx->desc, &ctx->img_off_dev,
                      &ctx->n_dev, &ctx->m_d1, &ctx->m_d2, &ctx->m_part, &ctx->m_terms,
                      &ctx->m_match, &ctx->m_dist};
    for (DevBuf* b : bufs) b->release();
    for (int i = 0; i <= T_N; i++)
        if (ctx->ev[i]) (void)hipEventDestroy(ctx->ev[i]);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return SGPU_OK;
}

const char* sgpu_last_error(const sgpu_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

static int extract_impl(sgpu_ctx* ctx, const void* images, bool is_f32, int n, int w, int h,
                        int stride, int flags) {
    if (!ctx) return SGPU_EINVAL;
    const bool staged = (flags & SGPU_INPUT_STAGED) != 0;
    if ((!images && !staged) || n <= 0 || w < 8 || h < 8 || stride < w)
        return ctx->fail(SGPU_EINVAL, "bad image arguments");
    if (staged && (is_f32 || ctx->staged_bytes < (size_t)n * h * stride))
        return ctx->fail(SGPU_EINVAL, "staged input does not match the batch");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const sgpu_options& O = ctx->opt;
    const sgp::Schedule& S = ctx->sched;
    const int d = S.dog_level_num, nlev = S.level_num;

    ctx->oct = sgp::make_octaves(w, h, O.octave_num, 0);
    const int noct = (int)ctx->oct.size();
    if (noct > sgk::kMaxOctaves) return ctx->fail(SGPU_EINVAL, "too many octaves");
    for (const auto& oc : ctx->oct)
        if (oc.w < 4 || oc.h < 4) return ctx->fail(SGPU_EINVAL, "image too small for the octave count");
    ctx->batch = n;
    ctx->w = w;
    ctx->h = h;

    // ---- layout: pyramid [octave][level][image][h][wa]; mask [octave][dog level][image][h][words]
    sgk::FeatureParams& fp = ctx->fp;
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
    ctx->total_rows = rows * n;
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
    fp.origin_offset = O.lowe_origin ? 0.0f : 0.5f;

    const size_t in_bytes = (size_t)n * h * stride * (is_f32 ? sizeof(float) : 1);
    ALLOCCHK(ctx, ctx->pyr.ensure((size_t)goff * sizeof(float)));
    ALLOCCHK(ctx, ctx->mask.ensure((size_t)moff * sizeof(uint32_t)));
    ALLOCCHK(ctx, ctx->row_count.ensure((size_t)ctx->total_rows * sizeof(uint32_t)));
    ALLOCCHK(ctx, ctx->row_base.ensure(((size_t)ctx->total_rows + 1) * sizeof(uint32_t)));
    ALLOCCHK(ctx, ctx->img_off_dev.ensure((size_t)(n + 1) * sizeof(int64_t)));
    ALLOCCHK(ctx, ctx->n_dev.ensure(16));

    HIPCHK(ctx, hipEventRecord(ctx->ev[0], st));
    const void* src_in = staged ? ctx->input.p : images;
    if (!(flags & (SGPU_INPUT_DEVICE | SGPU_INPUT_STAGED))) {
        ctx->staged_bytes = 0;
        ALLOCCHK(ctx, ctx->input.ensure(in_bytes));
        HIPCHK(ctx, hipMemcpyAsync(ctx->input.p, images, in_bytes, hipMemcpyHostToDevice, st));
        src_in = ctx->input.p;
    }
    const uint8_t* src8 = is_f32 ? nullptr : (const uint8_t*)src_in;
    const float* srcf = is_f32 ? (const float*)src_in : nullptr;
    HIPCHK(ctx, hipEventRecord(ctx->ev[1], st));

    // ---- Gaussian pyramid (BuildPyramid, PyramidCU.cpp:979-1044)
    float* pyr = ctx->pyr.as<float>();
    sgk::Taps taps;
    for (int o = 0; o < noct; o++) {
        const sgk::OctaveDesc& od = fp.oct[o];
        const long long npx = (long long)od.wa * od.h;
        float* lvl0 = pyr + od.gauss_off;
        if (o == 0) {
            int fw = sgp::make_filter(S.initial_smooth, O.filter_width_factor, taps.k);
            HIPCHK(ctx, sgk::launch_gauss(srcf, src8, stride, (long long)stride * h, lvl0, npx,
                                          od.wa, od.h, fw, taps, n, nullptr, 0, 0, 0, st));
        }
        for (int k = 1; k < nlev; k++) {
            int fw = sgp::make_filter(S.sigma[k - 1], O.filter_width_factor, taps.k);
            float* ds = nullptr;
            int dsw = 0, dsh = 0;
            long long ds_stride = 0;
            // level_ds - level_min (= d) feeds the next octave (PyramidCU.cpp:1024)
            if (k == S.level_ds - S.level_min && o + 1 < noct) {
                const sgk::OctaveDesc& nd = fp.oct[o + 1];
                ds = pyr + nd.gauss_off;
                dsw = nd.wa;
                dsh = nd.h;
                ds_stride = (long long)nd.wa * nd.h;
            }
            HIPCHK(ctx, sgk::launch_gauss(lvl0 + (k - 1) * od.level_stride, nullptr, od.wa, npx,
                                          lvl0 + k * od.level_stride, npx, od.wa, od.h, fw, taps,
                                          n, ds, dsw, dsh, ds_stride, st));
        }
    }
    HIPCHK(ctx, hipEventRecord(ctx->ev[2], st));

    // ---- extrema + row scan
    HIPCHK(ctx, hipMemsetAsync(ctx->row_count.p, 0, (size_t)ctx->total_rows * 4, st));
    // the strip extremum kernel only sets the bits of accepted pixels
    HIPCHK(ctx, hipMemsetAsync(ctx->mask.p, 0, (size_t)moff * sizeof(uint32_t), st));
    for (int o = 0; o < noct; o++)
        HIPCHK(ctx, sgk::launch_extrema(pyr, ctx->mask.as<uint32_t>(), ctx->row_count.as<uint32_t>(),
                                        fp, o, st));
    ALLOCCHK(ctx, ctx->scan_tmp.ensure((sgk::scan_tmp_words(ctx->total_rows) + 16) * 4));
    HIPCHK(ctx, sgk::launch_scan(ctx->row_count.as<uint32_t>(), ctx->row_base.as<uint32_t>(),
                                 ctx->total_rows, ctx->scan_tmp.as<uint32_t>(), st));
    uint32_t ncand = 0;
    HIPCHK(ctx, hipMemcpyAsync(&ncand, ctx->row_base.as<uint32_t>() + ctx->total_rows, 4,
                               hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipEventRecord(ctx->ev[3], st));
    HIPCHK(ctx, hipStreamSynchronize(st));
    ctx->n_cand = ncand;

    // ---- orientation (+ keypoint refinement), expansion, descriptors
    const size_t nc = std::max<uint32_t>(ncand, 1);
    ALLOCCHK(ctx, ctx->cand.ensure(nc * sizeof(float4)));
    ALLOCCHK(ctx, ctx->info.ensure(nc * sizeof(int2)));
    ALLOCCHK(ctx, ctx->ocount.ensure(nc * sizeof(uint32_t)));
    ALLOCCHK(ctx, ctx->eoff.ensure((nc + 1) * sizeof(uint32_t)));
    const size_t ne_cap = 2 * nc;
    ALLOCCHK(ctx, ctx->feat.ensure(ne_cap * sizeof(float4)));
    ALLOCCHK(ctx, ctx->feat_info.ensure(ne_cap * sizeof(int2)));
    ALLOCCHK(ctx, ctx->keys.ensure(ne_cap * sizeof(float4)));
    if (O.descriptors) ALLOCCHK(ctx, ctx->desc.ensure(ne_cap * 128 * sizeof(float)));
    ALLOCCHK(ctx, ctx->scan_tmp.ensure((sgk::scan_tmp_words(nc) + 16) * 4));
    const uint32_t* n_cand_dev = ctx->row_base.as<uint32_t>() + ctx->total_rows;
    HIPCHK(ctx, sgk::launch_orientation(pyr, ctx->mask.as<uint32_t>(), ctx->row_base.as<uint32_t>(),
                                        ctx->total_rows, n_cand_dev, (int)ncand, fp,
                                        ctx->cand.as<float4>(), ctx->info.as<int2>(),
                                        ctx->ocount.as<uint32_t>(), st));
    HIPCHK(ctx, hipEventRecord(ctx->ev[4], st));
    HIPCHK(ctx, sgk::launch_scan(ctx->ocount.as<uint32_t>(), ctx->eoff.as<uint32_t>(), ncand,
                                 ctx->scan_tmp.as<uint32_t>(), st));
    const uint32_t* n_feat_dev = ctx->eoff.as<uint32_t>() + ncand;
    HIPCHK(ctx, sgk::launch_expand(ctx->cand.as<float4>(), ctx->info.as<int2>(),
                                   ctx->eoff.as<uint32_t>(), n_cand_dev, (int)ncand, fp,
                                   ctx->feat.as<float4>(), ctx->feat_info.as<int2>(),
                                   ctx->keys.as<float4>(), st));
    HIPCHK(ctx, hipEventRecord(ctx->ev[5], st));
    if (O.descriptors)
        HIPCHK(ctx, sgk::launch_descriptor(pyr, ctx->feat.as<float4>(), ctx->feat_info.as<int2>(),
                                           n_feat_dev, (int)(2 * ncand), fp, ctx->desc.as<float>(),
                                           st));
    HIPCHK(ctx, hipEventRecord(ctx->ev[6], st));
    HIPCHK(ctx, sgk::launch_image_offsets(ctx->row_base.as<uint32_t>(), ctx->eoff.as<uint32_t>(), n,
                                          fp.rows_per_image, ctx->total_rows,
                                          ctx->img_off_dev.as<int64_t>(), st));
    ctx->img_off.assign(n + 1, 0);
    HIPCHK(ctx, hipMemcpyAsync(ctx->img_off.data(), ctx->img_off_dev.p, (n + 1) * sizeof(int64_t),
                               hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipEventRecord(ctx->ev[7], st));
    HIPCHK(ctx, hipStreamSynchronize(st));
    const int map[T_TOTAL + 1][2] = {{0, 1}, {1, 2}, {2, 3}, {3, 4}, {4, 5}, {5, 6}, {6, 7}, {0, 7}};
    for (int i = 0; i <= T_TOTAL; i++)
        (void)hipEventElapsedTime(&ctx->timing[i], ctx->ev[map[i][0]], ctx->ev[map[i][1]]);
    return SGPU_OK;
}

// SiftMatchGPU::SetDescriptors + GetSiftMatch (SiftMatchCU.cpp:71-179) in one call.
int sgpu_match(sgpu_ctx* ctx, const uint8_t* d1, int n1, const uint8_t* d2, int n2,
               float distmax, float ratiomax, int mbm, int max_match, int* out_pairs,
               int flags) {
    if (!ctx) return SGPU_EINVAL;
    if (n1 <= 0 || n2 <= 0) return 0;   // SiftMatchCU.cpp:142
    if (!d1 || !d2 || (max_match > 0 && !out_pairs)) return ctx->fail(SGPU_EINVAL, "bad match arguments");
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
    HIPCHK(ctx, hipEventRecord(ctx->ev[0], st));
    if (!(flags & SGPU_INPUT_DEVICE)) {
        ALLOCCHK(ctx, ctx->m_d1.ensure((size_t)n1 * 128));
        ALLOCCHK(ctx, ctx->m_d2.ensure((size_t)n2 * 128));
        HIPCHK(ctx, hipMemcpyAsync(ctx->m_d1.p, d1, (size_t)n1 * 128, hipMemcpyHostToDevice, st));
        HIPCHK(ctx, hipMemcpyAsync(ctx->m_d2.p, d2, (size_t)n2 * 128, hipMemcpyHostToDevice, st));
        a = ctx->m_d1.as<uint8_t>();
        b = ctx->m_d2.as<uint8_t>();
    }
    HIPCHK(ctx, hipEventRecord(ctx->ev[1], st));
    const int ca = sgk::match_chunks(n1, n2), cb = mbm ? sgk::match_chunks(n2, n1) : 0;
    const size_t part_n = std::max((size_t)ca * n1, (size_t)cb * n2);
    ALLOCCHK(ctx, ctx->m_part.ensure(part_n * sizeof(sgk::Top2)));
    ALLOCCHK(ctx, ctx->m_terms.ensure((size_t)2 * (n1 + n2) * sizeof(int)));
    ALLOCCHK(ctx, ctx->m_match.ensure((size_t)(n1 + n2) * sizeof(int)));
    int* row1 = ctx->m_terms.as<int>();          // 128 * sum(d1)
    int* col1 = row1 + n1;                       // 128 * sum(d1) - 2^21
    int* row2 = col1 + n1;
    int* col2 = row2 + n2;
    int* match1 = ctx->m_match.as<int>();
    int* match2 = match1 + n1;
    sgk::Top2* part = ctx->m_part.as<sgk::Top2>();
    HIPCHK(ctx, sgk::launch_rowsums(a, n1, row1, 128, 0, st));
    HIPCHK(ctx, sgk::launch_rowsums(b, n2, col2, 128, -2097152, st));
    HIPCHK(ctx, sgk::launch_match_rows(a, n1, b, n2, col2, ca, part, st));
    HIPCHK(ctx, sgk::launch_match_finish(part, n1, ca, row1, ctx->m_dist.as<float>(), distmax,
                                         ratiomax, match1, nullptr, st));
    if (mbm) {
        HIPCHK(ctx, sgk::launch_rowsums(b, n2, row2, 128, 0, st));
        HIPCHK(ctx, sgk::launch_rowsums(a, n1, col1, 128, -2097152, st));
        HIPCHK(ctx, sgk::launch_match_rows(b, n2, a, n1, col1, cb, part, st));
        HIPCHK(ctx, sgk::launch_match_finish(part, n2, cb, row2, ctx->m_dist.as<float>(), distmax,
                                             ratiomax, match2, nullptr, st));
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

int sgpu_stage_input(sgpu_ctx* ctx, const uint8_t* images, int n, int w, int h, int stride) {
    if (!ctx || !images || n <= 0 || stride < w) return SGPU_EINVAL;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    const size_t bytes = (size_t)n * h * stride;
    ALLOCCHK(ctx, ctx->input.ensure(bytes));
    HIPCHK(ctx, hipMemcpy(ctx->input.p, images, bytes, hipMemcpyHostToDevice));
    ctx->staged_bytes = bytes;
    return SGPU_OK;
}

int sgpu_extract(sgpu_ctx* ctx, const uint8_t* images, int n, int w, int h, int stride,
                 int flags) {
    return extract_impl(ctx, images, false, n, w, h, stride, flags);
}

int sgpu_extract_f32(sgpu_ctx* ctx, const float* images, int n, int w, int h, int stride,
                     int flags) {
    return extract_impl(ctx, images, true, n, w, h, stride, flags);
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
    const int64_t a = ctx->img_off[image], nf = ctx->img_off[image + 1] - a;
    if (nf <= 0) return SGPU_OK;
    if (keys)
        HIPCHK(ctx, hipMemcpyAsync(keys, ctx->keys.as<float4>() + a, nf * sizeof(float4),
                                   hipMemcpyDeviceToHost, ctx->stream));
    if (descriptors) {
        if (!ctx->opt.descriptors) return ctx->fail(SGPU_EINVAL, "descriptors disabled (-sd)");
        HIPCHK(ctx, hipMemcpyAsync(descriptors, ctx->desc.as<float>() + a * 128,
                                   nf * 128 * sizeof(float), hipMemcpyDeviceToHost, ctx->stream));
    }
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    return SGPU_OK;
}

int sgpu_device_features(sgpu_ctx* ctx, const float** keys, const float** descriptors,
                         const int64_t** image_offsets) {
    if (!ctx) return SGPU_EINVAL;
    if (keys) *keys = ctx->keys.as<float>();
    if (descriptors) *descriptors = ctx->opt.descriptors ? ctx->desc.as<float>() : nullptr;
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

int sgpu_debug_set_variant(int variant) {
    return sgk::set_variant(variant) == hipSuccess ? SGPU_OK : SGPU_ENODEV;
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
    const sgk::OctaveDesc& od = ctx->fp.oct[octave];
    const long long npx = (long long)od.wa * od.h;
    const float* src = ctx->pyr.as<float>() + od.gauss_off + level * od.level_stride + image * npx;
    HIPCHK(ctx, hipMemcpy(out, src, npx * sizeof(float), hipMemcpyDeviceToHost));
    return SGPU_OK;
}

int sgpu_debug_candidates(sgpu_ctx* ctx, int* ints, float* floats, int cap, int* n) {
    if (!ctx || !n) return SGPU_EINVAL;
    *n = (int)ctx->n_cand;
    if (!ints || !floats || cap < (int)ctx->n_cand) return ctx->n_cand ? SGPU_ERANGE : SGPU_OK;
    if (ctx->n_cand == 0) return SGPU_OK;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    DevBuf a, b;
    ALLOCCHK(ctx, a.ensure(ctx->n_cand * sizeof(int4)));
    ALLOCCHK(ctx, b.ensure(ctx->n_cand * sizeof(float4)));
    HIPCHK(ctx, sgk::launch_debug_candidates(ctx->pyr.as<float>(), ctx->mask.as<uint32_t>(),
                                             ctx->row_base.as<uint32_t>(), ctx->total_rows,
                                             ctx->row_base.as<uint32_t>() + ctx->total_rows,
                                             (int)ctx->n_cand, ctx->fp, a.as<int4>(), b.as<float4>(),
                                             ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ints, a.p, ctx->n_cand * sizeof(int4), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(floats, b.p, ctx->n_cand * sizeof(float4), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    a.release();
    b.release();
    return SGPU_OK;
}

}  // extern "C"
