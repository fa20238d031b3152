// siftgpu_api.cpp -- the reference's C++ API (include/SiftGPU.h) on top of the C ABI.
//
// Mirrors SiftGPU/SiftGPU.cpp (SiftGPU, SiftParam), SiftGPU/SiftMatch.cpp:549-687 (SiftMatchGPU
// front-end) and SiftGPU/SiftMatchCU.cpp (descriptor quantisation, max_sift clamp) with the same
// call semantics and return values.  Differences, by design:
//   * options are per instance (the reference keeps them in process-global statics,
//     GlobalUtil.cpp:50-141), so instances on different GPUs are independent;
//   * no OpenGL: CreateContextGL()/VerifyContextGL() create the HIP context and return
//     SIFTGPU_FULL_SUPPORTED (2) when a gfx950 device is usable, 0 otherwise;
//   * image files: PGM/PPM (P2/P3/P5/P6) as the reference's SIFTGPU_NO_DEVIL loader
//     (GLTexImage.cpp:1128-1189); DevIL formats are not available.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <new>
#include <string>
#include <vector>

#include "../../include/SiftGPU.h"
#include "../../include/sgpu.h"
#include "sift_params.h"

namespace {

constexpr unsigned kGL_LUMINANCE = 0x1909, kGL_LUMINANCE_ALPHA = 0x190A, kGL_RGB = 0x1907,
                   kGL_RGBA = 0x1908, kGL_BGR = 0x80E0, kGL_BGRA = 0x80E1;
constexpr unsigned kGL_UNSIGNED_BYTE = 0x1401, kGL_UNSIGNED_SHORT = 0x1403, kGL_FLOAT = 0x1406;

// Host-side input image, stored in the slot of the reference's GLTexInput* member.
struct HostImage {
    int w = 0, h = 0;
    bool is_float = false;
    int color = 0;                 // SGPU_RGB.. for u8 color data, 0 for luminance
    std::vector<uint8_t> u8;
    std::vector<float> f32;
};

// The object's feature arrays (the reference's host key / descriptor buffers, which
// GetFeatureVector copies out): page-locked and grow-only, so the per-image downloads run at
// DMA speed instead of through the runtime's pageable staging (C2: one image per RunSIFT).
// Falls back to ordinary memory if page-locked allocation fails.
class HostFloats {
  public:
    HostFloats() = default;
    HostFloats(const HostFloats&) = delete;
    HostFloats& operator=(const HostFloats&) = delete;
    ~HostFloats() { release(); }
    // capacity for n floats (contents not kept), size unchanged
    void reserve(size_t n) {
        if (n > cap_) {
            const size_t keep = n_;
            resize(n);
            n_ = keep;
        }
    }
    bool pinned() const { return pinned_; }
    void resize(size_t n) {
        if (n > cap_) {
            release();
            size_t c = std::max(n, cap_ + cap_ / 2);
            p_ = static_cast<float*>(sgpu_host_alloc(c * sizeof(float)));
            pinned_ = p_ != nullptr;
            if (!p_) p_ = static_cast<float*>(std::malloc(c * sizeof(float)));
            if (!p_) throw std::bad_alloc();
            cap_ = c;
        }
        n_ = n;
    }
    float* data() { return p_; }
    const float* data() const { return p_; }
    size_t size() const { return n_; }
  private:
    void release() {
        if (p_) {
            if (pinned_) sgpu_host_free(p_);
            else std::free(p_);
        }
        p_ = nullptr;
        cap_ = n_ = 0;
    }
    float* p_ = nullptr;
    size_t cap_ = 0, n_ = 0;
    bool pinned_ = false;
};

// Runtime state, stored in the slot of the reference's SiftPyramid* member.
struct Runtime {
    sgpu_options opt;
    int device = 0;
    sgpu_ctx* ctx = nullptr;
    int binary = 0;             // -b
    int verbose = 1;
    // GlobalUtil::_timingS (GlobalUtil.cpp:51, default 1; SiftGPU::SetVerbose, SiftGPU.cpp:401-429):
    // when 0 the reference skips its per-stage finish calls; here the extract records no stage
    // events (sgpu_set_stage_timing), so _timing[2..8] read 0 and the call is ~40 us shorter
    int timing_s = 1;
    int feature_num = 0;
    HostFloats keys, desc;
    // SetKeypointList (SiftPyramid::SetKeypointList, SiftPyramid.cpp:293-310): applied by the
    // next RunSIFT on a new image, then cleared (SiftPyramid.cpp:204)
    std::vector<float> pending;
    int pending_orientation = 1;
    bool have_image = false;    // a pyramid of the current image exists on the device
    // the current u8 gray image is staged in the context's device input: the reference uploads
    // an image into its input texture once, when it is loaded (SiftGPU.cpp:317-328,
    // GLTexImage.cpp:918-1009), and RunSIFT() on the loaded image reuses the texture
    bool staged = false;
    // host seconds of the last image load / conversion (SiftGPU::_timing[0], SiftGPU.cpp:249,328)
    // and of the last feature downloads (keys: _timing[7], descriptors: part of _timing[8])
    float t_load = 0.f, t_keys = 0.f, t_desc = 0.f;
    Runtime() { sgpu_default_options(&opt); }
};

struct ImageListImpl : std::vector<std::string> {};

Runtime* RT(SiftPyramid* p) { return reinterpret_cast<Runtime*>(p); }
HostImage* IMG(GLTexInput* p) { return reinterpret_cast<HostImage*>(p); }
ImageListImpl* LIST(ImageList* p) { return reinterpret_cast<ImageListImpl*>(p); }

constexpr int kMaxPath = 4096;

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// GLTexInput::LoadImageFile, SIFTGPU_NO_DEVIL branch (GLTexImage.cpp:1128-1189).
bool load_pnm(const char* path, HostImage* img) {
    FILE* f = fopen(path, "rb");
    if (!f) return false;
    char buf[8] = {0};
    int width, height, cn;
    if (fscanf(f, "%7s %d %d %d", buf, &width, &height, &cn) < 4 || cn > 255 || width < 0 ||
        height < 0) {
        fclose(f);
        std::cerr << "ERROR: fileformat not supported\n";
        return false;
    }
    std::vector<uint8_t> data((size_t)width * height);
    bool ok = true;
    if (!strcmp(buf, "P5")) {
        fgetc(f);
        ok = fread(data.data(), 1, data.size(), f) == data.size();
    } else if (!strcmp(buf, "P2")) {
        for (size_t i = 0; i < data.size(); i++) {
            int g = 0;
            if (fscanf(f, "%d", &g) != 1) { ok = false; break; }
            data[i] = (uint8_t)g;
        }
    } else if (!strcmp(buf, "P6")) {
        fgetc(f);
        for (size_t i = 0; i < data.size(); i++) {
            uint8_t p[3];
            if (fread(p, 1, 3, f) != 3) { ok = false; break; }
            data[i] = (uint8_t)int(0.10454f * p[2] + 0.60581f * p[1] + 0.28965f * p[0]);
        }
    } else if (!strcmp(buf, "P3")) {
        for (size_t i = 0; i < data.size(); i++) {
            int r, g, b;
            if (fscanf(f, "%d %d %d", &r, &g, &b) != 3) { ok = false; break; }
            data[i] = (uint8_t)int(0.10454f * b + 0.60581f * g + 0.28965f * r);
        }
    } else {
        std::cerr << "ERROR: fileformat not supported\n";
        ok = false;
    }
    fclose(f);
    if (!ok) return false;
    img->w = width;
    img->h = height;
    img->is_float = false;
    img->u8.swap(data);
    return true;
}

// GLTexInput::SetImageData for the CUDA path (GLTexImage.cpp:918-1009) with down-sampling 1:
// u8 luminance and u8 RGB/BGR/RGBA/BGRA stay u8 (converted to float luminance on the GPU with
// the reference's formulas); u16, float and luminance-alpha input is converted on the host
// (:808-916).
template <class T>
void to_float(const T* p, unsigned fmt, int w, int h, float factor, std::vector<float>* out) {
    out->resize((size_t)w * h);
    const int step = (fmt == kGL_LUMINANCE) ? 1 : (fmt == kGL_LUMINANCE_ALPHA) ? 2
                     : (fmt == kGL_RGB || fmt == kGL_BGR) ? 3 : 4;
    float* o = out->data();
    for (int i = 0; i < w * h; i++, p += step) {
        if (fmt == kGL_LUMINANCE || fmt == kGL_LUMINANCE_ALPHA) o[i] = p[0] / factor;
        else if (fmt == kGL_RGB || fmt == kGL_RGBA)
            o[i] = (19595 * p[0] + 38470 * p[1] + 7471 * p[2]) / (65535.0f * factor);
        else o[i] = (7471 * p[0] + 38470 * p[1] + 19595 * p[2]) / (65535.0f * factor);
    }
}

void to_float_f(const float* p, unsigned fmt, int w, int h, std::vector<float>* out) {
    out->resize((size_t)w * h);
    const int step = (fmt == kGL_LUMINANCE) ? 1 : (fmt == kGL_LUMINANCE_ALPHA) ? 2
                     : (fmt == kGL_RGB || fmt == kGL_BGR) ? 3 : 4;
    float* o = out->data();
    for (int i = 0; i < w * h; i++, p += step) {
        if (fmt == kGL_LUMINANCE || fmt == kGL_LUMINANCE_ALPHA) o[i] = p[0];
        else if (fmt == kGL_RGB || fmt == kGL_RGBA) o[i] = 0.299f * p[0] + 0.587f * p[1] + 0.114f * p[2];
        else o[i] = 0.114f * p[0] + 0.587f * p[1] + 0.299f * p[2];
    }
}

// The CUDA path's float luminance input without down-sampling is used in place, and with a
// width that is not a multiple of 4 the reference compacts its rows to the truncated width IN
// THE CALLER'S BUFFER (GLTexImage.cpp:994-1006, through the const pointer of RunSIFT): row i
// (i >= 1) moves from i * w to i * (w & ~3).  Reproduced, because a caller can observe it.
void compact_caller_rows(const void* data, int w, int h) {
    const int tw = w & ~3;
    if (tw == w) return;
    float* p = const_cast<float*>(static_cast<const float*>(data));
    for (int i = 1; i < h; ++i) {
        float* dst = p + (size_t)i * tw;
        const float* src = p + (size_t)i * w;
        for (int j = 0; j < tw; ++j) *dst++ = *src++;
    }
}

bool set_image(HostImage* img, int w, int h, const void* data, unsigned fmt, unsigned type,
               int down_sampled) {
    const bool fmt_ok = fmt == kGL_LUMINANCE || fmt == kGL_LUMINANCE_ALPHA || fmt == kGL_RGB ||
                        fmt == kGL_RGBA || fmt == kGL_BGR || fmt == kGL_BGRA;
    const bool type_ok = type == kGL_UNSIGNED_BYTE || type == kGL_UNSIGNED_SHORT || type == kGL_FLOAT;
    if (!fmt_ok || !type_ok) {
        std::cerr << "Input format not supported under current settings.\n";
        return false;
    }
    img->w = w;
    img->h = h;
    img->color = 0;
    if (fmt == kGL_LUMINANCE && type == kGL_UNSIGNED_BYTE) {
        img->is_float = false;
        img->u8.assign((const uint8_t*)data, (const uint8_t*)data + (size_t)w * h);
        return true;
    }
    if (type == kGL_UNSIGNED_BYTE && fmt != kGL_LUMINANCE_ALPHA) {
        // RGB / BGR / RGBA / BGRA u8: converted to luminance on the device (sgpu_extract_color)
        const int ch = (fmt == kGL_RGB || fmt == kGL_BGR) ? 3 : 4;
        img->is_float = false;
        img->color = fmt == kGL_RGB ? SGPU_RGB : fmt == kGL_BGR ? SGPU_BGR
                   : fmt == kGL_RGBA ? SGPU_RGBA : SGPU_BGRA;
        img->u8.assign((const uint8_t*)data, (const uint8_t*)data + (size_t)w * h * ch);
        return true;
    }
    img->is_float = true;
    if (type == kGL_UNSIGNED_BYTE) to_float((const uint8_t*)data, fmt, w, h, 255.0f, &img->f32);
    else if (type == kGL_UNSIGNED_SHORT) to_float((const uint16_t*)data, fmt, w, h, 65535.0f, &img->f32);
    else to_float_f((const float*)data, fmt, w, h, &img->f32);
    if (type == kGL_FLOAT && fmt == kGL_LUMINANCE && down_sampled == 0) {
        // the host copy keeps the caller's full rows (the pipeline truncates on the device);
        // the caller's buffer is compacted as the reference leaves it
        compact_caller_rows(data, w, h);
    }
    return true;
}

}  // namespace

// ---------------------------------------------------------------------------------- SiftParam
SiftParam::SiftParam() {
    _sigma = nullptr;
    _level_min = -1;
    _dog_level_num = 3;
    _level_max = 0;
    _sigma0 = 0;
    _sigman = 0;
    _edge_threshold = 0;
    _dog_threshold = 0;
    _sigma_skip0 = _sigma_skip1 = 0;
    _sigma_num = _level_num = _level_ds = 0;
}

float SiftParam::GetLevelSigma(int lev) {
    return _sigma0 * powf(2.0f, float(lev) / float(_dog_level_num));
}

float SiftParam::GetInitialSmoothSigma(int octave_min) {
    float sa = _sigma0 * powf(2.0f, float(_level_min) / float(_dog_level_num));
    float sb = _sigman / powf(2.0f, float(octave_min));
    return sa > sb + 0.001 ? sqrtf(sa * sa - sb * sb) : 0.0f;
}

void SiftParam::ParseSiftParam() {
    sgp::Options po;
    po.dog_level_num = _dog_level_num;
    po.dog_threshold = _dog_threshold;
    po.edge_threshold = _edge_threshold;
    sgp::Schedule s = sgp::make_schedule(po);
    _dog_level_num = s.dog_level_num;
    _level_max = s.level_max;
    _sigma0 = s.sigma0;
    _sigman = s.sigman;
    _level_num = s.level_num;
    _level_ds = s.level_ds;
    _sigma_skip0 = s.sigma_skip0;
    _sigma_skip1 = s.sigma_skip1;
    _sigma_num = s.level_max - s.level_min;
    delete[] _sigma;
    _sigma = new float[_sigma_num];
    for (int i = 0; i < _sigma_num; i++) _sigma[i] = s.sigma[i];
    _dog_threshold = s.dog_threshold;
    _edge_threshold = s.edge_threshold;
}

// ---------------------------------------------------------------------------------- SiftGPU
void* SiftGPU::operator new(size_t size) {
    void* p = malloc(size);
    if (!p) throw std::bad_alloc();
    return p;
}

SiftGPU::SiftGPU(int) {
    _texImage = reinterpret_cast<GLTexInput*>(new HostImage());
    _imgpath = new char[kMaxPath];
    _outpath = new char[kMaxPath];
    _imgpath[0] = _outpath[0] = 0;
    _initialized = 0;
    _image_loaded = 0;
    _current = 0;
    _list = reinterpret_cast<ImageList*>(new ImageListImpl());
    _pyramid = reinterpret_cast<SiftPyramid*>(new Runtime());
    for (float& t : _timing) t = 0;
}

SiftGPU::~SiftGPU() {
    Runtime* rt = RT(_pyramid);
    if (rt->ctx) sgpu_ctx_destroy(rt->ctx);
    delete rt;
    delete IMG(_texImage);
    delete LIST(_list);
    delete[] _imgpath;
    delete[] _outpath;
    delete[] _sigma;
}

void SiftGPU::PrintUsage() {
    std::cout << "SiftGPU (MI355X) usage: -i <files> -o <file> -f <float> -w <float> -dw <float>\n"
                 "  -fo <int> -no <int> -d <int> -t <float> -e <float> -m [int] -s [int] -sd -unn -b\n"
                 "  -loweo -ofix -sign -cuda [device] -v <int>\n";
}

void SiftGPU::InitSiftGPU() {
    if (_initialized) return;
    Runtime* rt = RT(_pyramid);
    _dog_level_num = rt->opt.dog_level_num;
    _dog_threshold = rt->opt.dog_threshold;
    _edge_threshold = rt->opt.edge_threshold;
    ParseSiftParam();
    if (!rt->ctx) {
        int rc = sgpu_ctx_create(rt->device, &rt->opt, &rt->ctx);
        if (rc != SGPU_OK) {
            std::cerr << "SiftGPU: no usable MI355X device " << rt->device << " (code " << rc << ")\n";
            rt->ctx = nullptr;
            return;
        }
        sgpu_set_stage_timing(rt->ctx, rt->timing_s);
    }
    _initialized = 1;
}

void SiftGPU::LoadImageList(const char* imlist) {
    std::ifstream in(imlist);
    std::string name;
    while (in >> name) LIST(_list)->push_back(name);
    if (!LIST(_list)->empty()) strncpy(_imgpath, LIST(_list)->at(0).c_str(), kMaxPath - 1);
    _image_loaded = 0;
}

void SiftGPU::SetImageList(int nimage, const char** filelist) {
    LIST(_list)->clear();
    for (int i = 0; i < nimage; i++) LIST(_list)->push_back(filelist[i]);
    _current = 0;
}

int SiftGPU::GetFeatureNum() { return RT(_pyramid)->feature_num; }

void SiftGPU::GetFeatureVector(SiftKeypoint* keys, float* descriptors) {
    Runtime* rt = RT(_pyramid);
    const size_t n = rt->feature_num;
    if (keys && n) memcpy(keys, rt->keys.data(), n * 4 * sizeof(float));
    if (descriptors && n && rt->opt.descriptors)
        memcpy(descriptors, rt->desc.data(), n * 128 * sizeof(float));
}

// SiftPyramid::SaveSIFT (SiftPyramid.cpp:313-387): Lowe's format, (y, x, s, o) per line.
void SiftGPU::SaveSIFT(const char* szFileName) {
    Runtime* rt = RT(_pyramid);
    const int n = rt->feature_num;
    if (n <= 0) return;
    const float* pk = rt->keys.data();
    const bool has_desc = rt->opt.descriptors != 0;
    if (rt->binary) {
        std::ofstream out(szFileName, std::ios::binary);
        out.write((const char*)&n, sizeof(int));
        const int dim = has_desc ? 128 : 0;
        out.write((const char*)&dim, sizeof(int));
        for (int i = 0; i < n; i++, pk += 4) {
            out.write((const char*)(pk + 1), sizeof(float));
            out.write((const char*)pk, sizeof(float));
            out.write((const char*)(pk + 2), 2 * sizeof(float));
            if (has_desc) out.write((const char*)(rt->desc.data() + (size_t)i * 128), 128 * sizeof(float));
        }
        return;
    }
    std::ofstream out(szFileName);
    out.flags(std::ios::fixed);
    if (has_desc) {
        const float* pd = rt->desc.data();
        out << n << " 128" << std::endl;
        for (int i = 0; i < n; i++, pk += 4) {
            out << std::setprecision(2) << pk[1] << " " << std::setprecision(2) << pk[0] << " "
                << std::setprecision(3) << pk[2] << " " << std::setprecision(3) << pk[3] << std::endl;
            for (int k = 0; k < 128; k++, pd++) {
                if (rt->opt.normalized) out << ((unsigned int)floor(0.5 + 512.0f * (*pd))) << " ";
                else out << std::setprecision(8) << pd[0] << " ";
                if ((k + 1) % 20 == 0) out << std::endl;
            }
            out << std::endl;
        }
    } else {
        out << n << " 0" << std::endl;
        for (int i = 0; i < n; i++, pk += 4)
            out << pk[1] << " " << pk[0] << " " << pk[2] << " " << pk[3] << std::endl;
    }
}

void SiftGPU::SetKeypointList(int num, const SiftKeypoint* keys, int keys_have_orientation) {
    if (num <= 0 || !keys) return;
    Runtime* rt = RT(_pyramid);
    rt->pending.assign((const float*)keys, (const float*)keys + 4 * (size_t)num);
    rt->pending_orientation = keys_have_orientation;
}

// Before a detecting extract: the object's page-locked key / descriptor buffers, sized for the
// last image's count + 25 % (at least 4,096 features), registered as the extract's host output
// (sgpu_set_host_output): the GPU writes them in the extract's own stream, and fetch_features
// then copies nothing when they fit.
static void arm_host_output(Runtime* rt) {
    // A/B hook: SGPU_HOST_OUTPUT=0 keeps the copies of sgpu_copy_features
    static const bool off = [] {
        const char* e = getenv("SGPU_HOST_OUTPUT");
        return e && e[0] == '0';
    }();
    if (off) return;
    const size_t hint = std::max<size_t>(4096, (size_t)rt->feature_num + (size_t)rt->feature_num / 4);
    rt->keys.reserve(hint * 4);
    if (rt->opt.descriptors) rt->desc.reserve(hint * 128);
    if (rt->keys.pinned() && (!rt->opt.descriptors || rt->desc.pinned()))
        sgpu_set_host_output(rt->ctx, rt->keys.data(), rt->opt.descriptors ? rt->desc.data() : nullptr,
                             (int)hint);
}

// Copy the context's current features (image 0) into the object's host buffers: the keys
// (the reference's DownloadKeypoints stage) and then the descriptors (downloaded inside its
// GetFeatureDescriptors stage, PyramidCU.cpp:434), each timed on the host.
static int fetch_features(Runtime* rt) {
    rt->feature_num = sgpu_feature_count(rt->ctx, 0);
    rt->keys.resize((size_t)rt->feature_num * 4);
    rt->desc.resize(rt->opt.descriptors ? (size_t)rt->feature_num * 128 : 0);
    // keys and descriptors in one call (one synchronisation); the key copy's event time is
    // _timing[7], the rest of the call goes with the descriptors into _timing[8]
    const double t0 = now_s();
    int rc = sgpu_copy_features(rt->ctx, 0, rt->keys.data(),
                                rt->opt.descriptors ? rt->desc.data() : nullptr);
    const double t = now_s() - t0;
    float ct[12] = {0};
    sgpu_last_timing(rt->ctx, ct, 12);
    rt->t_keys = std::min((float)t, ct[10] * 1e-3f);
    rt->t_desc = (float)t - rt->t_keys;
    return rc;
}

// Descriptors of a keypoint list on the current image (SiftGPU::RunSIFT(num, keys, ...)).
// keys_have_orientation: 0 computes the strongest orientation, -1 is the rectangle description
// (SIFT_RECT_DESCRIPTION, SiftPyramid.cpp:307-309, ProgramCU.cu:1104-1171), anything else keeps
// the given orientations.
static int describe_keys(Runtime* rt, const float* keys, int num, int has_orientation) {
    if (sgpu_extract_keypoints(rt->ctx, 0, keys, num, has_orientation) != SGPU_OK) {
        std::cerr << "SiftGPU: " << sgpu_last_error(rt->ctx) << "\n";
        return 0;
    }
    return fetch_features(rt) == SGPU_OK ? 1 : 0;
}

int SiftGPU::CreateContextGL() { return VerifyContextGL(); }

int SiftGPU::VerifyContextGL() {
    InitSiftGPU();
    return _initialized ? SIFTGPU_FULL_SUPPORTED : SIFTGPU_NOT_SUPPORTED;
}

int SiftGPU::IsFullSupported() { return _initialized ? 1 : 0; }

// SiftGPU::SetVerbose (SiftGPU.cpp:401-429): -1 cycles the levels, -2 silences the output but
// keeps the stage timing, otherwise output when > 0 and stage timing when > 1
void SiftGPU::SetVerbose(int verbose) {
    Runtime* rt = RT(_pyramid);
    if (verbose == -1) {
        if (rt->verbose) {
            rt->verbose = rt->timing_s;
            rt->timing_s = 0;
        } else {
            rt->verbose = 1;
            rt->timing_s = 1;
        }
    } else if (verbose == -2) {
        rt->verbose = 0;
        rt->timing_s = 1;
    } else {
        rt->verbose = verbose > 0;
        rt->timing_s = verbose > 1;
    }
    if (rt->ctx) sgpu_set_stage_timing(rt->ctx, rt->timing_s);
}

// SiftGPU::ParseParam (SiftGPU.cpp:801-1246): algorithm options go through sgpu_parse_args;
// file options (-i, -il, -o, -b) are handled here.
void SiftGPU::ParseParam(int argc, char** argv) {
    Runtime* rt = RT(_pyramid);
    if (!_initialized) {
        sgpu_parse_args(&rt->opt, argc, argv, &rt->device);
    } else {
        // after initialisation only the run-time options may change (SimpleSIFT.cpp:190-193)
        sgpu_options o = rt->opt;
        int dev = rt->device;
        sgpu_parse_args(&o, argc, argv, &dev);
        rt->opt.descriptor_window_factor = o.descriptor_window_factor;
        rt->opt.fixed_orientation = o.fixed_orientation;
        rt->opt.normalized = o.normalized;
        if (rt->ctx) sgpu_ctx_set_options(rt->ctx, &rt->opt);
    }
    for (int i = 0; i < argc; i++) {
        const char* a = argv[i];
        if (!a || a[0] != '-') continue;
        std::string k(a + 1);
        for (char& c : k) c = (char)tolower(c);
        if (k == "h" || k == "help") PrintUsage();
        else if (k == "b") rt->binary = 1;
        else if (k == "v" && i + 1 < argc) {   // SiftGPU.cpp:1207-1210
            int num = 0;
            if (sscanf(argv[i + 1], "%d", &num) == 1 && num >= 0 && num <= 4) SetVerbose(num);
        }
        else if (k == "i" && i + 1 < argc) {
            strncpy(_imgpath, argv[++i], kMaxPath - 1);
            LIST(_list)->push_back(argv[i]);
            while (i + 1 < argc && argv[i + 1][0] != '-') LIST(_list)->push_back(argv[++i]);
        } else if (k == "il" && i + 1 < argc) LoadImageList(argv[++i]);
        else if (k == "o" && i + 1 < argc) strncpy(_outpath, argv[++i], kMaxPath - 1);
    }
    if (_outpath[0] && LIST(_list)->size() > 1) _outpath[0] = 0;
}

int SiftGPU::RunSIFT(const char* imgpath) {
    if (imgpath && imgpath[0]) {
        strncpy(_imgpath, imgpath, kMaxPath - 1);
        _image_loaded = 0;
        return RunSIFT();
    }
    return 0;
}

int SiftGPU::RunSIFT(int index) {
    ImageListImpl* l = LIST(_list);
    if (l->empty()) return 0;
    index = index % (int)l->size();
    if (strcmp(_imgpath, l->at(index).c_str())) {
        strncpy(_imgpath, l->at(index).c_str(), kMaxPath - 1);
        _image_loaded = 0;
        _current = index;
    }
    return RunSIFT();
}

int SiftGPU::RunSIFT(int width, int height, const void* data, unsigned int gl_format,
                     unsigned int gl_type) {
    if (!_initialized) InitSiftGPU();
    if (!_initialized) return 0;
    if (width <= 0 || height <= 0 || !data) return 0;
    _imgpath[0] = 0;
    const double t0 = now_s();
    const sgpu_options& o = RT(_pyramid)->opt;
    const int down_sampled = sgp::plan_input(width, height, o.octave_min, o.max_dimension,
                                             o.preprocess_on_cpu).ds;
    if (!set_image(IMG(_texImage), width, height, data, gl_format, gl_type, down_sampled))
        return 0;
    RT(_pyramid)->t_load = (float)(now_s() - t0);
    RT(_pyramid)->staged = false;
    _image_loaded = 2;
    return RunSIFT();
}

int SiftGPU::RunSIFT() {
    if (_imgpath[0] == 0 && _image_loaded == 0) return 0;
    if (!_initialized) InitSiftGPU();
    if (!_initialized) return 0;
    Runtime* rt = RT(_pyramid);
    HostImage* img = IMG(_texImage);
    if (_image_loaded == 0) {
        const double t0 = now_s();
        if (!load_pnm(_imgpath, img)) {
            std::cerr << "Unable to open image " << _imgpath << "\n";
            return 0;
        }
        rt->t_load = (float)(now_s() - t0);
        _image_loaded = 1;
        rt->staged = false;
    } else if (_image_loaded == 1) {
        rt->t_load = 0.f;   // the file is already loaded (SiftGPU.cpp:348-351)
    }
    const int ch = img->color == SGPU_RGB || img->color == SGPU_BGR ? 3 : 4;
    int rc;
    if (rt->pending.empty()) arm_host_output(rt);
    if (!img->is_float && !img->color) {
        // u8 gray: uploaded once per image (the load, _timing[0]), then every RunSIFT() on it
        // starts from the device copy, as the reference's texture
        if (!rt->staged) {
            const double t0 = now_s();
            rc = sgpu_stage_input(rt->ctx, img->u8.data(), 1, img->w, img->h, img->w);
            rt->t_load += (float)(now_s() - t0);
            rt->staged = rc == SGPU_OK;
        }
        rc = rt->staged ? sgpu_extract(rt->ctx, nullptr, 1, img->w, img->h, img->w, SGPU_INPUT_STAGED)
                        : sgpu_extract(rt->ctx, img->u8.data(), 1, img->w, img->h, img->w,
                                       SGPU_INPUT_HOST);
    } else {
        rt->staged = false;   // a host-input extract reuses the context's input buffer
        rc = img->is_float
                 ? sgpu_extract_f32(rt->ctx, img->f32.data(), 1, img->w, img->h, img->w, SGPU_INPUT_HOST)
                 : sgpu_extract_color(rt->ctx, img->u8.data(), 1, img->w, img->h, img->w * ch,
                                      img->color, SGPU_INPUT_HOST);
    }
    if (rc != SGPU_OK) {
        std::cerr << "SiftGPU: " << sgpu_last_error(rt->ctx) << "\n";
        rt->staged = false;
        rt->feature_num = 0;
        rt->have_image = false;
        rt->pending.clear();
        return 0;
    }
    rt->have_image = true;
    if (!rt->pending.empty()) {
        // a list from SetKeypointList replaces detection on this image
        std::vector<float> keys;
        keys.swap(rt->pending);
        if (!describe_keys(rt, keys.data(), (int)(keys.size() / 4), rt->pending_orientation))
            return 0;
    } else if (fetch_features(rt) != SGPU_OK) {
        return 0;
    }
    // SiftGPU::_timing in the reference's slots, seconds (SiftGPU.cpp:249-255,328-351,368 ->
    // SiftPyramid::_timing[0..7], SiftPyramid.cpp:107,123,145,155,180,200,212; printed by
    // TestWin/speed.cpp:147-153): [0] load/convert the image on the host, [1] initialise the
    // pyramid (planned inside the extract here: 0), [2] build pyramid (with its input upload,
    // as ConvertInputToCU in BuildPyramid), [3] detection, [4] feature list, [5] orientation,
    // [6] multi-orientation feature list, [7] download keys, [8] descriptors (kernel + their
    // download), [9] display VBO (none: 0).  GPU stages from HIP events, downloads host-timed.
    float t[10] = {0};
    sgpu_last_timing(rt->ctx, t, 10);
    for (int i = 0; i < 10; i++) _timing[i] = 0;
    _timing[0] = rt->t_load;
    _timing[2] = (t[0] + t[1]) * 1e-3f;
    _timing[3] = (t[2] - t[9]) * 1e-3f;
    _timing[4] = t[9] * 1e-3f;
    _timing[5] = t[3] * 1e-3f;
    _timing[6] = t[4] * 1e-3f;
    _timing[7] = rt->t_keys;
    _timing[8] = t[5] * 1e-3f + rt->t_desc;
    if (rt->verbose > 0) std::cout << "[SiftGPU MI355X]: " << rt->feature_num << " features, " << t[7] << " ms\n";
    if (_outpath[0]) {
        SaveSIFT(_outpath);
        _outpath[0] = 0;
    }
    return 1;
}

// SiftGPU::RunSIFT(num, keys, keys_have_orientation) (SiftGPU.cpp:287-291): the list is
// described on the current image's pyramid (run_on_current: no new filtering).
int SiftGPU::RunSIFT(int num, const SiftKeypoint* keys, int keys_have_orientation) {
    if (num <= 0 || !keys) return 0;
    Runtime* rt = RT(_pyramid);
    if (!_initialized || !rt->have_image) return 0;
    return describe_keys(rt, (const float*)keys, num, keys_have_orientation);
}

int SiftGPU::GetImageCount() { return (int)LIST(_list)->size(); }
// SiftGPU::SetTightPyramid (SiftGPU.cpp:1430-1433) chooses how much slack ResizePyramid leaves
// for larger images; the context's buffers are grow-only and sized per batch, so it changes
// nothing here.
void SiftGPU::SetTightPyramid(int) {}
// SiftGPU::AllocatePyramid (SiftGPU.cpp:1435-1460): the pyramid (and every other buffer) for a
// width x height gray image is allocated now, so the first RunSIFT of that size allocates nothing
// (sgpu_reserve).  Like the reference's ResizePyramid it drops the current image's pyramid.
int SiftGPU::AllocatePyramid(int width, int height) {
    if (!_initialized) InitSiftGPU();
    if (!_initialized || width <= 0 || height <= 0) return 0;
    Runtime* rt = RT(_pyramid);
    rt->staged = false;
    rt->have_image = false;
    rt->feature_num = 0;
    return sgpu_reserve(rt->ctx, 1, width, height, width) == SGPU_OK;
}
// SiftGPU::SetMaxDimension (SiftGPU.cpp:1452-1458): below the GL texture limit (14096,
// GlobalUtil.cpp:88) it becomes _texMaxDim, which raises the first octave of larger inputs
// (PyramidCU.cpp:129-135).
void SiftGPU::SetMaxDimension(int sz) {
    if (sz >= 14096) return;
    Runtime* rt = RT(_pyramid);
    rt->opt.max_dimension = sz;
    if (rt->ctx) sgpu_ctx_set_options(rt->ctx, &rt->opt);
}

// ---------------------------------------------------------------------------------- matcher
namespace {
struct MatchState {
    sgpu_ctx* ctx = nullptr;
    int device = 0;
    int max_sift = 14096;
    int num[2] = {0, 0};
    int id[2] = {0, 0};
    std::vector<uint8_t> des[2];
    int have_loc[2] = {0, 0};
    std::vector<float> loc[2];   // packed (x, y) per feature
};
MatchState* MS(SiftMatchGPU* p) { return reinterpret_cast<MatchState*>(p); }
}  // namespace

void* SiftMatchGPU::operator new(size_t size) {
    void* p = malloc(size);
    if (!p) throw std::bad_alloc();
    return p;
}

SiftMatchGPU::SiftMatchGPU(int max_sift) {
    __max_sift = std::max(max_sift, 1024);   // SiftMatch.cpp:616
    __language = 0;
    __matcher = nullptr;
}

SiftMatchGPU::~SiftMatchGPU() {
    MatchState* m = MS(__matcher);
    if (m) {
        if (m->ctx) sgpu_ctx_destroy(m->ctx);
        delete m;
    }
}

int SiftMatchGPU::_CreateContextGL() { return _VerifyContextGL(); }

int SiftMatchGPU::_VerifyContextGL() {
    if (__matcher) return MS(__matcher)->ctx ? 1 : 0;
    MatchState* m = new MatchState();
    m->device = __language > SIFTMATCH_CUDA ? __language - SIFTMATCH_CUDA : 0;
    // SiftMatchCU::SiftMatchCU (SiftMatchCU.cpp:46): round up to a multiple of 32
    m->max_sift = __max_sift <= 0 ? 14096 : ((__max_sift + 31) / 32 * 32);
    if (sgpu_ctx_create(m->device, nullptr, &m->ctx) != SGPU_OK) {
        std::cerr << "SiftMatchGPU: no usable MI355X device " << m->device << "\n";
        m->ctx = nullptr;
    }
    __matcher = reinterpret_cast<SiftMatchGPU*>(m);
    return m->ctx ? 1 : 0;
}

void SiftMatchGPU::SetLanguage(int language) {
    if (__matcher) return;
    __language = language;
}

void SiftMatchGPU::SetDeviceParam(int argc, char** argv) {
    if (__matcher) return;
    sgpu_options o;
    sgpu_default_options(&o);
    int dev = -1;
    sgpu_parse_args(&o, argc, argv, &dev);
    if (dev >= 0) __language = SIFTMATCH_CUDA + dev;
}

void SiftMatchGPU::SetMaxSift(int max_sift) {
    max_sift = std::max(128, max_sift);
    if (__matcher) MS(__matcher)->max_sift = ((max_sift + 31) / 32) * 32;
    else __max_sift = max_sift;
}

// SiftMatchCU::SetDescriptors (SiftMatchCU.cpp:71-101)
void SiftMatchGPU::SetDescriptors(int index, int num, const unsigned char* descriptors, int id) {
    MatchState* m = MS(__matcher);
    if (!m || !m->ctx) return;
    index = std::min(std::max(index, 0), 1);
    m->have_loc[index] = 0;   // SiftMatchCU.cpp:77
    if (id != -1 && id == m->id[index]) return;
    m->id[index] = id;
    if (num > m->max_sift) num = m->max_sift;
    m->num[index] = num;
    m->des[index].assign(descriptors, descriptors + (size_t)num * 128);
}

void SiftMatchGPU::SetDescriptors(int index, int num, const float* descriptors, int id) {
    MatchState* m = MS(__matcher);
    if (!m || !m->ctx) return;
    index = std::min(std::max(index, 0), 1);
    if (num > m->max_sift) num = m->max_sift;
    std::vector<uint8_t> q((size_t)num * 128);
    sgpu_quantize_descriptors(descriptors, q.size(), q.data());
    SetDescriptors(index, num, q.data(), id);   // the id cache applies as SiftMatchCU.cpp:100
}

int SiftMatchGPU::GetSiftMatch(int max_match, int match_buffer[][2], float distmax,
                               float ratiomax, int mutual_best_match) {
    MatchState* m = MS(__matcher);
    if (!m || !m->ctx || m->num[0] <= 0 || m->num[1] <= 0) return 0;
    int r = sgpu_match(m->ctx, m->des[0].data(), m->num[0], m->des[1].data(), m->num[1], distmax,
                       ratiomax, mutual_best_match, max_match, &match_buffer[0][0], SGPU_INPUT_HOST);
    return r < 0 ? 0 : r;
}

// SiftMatchCU::SetFeautreLocation (SiftMatchCU.cpp:104-122): (x, y) then `gap` skipped floats
// per feature, for the current descriptor count of that set.
void SiftMatchGPU::SetFeautreLocation(int index, const float* locations, int gap) {
    MatchState* m = MS(__matcher);
    if (!m || !m->ctx || !locations) return;
    index = std::min(std::max(index, 0), 1);
    const int n = m->num[index];
    if (n <= 0) return;
    std::vector<float>& l = m->loc[index];
    l.resize((size_t)n * 2);
    for (int i = 0; i < n; i++) {
        l[2 * i] = locations[(size_t)i * (2 + gap)];
        l[2 * i + 1] = locations[(size_t)i * (2 + gap) + 1];
    }
    m->have_loc[index] = 1;
}

// SiftMatch.cpp:663-677 (NULL matrices) + SiftMatchCU::GetGuidedSiftMatch (:126-136).
int SiftMatchGPU::GetGuidedSiftMatch(int max_match, int match_buffer[][2], float H[3][3],
                                     float F[3][3], float distmax, float ratiomax,
                                     float hdistmax, float fdistmax, int mutual_best_match) {
    if (H == NULL && F == NULL)
        return GetSiftMatch(max_match, match_buffer, distmax, ratiomax, mutual_best_match);
    MatchState* m = MS(__matcher);
    if (!m || !m->ctx || m->num[0] <= 0 || m->num[1] <= 0) return 0;
    if (!m->have_loc[0] || !m->have_loc[1]) return 0;
    int r = sgpu_match_guided(m->ctx, m->des[0].data(), m->num[0], m->des[1].data(), m->num[1],
                              m->loc[0].data(), m->loc[1].data(), H ? &H[0][0] : nullptr,
                              F ? &F[0][0] : nullptr, distmax, ratiomax, hdistmax, fdistmax,
                              mutual_best_match, max_match, &match_buffer[0][0], SGPU_INPUT_HOST);
    return r < 0 ? 0 : r;
}

// ---------------------------------------------------------------------------------- factories
void* ComboSiftGPU::operator new(size_t size) {
    void* p = malloc(size);
    if (!p) throw std::bad_alloc();
    return p;
}

SiftGPU* CreateNewSiftGPU(int np) { return new SiftGPU(np); }
SiftMatchGPU* CreateNewSiftMatchGPU(int max_sift) { return new SiftMatchGPU(max_sift); }
ComboSiftGPU* CreateComboSiftGPU() { return new ComboSiftGPU(); }
ComboSiftGPU* CreateRemoteSiftGPU(int, char*) { return new ComboSiftGPU(); }
int CreateLiteWindow(LiteWindow*) { return 0; }
void RunServerLoop(int, int, char**) {
    std::cerr << "RunServerLoop: no remote server on this platform\n";
}
