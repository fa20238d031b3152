// sift_params.h -- host-side SIFT parameter schedule and pyramid geometry.
//
// Restates the reference's scalar set-up (no per-pixel work happens here):
//   * sigma schedule       SiftGPU.cpp:446-498 (SiftParam::ParseSiftParam, GetInitialSmoothSigma)
//                          and SiftGPU.cpp:1285-1288 (GetLevelSigma)
//   * Gaussian taps        ProgramCU.cu:375-403 (ProgramCU::CreateFilterKernel)
//   * octave geometry      PyramidCU.cpp:89-271 (InitPyramid / ResizePyramid), width padding
//                          wa = ((w+3)/4)*4 at PyramidCU.cpp:242, TruncateWidthCU GLTexImage.h:125
//   * global defaults      GlobalUtil.cpp:50-135
// Used by the product host code (sgpu_capi) and by the CPU oracle, so both see the same taps.
#pragma once
#include <cmath>
#include <vector>

namespace sgp {

constexpr int kMaxFilterWidth = 33;  // ProgramCU.cu:40
constexpr int kMinFilterWidth = 5;   // ProgramCU.cu:41

// User-visible options.  Field meaning and defaults follow GlobalUtil.cpp:50-135 and the
// ParseParam switch at SiftGPU.cpp:801-1246 (the CLI letters are in the comments).
struct Options {
    float filter_width_factor = 4.0f;       // -f   GlobalUtil.cpp:61
    float descriptor_window_factor = 3.0f;  // -dw  GlobalUtil.cpp:62
    int subpixel = 1;                       // -s   GlobalUtil.cpp:63
    int max_orientation = 2;                // -m   GlobalUtil.cpp:64
    int fixed_orientation = 0;              // -ofix GlobalUtil.cpp:117
    int octave_min = 0;                     // -fo  GlobalUtil.cpp:111, -2 .. (SiftGPU.cpp:1074-1077)
    int octave_num = -1;                    // -no  GlobalUtil.cpp:112
    int dog_level_num = 3;                  // -d   SiftGPU.cpp:436
    float dog_threshold = 0.0f;             // -t   0 -> 0.02/d (SiftGPU.cpp:495)
    float edge_threshold = 0.0f;            // -e   0 -> 10     (SiftGPU.cpp:497)
    float orientation_window_factor = 2.0f; // -w   GlobalUtil.cpp:131
    float orientation_gaussian_factor = 1.5f; // GlobalUtil.cpp:132
    int lowe_origin = 0;                    // -loweo GlobalUtil.cpp:118
    int normalized = 1;                     // -unn/-ndes GlobalUtil.cpp:119
    int descriptors = 1;                    // -sd  (_DescriptorPPT != 0), GlobalUtil.cpp:99
    int keep_extremum_sign = 0;             // -sign GlobalUtil.cpp:122
    int circular_window = 0;                // 1: GLSL/upstream circular orientation window
                                            //    (ProgramCU-0.cu:834); 0: active ProgramCU.cu
};

// Derived scalar schedule (SiftParam after ParseSiftParam).
struct Schedule {
    int dog_level_num, level_min, level_max, level_num, level_ds;
    float sigma0, sigman, sigmak, dsigma0;
    float sigma_skip0, sigma_skip1;
    float sigma[16];        // filter sigma to go from level i to i+1 (i = level_min .. level_max-1)
    float dog_threshold, edge_threshold;
    float initial_smooth;   // GetInitialSmoothSigma(octave_min)
};

inline Schedule make_schedule(const Options& o) {
    Schedule s{};
    s.dog_level_num = o.dog_level_num > 0 ? o.dog_level_num : 3;
    s.level_min = -1;
    s.level_max = s.dog_level_num + 1;
    s.sigma0 = 1.6f * powf(2.0f, 1.0f / s.dog_level_num);
    s.sigman = 0.5f;
    s.level_num = s.level_max - s.level_min + 1;
    s.level_ds = s.level_min + s.dog_level_num;
    if (s.level_ds > s.level_max) s.level_ds = s.level_max;
    s.sigmak = powf(2.0f, 1.0f / s.dog_level_num);
    s.dsigma0 = s.sigma0 * sqrtf(1.0f - 1.0f / (s.sigmak * s.sigmak));
    float sa = s.sigma0 * powf(s.sigmak, (float)s.level_min);
    float sb = s.sigman / powf(2.0f, (float)o.octave_min);
    s.sigma_skip0 = sa > sb + 0.001 ? sqrtf(sa * sa - sb * sb) : 0.0f;
    sa = s.sigma0 * powf(s.sigmak, (float)s.level_min);
    sb = s.sigma0 * powf(s.sigmak, (float)(s.level_ds - s.dog_level_num));
    s.sigma_skip1 = sa > sb + 0.001 ? sqrtf(sa * sa - sb * sb) : 0.0f;
    for (int i = s.level_min + 1; i <= s.level_max; i++)
        s.sigma[i - s.level_min - 1] = s.dsigma0 * powf(s.sigmak, (float)i);
    s.dog_threshold = o.dog_threshold > 0 ? o.dog_threshold : 0.02f / s.dog_level_num;
    s.edge_threshold = o.edge_threshold > 0 ? o.edge_threshold : 10.0f;
    {  // GetInitialSmoothSigma(octave_min), SiftGPU.cpp:446-452
        float a = s.sigma0 * powf(2.0f, float(s.level_min) / float(s.dog_level_num));
        float b = s.sigman / powf(2.0f, float(o.octave_min));
        s.initial_smooth = a > b + 0.001 ? sqrtf(a * a - b * b) : 0.0f;
    }
    return s;
}

// GetLevelSigma(lev), SiftGPU.cpp:1285-1288.
inline float level_sigma(const Schedule& s, int lev) {
    return s.sigma0 * powf(2.0f, float(lev) / float(s.dog_level_num));
}

// CreateFilterKernel, ProgramCU.cu:375-403.  Returns the tap count; taps[0..width).
inline int make_filter(float sigma, float factor, float* taps) {
    int sz = int(std::ceil(factor * sigma - 0.5));
    int width = 2 * sz + 1;
    if (width > kMaxFilterWidth) { sz = kMaxFilterWidth >> 1; width = kMaxFilterWidth; }
    else if (width < kMinFilterWidth) { sz = kMinFilterWidth >> 1; width = kMinFilterWidth; }
    float rv = 1.0f / (sigma * sigma), v, ksum = 0;
    for (int i = -sz; i <= sz; ++i) {
        taps[i + sz] = v = expf(-0.5f * i * i * rv);
        ksum += v;
    }
    rv = 1.0f / ksum;
    for (int i = 0; i < width; i++) taps[i] *= rv;
    return width;
}

// One octave of the pyramid as the reference allocates it (PyramidCU.cpp:240-261):
// every level image is wa x h floats with wa = ((w+3)/4)*4.
struct Octave { int w, h, wa; };

// How the reference turns a w x h input into the first octave (GLTexInput::SetImageData,
// GLTexImage.cpp:918-1009, then PyramidCU::InitPyramid, PyramidCU.cpp:89-135):
//   * ds: with -fo > 0 and pre-processing on the CPU (-prep, the default: GlobalUtil.cpp:81) or
//     an input beyond _texMaxDim, the input is first sampled by 2^fo -- pixel (r << fo, c << fo)
//     -- and its width truncated to a multiple of 4 (DownSamplePixelDataI2F/F); the pyramid
//     then starts at octave 0 of that image with _down_sample_factor = fo;
//   * octave_min: otherwise -fo (>= -3) on the truncated input; in both cases raised by one
//     while the first octave is wider or taller than _texMaxDim (-maxd, 13200 in this fork,
//     GlobalUtil.cpp:86).
// Coordinates and the initial smoothing then use 2^(octave_min + ds)
// (GetInitialSmoothSigma(_octave_min + _down_sample_factor), PyramidCU.cpp:1009-1019, 463, 542).
struct InputPlan {
    int ds;           // CPU-side sampling exponent (0: none)
    int w, h;         // the image the pyramid starts from (after sampling; w % 4 == 0)
    int octave_min;   // first octave relative to that image
};

inline InputPlan plan_input(int w, int h, int fo, int max_dim, int prep_on_cpu) {
    InputPlan p;
    p.ds = (fo > 0 && (w > max_dim || h > max_dim || prep_on_cpu)) ? fo : 0;
    p.w = (w >> p.ds) & ~3;   // TruncateWidthCU (GLTexImage.h:125)
    p.h = h >> p.ds;
    p.octave_min = p.ds > 0 ? 0 : (fo < -3 ? -3 : fo);
    int wp = p.octave_min >= 0 ? p.w >> p.octave_min : p.w << -p.octave_min;
    int hp = p.octave_min >= 0 ? p.h >> p.octave_min : p.h << -p.octave_min;
    while (wp > max_dim || hp > max_dim) {
        p.octave_min++;
        wp >>= 1;
        hp >>= 1;
    }
    return p;
}

// Octave geometry for an input of w x h pixels (after plan_input).  The first octave is
// octave_min (-fo): its size is the truncated input shifted by octave_min, up-sampled for
// octave_min < 0 (PyramidCU::InitPyramid, PyramidCU.cpp:89-112; SiftGPU::AllocatePyramid,
// SiftGPU.cpp:1435-1448).  octave_num <= 0 selects floor(log2(min(w,h))) - 3 of that size
// (SiftPyramid::GetRequiredOctaveNum, SiftPyramid.cpp:279-285).
inline std::vector<Octave> make_octaves(int w, int h, int octave_num, int octave_min = 0) {
    w &= ~3;  // TruncateWidthCU (GLTexImage.h:125) via PyramidCU::InitPyramid:95
    int wp = octave_min >= 0 ? w >> octave_min : w << -octave_min;
    int hp = octave_min >= 0 ? h >> octave_min : h << -octave_min;
    int n = octave_num;
    if (n < 1) {
        int m = wp < hp ? wp : hp;
        n = (int)std::floor(std::log(double(m)) / std::log(2.0)) - 3;
        if (n < 1) n = 1;
    }
    std::vector<Octave> out;
    for (int i = 0; i < n; i++) {
        out.push_back(Octave{wp, hp, ((wp + 3) / 4) * 4});
        wp >>= 1;
        hp >>= 1;
    }
    return out;
}

}  // namespace sgp
