// sift_oracle.h -- CPU restatement of the SiftGPU CUDA hot path.
//
// TEST INFRASTRUCTURE ONLY.  This is the checker the HIP path is compared against; it is never
// linked into libsiftgpu.so and nothing in the product calls it.  Only tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it (oracle/liboracle.so).
//
// Parity status: the reference (CUDA + OpenGL) cannot be compiled or run anywhere in this
// pipeline (no nvcc, no NVIDIA GPU, GL/glew.h and DevIL absent), and it ships
// no tests or fixtures.  The restatement is pinned by the known-answer values the reference
// itself states (sigma schedule SiftGPU.cpp:459-497, octave geometry PyramidCU.cpp:985,
// histopyramid widths PyramidCU.cpp:346-348/773) and cross-checked against an independent
// float64 NumPy restatement (tests/ref_numpy.py); everything beyond those pins is
// "parity unpinned" against the CUDA binary itself.  See DESIGN.md §3.
#pragma once
#include <cstdint>
#include <vector>

#include "../include/sgpu.h"
#include "../modify-sift-gpu_amd/csrc/sift_params.h"

namespace oracle {

struct Image {
    int w = 0, h = 0;
    std::vector<float> px;
    float at(int x, int y) const { return px[(size_t)y * w + x]; }
};

struct Candidate {   // one entry of the reference's per-level feature list (int4 + key float4)
    int col, row;
    float dx, dy, ds;
};

struct LevelResult {
    int octave, level;                 // level j in [0, dog_level_num)
    std::vector<Candidate> candidates; // raster order (histopyramid output, ListGen_Kernel)
    std::vector<float> oriented;       // 4 floats per candidate after ComputeOrientation_Kernel
                                       // (x, y, s, packed-orientation bits or angle)
};

struct Result {
    std::vector<sgp::Octave> octaves;
    std::vector<std::vector<Image>> gauss;  // [octave][level]
    std::vector<LevelResult> levels;        // octave-major
    std::vector<float> keys;                // 4 per feature (x, y, s, o), image coordinates
    std::vector<float> feat_oct;            // 4 per feature, octave coordinates (descriptor input)
    std::vector<int> feat_level;            // level index (octave*d + j) per feature
    std::vector<float> desc;                // 128 per feature
};

// Runs the whole pipeline on one gray u8 image.  keep_intermediates=false drops the pyramid.
// With img_f32 (and img == nullptr) the input is float luminance, row stride `stride` floats
// (the GL_FLOAT / host-converted path of GLTexInput::SetImageData, GLTexImage.cpp:981-1006).
Result extract(const uint8_t* img, int w, int h, int stride, const sgpu_options& opt,
               bool keep_intermediates = true, const float* img_f32 = nullptr);

// Descriptors (and, without orientations, the strongest orientation) of caller-supplied
// keypoints on image img (SiftGPU::RunSIFT(num, keys, keys_have_orientation)).  Returns the
// descriptors [num][128] in input order; *keys_out gets the keys as the reference returns them.
std::vector<float> describe_keys(const uint8_t* img, int w, int h, int stride,
                                 const sgpu_options& opt, const float* keys, int num,
                                 int has_orientation, std::vector<float>* keys_out);

// Matcher (SiftMatchCU::GetSiftMatch + GetBestMatch).  Returns pairs {i, j}, ascending i.
std::vector<int> match(const uint8_t* d1, int n1, const uint8_t* d2, int n2, float distmax,
                       float ratiomax, int mbm, int max_match);

// Guided matching (SiftMatchCU::GetGuidedSiftMatch): loc1/loc2 (x, y) per feature, H and F
// row-major 3x3.
std::vector<int> match_guided(const uint8_t* d1, int n1, const uint8_t* d2, int n2,
                              const float* loc1, const float* loc2, const float* H,
                              const float* F, float distmax, float ratiomax, float hdistmax,
                              float fdistmax, int mbm, int max_match);
bool guided_pass(const float* H, const float* F, float x1, float y1, float x2, float y2,
                 float hdistmax, float fdistmax);

// acos distance table shared with the HIP path's definition: dist[v] for dot v in [0, 262144].
float match_distance(int dot);

}  // namespace oracle
