// perturb.h -- test infrastructure only (oracle/Makefile: liboracle_perturb.so, force-included
// into sift_oracle.cpp with -include).  The oracle's transcendentals with the error bounds of the
// CUDA device functions the reference calls, to measure how far the parity of this repository
// (HIP path == oracle, bit for bit) can be trusted against the real CUDA binary, which cannot be
// built here (tests/parity_trust.py):
//   __sincosf (ProgramCU.cu:1024)  absolute error up to 2^-21.41 on [-pi, pi]
//   expf                           2 ulp      atan2f   3 ulp
//   powf                           2 ulp      rsqrtf   2 ulp
// Each result moves by a pseudo-random, input-determined amount within its bound, so a run is
// reproducible and the perturbation is independent between call sites.
#pragma once
#include <math.h>
#include "../modify-sift-gpu_amd/csrc/sift_math.h"

namespace sgm {
inline uint32_t pert_hash_(uint32_t x, uint32_t salt) {
    x ^= salt * 0x9e3779b9u;
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
// r moved by k ulp, k uniform in [-max_ulp, max_ulp] from the input bits
inline float pert_ulp_(float r, uint32_t in_bits, uint32_t salt, int max_ulp) {
    const int k = (int)(pert_hash_(in_bits, salt) % (uint32_t)(2 * max_ulp + 1)) - max_ulp;
    for (int i = 0; i < k; i++) r = nextafterf(r, INFINITY);
    for (int i = 0; i > k; i--) r = nextafterf(r, -INFINITY);
    return r;
}
inline float pert_exp_(float x) { return pert_ulp_(exp_(x), as_uint(x), 1u, 2); }
inline float pert_atan2_(float y, float x) {
    return pert_ulp_(atan2_(y, x), as_uint(y) * 31u + as_uint(x), 2u, 3);
}
inline float pert_pow_(float a, float b) {
    return pert_ulp_(pow_(a, b), as_uint(a) * 31u + as_uint(b), 3u, 2);
}
inline float pert_rsqrt_(float x) { return pert_ulp_(rsqrt_(x), as_uint(x), 4u, 2); }
inline void pert_sincos_(float x, float* s, float* c) {
    sincos_(x, s, c);
    const float e = 3.6e-7f;   // 2^-21.41
    const uint32_t h = pert_hash_(as_uint(x), 5u);
    *s += e * ((float)(h & 0xffffu) / 32767.5f - 1.0f);
    *c += e * ((float)(h >> 16) / 32767.5f - 1.0f);
}
}  // namespace sgm

#define exp_(x) pert_exp_(x)
#define atan2_(y, x) pert_atan2_(y, x)
#define pow_(a, b) pert_pow_(a, b)
#define rsqrt_(x) pert_rsqrt_(x)
#define sincos_(x, s, c) pert_sincos_(x, s, c)
