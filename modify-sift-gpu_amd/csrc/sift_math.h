// sift_math.h -- deterministic float32 math shared by the HIP kernels and the CPU oracle.
//
// Why this exists: the reference (SiftGPU/ProgramCU.cu) calls CUDA device libm (atan2f, expf,
// powf, __sincosf, rsqrt).  Neither CUDA's nor ROCm's device libm is bit-reproducible on the
// host, so every transcendental that runs per pixel / per feature is written here with only
// IEEE-exact primitives (+ - * /, fmaf, sqrtf, floorf, bit casts).  Compiled with
// -ffp-contract=off on both sides (g++ for the oracle, hipcc for gfx950) the HIP path and the
// oracle then produce identical bits.  Accuracy is ~1-2 ulp against libm (tests check that).
//
// SG_HD marks functions usable in host and device code; the header is plain C++ otherwise.
#pragma once
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define SG_HD __host__ __device__ __forceinline__
#else
#define SG_HD inline
#endif

namespace sgm {

SG_HD float as_float(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
SG_HD uint32_t as_uint(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

SG_HD float fma_(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
SG_HD float floor_(float x) { return __builtin_floorf(x); }
SG_HD float sqrt_(float x) { return __builtin_sqrtf(x); }
SG_HD float fabs_(float x) { return __builtin_fabsf(x); }
// IEEE minNum / maxNum (CUDA min()/max() on floats): a NaN operand is ignored.
SG_HD float fmin_(float a, float b) { return __builtin_fminf(a, b); }
SG_HD float fmax_(float a, float b) { return __builtin_fmaxf(a, b); }

// 2^k for integer k in [-149, 127], exact.
SG_HD float exp2i_(int k) {
    if (k >= -126) return as_float((uint32_t)(k + 127) << 23);
    return as_float(1u << (k + 149));  // subnormal power of two
}

// e^x core: Cody-Waite reduction x = k ln2 + r, |r| <= ln2/2, degree-7 Taylor in Horner form.
// Returns the polynomial; *ki = k.
SG_HD float exp_poly_(float x, int* ki) {
    const float kLog2e = 1.44269502f;
    const float kLn2Hi = 0.693145752f;      // 12 significant bits: k * kLn2Hi exact
    const float kLn2Lo = 1.42860677e-06f;
    float k = floor_(fma_(x, kLog2e, 0.5f));
    float r = fma_(k, -kLn2Hi, x);
    r = fma_(k, -kLn2Lo, r);
    float p = 1.98412698e-4f;               // 1/7!
    p = fma_(p, r, 1.38888889e-3f);         // 1/6!
    p = fma_(p, r, 8.33333333e-3f);         // 1/5!
    p = fma_(p, r, 4.16666667e-2f);         // 1/4!
    p = fma_(p, r, 1.66666667e-1f);         // 1/3!
    p = fma_(p, r, 0.5f);
    p = fma_(p, r, 1.0f);
    p = fma_(p, r, 1.0f);
    *ki = (int)k;
    return p;
}

// e^x.
SG_HD float exp_(float x) {
    if (!(x == x)) return x;  // NaN
    if (x > 88.7228394f) return as_float(0x7f800000u);
    if (x < -103.972084f) return 0.0f;
    int ki;
    const float p = exp_poly_(x, &ki);
    // scale in two exact steps so that subnormal results round once.
    if (ki < -125) return (p * exp2i_(ki + 64)) * exp2i_(-64);
    if (ki > 127) return (p * exp2i_(ki - 1)) * 2.0f;
    return p * exp2i_(ki);
}

// e^x for x in [-80, 80] (the Gaussian window weights): the same bits as exp_ there, without
// its range branches.
SG_HD float exp_mid_(float x) {
    int ki;
    const float p = exp_poly_(x, &ki);
    return p * as_float((uint32_t)(ki + 127) << 23);
}

// natural log for x > 0 (finite).  x = m 2^e with m in [sqrt(1/2), sqrt(2)), atanh series.
SG_HD float log_(float x) {
    if (!(x > 0.0f)) return (x == 0.0f) ? -as_float(0x7f800000u) : as_float(0x7fc00000u);
    if (x == as_float(0x7f800000u)) return x;
    uint32_t u = as_uint(x);
    int e = 0;
    if (u < 0x00800000u) { x = x * 16777216.0f; u = as_uint(x); e = -24; }  // subnormal
    e += (int)(u >> 23) - 127;
    u = (u & 0x007fffffu) | 0x3f800000u;
    float m = as_float(u);                  // [1, 2)
    if (m > 1.41421356f) { m = m * 0.5f; e += 1; }
    float f = m - 1.0f;
    float s = f / (2.0f + f);
    float z = s * s;
    float p = 0.0769230769f;                // 1/13
    p = fma_(p, z, 0.0909090909f);          // 1/11
    p = fma_(p, z, 0.111111111f);
    p = fma_(p, z, 0.142857143f);
    p = fma_(p, z, 0.2f);
    p = fma_(p, z, 0.333333333f);
    p = fma_(p, z, 1.0f);
    float lg = 2.0f * s * p;
    const float kLn2Hi = 0.693145752f, kLn2Lo = 1.42860677e-06f;
    float fe = (float)e;
    return fma_(fe, kLn2Hi, fma_(fe, kLn2Lo, lg));
}

// a^b for a > 0 (the only use is pow(sigma_step, ds), ProgramCU.cu:847).
SG_HD float pow_(float a, float b) { return exp_(b * log_(a)); }

// atan2(y, x) in (-pi, pi].  With a = min(|x|,|y|), b = max(|x|,|y|): t = a / b, or
// t = (a - b) / (a + b) (angle - pi/4) when a > tan(pi/8) b, so |t| <= tan(pi/8); odd Taylor
// series to t^19.  One division and no data-dependent branches (selects only).
SG_HD float atan2_(float y, float x) {
    const float kPi = 3.14159265f, kPi2 = 1.57079633f, kPi4 = 0.785398163f;
    const float ax = fabs_(x), ay = fabs_(y);
    const bool swap = ay > ax;
    const float mx = swap ? ay : ax, mn = swap ? ax : ay;
    const bool red = mn > 0.414213562f * mx;
    const float t = (red ? mn - mx : mn) / (red ? mn + mx : mx);
    const float z = t * t;
    float p = -0.0526315789f;            // -1/19
    p = fma_(p, z, 0.0588235294f);       //  1/17
    p = fma_(p, z, -0.0666666667f);      // -1/15
    p = fma_(p, z, 0.0769230769f);       //  1/13
    p = fma_(p, z, -0.0909090909f);      // -1/11
    p = fma_(p, z, 0.111111111f);        //  1/9
    p = fma_(p, z, -0.142857143f);       // -1/7
    p = fma_(p, z, 0.2f);                //  1/5
    p = fma_(p, z, -0.333333333f);       // -1/3
    float r = fma_(p * z, t, t) + (red ? kPi4 : 0.0f);
    r = swap ? kPi2 - r : r;
    const bool xneg = (as_uint(x) >> 31) != 0;
    r = xneg ? kPi - r : r;
    r = mx == 0.0f ? (xneg ? kPi : 0.0f) : r;
    r = (as_uint(y) >> 31) ? -r : r;
    return (ax == ax && ay == ay) ? r : x + y;
}

// sin and cos of x (|x| < 1e5), Cody-Waite with a 3-part pi/2.
SG_HD void sincos_(float x, float* s, float* c) {
    const float k2Pi = 0.636619772f;
    const float kP1 = 1.5703125f, kP2 = 4.83751297e-04f, kP3 = 7.54978942e-08f;
    float k = floor_(fma_(x, k2Pi, 0.5f));
    float r = fma_(k, -kP1, x);
    r = fma_(k, -kP2, r);
    r = fma_(k, -kP3, r);
    float z = r * r;
    float ps = -2.50521084e-08f;             // -1/11!
    ps = fma_(ps, z, 2.75573192e-06f);       //  1/9!
    ps = fma_(ps, z, -1.98412698e-04f);      // -1/7!
    ps = fma_(ps, z, 8.33333333e-03f);       //  1/5!
    ps = fma_(ps, z, -1.66666667e-01f);      // -1/3!
    float sr = fma_(ps * z, r, r);
    float pc = 2.08767570e-09f;              //  1/12!
    pc = fma_(pc, z, -2.75573192e-07f);      // -1/10!
    pc = fma_(pc, z, 2.48015873e-05f);       //  1/8!
    pc = fma_(pc, z, -1.38888889e-03f);      // -1/6!
    pc = fma_(pc, z, 4.16666667e-02f);       //  1/4!
    pc = fma_(pc, z, -0.5f);
    float cr = fma_(pc, z, 1.0f);
    int q = ((int)k) & 3;
    float so, co;
    if (q == 0) { so = sr; co = cr; }
    else if (q == 1) { so = cr; co = -sr; }
    else if (q == 2) { so = -sr; co = -cr; }
    else { so = -cr; co = sr; }
    *s = so; *c = co;
}

// 1/sqrt(x) with two IEEE roundings (replaces CUDA rsqrt, ProgramCU.cu:1187,1200).
SG_HD float rsqrt_(float x) { return 1.0f / sqrt_(x); }

}  // namespace sgm
