// sift_keys.h -- device-side keypoint helpers shared by the product kernels (sift_kernels.hip)
// and the test-hook library's candidate dump (sgpu_debug.hip): ComputeKEY_Kernel's state machine
// (key_test) and the (image, octave, level, row, column) of a scanned keypoint slot (locate,
// key_at).  Included after sift_kernels.h and sift_math.h (`using namespace sgm`).
#pragma once

namespace sgk {
namespace {

// ------------------------------------------------------------------------------------------
// ComputeKEY_Kernel (ProgramCU.cu:553-671): extremum state machine + edge test + subpixel
// solve on 27 DoG values.  get(m, r, c): m = 0 previous / 1 current / 2 next DoG level,
// r, c in {0,1,2} around the pixel.  The READ_CMP_DOG_DATA order (:534-550) is kept because it
// decides ties.
struct KeyOut { float result, dx, dy, ds; };

template <class Get>
__device__ __forceinline__ KeyOut key_test(Get get, float t0, float t, float edge, int subpixel) {
    KeyOut o{0.f, 0.f, 0.f, 0.f};
    const float v = get(1, 1, 1);
    if (fabs_(v) <= t0) return o;
    const float l = get(1, 1, 0), r = get(1, 1, 2);
    float nmax = fmax_(l, r), nmin = fmin_(l, r);
    if (v <= nmax && v >= nmin) return o;
    // the 9 row-triples in reference order: cur r0, cur r2, [edge test], prev r0..2, next r0..2
    const int seq_m[8] = {1, 1, 0, 0, 0, 2, 2, 2};
    const int seq_r[8] = {0, 2, 0, 1, 2, 0, 1, 2};
#pragma unroll
    for (int s = 0; s < 8; s++) {
        if (s == 2) {
            const float vx2 = v * 2.0f;
            const float fxx = l + r - vx2;
            const float fyy = get(1, 0, 1) + get(1, 2, 1) - vx2;
            const float fxy = 0.25f * (get(1, 2, 2) + get(1, 0, 0) - get(1, 2, 0) - get(1, 0, 2));
            const float temp1 = fma_(fxx, fyy, -(fxy * fxy));
            const float temp2 = (fxx + fyy) * (fxx + fyy);
            if (temp1 <= 0 || temp2 > edge * temp1) return o;
        }
        const float a = get(seq_m[s], seq_r[s], 0), bb = get(seq_m[s], seq_r[s], 1),
                    cc = get(seq_m[s], seq_r[s], 2);
        if (v > nmax) {
            nmax = fmax_(fmax_(fmax_(nmax, a), bb), cc);
            if (v < nmax) return o;
        } else {
            nmin = fmin_(fmin_(fmin_(nmin, a), bb), cc);
            if (v > nmin) return o;
        }
    }
    bool ok = true;
    float dx = 0.f, dy = 0.f, ds = 0.f;
    if (subpixel) {
        const float vx2 = v * 2.0f;
        const float fxx = l + r - vx2;
        const float fyy = get(1, 0, 1) + get(1, 2, 1) - vx2;
        const float fxy = 0.25f * (get(1, 2, 2) + get(1, 0, 0) - get(1, 2, 0) - get(1, 0, 2));
        const float fx = 0.5f * (r - l);
        const float fy = 0.5f * (get(1, 2, 1) - get(1, 0, 1));
        const float pc = get(0, 1, 1), nc = get(2, 1, 1);
        const float fs = 0.5f * (nc - pc);
        const float fss = (nc + pc - vx2);
        const float fxs = 0.25f * (get(2, 1, 2) + get(0, 1, 0) - get(2, 1, 0) - get(0, 1, 2));
        const float fys = 0.25f * (get(2, 2, 1) + get(0, 0, 1) - get(2, 0, 1) - get(0, 2, 1));
        float4 A0 = fxx > 0 ? make_float4(fxx, fxy, fxs, -fx) : make_float4(-fxx, -fxy, -fxs, fx);
        float4 A1 = fxy > 0 ? make_float4(fxy, fyy, fys, -fy) : make_float4(-fxy, -fyy, -fys, fy);
        float4 A2 = fxs > 0 ? make_float4(fxs, fys, fss, -fs) : make_float4(-fxs, -fys, -fss, fs);
        const float maxa = fmax_(fmax_(A0.x, A1.x), A2.x);
        if ((double)maxa >= 1e-10) {   // double compare, as the reference's literal
            if (maxa == A1.x) { float4 T = A1; A1 = A0; A0 = T; }
            else if (maxa == A2.x) { float4 T = A2; A2 = A0; A0 = T; }
            A0.y /= A0.x; A0.z /= A0.x; A0.w /= A0.x;
            A1.y = fma_(-A1.x, A0.y, A1.y); A1.z = fma_(-A1.x, A0.z, A1.z); A1.w = fma_(-A1.x, A0.w, A1.w);
            A2.y = fma_(-A2.x, A0.y, A2.y); A2.z = fma_(-A2.x, A0.z, A2.z); A2.w = fma_(-A2.x, A0.w, A2.w);
            if (fabs_(A2.y) > fabs_(A1.y)) { float4 T = A2; A2 = A1; A1 = T; }
            if ((double)fabs_(A1.y) >= 1e-10) {
                A1.z /= A1.y; A1.w /= A1.y;
                A2.z = fma_(-A2.y, A1.z, A2.z); A2.w = fma_(-A2.y, A1.w, A2.w);
                if ((double)fabs_(A2.z) >= 1e-10) {
                    ds = A2.w / A2.z;
                    dy = fma_(-ds, A1.z, A1.w);
                    dx = fma_(-dy, A0.y, fma_(-ds, A0.z, A0.w));
                    const float dot = fma_(ds, fs, fma_(dx, fx, dy * fy));
                    ok = fabs_(fma_(0.5f, dot, v)) > t && fabs_(ds) < 1.0f &&
                         fabs_(dx) < 1.0f && fabs_(dy) < 1.0f;
                }
            }
        }
    }
    if (ok) o.result = v > nmax ? 1.0f : -1.0f;
    o.dx = dx; o.dy = dy; o.ds = ds;
    return o;
}

// Locate keypoint f: the row whose scanned base <= f (binary search), then the k-th set bit.
struct KeyLoc { int b, o, j, row, col; };

// (image, octave, level, row) of global row id `lo` = the index into row_count / row_base
__device__ __forceinline__ KeyLoc row_loc(int lo, const FeatureParams& fp) {
    KeyLoc L;
    L.b = lo / fp.rows_per_image;
    int rem = lo - L.b * fp.rows_per_image;
    int o = 0;
    while (o + 1 < fp.n_octaves && fp.row_off[o + 1] <= rem) o++;
    L.o = o;
    rem -= fp.row_off[o];
    const OctaveDesc& od = fp.oct[o];
    L.j = rem / od.h;
    L.row = rem - L.j * od.h;
    L.col = 0;
    return L;
}

// Locate keypoint f by binary search over the scanned row counts and the k-th set bit of its
// mask row.  (A separate list kernel that writes every keypoint's (row, column) from the mask
// measured 84 us per 128 x 1080p against the ~24 us the searches cost inside k_orientation.)
__device__ __forceinline__ KeyLoc locate(uint32_t f, const uint32_t* __restrict__ row_base,
                                         int total_rows, const uint32_t* __restrict__ mask,
                                         const FeatureParams& fp) {
    int lo = 0, hi = total_rows;   // find last index with row_base[idx] <= f
    while (hi - lo > 1) {
        int mid = (lo + hi) >> 1;
        if (row_base[mid] <= f) lo = mid; else hi = mid;
    }
    KeyLoc L = row_loc(lo, fp);
    uint32_t k = f - row_base[lo];
    const OctaveDesc& od = fp.oct[L.o];
    const uint32_t* mrow = mask + od.mask_off + L.j * od.mask_level_stride +
                           ((long long)L.b * od.h + L.row) * od.nwords;
    int col = 0;
    for (int w = 0; w < od.nwords; w++) {
        uint32_t m = mrow[w];
        uint32_t c = __popc(m);
        if (k < c) {
            for (uint32_t q = 0; q < k; q++) m &= m - 1;
            col = w * 32 + (__ffs(m) - 1);
            break;
        }
        k -= c;
    }
    L.col = col;
    return L;
}

// Recompute (result, dx, dy, ds) of a located keypoint from the Gaussian planes.
__device__ __forceinline__ KeyOut key_at(const float* __restrict__ pyr, const FeatureParams& fp,
                                         const KeyLoc& L) {
    const OctaveDesc& od = fp.oct[L.o];
    const long long npx = (long long)od.wa * od.h;
    const float* g = pyr + od.gauss_off + (long long)L.b * npx + (long long)L.row * od.wa + L.col;
    // DoG plane (1 + j + m) = G[1+j+m] - G[j+m]
    auto get = [&](int m, int r, int c) {
        const long long p = (long long)(r - 1) * od.wa + (c - 1);
        const float* gm = g + (long long)(L.j + m) * od.level_stride;
        return gm[od.level_stride + p] - gm[p];
    };
    return key_test(get, fp.t0, fp.t, fp.edge, fp.subpixel);
}

}  // namespace
}  // namespace sgk
