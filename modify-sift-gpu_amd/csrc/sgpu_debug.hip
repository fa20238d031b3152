// sgpu_debug.hip -- test hooks kept out of the product library: lib/libsiftgpu_debug.so, loaded
// by sgpu_debug_candidates (sgpu_capi.cpp) on first use.  The keypoint candidates of the
// orientation stage with their ComputeKEY results, for tests/test_gpu_parity.py's bitwise
// candidate checks against the oracle (ProgramCU.cu:553-671 via sift_keys.h).
#include <cstdint>

#include "sift_kernels.h"
#include "sift_math.h"

using namespace sgm;

#include "sift_keys.h"

namespace sgk {
namespace {

__global__ __launch_bounds__(64) void k_debug_candidates(
    const float* __restrict__ pyr, const uint32_t* __restrict__ mask,
    const uint32_t* __restrict__ row_base, int total_rows, const uint32_t* __restrict__ n_cand_dev,
    const FeatureParams fp, int4* __restrict__ ints, float4* __restrict__ floats) {
    const uint32_t f = blockIdx.x * 64 + threadIdx.x;
    if (f >= *n_cand_dev) return;
    const KeyLoc L = locate(f, row_base, total_rows, mask, fp);
    const KeyOut kv = key_at(pyr, fp, L);
    ints[f] = make_int4(L.col, L.row, L.o * fp.d + L.j, L.b);
    floats[f] = make_float4(kv.dx, kv.dy, kv.ds, kv.result);
}

}  // namespace
}  // namespace sgk

extern "C" __attribute__((visibility("default"))) hipError_t sgpu_testhook_candidates(
    const float* pyr, const uint32_t* mask, const uint32_t* row_base, int total_rows,
    const uint32_t* n_cand_dev, int n_cand_cap, const sgk::FeatureParams* fp, int4* ints,
    float4* floats, hipStream_t stream) {
    if (n_cand_cap <= 0) return hipSuccess;
    hipLaunchKernelGGL(sgk::k_debug_candidates, dim3((n_cand_cap + 63) / 64), dim3(64), 0, stream,
                       pyr, mask, row_base, total_rows, n_cand_dev, *fp, ints, floats);
    return hipGetLastError();
}
