// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths the
// pyramid kernels use (MI355X_MICROARCH.md, HBM section: FETCH_SIZE reports 1/2 of the bytes of a
// 16-B-per-lane streaming read; other widths uncalibrated).  Each kernel streams a known byte
// count once over a 1 GiB buffer (well past the 256 MiB Infinity Cache):
//   read16 / read8 / read4  -- one float4 / float2 / u32 load per lane, grid-strided, coalesced
//   write16 / write8 / write4 -- the same widths as stores
// Run under separate --pmc FETCH_SIZE and --pmc WRITE_SIZE passes (tests/pmc_calib.sh); the
// summary divides each counter by the known bytes.
//   hipcc -O3 --offload-arch=gfx950 pmc_calib.hip -o pmc_calib && ./pmc_calib
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

template <class T>
__device__ __forceinline__ float fold(T v) { return (float)v; }
template <>
__device__ __forceinline__ float fold(f4 v) { return v.x + v.y + v.z + v.w; }
template <>
__device__ __forceinline__ float fold(f2 v) { return v.x + v.y; }
template <>
__device__ __forceinline__ float fold(uint32_t v) { return (float)(v & 255u); }

template <class T>
__global__ __launch_bounds__(256) void k_read(const T* __restrict__ a, size_t n, float* __restrict__ out) {
    float s = 0.f;
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        s += fold(a[i]);
    if (s == 1234.5f) out[0] = s;   // keeps the loads live, never true for the zeroed buffer
}

template <class T>
__global__ __launch_bounds__(256) void k_write(T* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        b[i] = T{};
}

#define CHK(x)                                                                   \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
            return 1;                                                            \
        }                                                                        \
    } while (0)

int main() {
    const size_t bytes = (size_t)1 << 30;
    void* buf = nullptr;
    float* out = nullptr;
    CHK(hipMalloc(&buf, bytes));
    CHK(hipMalloc(&out, 256));
    CHK(hipMemset(buf, 0, bytes));
    CHK(hipDeviceSynchronize());
    const dim3 grid(8192), block(256);
    // each kernel once; the profiler attributes counters per dispatch
    hipLaunchKernelGGL(k_read<f4>, grid, block, 0, 0, (const f4*)buf, bytes / 16, out);
    hipLaunchKernelGGL(k_read<f2>, grid, block, 0, 0, (const f2*)buf, bytes / 8, out);
    hipLaunchKernelGGL(k_read<uint32_t>, grid, block, 0, 0, (const uint32_t*)buf, bytes / 4, out);
    hipLaunchKernelGGL(k_write<f4>, grid, block, 0, 0, (f4*)buf, bytes / 16);
    hipLaunchKernelGGL(k_write<f2>, grid, block, 0, 0, (f2*)buf, bytes / 8);
    hipLaunchKernelGGL(k_write<uint32_t>, grid, block, 0, 0, (uint32_t*)buf, bytes / 4);
    CHK(hipGetLastError());
    CHK(hipDeviceSynchronize());
    printf("pmc_calib: 6 kernels, %zu bytes each\n", bytes);
    CHK(hipFree(buf));
    CHK(hipFree(out));
    return 0;
}
