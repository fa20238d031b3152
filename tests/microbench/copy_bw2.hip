// HBM calibration, round 2: which copy form reaches the guide's 6.29 TB/s (MI355X_MICROARCH.md,
// "float4 copy") on 128 x 1920 x 1080 f32 (1.06 GB read + 1.06 GB written).
//   hipcc -O3 --offload-arch=gfx950 copy_bw2.hip -o copy_bw2 && ./copy_bw2
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

// one float4 per thread, no loop
__global__ __launch_bounds__(256) void copy_flat(const f4* __restrict__ a, f4* __restrict__ b, size_t n) {
    const size_t i = blockIdx.x * (size_t)256 + threadIdx.x;
    if (i < n) b[i] = a[i];
}
// U float4 per thread, loads first (U in flight), blocks of 256*U consecutive float4
template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_unroll(const f4* __restrict__ a, f4* __restrict__ b, size_t n) {
    const size_t base = blockIdx.x * (size_t)(256 * U) + threadIdx.x;
    f4 v[U];
#pragma unroll
    for (int k = 0; k < U; k++) {
        const size_t i = base + (size_t)k * 256;
        if (NT) v[k] = i < n ? __builtin_nontemporal_load(a + i) : f4{0, 0, 0, 0};
        else v[k] = i < n ? a[i] : f4{0, 0, 0, 0};
    }
#pragma unroll
    for (int k = 0; k < U; k++) {
        const size_t i = base + (size_t)k * 256;
        if (i < n) {
            if (NT) __builtin_nontemporal_store(v[k], b + i);
            else b[i] = v[k];
        }
    }
}
// read-only: sum of float4 (HBM read rate)
__global__ __launch_bounds__(256) void read_unroll(const f4* __restrict__ a, float* __restrict__ out, size_t n) {
    const size_t base = blockIdx.x * (size_t)(256 * 4) + threadIdx.x;
    f4 s = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const size_t i = base + (size_t)k * 256;
        if (i < n) s += a[i];
    }
    const float t = s.x + s.y + s.z + s.w;
    if (t == 12345.f) out[0] = t;
}
// write-only
__global__ __launch_bounds__(256) void write_unroll(f4* __restrict__ b, size_t n) {
    const size_t base = blockIdx.x * (size_t)(256 * 4) + threadIdx.x;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const size_t i = base + (size_t)k * 256;
        if (i < n) b[i] = f4{1, 2, 3, 4};
    }
}

int main() {
    const size_t n = (size_t)1920 * 1080 * 128;   // floats
    const size_t n4 = n / 4;
    float *a, *b, *o;
    hipMalloc(&a, n * 4);
    hipMalloc(&b, n * 4);
    hipMalloc(&o, 64);
    hipMemset(a, 0, n * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char* name, double bytes, auto launch) {
        launch();
        hipDeviceSynchronize();
        float best = 1e9f;
        for (int r = 0; r < 7; r++) {
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            best = ms < best ? ms : best;
        }
        printf("%-36s %8.1f us  %6.2f TB/s\n", name, best * 1e3, bytes / (best * 1e-3) / 1e12);
    };
    const double cp = 2.0 * n * 4;
    run("copy flat float4", cp, [&] { copy_flat<<<(unsigned)((n4 + 255) / 256), 256>>>((const f4*)a, (f4*)b, n4); });
    run("copy unroll2 float4", cp, [&] { copy_unroll<2, false><<<(unsigned)((n4 + 511) / 512), 256>>>((const f4*)a, (f4*)b, n4); });
    run("copy unroll4 float4", cp, [&] { copy_unroll<4, false><<<(unsigned)((n4 + 1023) / 1024), 256>>>((const f4*)a, (f4*)b, n4); });
    run("copy unroll8 float4", cp, [&] { copy_unroll<8, false><<<(unsigned)((n4 + 2047) / 2048), 256>>>((const f4*)a, (f4*)b, n4); });
    run("copy unroll4 float4 nontemporal", cp, [&] { copy_unroll<4, true><<<(unsigned)((n4 + 1023) / 1024), 256>>>((const f4*)a, (f4*)b, n4); });
    run("read unroll4 float4", n * 4.0, [&] { read_unroll<<<(unsigned)((n4 + 1023) / 1024), 256>>>((const f4*)a, o, n4); });
    run("write unroll4 float4", n * 4.0, [&] { write_unroll<<<(unsigned)((n4 + 1023) / 1024), 256>>>((f4*)b, n4); });
    return 0;
}
