// HBM calibration on the GPU box: linear float4 / float copies and the strip-walk pattern of the
// Gaussian kernel (64-column strips, rows walked top to bottom), all on 128 x 1920 x 1080 f32.
//   hipcc -O3 --offload-arch=gfx950 copy_bw.hip -o copy_bw && ./copy_bw
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void copy4(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b[i] = a[i];
}
__global__ void copy1(const float* __restrict__ a, float* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b[i] = a[i];
}
// one WG per (image, 64-col strip): 256 threads = 4 rows x 64 columns per step, f32
__global__ void strip_copy(const float* __restrict__ a, float* __restrict__ b, int W, int H) {
    const int strips = W / 64;
    const int sx = blockIdx.x % strips, img = blockIdx.x / strips;
    const float* s = a + (size_t)img * W * H + sx * 64;
    float* d = b + (size_t)img * W * H + sx * 64;
    const int c = threadIdx.x & 63, r0 = threadIdx.x >> 6;
    for (int y = r0; y < H; y += 16) {
        float v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) v[k] = (y + 4 * k < H) ? s[(size_t)(y + 4 * k) * W + c] : 0.f;
#pragma unroll
        for (int k = 0; k < 4; k++) if (y + 4 * k < H) d[(size_t)(y + 4 * k) * W + c] = v[k];
    }
}
// same with 128-column strips, float2 per lane
__global__ void strip_copy2(const float* __restrict__ a, float* __restrict__ b, int W, int H) {
    const int strips = W / 128;
    const int sx = blockIdx.x % strips, img = blockIdx.x / strips;
    const float2* s = reinterpret_cast<const float2*>(a + (size_t)img * W * H + sx * 128);
    float2* d = reinterpret_cast<float2*>(b + (size_t)img * W * H + sx * 128);
    const int c = threadIdx.x & 63, r0 = threadIdx.x >> 6;
    const int W2 = W / 2;
    for (int y = r0; y < H; y += 16) {
        float2 v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) v[k] = (y + 4 * k < H) ? s[(size_t)(y + 4 * k) * W2 + c] : make_float2(0.f, 0.f);
#pragma unroll
        for (int k = 0; k < 4; k++) if (y + 4 * k < H) d[(size_t)(y + 4 * k) * W2 + c] = v[k];
    }
}

int main() {
    const int W = 1920, H = 1080, N = 128;
    const size_t n = (size_t)W * H * N;
    float *a, *b;
    hipMalloc(&a, n * 4);
    hipMalloc(&b, n * 4);
    hipMemset(a, 0, n * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char* name, auto launch) {
        launch();
        hipDeviceSynchronize();
        float best = 1e9f;
        for (int r = 0; r < 5; r++) {
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            best = ms < best ? ms : best;
        }
        printf("%-28s %8.1f us  %6.2f TB/s (read+write)\n", name, best * 1e3, 2.0 * n * 4 / (best * 1e-3) / 1e12);
    };
    run("copy float4 grid-stride", [&] { copy4<<<8192, 256>>>((const float4*)a, (float4*)b, n / 4); });
    run("copy float grid-stride", [&] { copy1<<<8192, 256>>>(a, b, n); });
    run("strip copy 64 cols f32", [&] { strip_copy<<<N * (W / 64), 256>>>(a, b, W, H); });
    run("strip copy 128 cols f2", [&] { strip_copy2<<<N * (W / 128), 256>>>(a, b, W, H); });
    return 0;
}
