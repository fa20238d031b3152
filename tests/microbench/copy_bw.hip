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

// wave-owned strips (the k_gauss_wave pattern): each wave walks one strip of SW columns over a
// band of BR rows, float4 per lane (SW / 4 lanes per row, 256 / SW rows per load), 8-row chunks
// with the next chunk's loads issued before the current chunk's stores
template <int SW>
__global__ __launch_bounds__(256) void wave_strip(const float* __restrict__ a, float* __restrict__ b,
                                                  int W, int H, int BR) {
    constexpr int LPR = SW / 4;          // lanes per row
    constexpr int RPL = 64 / LPR;        // rows per load instruction
    constexpr int LD = 8 / RPL > 0 ? 8 / RPL : 1;   // loads per 8-row chunk
    const int lane = threadIdx.x & 63;
    const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int strips = W / SW, bands = (H + BR - 1) / BR;
    const int sx = gw % strips, rest = gw / strips, band = rest % bands, img = rest / bands;
    if (img >= 128) return;
    const float4* s = reinterpret_cast<const float4*>(a + (size_t)img * W * H + sx * SW);
    float4* d = reinterpret_cast<float4*>(b + (size_t)img * W * H + sx * SW);
    const int W4 = W / 4, c = lane % LPR, rr = lane / LPR;
    const int y0 = band * BR, y1 = min(H, y0 + BR);
    float4 cur[LD], nxt[LD];
#pragma unroll
    for (int k = 0; k < LD; k++) cur[k] = s[(size_t)min(y0 + k * RPL + rr, H - 1) * W4 + c];
    for (int y = y0; y < y1; y += LD * RPL) {
#pragma unroll
        for (int k = 0; k < LD; k++) nxt[k] = s[(size_t)min(y + LD * RPL + k * RPL + rr, H - 1) * W4 + c];
#pragma unroll
        for (int k = 0; k < LD; k++) {
            const int yy = y + k * RPL + rr;
            if (yy < y1) d[(size_t)yy * W4 + c] = cur[k];
        }
#pragma unroll
        for (int k = 0; k < LD; k++) cur[k] = nxt[k];
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
    for (int br : {270, 540, 1080}) {
        char nm[64];
        auto waves = [&](int sw) { return (size_t)N * (W / sw) * ((H + br - 1) / br); };
        snprintf(nm, sizeof nm, "wave strip 64 cols, %d rows", br);
        run(nm, [&] { wave_strip<64><<<(waves(64) + 3) / 4, 256>>>(a, b, W, H, br); });
        snprintf(nm, sizeof nm, "wave strip 128 cols, %d rows", br);
        run(nm, [&] { wave_strip<128><<<(waves(128) + 3) / 4, 256>>>(a, b, W, H, br); });
        snprintf(nm, sizeof nm, "wave strip 256 cols, %d rows", br);
        run(nm, [&] { wave_strip<256><<<(waves(256) + 3) / 4, 256>>>(a, b, W, H, br); });
    }
    return 0;
}
