// Read-pattern calibration on the GPU box: the extremum kernel reads 6 Gaussian planes
// (128 x 1920 x 1080 f32 each) in 64x16 tiles with a 1-pixel halo.  Compares a linear float4
// read of the same bytes, a plain row-aligned tile walk, and the halo tile walk.
//   hipcc -O3 --offload-arch=gfx950 read_bw.hip -o read_bw && ./read_bw
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void read_linear(const float4* __restrict__ a, size_t n, float* out) {
    float s = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        float4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 1234.5f) out[0] = s;
}

// one WG per (image, 64-col strip, strip of rows); 6 planes; tiles of 64 x 16 (+halo)
template <bool HALO>
__global__ void read_tiles(const float* __restrict__ g, long long plane, int W, int H, int rows, float* out) {
    const int strips_x = W / 64, strips_y = (H + rows - 1) / rows;
    const int sx = blockIdx.x % strips_x, rest = blockIdx.x / strips_x;
    const int sy = rest % strips_y, b = rest / strips_y;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const float* g0 = g + (size_t)b * W * H;
    float s = 0.f;
    const int yb = sy * rows, ye = min(H, yb + rows);
    for (int y0 = yb; y0 < ye; y0 += 16) {
        const int nr = HALO ? 18 : 16;
        for (int ty = wave; ty < nr; ty += 4) {
            int gy = y0 + ty - (HALO ? 1 : 0);
            gy = gy < 0 ? 0 : (gy >= H ? H - 1 : gy);
            const float* q = g0 + (size_t)gy * W + sx * 64 + lane;
#pragma unroll
            for (int m = 0; m < 6; m++) s += q[m * plane];
        }
    }
    if (s == 1234.5f) out[0] = s;
}

int main() {
    const int W = 1920, H = 1080, N = 128;
    const size_t plane = (size_t)W * H * N;
    float *a, *o;
    hipMalloc(&a, plane * 6 * 4);
    hipMalloc(&o, 64);
    hipMemset(a, 0, plane * 6 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char* name, double bytes, auto launch) {
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
        printf("%-32s %8.1f us  %6.2f TB/s\n", name, best * 1e3, bytes / (best * 1e-3) / 1e12);
    };
    const double bytes = 6.0 * plane * 4;
    run("read linear float4 (6 planes)", bytes, [&] { read_linear<<<8192, 256>>>((const float4*)a, plane * 6 / 4, o); });
    const int strips = N * (W / 64);
    for (int rows : {1080, 544, 272}) {
        const int sy = (H + rows - 1) / rows;
        char nm[64];
        snprintf(nm, 64, "tiles no halo rows=%d", rows);
        run(nm, bytes, [&] { read_tiles<false><<<strips * sy, 256>>>(a, (long long)plane, W, H, rows, o); });
        snprintf(nm, 64, "tiles halo rows=%d", rows);
        run(nm, bytes, [&] { read_tiles<true><<<strips * sy, 256>>>(a, (long long)plane, W, H, rows, o); });
    }
    return 0;
}
