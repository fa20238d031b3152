// Round 4: does the plane LAYOUT bound the Gaussian's strip walk?  The level kernel walks
// 64-column strips top to bottom in 8-row chunks (4 chunks in flight per wave, 12 waves per CU);
// round 1 measured that access pattern at ~5.0 TB/s as a copy against 6.3 for a flat copy.  This
// copies 128 x 1920 x 1080 f32 with that walk over three layouts of the same plane:
//   rm     row-major [img][y][x] (the shipped layout)
//   sm     strip-major [img][x / 64][y][x % 64]: a wave's own columns are one contiguous stream
//   tile   [img][y / 8][x / 64][y % 8][x % 64]: 2 KB tiles of 8 rows x 64 columns
// each without and with the Gaussian's horizontal halo (16 columns a side read per row, FW 25).
//   hipcc -O3 --offload-arch=gfx950 layout_bw.hip -o layout_bw && ./layout_bw
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int W = 1920, H = 1080, N = 128;

template <int L>
__device__ __forceinline__ size_t addr(int y, int col) {
    if (L == 0) return (size_t)y * W + col;
    if (L == 1) return ((size_t)(col >> 6) * H + y) * 64 + (col & 63);
    return (((size_t)(y >> 3) * (W / 64) + (col >> 6)) * 8 + (y & 7)) * 64 + (col & 63);
}

// one wave per (image, strip, band); half-wave g handles row 2p + g of a row pair, lane j < NQ of
// it one aligned quad; lanes j in [HALO/4, HALO/4 + 16) own the strip's 64 columns and store them
template <int L, int HALO>
__global__ __launch_bounds__(256) void walk(const float* __restrict__ a, float* __restrict__ b, int BR,
                                            float* __restrict__ sink) {
    extern __shared__ float lds_pad[];   // only sizes the occupancy (12 waves per CU)
    constexpr int NQ = 16 + 2 * HALO / 4;
    const int lane = threadIdx.x & 63;
    const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int strips = W / 64, bands = (H + BR - 1) / BR;
    const int sx = gw % strips, rest = gw / strips, band = rest % bands, img = rest / bands;
    if (img >= N) return;
    const float* s = a + (size_t)img * W * H;
    float* d = b + (size_t)img * W * H;
    const int g = lane >> 5, j = min(lane & 31, NQ - 1);
    const int col = min(max(sx * 64 - HALO + 4 * j, 0), W - 4);
    const int y0 = band * BR, y1 = min(H, y0 + BR);
    const int nch = (y1 - y0 + 7) / 8;
    float4 st[4][4];
    float4 hs = {0, 0, 0, 0};
    auto load = [&](float4 (&r)[4], int c) {
#pragma unroll
        for (int p = 0; p < 4; p++) {
            const int y = min(y0 + 8 * c + 2 * p + g, H - 1);
            r[p] = *reinterpret_cast<const float4*>(s + addr<L>(y, col));
        }
    };
    // every lane stores (V-pass form: 32 lanes x 2 columns per row, two rows per instruction) and
    // every condition is uniform, so the compiler can count the loads still in flight
    const int scol = sx * 64 + 2 * (lane & 31);
    auto step = [&](float4 (&r)[4], int c) {
        if (c < nch) {
#pragma unroll
            for (int p = 0; p < 4; p++) {
                const int y = y0 + 8 * c + 2 * p + g;
                *reinterpret_cast<float2*>(d + addr<L>(y, scol)) = make_float2(r[p].x, r[p].y);
                hs.x += r[p].z + r[p].w;
            }
        }
        load(r, c + 4);
    };
#pragma unroll
    for (int k = 0; k < 4; k++) load(st[k], k);
    for (int c = 0; c < nch; c += 4) {
        step(st[0], c + 0);
        step(st[1], c + 1);
        step(st[2], c + 2);
        step(st[3], c + 3);
    }
    if (hs.x == 1234.5f) sink[0] = hs.x;
    if (lds_pad[threadIdx.x] == 1234.5f) sink[1] = 1.f;
}


// round-4 variants of the row-major walk (halo 16 columns a side, the FW 25 case):
//   SW  store width per lane in floats (2: the level kernel's V-pass form, 4: 16 lanes per row)
//   NT  non-temporal stores
//   NC  chunks in flight (register sets)
template <int SW, bool NT, int NC>
__global__ __launch_bounds__(256) void walk2(const float* __restrict__ a, float* __restrict__ b, int BR,
                                             float* __restrict__ sink) {
    extern __shared__ float lds_pad[];
    constexpr int HALO = 16, NQ = 16 + 2 * HALO / 4;
    const int lane = threadIdx.x & 63;
    const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int strips = W / 64, bands = (H + BR - 1) / BR;
    const int sx = gw % strips, rest = gw / strips, band = rest % bands, img = rest / bands;
    if (img >= N) return;
    const float* s = a + (size_t)img * W * H;
    float* d = b + (size_t)img * W * H;
    const int g = lane >> 5, j = min(lane & 31, NQ - 1);
    const int col = min(max(sx * 64 - HALO + 4 * j, 0), W - 4);
    const int y0 = band * BR, y1 = min(H, y0 + BR);
    const int nch = (y1 - y0 + 7) / 8;
    float4 st[NC][4];
    float hs = 0.f;
    auto load = [&](float4 (&r)[4], int c) {
#pragma unroll
        for (int p = 0; p < 4; p++) {
            const int y = min(y0 + 8 * c + 2 * p + g, H - 1);
            r[p] = *reinterpret_cast<const float4*>(s + (size_t)y * W + col);
        }
    };
    // SW 2: lane (32 g + l) stores columns 2l, 2l+1 of rows 2p + g; SW 4: lane (16 q + l) stores
    // columns 4l .. 4l+3 of rows 4 (p / 2) + q, two instructions per 4 rows
    const int scol2 = sx * 64 + 2 * (lane & 31);
    const int scol4 = sx * 64 + 4 * (lane & 15), q4 = lane >> 4;
    auto step = [&](float4 (&r)[4], int c) {
        if (c < nch) {
#pragma unroll
            for (int p = 0; p < 4; p++) {
                hs += r[p].z + r[p].w;
                if (SW == 2) {
                    const int y = y0 + 8 * c + 2 * p + g;
                    typedef float v2 __attribute__((ext_vector_type(2)));
                    v2* q = reinterpret_cast<v2*>(d + (size_t)y * W + scol2);
                    const v2 v = {r[p].x, r[p].y};
                    if (NT) __builtin_nontemporal_store(v, q); else *q = v;
                } else if ((p & 1) == 0) {
                    const int y = y0 + 8 * c + 4 * (p >> 1) + q4;
                    typedef float v4 __attribute__((ext_vector_type(4)));
                    v4* q = reinterpret_cast<v4*>(d + (size_t)y * W + scol4);
                    const v4 v = {r[p].x, r[p].y, r[p + 1].x, r[p + 1].y};
                    if (NT) __builtin_nontemporal_store(v, q); else *q = v;
                }
            }
        }
        load(r, c + NC);
    };
#pragma unroll
    for (int k = 0; k < NC; k++) load(st[k], k);
    for (int c = 0; c < nch; c += NC) {
#pragma unroll
        for (int k = 0; k < NC; k++) step(st[k], c + k);
    }
    if (hs == 1234.5f) sink[0] = hs;
    if (lds_pad[threadIdx.x] == 1234.5f) sink[1] = 1.f;
}

typedef float f4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void copy_flat(const f4* __restrict__ a, f4* __restrict__ b, size_t n) {
    const size_t i = blockIdx.x * (size_t)256 + threadIdx.x;
    if (i < n) b[i] = a[i];
}

int main() {
    const size_t n = (size_t)W * H * N;
    float *a, *b, *sink;
    hipMalloc(&a, n * 4);
    hipMalloc(&b, n * 4);
    hipMalloc(&sink, 64);
    hipMemset(a, 0, n * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char* name, auto launch) {
        launch();
        hipDeviceSynchronize();
        float best = 1e9f, sum = 0;
        for (int r = 0; r < 9; r++) {
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            best = ms < best ? ms : best;
            sum += ms;
        }
        printf("%-34s best %7.1f us %5.2f TB/s   mean %7.1f us\n", name, best * 1e3,
               2.0 * n * 4 / (best * 1e-3) / 1e12, sum / 9 * 1e3);
        fflush(stdout);
    };
    run("flat float4 copy", [&] { copy_flat<<<(n / 4 + 255) / 256, 256>>>((const f4*)a, (f4*)b, n / 4); });
    const size_t lds = 47 * 1024;   // 3 workgroups (12 waves) per CU, as k_gauss_lean
    {
        const int br = 1080, waves = N * (W / 64), blocks = (waves + 3) / 4;
        char nm[80];
        run("rm   halo 16 band 1080 (round 4 ref)", [&] { walk<0, 16><<<blocks, 256, lds>>>(a, b, br, sink); });
#define RUN2(SW, NT, NC, L, LN)                                                                  \
        snprintf(nm, sizeof nm, "walk2 st%d nt%d nc%d %s", SW, NT, NC, LN);                     \
        run(nm, [&] { walk2<SW, NT, NC><<<blocks, 256, L>>>(a, b, br, sink); });
        RUN2(2, 0, 4, lds, "12w") RUN2(4, 0, 4, lds, "12w") RUN2(2, 1, 4, lds, "12w")
        RUN2(4, 1, 4, lds, "12w") RUN2(2, 0, 6, lds, "12w") RUN2(2, 0, 2, lds, "12w")
        RUN2(2, 0, 4, 0, "nolds") RUN2(4, 1, 4, 0, "nolds") RUN2(2, 0, 4, 64 * 1024, "8w")
    }
    return 0;
}
