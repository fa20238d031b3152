// Does the 256 MiB Infinity Cache (MALL) serve a level that was written just before it is read?
// A pyramid-like chain of copies, plane k-1 -> plane k (k = 1..5), over 128 images of
// 1920 x 1080 f32, in three schedules:
//   level-major : one launch per level over all 128 images (what the pyramid does today);
//   group-major : G images at a time, their 5 levels back to back (small launches);
//   diagonal    : launch t copies level k of group t-k for every k at once (5 groups per launch),
//                 so a plane is read one launch after it was written.
// Bytes moved are the same in every schedule (2 x 4 B per pixel and level); a schedule whose
// reads hit the cache finishes sooner.
//   hipcc -O3 --offload-arch=gfx950 mall_chain.hip -o mall_chain && ./mall_chain
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

struct Seg { const f4* src; f4* dst; long long n; long long blk0; };
struct Segs { Seg s[8]; int ns; };

// U float4 per thread; blocks are dealt to the segments in order
template <int U>
__global__ __launch_bounds__(256) void copy_segs(Segs S) {
    const long long b = blockIdx.x;
    int k = 0;
    while (k + 1 < S.ns && b >= S.s[k + 1].blk0) k++;
    const Seg g = S.s[k];
    const long long base = (b - g.blk0) * (256LL * U) + threadIdx.x;
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const long long i = base + (long long)u * 256;
        v[u] = i < g.n ? g.src[i] : f4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        const long long i = base + (long long)u * 256;
        if (i < g.n) g.dst[i] = v[u];
    }
}

constexpr int U = 4;
static void launch(const std::vector<Seg>& segs, hipStream_t st) {
    Segs S{};
    long long blk = 0;
    S.ns = (int)segs.size();
    for (int i = 0; i < S.ns; i++) {
        S.s[i] = segs[i];
        S.s[i].blk0 = blk;
        blk += (segs[i].n + 256LL * U - 1) / (256LL * U);
    }
    hipLaunchKernelGGL((copy_segs<U>), dim3((unsigned)blk), dim3(256), 0, st, S);
}

int main() {
    const int NI = 128, NL = 6;
    const long long img = 1920LL * 1080 / 4;           // float4 per image
    const long long plane = img * NI;
    f4* buf;
    if (hipMalloc(&buf, plane * NL * sizeof(f4)) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipMemset(buf, 0, plane * NL * sizeof(f4));
    auto P = [&](int lvl, int i0) { return buf + lvl * plane + i0 * img; };
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const double bytes = 2.0 * 4 * 1920.0 * 1080 * NI * (NL - 1);
    auto timeit = [&](const char* name, auto&& body) {
        body();   // warm-up
        hipDeviceSynchronize();
        float best = 1e9f;
        for (int r = 0; r < 5; r++) {
            hipEventRecord(e0, 0);
            body();
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            best = ms < best ? ms : best;
        }
        printf("%-28s %8.3f ms  %6.2f TB/s (bytes moved / time)\n", name, best, bytes / best / 1e9);
    };
    timeit("level-major", [&] {
        for (int k = 1; k < NL; k++) launch({Seg{P(k - 1, 0), P(k, 0), plane, 0}}, 0);
    });
    for (int G : {1, 2, 4, 8, 16}) {
        char nm[64];
        snprintf(nm, sizeof nm, "group-major G=%d", G);
        timeit(nm, [&] {
            for (int g = 0; g < NI; g += G)
                for (int k = 1; k < NL; k++) launch({Seg{P(k - 1, g), P(k, g), img * G, 0}}, 0);
        });
    }
    for (int G : {1, 2, 4, 8, 16}) {
        char nm[64];
        snprintf(nm, sizeof nm, "diagonal G=%d", G);
        const int ng = NI / G;
        timeit(nm, [&] {
            for (int t = 0; t < ng + NL - 2; t++) {
                std::vector<Seg> segs;
                for (int k = 1; k < NL; k++) {
                    const int g = t - (k - 1);
                    if (g >= 0 && g < ng) segs.push_back(Seg{P(k - 1, g * G), P(k, g * G), img * G, 0});
                }
                launch(segs, 0);
            }
        });
    }
    hipFree(buf);
    return 0;
}
