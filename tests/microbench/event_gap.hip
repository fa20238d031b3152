// Round 4: does a stage event cost GPU time between two kernels of a stream?  20 short kernels
// back to back (a) alone, (b) with hipEventRecord between each (default / device-release /
// untimed events), (c) launched through hipExtLaunchKernelGGL with start/stop events.
//   hipcc -O3 --offload-arch=gfx950 event_gap.hip -o event_gap && ./event_gap
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>

__global__ void k_short(float* p, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) p[i] = p[i] * 1.0001f + 1.0f;
}

int main() {
    const int n = 1 << 16, K = 20;
    float* p;
    hipMalloc(&p, n * 4);
    hipMemset(p, 0, n * 4);
    hipStream_t st;
    hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    hipEvent_t a, b, ev[3][K + 1];
    hipEventCreate(&a);
    hipEventCreate(&b);
    const unsigned flags[3] = {hipEventDefault, hipEventReleaseToDevice, hipEventDisableTiming};
    for (int f = 0; f < 3; f++)
        for (int k = 0; k <= K; k++) hipEventCreateWithFlags(&ev[f][k], flags[f]);
    auto run = [&](const char* name, int mode) {
        float best = 1e9f;
        for (int rep = 0; rep < 7; rep++) {
            hipEventRecord(a, st);
            for (int k = 0; k < K; k++) {
                if (mode == 4) {
                    hipExtLaunchKernelGGL(k_short, dim3(n / 256), dim3(256), 0, st, ev[0][k], ev[0][k + 1], 0, p, n);
                } else {
                    if (mode >= 1 && mode <= 3) hipEventRecord(ev[mode - 1][k], st);
                    k_short<<<n / 256, 256, 0, st>>>(p, n);
                }
            }
            hipEventRecord(b, st);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            best = ms < best ? ms : best;
        }
        printf("%-40s %7.2f us per kernel\n", name, best * 1e3 / K);
        fflush(stdout);
    };
    run("no events", 0);
    run("hipEventRecord default", 1);
    run("hipEventRecord release-to-device", 2);
    run("hipEventRecord untimed", 3);
    run("hipExtLaunchKernelGGL start/stop", 4);
    run("no events (again)", 0);
    return 0;
}
