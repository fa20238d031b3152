// oracle_bench.cpp -- CPU baseline driver over the oracle (TEST / BENCH INFRASTRUCTURE ONLY).
//
// bench.py's cpu_baseline leg times oracle::extract on the host cores: one image per OpenMP
// thread, the batching the survey specifies for config C3.
#include <omp.h>

#include <chrono>
#include <cstdint>

#include "sift_oracle.h"

extern "C" {

// Extract n images (same size) with `threads` OpenMP threads; returns wall seconds and the
// total feature count in *features.
double oracle_bench_extract(const uint8_t* images, int n, int w, int h, int stride,
                            const sgpu_options* opt, int threads, long long* features) {
    long long total = 0;
    auto t0 = std::chrono::steady_clock::now();
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1) reduction(+ : total)
    for (int i = 0; i < n; i++) {
        oracle::Result R =
            oracle::extract(images + (size_t)i * stride * h, w, h, stride, *opt, false);
        total += (long long)R.feat_level.size();
    }
    auto t1 = std::chrono::steady_clock::now();
    *features = total;
    return std::chrono::duration<double>(t1 - t0).count();
}

}  // extern "C"
