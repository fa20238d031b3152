// oracle_bench.cpp -- CPU baseline driver over the oracle (TEST / BENCH INFRASTRUCTURE ONLY).
//
// bench.py's cpu_baseline legs time the oracle on the host cores: oracle::extract with one image
// per OpenMP thread (configs C3 and C4), and the matcher's row side -- the integer dot products
// of MultiplyDescriptor_Kernel and RowMatch_Kernel's running (max, argmax, second), ProgramCU.cu:
// 1466-1564, 1785-1841 -- row-blocked over OpenMP threads (config C5), SURVEY.md §8d.
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

// Row side of SiftMatch for rows [0, rows) of d1 against all n2 columns of d2 (u8 descriptors,
// 128 bytes each): exact int32 dots, the reference's running top-2 with strict '>' from
// (0, -1, 0).  Returns wall seconds; *checksum = sum of the argmax indices (keeps the loop live).
double oracle_bench_match_rows(const uint8_t* d1, int rows, const uint8_t* d2, int n2,
                               int threads, long long* checksum) {
    long long cs = 0;
    auto t0 = std::chrono::steady_clock::now();
#pragma omp parallel for num_threads(threads) schedule(static, 16) reduction(+ : cs)
    for (int i = 0; i < rows; i++) {
        const uint8_t* a = d1 + (size_t)i * 128;
        int best = 0, second = 0, idx = -1;
        for (int j = 0; j < n2; j++) {
            const uint8_t* b = d2 + (size_t)j * 128;
            int dot = 0;
            for (int k = 0; k < 128; k++) dot += (int)a[k] * (int)b[k];
            if (dot > best) { second = best; best = dot; idx = j; }
            else if (dot > second) second = dot;
        }
        cs += idx + (second & 1);
    }
    auto t1 = std::chrono::steady_clock::now();
    *checksum = cs;
    return std::chrono::duration<double>(t1 - t0).count();
}

}  // extern "C"
