// speed_replica.cpp -- the reference's TestWin/speed.cpp:60-155 protocol against our
// include/SiftGPU.h, directly linked (`SiftGPU sift;`, as speed.cpp:71 does):
//   ParseParam(argv) -> SetVerbose(0) -> CreateContextGL -> RunSIFT() (loads the -i image) ->
//   RunSIFT() (warm-up) -> REPEAT x RunSIFT() timed as a whole (the GetFeatureNum stability
//   check of speed.cpp:108-114 after each) -> REPEAT x RunSIFT() again, summing _timing[0..9]
//   per run (speed.cpp:122-135).
// Prints one JSON object: feature count, average ms per RunSIFT, per-stage averages in the
// reference's _timing slots (SiftGPU.cpp:368; printed by speed.cpp:147-153), and whether every
// run reproduced the first feature count.
//   usage: speed_replica [REPEAT] -- <SiftGPU options, e.g. -i img.pgm -fo 0 -no 4 -d 3>
#include <sys/time.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "SiftGPU.h"

static double now_ms() {
    timeval tv;
    gettimeofday(&tv, nullptr);
    return tv.tv_sec * 1e3 + tv.tv_usec * 1e-3;
}

int main(int argc, char** argv) {
    int repeat = 30;   // SIFTGPU_REPEAT, speed.cpp:59
    int first = 1;
    if (argc > 1 && strcmp(argv[1], "--") != 0) repeat = atoi(argv[first++]);
    if (first < argc && strcmp(argv[first], "--") == 0) first++;
    SiftGPU sift;
    sift.ParseParam(argc - first, argv + first);
    sift.SetVerbose(0);
    if (sift.CreateContextGL() == 0) return 3;
    if (sift.RunSIFT() == 0) return 4;
    const double load_ms = sift._timing[0] * 1e3;
    sift.RunSIFT();   // "run one more time to get all texture allocated"
    const int num = sift.GetFeatureNum();
    bool stable = true;
    const double t0 = now_ms();
    for (int i = 0; i < repeat; i++) {
        sift.RunSIFT();
        stable = stable && sift.GetFeatureNum() == num;
    }
    const double avg_ms = (now_ms() - t0) / repeat;
    sift.SetVerbose(-2);
    double timing[10] = {0};
    const double t1 = now_ms();
    for (int k = 0; k < repeat; k++) {
        sift.RunSIFT();
        for (int j = 0; j < 10; j++) timing[j] += sift._timing[j];
        stable = stable && sift.GetFeatureNum() == num;
    }
    // the second loop runs with the stage timing on (SetVerbose(-2)): its own wall time per run
    const double timed_ms = (now_ms() - t1) / repeat;
    static const char* names[10] = {"load_image", "init_pyramid", "build_pyramid", "detection",
                                     "feature_list", "orientation", "mo_feature_list",
                                     "download_keys", "descriptor", "vbo"};
    printf("{\"features\": %d, \"repeat\": %d, \"avg_ms\": %.6f, \"hz\": %.3f, \"stable\": %s, "
           "\"first_load_ms\": %.6f, \"timed_avg_ms\": %.6f, \"timing_ms\": {",
           num, repeat, avg_ms, 1e3 / avg_ms, stable ? "true" : "false", load_ms, timed_ms);
    for (int j = 0; j < 10; j++)
        printf("%s\"%s\": %.6f", j ? ", " : "", names[j], timing[j] / repeat * 1e3);
    printf("}}\n");
    return stable ? 0 : 5;
}
