// keypoint_replica.cpp -- the reference's caller-supplied keypoint entry points through our
// SiftGPU.h (SiftGPU.h:150, 181; SiftGPU.cpp:287-291, 383-386), driven as an application would:
//   A: RunSIFT(image); RunSIFT(num, keys, 1)       (describe on the current image)
//   B: SetKeypointList(num, keys, 0); RunSIFT(image)  (list applied to the next image, the
//                                                      strongest orientation computed)
//   usage: keypoint_replica <libsiftgpu.so> <img.pgm> <keys.f32> <n> <outA.f32> <outB.f32>
// Each output file holds num x 4 key floats then num x 128 descriptor floats.
#include <dlfcn.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "SiftGPU.h"

static bool dump(SiftGPU* sift, const char* path, int n) {
    if (sift->GetFeatureNum() != n) return false;
    std::vector<SiftGPU::SiftKeypoint> k(n);
    std::vector<float> d((size_t)n * 128);
    sift->GetFeatureVector(k.data(), d.data());
    FILE* f = fopen(path, "wb");
    if (!f) return false;
    fwrite(k.data(), sizeof(float), (size_t)n * 4, f);
    fwrite(d.data(), sizeof(float), d.size(), f);
    fclose(f);
    return true;
}

int main(int argc, char** argv) {
    if (argc < 7) return 2;
    void* h = dlopen(argv[1], RTLD_LAZY);
    if (!h) { fprintf(stderr, "%s\n", dlerror()); return 3; }
    auto create = (SiftGPU * (*)(int)) dlsym(h, "CreateNewSiftGPU");
    const int n = atoi(argv[4]);
    std::vector<SiftGPU::SiftKeypoint> keys(n);
    FILE* f = fopen(argv[3], "rb");
    if (!f || fread(keys.data(), sizeof(float), (size_t)n * 4, f) != (size_t)n * 4) return 4;
    fclose(f);
    SiftGPU* sift = create(1);
    char a0[] = "-v", a1[] = "0";
    char* av[] = {a0, a1};
    sift->ParseParam(2, av);
    if (sift->CreateContextGL() != SiftGPU::SIFTGPU_FULL_SUPPORTED) return 5;
    if (sift->RunSIFT(n, keys.data(), 1)) return 6;          // no image yet: must fail
    if (!sift->RunSIFT(argv[2])) return 7;
    if (!sift->RunSIFT(n, keys.data(), 1)) return 8;
    if (!dump(sift, argv[5], n)) return 9;
    sift->SetKeypointList(n, keys.data(), 0);
    if (!sift->RunSIFT(argv[2])) return 10;
    if (!dump(sift, argv[6], n)) return 11;
    if (!sift->RunSIFT(argv[2])) return 12;                   // the list was consumed
    printf("OK %d %d\n", n, sift->GetFeatureNum());
    delete sift;
    dlclose(h);
    return 0;
}
