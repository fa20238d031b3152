// float_input_replica.cpp -- SiftGPU::RunSIFT(w, h, data, GL_LUMINANCE, GL_FLOAT) through our
// include/SiftGPU.h, for the reference's in-place row compaction of float luminance input whose
// width is not a multiple of 4 (GLTexImage.cpp:994-1006).
//   usage: float_input_replica <libsiftgpu.so> <img.f32> <w> <h> <buffer_after.f32> <keys.f32>
// Reads w*h floats, runs SIFT on them, writes the caller's buffer as RunSIFT left it and the
// keypoints; prints "RESULT num".
#include <dlfcn.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "SiftGPU.h"

int main(int argc, char** argv) {
    if (argc < 7) return 2;
    void* h = dlopen(argv[1], RTLD_LAZY);
    if (!h) { fprintf(stderr, "%s\n", dlerror()); return 3; }
    SiftGPU* (*create)(int) = (SiftGPU * (*)(int)) dlsym(h, "CreateNewSiftGPU");
    const int w = atoi(argv[3]), ht = atoi(argv[4]);
    std::vector<float> img((size_t)w * ht);
    FILE* f = fopen(argv[2], "rb");
    if (!f || fread(img.data(), sizeof(float), img.size(), f) != img.size()) return 4;
    fclose(f);
    SiftGPU* sift = create(1);
    char a0[] = "-v", a1[] = "0";
    char* av[] = {a0, a1};
    sift->ParseParam(2, av);
    if (sift->CreateContextGL() != SiftGPU::SIFTGPU_FULL_SUPPORTED) return 5;
    if (!sift->RunSIFT(w, ht, img.data(), 0x1909 /* GL_LUMINANCE */, 0x1406 /* GL_FLOAT */)) return 6;
    const int num = sift->GetFeatureNum();
    std::vector<SiftGPU::SiftKeypoint> keys(num > 0 ? num : 1);
    sift->GetFeatureVector(keys.data(), nullptr);
    f = fopen(argv[5], "wb");
    fwrite(img.data(), sizeof(float), img.size(), f);
    fclose(f);
    f = fopen(argv[6], "wb");
    fwrite(keys.data(), sizeof(float) * 4, (size_t)num, f);
    fclose(f);
    printf("RESULT %d\n", num);
    delete sift;
    dlclose(h);
    return 0;
}
