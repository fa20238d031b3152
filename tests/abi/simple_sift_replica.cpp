// simple_sift_replica.cpp -- the call sequence of the reference's TestWin/SimpleSIFT.cpp:92-332
// (dlopen, factories, ParseParam with its argv, CreateContextGL == FULL_SUPPORTED, RunSIFT on two
// image files, SaveSIFT, GetFeatureNum, GetFeatureVector, VerifyContextGL, SetDescriptors x2,
// GetSiftMatch), written against include/SiftGPU.h.  Used by the GPU tests: the reference file
// itself does not exist on the GPU box.
//   usage: simple_sift_replica <libsiftgpu.so> <img1.pgm> <img2.pgm> <out1.sift> <out2.sift>
// Prints "RESULT num1 num2 num_match" and one "PAIR i j" line per match on success (the
// library's own -v 1 progress text goes to the same stdout).
#include <dlfcn.h>

#include <cstdio>
#include <vector>

#include "SiftGPU.h"

int main(int argc, char** argv) {
    if (argc < 6) return 2;
    void* hsiftgpu = dlopen(argv[1], RTLD_LAZY);
    if (!hsiftgpu) { fprintf(stderr, "%s\n", dlerror()); return 3; }
    SiftGPU* (*pCreateNewSiftGPU)(int) = (SiftGPU * (*)(int)) dlsym(hsiftgpu, "CreateNewSiftGPU");
    SiftMatchGPU* (*pCreateNewSiftMatchGPU)(int) =
        (SiftMatchGPU * (*)(int)) dlsym(hsiftgpu, "CreateNewSiftMatchGPU");
    SiftGPU* sift = pCreateNewSiftGPU(1);
    SiftMatchGPU* matcher = pCreateNewSiftMatchGPU(14096);
    std::vector<float> descriptors1(1), descriptors2(1);
    std::vector<SiftGPU::SiftKeypoint> keys1(1), keys2(1);
    int num1 = 0, num2 = 0;
    // SimpleSIFT.cpp:145, verbatim (the " -fo" with a leading space is skipped by ParseParam)
    char a0[] = "-cuda", a1[] = " -fo", a2[] = "-1", a3[] = "-v", a4[] = "1";
    char* av[] = {a0, a1, a2, a3, a4};
    sift->ParseParam(5, av);
    if (sift->CreateContextGL() != SiftGPU::SIFTGPU_FULL_SUPPORTED) return 4;
    if (sift->RunSIFT(argv[2])) {
        sift->SaveSIFT(argv[4]);
        num1 = sift->GetFeatureNum();
        keys1.resize(num1);
        descriptors1.resize(128 * num1);
        sift->GetFeatureVector(&keys1[0], &descriptors1[0]);
    }
    if (sift->RunSIFT(argv[3])) {
        sift->SaveSIFT(argv[5]);
        num2 = sift->GetFeatureNum();
        keys2.resize(num2);
        descriptors2.resize(128 * num2);
        sift->GetFeatureVector(&keys2[0], &descriptors2[0]);
    }
    matcher->VerifyContextGL();
    matcher->SetDescriptors(0, num1, &descriptors1[0]);
    matcher->SetDescriptors(1, num2, &descriptors2[0]);
    int(*match_buf)[2] = new int[num1][2];
    int num_match = matcher->GetSiftMatch(num1, match_buf);
    printf("RESULT %d %d %d\n", num1, num2, num_match);
    for (int i = 0; i < num_match; ++i) printf("PAIR %d %d\n", match_buf[i][0], match_buf[i][1]);
    delete[] match_buf;
    delete sift;
    delete matcher;
    dlclose(hsiftgpu);
    return 0;
}
