// allocate_replica.cpp -- SiftGPU::AllocatePyramid (SiftGPU.h:193, SiftGPU.cpp:1435-1460) through
// include/SiftGPU.h: CreateContextGL, AllocatePyramid(w, h) for the image's size, then RunSIFT
// of the image.  The library's allocation counter (sgpu_debug_alloc_count, a test hook of the
// same libsiftgpu.so) must not move during that first RunSIFT: the pyramid and every other
// buffer were allocated by AllocatePyramid.  A second AllocatePyramid of the same size
// allocates nothing either (the buffers are grow-only).
//   usage: allocate_replica <img.pgm> <w> <h>
// Prints one line: "ALLOC reserve=<1|0> during_reserve=<n> during_run=<n> again=<n> features=<n>".
#include <cstdio>
#include <cstdlib>

#include "SiftGPU.h"

extern "C" long long sgpu_debug_alloc_count(void);

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    const int w = atoi(argv[2]), h = atoi(argv[3]);
    SiftGPU* sift = CreateNewSiftGPU(1);
    char a0[] = "-fo", a1[] = "0", a2[] = "-v", a3[] = "0";
    char* args[] = {a0, a1, a2, a3};
    sift->ParseParam(4, args);
    if (sift->CreateContextGL() != SiftGPU::SIFTGPU_FULL_SUPPORTED) return 3;
    const long long c0 = sgpu_debug_alloc_count();
    const int ok = sift->AllocatePyramid(w, h);
    const long long c1 = sgpu_debug_alloc_count();
    if (!sift->RunSIFT(argv[1])) return 4;
    const long long c2 = sgpu_debug_alloc_count();
    const int ok2 = sift->AllocatePyramid(w, h);
    const long long c3 = sgpu_debug_alloc_count();
    if (!sift->RunSIFT()) return 5;
    const long long c4 = sgpu_debug_alloc_count();
    printf("ALLOC reserve=%d during_reserve=%lld during_run=%lld again=%lld features=%d\n",
           ok && ok2, c1 - c0, c2 - c1, (c3 - c2) + (c4 - c3), sift->GetFeatureNum());
    delete sift;
    return 0;
}
