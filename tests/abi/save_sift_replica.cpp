// save_sift_replica.cpp -- SiftGPU::SaveSIFT through include/SiftGPU.h, as the reference's
// SimpleSIFT.cpp:211 uses it: ParseParam (with -b / -unn / -sd / -fo / -maxd / -tc... from the
// command line), CreateContextGL, RunSIFT(file), SaveSIFT(out).  "=maxd N" calls
// SetMaxDimension(N) before the run (SiftGPU.cpp:1452-1458).
//   usage: save_sift_replica <img.pgm> <out.sift> [options...]
// Prints "NUM n" on success.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "SiftGPU.h"

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    SiftGPU* sift = CreateNewSiftGPU(1);
    std::vector<char*> av;
    int maxd = 0;
    for (int i = 3; i < argc; i++) {
        if (!strcmp(argv[i], "=maxd") && i + 1 < argc) { maxd = atoi(argv[++i]); continue; }
        av.push_back(argv[i]);
    }
    char v0[] = "-v", v1[] = "0";
    av.push_back(v0);
    av.push_back(v1);
    sift->ParseParam((int)av.size(), av.data());
    if (maxd > 0) sift->SetMaxDimension(maxd);
    if (sift->CreateContextGL() != SiftGPU::SIFTGPU_FULL_SUPPORTED) return 4;
    if (!sift->RunSIFT(argv[1])) return 5;
    sift->SaveSIFT(argv[2]);
    printf("NUM %d\n", sift->GetFeatureNum());
    delete sift;
    return 0;
}
