// abi_check.cpp -- vtable / data-layout compatibility check of libsiftgpu.so.
//
// Compiled twice by tests/test_capi.py: once against include/SiftGPU.h and, when the reference
// checkout is present (this container only), against the reference's own SiftGPU/SiftGPU.h.
// The program loads the library the way TestWin/SimpleSIFT.cpp:92-121 does (dlopen + dlsym of
// the extern "C" factories) and calls virtual methods that need no GPU, so a slot mismatch
// between the two headers shows up as a wrong result or a crash.
#include <dlfcn.h>

#include <cstdio>
#include <cstring>

#include "SiftGPU.h"

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    void* h = dlopen(argv[1], RTLD_LAZY);
    if (!h) { fprintf(stderr, "dlopen: %s\n", dlerror()); return 3; }
    SiftGPU* (*pCreateNewSiftGPU)(int) = (SiftGPU * (*)(int)) dlsym(h, "CreateNewSiftGPU");
    SiftMatchGPU* (*pCreateNewSiftMatchGPU)(int) =
        (SiftMatchGPU * (*)(int)) dlsym(h, "CreateNewSiftMatchGPU");
    ComboSiftGPU* (*pCombo)() = (ComboSiftGPU * (*)()) dlsym(h, "CreateComboSiftGPU");
    if (!pCreateNewSiftGPU || !pCreateNewSiftMatchGPU || !pCombo) return 4;
    SiftGPU* sift = pCreateNewSiftGPU(1);
    const char* files[3] = {"a.pgm", "b.pgm", "c.pgm"};
    sift->SetImageList(3, files);                       // vtable slot 0
    if (sift->GetImageCount() != 3) return 10;          // slot 20
    if (sift->GetFeatureNum() != 0) return 11;          // slot 1
    char a0[] = "-fo", a1[] = "0", a2[] = "-v", a3[] = "0", a4[] = "-i", a5[] = "x.pgm";
    char* av[] = {a0, a1, a2, a3, a4, a5};
    sift->ParseParam(6, av);                            // slot 9
    if (strcmp(sift->GetCurrentImagePath(), "x.pgm") != 0) return 12;   // _imgpath offset
    for (int i = 0; i < 10; i++)
        if (sift->_timing[i] != 0.0f) return 13;        // _timing offset
    if (sift->GetImageCount() != 4) return 14;
    if (sift->RunSIFT(0, (const SiftGPU::SiftKeypoint*)0) != 0) return 15;   // num <= 0 -> 0
    delete sift;                                        // virtual destructor

    SiftMatchGPU* m = pCreateNewSiftMatchGPU(4096);
    m->SetMaxSift(2048);
    int buf[4][2];
    // without a verified context the matcher reports 0 matches (SiftMatchCU.cpp:141-142)
    delete m;

    ComboSiftGPU* c = pCombo();
    SiftGPU* cs = c;
    SiftMatchGPU* cm = c;
    cs->SetImageList(1, files);
    if (cs->GetImageCount() != 1) return 16;
    cm->SetMaxSift(1024);
    (void)buf;
    delete cs;
    printf("abi ok\n");
    return 0;
}
