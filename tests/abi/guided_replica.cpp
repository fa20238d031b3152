// guided_replica.cpp -- guided matching through our SiftGPU.h as an application drives it
// (SiftGPU.h:313-335): SetDescriptors + SetFeatureLocation(index, SiftKeypoint*) (gap 2) per set,
// then GetGuidedSiftMatch with H and F, H only, F only, neither.
//   usage: guided_replica <libsiftgpu.so> <scene.bin>
// scene.bin: int32 n1, n2; u8 q1[n1][128], q2[n2][128]; float keys1[n1][4], keys2[n2][4];
//            float H[9], F[9], distmax, ratiomax, hdistmax, fdistmax; int32 mbm.
// Prints "CASE <k> <count>" then "PAIR i j" lines per case.
#include <dlfcn.h>

#include <cstdio>
#include <vector>

#include "SiftGPU.h"

template <class T>
static bool rd(FILE* f, T* p, size_t n) { return fread(p, sizeof(T), n, f) == n; }

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    void* h = dlopen(argv[1], RTLD_LAZY);
    if (!h) { fprintf(stderr, "%s\n", dlerror()); return 3; }
    auto create = (SiftMatchGPU * (*)(int)) dlsym(h, "CreateNewSiftMatchGPU");
    FILE* f = fopen(argv[2], "rb");
    int n[2];
    if (!f || !rd(f, n, 2)) return 4;
    std::vector<unsigned char> q1((size_t)n[0] * 128), q2((size_t)n[1] * 128);
    std::vector<SiftGPU::SiftKeypoint> k1(n[0]), k2(n[1]);
    float H[3][3], F[3][3], th[4];
    int mbm;
    if (!rd(f, q1.data(), q1.size()) || !rd(f, q2.data(), q2.size()) ||
        !rd(f, (float*)k1.data(), (size_t)n[0] * 4) || !rd(f, (float*)k2.data(), (size_t)n[1] * 4) ||
        !rd(f, &H[0][0], 9) || !rd(f, &F[0][0], 9) || !rd(f, th, 4) || !rd(f, &mbm, 1))
        return 5;
    fclose(f);
    SiftMatchGPU* m = create(n[0] > n[1] ? n[0] : n[1]);
    if (!m->VerifyContextGL()) return 6;
    m->SetDescriptors(0, n[0], q1.data());
    m->SetDescriptors(1, n[1], q2.data());
    std::vector<int> buf((size_t)2 * n[0]);
    int (*mb)[2] = reinterpret_cast<int (*)[2]>(buf.data());
    // locations are required after SetDescriptors (SiftMatchCU.cpp:77, 131)
    if (m->GetGuidedSiftMatch(n[0], mb, H, F, th[0], th[1], th[2], th[3], mbm) != 0) return 7;
    m->SetFeatureLocation(0, k1.data());
    m->SetFeatureLocation(1, k2.data());
    float (*Hs[4])[3] = {H, H, nullptr, nullptr};
    float (*Fs[4])[3] = {F, nullptr, F, nullptr};
    for (int c = 0; c < 4; c++) {
        const int cnt = m->GetGuidedSiftMatch(n[0], mb, Hs[c], Fs[c], th[0], th[1], th[2], th[3], mbm);
        printf("CASE %d %d\n", c, cnt);
        for (int i = 0; i < cnt; i++) printf("PAIR %d %d\n", mb[i][0], mb[i][1]);
    }
    delete m;
    dlclose(h);
    return 0;
}
