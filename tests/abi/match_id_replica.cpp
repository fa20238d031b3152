// match_id_replica.cpp -- SiftMatchGPU::SetDescriptors' id cache (SiftMatchCU.cpp:71-101): a
// float or u8 upload with the id the slot already holds (id != -1) leaves the slot unchanged.
//   usage: match_id_replica <set1.f32> <n1> <set2.f32> <n2> <set3.f32> <n3>
// (raw float32 [n][128] files).  Prints "COUNT <label> <num_match>" after each match.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "SiftGPU.h"

static std::vector<float> load(const char* path, int n) {
    std::vector<float> v((size_t)n * 128);
    FILE* f = fopen(path, "rb");
    if (!f || fread(v.data(), sizeof(float), v.size(), f) != v.size()) exit(3);
    fclose(f);
    return v;
}

int main(int argc, char** argv) {
    if (argc < 7) return 2;
    const int n1 = atoi(argv[2]), n2 = atoi(argv[4]), n3 = atoi(argv[6]);
    std::vector<float> a = load(argv[1], n1), b = load(argv[3], n2), c = load(argv[5], n3);
    SiftMatchGPU* m = CreateNewSiftMatchGPU(8192);
    if (!m->VerifyContextGL()) return 4;
    std::vector<int> buf((size_t)8192 * 2);
    int(*mb)[2] = reinterpret_cast<int(*)[2]>(buf.data());
    m->SetDescriptors(0, n1, a.data(), 5);
    m->SetDescriptors(1, n2, b.data(), 7);
    printf("COUNT ab %d\n", m->GetSiftMatch(8192, mb));
    m->SetDescriptors(0, n3, c.data(), 5);      // same id: the slot keeps set a
    printf("COUNT cached %d\n", m->GetSiftMatch(8192, mb));
    m->SetDescriptors(0, n3, c.data(), 6);      // new id: replaced
    printf("COUNT cb %d\n", m->GetSiftMatch(8192, mb));
    m->SetDescriptors(0, n1, a.data(), -1);     // -1: always replaced
    m->SetDescriptors(0, n3, c.data(), -1);
    printf("COUNT cb_again %d\n", m->GetSiftMatch(8192, mb));
    delete m;
    return 0;
}
