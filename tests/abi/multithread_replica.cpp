// multithread_replica.cpp -- the reference's TestWin/MultiThreadSIFT.cpp pattern through
// include/SiftGPU.h: one SiftGPU per thread, initialisation serialised by a global mutex
// (MultiThreadSIFT.cpp:90-100: ParseParam {-fo -1 -v 0 -cuda <dev>}, CreateContextGL, RunSIFT
// of the thread's file), then each thread repeats RunSIFT() on its image (RunTask,
// MultiThreadSIFT.cpp:178-186) concurrently with the others.  Every repetition must give the
// bits of the thread's first run; the last one is written as raw keys + descriptors.
//   usage: multithread_replica <device> <repeats> <img1.pgm> <out1.bin> [<img2.pgm> <out2.bin> ...]
// Prints "THREAD i num equal" per thread.
#include <pthread.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "SiftGPU.h"

static pthread_mutex_t g_init = PTHREAD_MUTEX_INITIALIZER;

struct Task {
    int device = 0, repeats = 0, index = 0;
    const char* image = nullptr;
    const char* out = nullptr;
    SiftGPU* sift = nullptr;
    int num = -1, equal = 0;
};

static void features(SiftGPU* s, std::vector<float>* k, std::vector<float>* d) {
    const int n = s->GetFeatureNum();
    k->assign((size_t)n * 4, 0.f);
    d->assign((size_t)n * 128, 0.f);
    if (n) s->GetFeatureVector(reinterpret_cast<SiftGPU::SiftKeypoint*>(k->data()), d->data());
}

static void* run(void* p) {
    Task* t = static_cast<Task*>(p);
    {
        pthread_mutex_lock(&g_init);
        char dev[16];
        snprintf(dev, sizeof(dev), "%d", t->device);
        char a0[] = "-fo", a1[] = "-1", a2[] = "-v", a3[] = "0", a4[] = "-cuda";
        char* argv[] = {a0, a1, a2, a3, a4, dev};
        t->sift = new SiftGPU;
        t->sift->ParseParam(6, argv);
        const bool ok = t->sift->CreateContextGL() == SiftGPU::SIFTGPU_FULL_SUPPORTED &&
                        t->sift->RunSIFT(t->image);
        pthread_mutex_unlock(&g_init);
        if (!ok) return nullptr;
    }
    std::vector<float> k0, d0, k, d;
    features(t->sift, &k0, &d0);
    t->equal = 1;
    for (int r = 0; r < t->repeats; r++) {
        if (!t->sift->RunSIFT()) { t->equal = 0; break; }
        features(t->sift, &k, &d);
        if (k != k0 || d != d0 ||
            memcmp(k.data(), k0.data(), k.size() * 4) || memcmp(d.data(), d0.data(), d.size() * 4))
            t->equal = 0;
    }
    t->num = (int)(k0.size() / 4);
    FILE* f = fopen(t->out, "wb");
    if (f) {
        fwrite(k0.data(), 4, k0.size(), f);
        fwrite(d0.data(), 4, d0.size(), f);
        fclose(f);
    }
    delete t->sift;
    return nullptr;
}

int main(int argc, char** argv) {
    if (argc < 5 || (argc - 3) % 2) return 2;
    const int device = atoi(argv[1]), repeats = atoi(argv[2]);
    const int nt = (argc - 3) / 2;
    std::vector<Task> tasks(nt);
    std::vector<pthread_t> th(nt);
    for (int i = 0; i < nt; i++) {
        tasks[i].device = device;
        tasks[i].repeats = repeats;
        tasks[i].index = i;
        tasks[i].image = argv[3 + 2 * i];
        tasks[i].out = argv[4 + 2 * i];
        pthread_create(&th[i], nullptr, run, &tasks[i]);
    }
    for (int i = 0; i < nt; i++) pthread_join(th[i], nullptr);
    for (int i = 0; i < nt; i++) printf("THREAD %d %d %d\n", i, tasks[i].num, tasks[i].equal);
    return 0;
}
