/* synth.c -- fast deterministic synthetic test / bench images (SURVEY.md section 8d "Synthetic
 * inputs"): background 128, 400 anisotropic Gaussian blobs (amplitude U(-96, 96), sigma
 * U(2, 40) px scaled by min(w, h) / 1080), 200 rotated rectangles (step U(-64, 64)), i.i.d.
 * N(0, 4^2) noise, rounded and clamped to u8.  Same recipe as sift_synth.synth_image, with its
 * own generator (PCG32 + Box-Muller), so the images differ from the NumPy ones but are a pure
 * function of the seed.  Test / bench data only; nothing in the product uses it.
 *   gcc -O3 -fopenmp -shared -fPIC -o libsynth.so synth.c -lm
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct { uint64_t state, inc; } pcg32;

static uint32_t pcg_next(pcg32* r) {
    uint64_t old = r->state;
    r->state = old * 6364136223846793005ULL + r->inc;
    uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
    uint32_t rot = (uint32_t)(old >> 59u);
    return (xs >> rot) | (xs << ((-rot) & 31));
}

static void pcg_seed(pcg32* r, uint64_t seed, uint64_t stream) {
    r->state = 0;
    r->inc = (stream << 1u) | 1u;
    pcg_next(r);
    r->state += seed;
    pcg_next(r);
}

static double uni(pcg32* r, double a, double b) {   /* [a, b) */
    return a + (b - a) * (pcg_next(r) * (1.0 / 4294967296.0));
}

static double gauss(pcg32* r) {
    double u1 = (pcg_next(r) + 1.0) * (1.0 / 4294967297.0);
    double u2 = pcg_next(r) * (1.0 / 4294967296.0);
    return sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
}

static void synth_one(uint8_t* out, int w, int h, uint64_t seed, int n_blobs, int n_rects,
                      double noise) {
    float* img = (float*)malloc((size_t)w * h * sizeof(float));
    for (size_t i = 0; i < (size_t)w * h; i++) img[i] = 128.0f;
    pcg32 r;
    pcg_seed(&r, seed, 54u);
    double scale = (w < h ? w : h) / 1080.0;
    if (scale < 0.15) scale = 0.15;
    for (int b = 0; b < n_blobs; b++) {
        double cx = uni(&r, 0, w), cy = uni(&r, 0, h), amp = uni(&r, -96, 96);
        double sx = uni(&r, 2, 40) * scale, sy = uni(&r, 2, 40) * scale, th = uni(&r, 0, M_PI);
        double rr = 4.0 * (sx > sy ? sx : sy);
        int x0 = (int)fmax(0, cx - rr), x1 = (int)fmin(w, cx + rr + 1);
        int y0 = (int)fmax(0, cy - rr), y1 = (int)fmin(h, cy + rr + 1);
        double c = cos(th), s = sin(th), ax = 0.5 / (sx * sx), ay = 0.5 / (sy * sy);
        for (int y = y0; y < y1; y++)
            for (int x = x0; x < x1; x++) {
                double dx = x - cx, dy = y - cy;
                double u = c * dx + s * dy, v = -s * dx + c * dy;
                img[(size_t)y * w + x] += (float)(amp * exp(-(u * u * ax + v * v * ay)));
            }
    }
    for (int q = 0; q < n_rects; q++) {
        double cx = uni(&r, 0, w), cy = uni(&r, 0, h), step = uni(&r, -64, 64);
        double hw = uni(&r, 3, 60) * scale, hh = uni(&r, 3, 60) * scale, th = uni(&r, 0, M_PI);
        double rr = hypot(hw, hh) + 1;
        int x0 = (int)fmax(0, cx - rr), x1 = (int)fmin(w, cx + rr + 1);
        int y0 = (int)fmax(0, cy - rr), y1 = (int)fmin(h, cy + rr + 1);
        double c = cos(th), s = sin(th);
        for (int y = y0; y < y1; y++)
            for (int x = x0; x < x1; x++) {
                double dx = x - cx, dy = y - cy;
                double u = c * dx + s * dy, v = -s * dx + c * dy;
                if (fabs(u) <= hw && fabs(v) <= hh) img[(size_t)y * w + x] += (float)step;
            }
    }
    for (size_t i = 0; i < (size_t)w * h; i++) {
        double v = nearbyint(img[i] + noise * gauss(&r));
        out[i] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
    }
    free(img);
}

/* n images [n][h][w], image i from seed seed0 + i, on `threads` OpenMP threads (>= 1). */
void synth_batch_u8(uint8_t* out, int n, int w, int h, uint64_t seed0, int threads) {
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads > 0 ? threads : 1)
    for (int i = 0; i < n; i++)
        synth_one(out + (size_t)i * w * h, w, h, seed0 + (uint64_t)i, 400, 200, 4.0);
}
