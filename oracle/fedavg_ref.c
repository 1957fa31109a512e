/*
 * ORACLE — plain-C restatement of the reference FedAvg / FedLesScan fold.
 *
 * TEST INFRASTRUCTURE ONLY: loaded by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py (as the multi-core CPU baseline, kind "port").
 * The product library (fedlesscan_amd/csrc) never links or calls it.
 *
 * Restates, per output column p and clients in list order i = 0..N-1:
 *   fed_avg_aggregator.py:24-42          out = reduce(add, [x_i * n_i]) / sum(n)
 *   stall_aware_aggregation.py:42-67     out = reduce(add, [(x_i * n_i) * s_i]) / sum(n)
 * with a_i = fl32(n_i), s_i = fl32((r_i+1)/(R+1)) and divisor = fl32(sum n_i)
 * computed by the caller exactly as numpy would (weak Python scalars).
 * Separate multiply and add (built with -ffp-contract=off), IEEE divide.
 * Parity: pinned against tests/golden (reference-generated) by
 * tests/test_oracle_golden.py.
 *
 * Columns are independent, so the loop is blocked over columns (OpenMP) and
 * every column still folds its clients strictly left to right.
 */
#include <stdint.h>
#include <string.h>
#include <math.h>
#include <omp.h>

#define COLBLK 2048

static void set_threads(int nthreads) {
    if (nthreads > 0) omp_set_num_threads(nthreads);
}

int oracle_max_threads(void) { return omp_get_max_threads(); }

void oracle_fedavg_f32(const float* X, int64_t N, int64_t P, int64_t ldx,
                       const float* a, const float* s, float divisor, float* out,
                       int nthreads) {
    set_threads(nthreads);
    int64_t nblk = (P + COLBLK - 1) / COLBLK;
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < nblk; ++b) {
        int64_t c0 = b * COLBLK;
        int64_t c1 = c0 + COLBLK < P ? c0 + COLBLK : P;
        int64_t w = c1 - c0;
        float acc[COLBLK];
        for (int64_t i = 0; i < N; ++i) {
            const float* row = X + i * ldx + c0;
            float ai = a[i];
            float si = s ? s[i] : 1.0f;
            if (i == 0) {
                for (int64_t j = 0; j < w; ++j) {
                    float t = row[j] * ai;
                    if (s) t = t * si;
                    acc[j] = t;
                }
            } else {
                for (int64_t j = 0; j < w; ++j) {
                    float t = row[j] * ai;
                    if (s) t = t * si;
                    acc[j] = acc[j] + t;
                }
            }
        }
        for (int64_t j = 0; j < w; ++j) out[c0 + j] = acc[j] / divisor;
    }
}

void oracle_fedavg_f64(const double* X, int64_t N, int64_t P, int64_t ldx,
                       const double* a, const double* s, double divisor, double* out,
                       int nthreads) {
    set_threads(nthreads);
    int64_t nblk = (P + COLBLK - 1) / COLBLK;
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < nblk; ++b) {
        int64_t c0 = b * COLBLK;
        int64_t c1 = c0 + COLBLK < P ? c0 + COLBLK : P;
        int64_t w = c1 - c0;
        double acc[COLBLK];
        for (int64_t i = 0; i < N; ++i) {
            const double* row = X + i * ldx + c0;
            double ai = a[i];
            double si = s ? s[i] : 1.0;
            for (int64_t j = 0; j < w; ++j) {
                double t = row[j] * ai;
                if (s) t = t * si;
                acc[j] = (i == 0) ? t : acc[j] + t;
            }
        }
        for (int64_t j = 0; j < w; ++j) out[c0 + j] = acc[j] / divisor;
    }
}

static inline float bf16_to_f32(uint16_t b) {
    uint32_t u = (uint32_t)b << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}

static inline uint16_t f32_to_bf16_rne(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    if (isnan(f)) return (uint16_t)((u >> 16) | 0x40);
    return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}

/* bf16 extension: exact upcast to f32, then the f32 fold (no reference path). */
void oracle_fedavg_bf16(const uint16_t* X, int64_t N, int64_t P, int64_t ldx,
                        const float* a, const float* s, float divisor, float* out,
                        uint16_t* out_bf16, int nthreads) {
    set_threads(nthreads);
    int64_t nblk = (P + COLBLK - 1) / COLBLK;
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < nblk; ++b) {
        int64_t c0 = b * COLBLK;
        int64_t c1 = c0 + COLBLK < P ? c0 + COLBLK : P;
        int64_t w = c1 - c0;
        float acc[COLBLK];
        for (int64_t i = 0; i < N; ++i) {
            const uint16_t* row = X + i * ldx + c0;
            float ai = a[i];
            float si = s ? s[i] : 1.0f;
            for (int64_t j = 0; j < w; ++j) {
                float t = bf16_to_f32(row[j]) * ai;
                if (s) t = t * si;
                acc[j] = (i == 0) ? t : acc[j] + t;
            }
        }
        for (int64_t j = 0; j < w; ++j) {
            float o = acc[j] / divisor;
            out[c0 + j] = o;
            if (out_bf16) out_bf16[c0 + j] = f32_to_bf16_rne(o);
        }
    }
}

/* ---- synthetic generator, identical to fedlesscan_amd/synth.py ---------- */
#define GOLDEN 0x9E3779B97F4A7C15ULL
static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

void oracle_synth_f32(float* X, int64_t nrows, int64_t ncols, int64_t ldx, uint64_t seed,
                      int64_t row0, int64_t col0, int nthreads) {
    set_threads(nthreads);
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < nrows; ++r) {
        uint64_t key = mix64((seed * GOLDEN) ^ mix64((uint64_t)(row0 + r) + 1));
        float* row = X + r * ldx;
        for (int64_t j = 0; j < ncols; ++j) {
            uint64_t h = mix64(key + (uint64_t)(col0 + j + 1) * GOLDEN);
            int64_t v = (int64_t)(h & 0x1FFFFF) + (int64_t)((h >> 21) & 0x1FFFFF) +
                        (int64_t)((h >> 42) & 0x1FFFFF) - 3 * (1 << 20);
            row[j] = (float)v * 0x1p-24f;
        }
    }
}

void oracle_synth_bf16(uint16_t* X, int64_t nrows, int64_t ncols, int64_t ldx, uint64_t seed,
                       int64_t row0, int64_t col0, int nthreads) {
    set_threads(nthreads);
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < nrows; ++r) {
        uint64_t key = mix64((seed * GOLDEN) ^ mix64((uint64_t)(row0 + r) + 1));
        uint16_t* row = X + r * ldx;
        for (int64_t j = 0; j < ncols; ++j) {
            uint64_t h = mix64(key + (uint64_t)(col0 + j + 1) * GOLDEN);
            int64_t v = (int64_t)(h & 0x1FFFFF) + (int64_t)((h >> 21) & 0x1FFFFF) +
                        (int64_t)((h >> 42) & 0x1FFFFF) - 3 * (1 << 20);
            row[j] = f32_to_bf16_rne((float)v * 0x1p-24f);
        }
    }
}
