/*
 * tcsc_oracle.c -- CPU restatement of the reference TCSC path.
 * TEST INFRASTRUCTURE ONLY (see tcsc_oracle.h for scope and pinning).
 *
 * Built with the reference's arithmetic flags (Makefile:5, gcc spelling):
 * -O3 -fno-tree-vectorize -fno-tree-slp-vectorize, no fast-math, so each
 * float add/sub is one IEEE binary32 operation in program order.
 */
#include "tcsc_oracle.h"

#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#if defined(__x86_64__)
#include <x86intrin.h>
#endif

/* ---------------------------------------------------------------- inputs -- */

uint64_t oracle_splitmix64(uint64_t *state)
{
    uint64_t z = (*state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

uint64_t oracle_below(uint64_t *state, uint64_t n)
{
    if (n <= 1)
        return 0;
    const uint64_t thresh = (0 - n) % n; /* 2^64 mod n: reject to stay unbiased */
    uint64_t x;
    do {
        x = oracle_splitmix64(state);
    } while (x < thresh);
    return x % n;
}

/* sparseUtils.h:52-87 (uniformDistribution=false). */
void oracle_gen_ternary(int K, int N, int s, uint64_t seed, int32_t *W)
{
    memset(W, 0, sizeof(int32_t) * (size_t)K * (size_t)N);
    uint64_t st = seed;
    const int per_row = (s > 0) ? N / s : 0;
    const int half = per_row / 2;
    const int vari = per_row / 20 + 1; /* variRange(0, W/nonZero/20 + 1), :56 */
    for (int k = 0; k < K; k++) {
        int32_t *row = W + (size_t)k * N;
        const int v = (int)oracle_below(&st, (uint64_t)vari + 1);
        int npos = half + v, nneg = half - v; /* :60-61 */
        if (npos > N) npos = N;
        if (nneg < 0) nneg = 0;
        if (nneg > N - npos) nneg = N - npos;
        for (int c = 0; c < npos;) { /* :64-73 */
            const int col = (int)oracle_below(&st, (uint64_t)N);
            if (row[col] == 0) { row[col] = 1; c++; }
        }
        for (int c = 0; c < nneg;) { /* :76-85 */
            const int col = (int)oracle_below(&st, (uint64_t)N);
            if (row[col] == 0) { row[col] = -1; c++; }
        }
    }
}

void oracle_init_x_int(int64_t len, int range, uint64_t seed, float *X)
{
    uint64_t st = seed;
    for (int64_t i = 0; i < len; i++)
        X[i] = (float)((int64_t)oracle_below(&st, 2ull * (uint64_t)range + 1) - range);
}

void oracle_init_x_frac(int64_t len, uint64_t seed, float *X)
{
    uint64_t st = seed;
    for (int64_t i = 0; i < len; i++) {
        const int64_t mant = (int64_t)oracle_below(&st, 1ull << 24) - (1ll << 23);
        const int e = (int)oracle_below(&st, 24);
        float v = (float)mant;
        for (int j = 0; j < e; j++) v *= 0.5f; /* exact scaling by 2^-e */
        X[i] = v;
    }
}

/* ----------------------------------------------------------------- formats -- */

void oracle_tcsc_count(const int32_t *W, int K, int N, int64_t *nnz_pos, int64_t *nnz_neg)
{
    int64_t p = 0, q = 0;
    for (int64_t i = 0; i < (int64_t)K * N; i++) {
        p += (W[i] == 1);
        q += (W[i] == -1);
    }
    *nnz_pos = p;
    *nnz_neg = q;
}

/* TCSC.h:13-41 */
void oracle_tcsc_encode(const int32_t *W, int K, int N,
                        int32_t *csp, int32_t *csn, int32_t *rip, int32_t *rin)
{
    int32_t cp = 0, cn = 0;
    for (int n = 0; n < N; n++) {
        csp[n] = cp; /* :20-21 */
        csn[n] = cn;
        for (int k = 0; k < K; k++) { /* :23-36 */
            const int32_t v = W[(size_t)k * N + n];
            if (v == 1) rip[cp++] = k;
            else if (v == -1) rin[cn++] = k;
        }
    }
    csp[N] = cp; /* :39-40 */
    csn[N] = cn;
}

int64_t oracle_tcsc_size_bytes(int N, int64_t nnz_pos, int64_t nnz_neg)
{
    return 4 * (2 * ((int64_t)N + 1) + nnz_pos + nnz_neg); /* TCSC.h:43-49 */
}

void oracle_tcsc_decode(const int32_t *csp, const int32_t *csn, const int32_t *rip,
                        const int32_t *rin, int K, int N, int32_t *W)
{
    memset(W, 0, sizeof(int32_t) * (size_t)K * (size_t)N);
    for (int n = 0; n < N; n++) {
        for (int32_t i = csp[n]; i < csp[n + 1]; i++) W[(size_t)rip[i] * N + n] = 1;
        for (int32_t i = csn[n]; i < csn[n + 1]; i++) W[(size_t)rin[i] * N + n] = -1;
    }
}

void oracle_blocked_tcsc_count(const int32_t *W, int K, int N, int B, int64_t *nnz_pos,
                               int64_t *nnz_neg)
{
    (void)B;
    oracle_tcsc_count(W, K, N, nnz_pos, nnz_neg);
}

/* BlockedTCSC.h:15-41 */
void oracle_blocked_tcsc_encode(const int32_t *W, int K, int N, int B,
                                int32_t *csp, int32_t *csn, int32_t *rip, int32_t *rin)
{
    int32_t cp = 0, cn = 0;
    int64_t slot = 0;
    for (int kb = 0; kb < K / B; kb++) {
        for (int n = 0; n < N; n++) {
            csp[slot] = cp;
            csn[slot] = cn;
            slot++;
            for (int i = 0; i < B; i++) {
                const int k = kb * B + i;
                const int32_t v = W[(size_t)k * N + n];
                if (v == 1) rip[cp++] = k;
                else if (v == -1) rin[cn++] = k;
            }
        }
    }
    csp[slot] = cp;
    csn[slot] = cn;
}

void oracle_csc_packed_encode(const int32_t *W, int K, int N, int32_t *col_ptr, int32_t *row_idx,
                              uint8_t *packed)
{
    static const int pw[5] = {1, 3, 9, 27, 81};
    int64_t e = 0;
    for (int n = 0; n < N; n++) {
        col_ptr[n] = (int32_t)e;
        for (int k = 0; k < K; k++) {
            const int32_t v = W[(size_t)k * N + n];
            if (v == 1 || v == -1) {
                row_idx[e] = k;
                if (e % 5 == 0) packed[e / 5] = 0;
                packed[e / 5] = (uint8_t)(packed[e / 5] + (v + 1) * pw[e % 5]);
                e++;
            }
        }
    }
    col_ptr[N] = (int32_t)e;
}

int oracle_csc_packed_value(const uint8_t *packed, int64_t i)
{
    int b = packed[i / 5];
    for (int j = 0; j < (int)(i % 5); j++) b /= 3;
    return b % 3 - 1;
}

/* ----------------------------------------------------------------- kernels -- */

static inline float base_tcsc_one(const float *xrow, const int32_t *csp, const int32_t *csn,
                                  const int32_t *rip, const int32_t *rin, int n)
{
    float y = 0.0f; /* comp.h:41 */
    for (int32_t k = csp[n]; k < csp[n + 1]; k++) /* comp.h:44-51 */
        y += xrow[rip[k]];
    for (int32_t k = csn[n]; k < csn[n + 1]; k++) /* comp.h:54-61 */
        y -= xrow[rin[k]];
    return y;
}

/* comp.h:25-69 */
void oracle_base_tcsc(const float *X, const int32_t *csp, const int32_t *csn, const int32_t *rip,
                      const int32_t *rin, const float *b, float *Y, int M, int N, int K)
{
    for (int m = 0; m < M; m++) {
        const float *xrow = X + (size_t)m * K;
        float *yrow = Y + (size_t)m * N;
        for (int n = 0; n < N; n++)
            yrow[n] = base_tcsc_one(xrow, csp, csn, rip, rin, n) + b[n]; /* comp.h:63 */
    }
}

void oracle_base_tcsc_omp(const float *X, const int32_t *csp, const int32_t *csn,
                          const int32_t *rip, const int32_t *rin, const float *b, float *Y,
                          int M, int N, int K, int nthreads)
{
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(static)
#else
    (void)nthreads;
#endif
    for (int m = 0; m < M; m++) {
        const float *xrow = X + (size_t)m * K;
        float *yrow = Y + (size_t)m * N;
        for (int n = 0; n < N; n++)
            yrow[n] = base_tcsc_one(xrow, csp, csn, rip, rin, n) + b[n];
    }
}

/* comp.h:1227-1438 with K_UNROLL_FACTOR = 4, M_UNROLL_FACTOR = 4 */
#define KU 4
#define MU 4
void oracle_double_unrolled_tcsc_k4m4(const float *X, const int32_t *csp, const int32_t *csn,
                                      const int32_t *rip, const int32_t *rin, const float *b,
                                      float *Y, int M, int N, int K)
{
    int m;
    for (m = 0; m <= M - MU; m += MU) { /* :1240 */
        for (int n = 0; n < N; n++) {
            float yp[MU][KU], yn[MU][KU];
            for (int v = 0; v < MU; v++)
                for (int u = 0; u < KU; u++) yp[v][u] = yn[v][u] = 0.0f;
            int kp = csp[n];
            const int ep = csp[n + 1];
            for (; kp + KU <= ep; kp += KU) /* :1261-1273 */
                for (int u = 0; u < KU; u++) {
                    const int r = rip[kp + u];
                    for (int v = 0; v < MU; v++) yp[v][u] += X[(size_t)(m + v) * K + r];
                }
            float ypf[MU];
            for (int v = 0; v < MU; v++) { /* :1276-1286 */
                ypf[v] = 0.0f;
                for (int u = 0; u < KU; u++) ypf[v] += yp[v][u];
            }
            for (; kp < ep; kp++) { /* :1289-1298 */
                const int r = rip[kp];
                for (int v = 0; v < MU; v++) ypf[v] += X[(size_t)(m + v) * K + r];
            }
            int kn = csn[n];
            const int en = csn[n + 1];
            for (; kn + KU <= en; kn += KU) /* :1304-1316 */
                for (int u = 0; u < KU; u++) {
                    const int r = rin[kn + u];
                    for (int v = 0; v < MU; v++) yn[v][u] += X[(size_t)(m + v) * K + r];
                }
            float ynf[MU];
            for (int v = 0; v < MU; v++) { /* :1319-1329 */
                ynf[v] = 0.0f;
                for (int u = 0; u < KU; u++) ynf[v] += yn[v][u];
            }
            for (; kn < en; kn++) { /* :1332-1341 */
                const int r = rin[kn];
                for (int v = 0; v < MU; v++) ynf[v] += X[(size_t)(m + v) * K + r];
            }
            for (int v = 0; v < MU; v++) /* :1344-1350 */
                Y[(size_t)(m + v) * N + n] = (ypf[v] - ynf[v]) + b[n];
        }
    }
    for (; m < M; m++) { /* cleanup rows, :1355-1436 */
        const float *xr = X + (size_t)m * K;
        for (int n = 0; n < N; n++) {
            float yp[KU] = {0}, yn[KU] = {0};
            int kp = csp[n];
            const int ep = csp[n + 1];
            for (; kp + KU <= ep; kp += KU)
                for (int u = 0; u < KU; u++) yp[u] += xr[rip[kp + u]];
            float ypf = 0.0f;
            for (int u = 0; u < KU; u++) ypf += yp[u];
            for (; kp < ep; kp++) ypf += xr[rip[kp]];
            int kn = csn[n];
            const int en = csn[n + 1];
            for (; kn + KU <= en; kn += KU)
                for (int u = 0; u < KU; u++) yn[u] += xr[rin[kn + u]];
            float ynf = 0.0f;
            for (int u = 0; u < KU; u++) ynf += yn[u];
            for (; kn < en; kn++) ynf += xr[rin[kn]];
            Y[(size_t)m * N + n] = (ypf - ynf) + b[n];
        }
    }
}
#undef KU
#undef MU

/* comp_prelu.h:12-70 */
void oracle_base_tcsc_prelu(const float *X, const int32_t *csp, const int32_t *csn,
                            const int32_t *rip, const int32_t *rin, const float *b,
                            const float *alpha, float *Y, int M, int N, int K)
{
    for (int m = 0; m < M; m++) {
        const float *xrow = X + (size_t)m * K;
        float *yrow = Y + (size_t)m * N;
        for (int n = 0; n < N; n++) {
            float y = base_tcsc_one(xrow, csp, csn, rip, rin, n);
            y = y + b[n];                            /* :50 */
            yrow[n] = (y > 0) ? y : alpha[n] * y;    /* :57-67 */
        }
    }
}

/* comp.h:607-658; assumes Y zero-initialised as main.cpp:211 does. */
void oracle_base_blocked_tcsc(const float *X, const int32_t *csp, const int32_t *csn,
                              const int32_t *rip, const int32_t *rin, const float *b, float *Y,
                              int M, int N, int K, int B)
{
    for (int m = 0; m < M; m++) {
        const float *xrow = X + (size_t)m * K;
        float *yrow = Y + (size_t)m * N;
        for (int n = 0; n < N; n++) yrow[n] = 0.0f;
        for (int kb = 0; kb < K / B; kb++) {
            for (int n = 0; n < N; n++) {
                const int64_t s = (int64_t)kb * N + n;
                float y = 0.0f;
                for (int32_t k = csp[s]; k < csp[s + 1]; k++) y += xrow[rip[k]];
                for (int32_t k = csn[s]; k < csn[s + 1]; k++) y -= xrow[rin[k]];
                yrow[n] += y; /* :641 */
            }
        }
        for (int n = 0; n < N; n++) yrow[n] += b[n]; /* :648-654 */
    }
}

void oracle_base_csc_packed(const float *X, const int32_t *col_ptr, const int32_t *row_idx,
                            const uint8_t *packed, const float *b, float *Y, int M, int N, int K)
{
    for (int m = 0; m < M; m++) {
        const float *xrow = X + (size_t)m * K;
        for (int n = 0; n < N; n++) {
            float y = 0.0f;
            for (int32_t i = col_ptr[n]; i < col_ptr[n + 1]; i++)
                if (oracle_csc_packed_value(packed, i) == 1) y += xrow[row_idx[i]];
            for (int32_t i = col_ptr[n]; i < col_ptr[n + 1]; i++)
                if (oracle_csc_packed_value(packed, i) == -1) y -= xrow[row_idx[i]];
            Y[(size_t)m * N + n] = y + b[n];
        }
    }
}

/* sparseUtils.h:92-108 */
void oracle_gemm_dense(const float *X, const float *W, const float *b, float *Y, int M, int N, int K)
{
    for (int m = 0; m < M; m++)
        for (int n = 0; n < N; n++) {
            float y = 0.0f;
            for (int k = 0; k < K; k++) y += X[(size_t)m * K + k] * W[(size_t)k * N + n];
            Y[(size_t)m * N + n] = y + b[n];
        }
}

/* ------------------------------------------------------------------ timing -- */

/* The reference's measurement method, perf.cpp:37-71 (rdtsc) with CALIBRATE
 * on (Makefile:11-16): starting at NUM_RUNS = 1 (perf.cpp:28) the run count
 * doubles until one batch of runs takes >= CYCLES_REQUIRED TSC cycles
 * (perf.cpp:29, 1e8) or 2^14 runs, then that many runs are timed again and
 * the average is returned.  Here the TSC is read with __rdtsc() (tsc_x86.h
 * uses rdtsc behind cpuid serialisation) and the wall-clock seconds of the
 * timed batch are reported beside the cycles, because the TSC rate of the host
 * is not known a priori.  kernel: 0 BaseTCSC (comp.h:25-69), 1 BaseTCSC with
 * OpenMP over rows (`threads`), 2 DoubleUnrolledTCSC<4,4> (comp.h:1227-1438). */
static uint64_t tsc_now(void)
{
#if defined(__x86_64__)
    return __rdtsc();
#else
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
#endif
}

static double wall_now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void run_kernel(int kernel, int threads, const float *X, const int32_t *csp, const int32_t *csn,
                       const int32_t *rip, const int32_t *rin, const float *b, float *Y, int M, int N, int K)
{
    if (kernel == 1) oracle_base_tcsc_omp(X, csp, csn, rip, rin, b, Y, M, N, K, threads);
    else if (kernel == 2) oracle_double_unrolled_tcsc_k4m4(X, csp, csn, rip, rin, b, Y, M, N, K);
    else oracle_base_tcsc(X, csp, csn, rip, rin, b, Y, M, N, K);
}

double oracle_perf_calibrated(int kernel, int threads, double cycles_required, const float *X,
                              const int32_t *csp, const int32_t *csn, const int32_t *rip, const int32_t *rin,
                              const float *b, float *Y, int M, int N, int K, int64_t *num_runs,
                              double *cycles_per_run)
{
    int64_t runs = 1; /* NUM_RUNS, perf.cpp:28 */
    while (runs < (1 << 14)) { /* perf.cpp:46-60 */
        const uint64_t t0 = tsc_now();
        for (int64_t i = 0; i < runs; i++) run_kernel(kernel, threads, X, csp, csn, rip, rin, b, Y, M, N, K);
        if ((double)(tsc_now() - t0) >= cycles_required) break;
        runs *= 2;
    }
    const double w0 = wall_now();
    const uint64_t t0 = tsc_now(); /* perf.cpp:62-69 */
    for (int64_t i = 0; i < runs; i++) run_kernel(kernel, threads, X, csp, csn, rip, rin, b, Y, M, N, K);
    const uint64_t cyc = tsc_now() - t0;
    const double secs = wall_now() - w0;
    if (num_runs) *num_runs = runs;
    if (cycles_per_run) *cycles_per_run = (double)cyc / (double)runs;
    return secs / (double)runs;
}
