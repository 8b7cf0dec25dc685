/*
 * Host vector kernels: the OpenCL demo's element-wise multiply (ref 6-opencl-region-growing/
 * multiply_opencl.c:10-14) and the north-star "vector-add + dot 1e7 f32 on CPU/OpenMP" plumbing config.
 * Streaming loops are OpenMP static-partitioned and `omp simd` vectorised (AVX2 with -march=x86-64-v3).
 * Dot/sum accumulate in f64 per thread, so the result does not depend on the thread count beyond the
 * final (deterministic, thread-ordered) combine.
 */
#include <stdlib.h>
#include <sys/time.h>
#include "pcmx_cpu.h"
#ifdef _OPENMP
#include <omp.h>
#endif

int pcmx_omp_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

double pcmx_wtime(void) {
    struct timeval tv;
    gettimeofday(&tv, NULL);
    return (double)tv.tv_sec + 1e-6 * (double)tv.tv_usec;
}

void pcmx_vmul_host(const float* a, const float* b, float* r, long long n) {
#pragma omp simd
    for (long long i = 0; i < n; ++i) r[i] = a[i] * b[i];
}

static int nthreads_or_default(int n_threads) { return n_threads > 0 ? n_threads : pcmx_omp_max_threads(); }

void pcmx_vadd_omp(const float* a, const float* b, float* r, long long n, int n_threads) {
#pragma omp parallel for simd schedule(static) num_threads(nthreads_or_default(n_threads))
    for (long long i = 0; i < n; ++i) r[i] = a[i] + b[i];
}

void pcmx_axpy_omp(float alpha, const float* x, float* y, long long n, int n_threads) {
#pragma omp parallel for simd schedule(static) num_threads(nthreads_or_default(n_threads))
    for (long long i = 0; i < n; ++i) y[i] = alpha * x[i] + y[i];
}

double pcmx_dot_omp(const float* a, const float* b, long long n, int n_threads) {
    const int nt = nthreads_or_default(n_threads);
    double partial[256] = {0};
#pragma omp parallel num_threads(nt)
    {
        int t = 0, T = 1;
#ifdef _OPENMP
        t = omp_get_thread_num();
        T = omp_get_num_threads();
#endif
        long long lo = n * t / T, hi = n * (t + 1) / T;
        double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        long long i = lo;
        for (; i + 8 <= hi; i += 8)
#pragma omp simd
            for (int k = 0; k < 8; ++k) acc[k] += (double)a[i + k] * (double)b[i + k];
        double s = 0.0;
        for (; i < hi; ++i) s += (double)a[i] * (double)b[i];
        for (int k = 0; k < 8; ++k) s += acc[k];
        if (t < 256) partial[t] = s;
    }
    double s = 0.0;
    for (int t = 0; t < nt && t < 256; ++t) s += partial[t];
    return s;
}

double pcmx_sum_omp(const float* a, long long n, int n_threads) {
    const int nt = nthreads_or_default(n_threads);
    double s = 0.0;
#pragma omp parallel for simd reduction(+ : s) schedule(static) num_threads(nt)
    for (long long i = 0; i < n; ++i) s += (double)a[i];
    return s;
}
