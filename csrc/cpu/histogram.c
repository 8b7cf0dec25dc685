/*
 * Histogram equalisation on the host (components C6-C8):
 *   serial   ref 4-histogram-equalization-openmp-pthreads/histogram_serial.c:11-42
 *   OpenMP   ref histogram_omp.c:25-46     (the reference serialises every pixel through `omp critical`,
 *                                           B16; here each thread fills a private histogram and the
 *                                           partials are summed once — no lock in the pixel loop)
 *   pthreads ref histogram_pthreads.c:24-68 (cyclic partition and private histograms kept; the barrier is
 *                                           a generation-counting barrier, safe against spurious wakeups, B15)
 *
 * Transfer function: tf[v] = sum_{j<=v} fl(fl(255*h[j]) / npix), summed in f32 in increasing j — the
 * same rounding sequence as the reference's triangular loop, so outputs are bit-identical.
 * 256 bins (B14: the reference's 255-entry table overflows on pixel value 255).
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include "pcmx_cpu.h"
#ifdef _OPENMP
#include <omp.h>
#endif

void pcmx_histogram_u8(const unsigned char* img, int npix, int* hist) {
    /* 4 interleaved sub-histograms break the store->load dependency on runs of equal pixels */
    int h4[4][PCMX_HIST_BINS];
    memset(h4, 0, sizeof h4);
    int i = 0;
    for (; i + 4 <= npix; i += 4) {
        h4[0][img[i]]++;
        h4[1][img[i + 1]]++;
        h4[2][img[i + 2]]++;
        h4[3][img[i + 3]]++;
    }
    for (; i < npix; ++i) h4[0][img[i]]++;
    for (int b = 0; b < PCMX_HIST_BINS; ++b) hist[b] = h4[0][b] + h4[1][b] + h4[2][b] + h4[3][b];
}

void pcmx_transfer_function(const int* hist, int npix, float* tf) {
    float run = 0.0f;
    for (int v = 0; v < PCMX_HIST_BINS; ++v) {
        run += (255.0f * (float)hist[v]) / (float)npix;
        tf[v] = run;
    }
}

static void apply_tf(const unsigned char* img, unsigned char* out, long lo, long hi, long step, const float* tf) {
    for (long i = lo; i < hi; i += step) out[i] = (unsigned char)tf[img[i]];
}

void pcmx_histeq_serial(const unsigned char* img, unsigned char* out, int npix) {
    int hist[PCMX_HIST_BINS];
    float tf[PCMX_HIST_BINS];
    pcmx_histogram_u8(img, npix, hist);
    pcmx_transfer_function(hist, npix, tf);
    apply_tf(img, out, 0, npix, 1, tf);
}

void pcmx_histeq_omp(const unsigned char* img, unsigned char* out, int npix, int n_threads) {
    int hist[PCMX_HIST_BINS];
    float tf[PCMX_HIST_BINS];
    memset(hist, 0, sizeof hist);
    if (n_threads < 1) n_threads = 1;
#pragma omp parallel num_threads(n_threads)
    {
        int local[PCMX_HIST_BINS];
        memset(local, 0, sizeof local);
#pragma omp for schedule(static) nowait
        for (int i = 0; i < npix; ++i) local[img[i]]++;
        for (int b = 0; b < PCMX_HIST_BINS; ++b)
            if (local[b]) {
#pragma omp atomic
                hist[b] += local[b];
            }
#pragma omp barrier
#pragma omp single
        pcmx_transfer_function(hist, npix, tf);
#pragma omp for schedule(static)
        for (int i = 0; i < npix; ++i) out[i] = (unsigned char)tf[img[i]];
    }
}

/* ------------------------------------------------------------------ pthreads version */

typedef struct {
    pthread_mutex_t mu;
    pthread_cond_t cv;
    int count, parties;
    unsigned long generation;
} gen_barrier_t;

static void gen_barrier_wait(gen_barrier_t* b) {
    pthread_mutex_lock(&b->mu);
    unsigned long gen = b->generation;
    if (++b->count == b->parties) {
        b->count = 0;
        b->generation++;
        pthread_cond_broadcast(&b->cv);
    } else {
        while (gen == b->generation) pthread_cond_wait(&b->cv, &b->mu);
    }
    pthread_mutex_unlock(&b->mu);
}

typedef struct {
    const unsigned char* img;
    unsigned char* out;
    int npix, n_threads;
    int hist[PCMX_HIST_BINS];
    float tf[PCMX_HIST_BINS];
    pthread_mutex_t merge;
    gen_barrier_t bar;
} histeq_job_t;

typedef struct {
    histeq_job_t* job;
    long tid;
} histeq_arg_t;

static void* histeq_worker(void* p) {
    histeq_arg_t* a = (histeq_arg_t*)p;
    histeq_job_t* j = a->job;
    const long t = a->tid, n = j->n_threads;
    int local[PCMX_HIST_BINS];
    memset(local, 0, sizeof local);
    for (long i = t; i < j->npix; i += n) local[j->img[i]]++; /* cyclic partition, as the reference */
    pthread_mutex_lock(&j->merge);
    for (int b = 0; b < PCMX_HIST_BINS; ++b) j->hist[b] += local[b];
    pthread_mutex_unlock(&j->merge);
    gen_barrier_wait(&j->bar);
    /* each thread owns tf entries v = t, t+n, ... computed as the in-order f32 prefix (bit-exact) */
    for (long v = t; v < PCMX_HIST_BINS; v += n) {
        float run = 0.0f;
        for (long k = 0; k <= v; ++k) run += (255.0f * (float)j->hist[k]) / (float)j->npix;
        j->tf[v] = run;
    }
    gen_barrier_wait(&j->bar);
    apply_tf(j->img, j->out, t, j->npix, n, j->tf);
    return NULL;
}

void pcmx_histeq_pthreads(const unsigned char* img, unsigned char* out, int npix, int n_threads) {
    if (n_threads < 1) n_threads = 1;
    histeq_job_t job;
    memset(&job, 0, sizeof job);
    job.img = img, job.out = out, job.npix = npix, job.n_threads = n_threads;
    pthread_mutex_init(&job.merge, NULL);
    pthread_mutex_init(&job.bar.mu, NULL);
    pthread_cond_init(&job.bar.cv, NULL);
    job.bar.parties = n_threads;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)n_threads);
    histeq_arg_t* args = (histeq_arg_t*)malloc(sizeof(histeq_arg_t) * (size_t)n_threads);
    for (long t = 0; t < n_threads; ++t) {
        args[t].job = &job;
        args[t].tid = t;
        pthread_create(&th[t], NULL, histeq_worker, &args[t]);
    }
    for (int t = 0; t < n_threads; ++t) pthread_join(th[t], NULL);
    pthread_cond_destroy(&job.bar.cv);
    pthread_mutex_destroy(&job.bar.mu);
    pthread_mutex_destroy(&job.merge);
    free(th);
    free(args);
}
