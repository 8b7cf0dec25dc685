/*
 * pcmx_cpu.h — host-side C API of the pcmx framework (libpcmx_cpu.so).
 *
 * Keeps the reference's C entry-point signatures and output formats:
 *   BMP I/O            read_bmp / write_bmp  (ref 2-mpi-region-growing/bmp.c:6-71, bmp.h:6-35)
 *   dense matrix_t     new_matrix … free_matrix (ref 1-introduction/matrix.c:4-114)
 *   CSR / banded SpMV  create_csr_matrix, multiply_naive, multiply, compare (ref 3-serial-optimization/spmv.c)
 *   histogram equal.   serial / OpenMP / pthreads (ref 4-histogram-equalization-openmp-pthreads/*.c)
 *   vector ops         vmul / vadd / dot on the host (ref 6-opencl-region-growing/multiply_opencl.c:10-14)
 *   serial oracles     2D/3D flood fill, software ray caster, volume generator
 *                      (ref 2-mpi-region-growing/region.c:493-533, 5-cuda-region-growing/raycast.cu:114-318)
 *
 * The implementations are new: contiguous storage, OpenMP/AVX2 where it pays, bug fixes documented
 * in docs/COMPAT.md (B1..B27 of SURVEY.md appendix A).
 */
#ifndef PCMX_CPU_H
#define PCMX_CPU_H

#include <stdint.h>
#include <stddef.h>
#include <sys/time.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ BMP (C1) */
/* Writes ./out.bmp: 8-bit gray, 1078-byte header+palette, file_size = w*h + 56 (reference formula). */
void write_bmp(unsigned char* data, int width, int height);
/* Reads width@18, height@22, pixel offset@10 then width*height bytes (row padding ignored). */
unsigned char* read_bmp(char* filename);
/* Extended forms: explicit path, dimensions out, status return (0 ok, <0 error). */
int pcmx_write_bmp_path(const char* path, const unsigned char* data, int width, int height);
unsigned char* pcmx_read_bmp_dims(const char* path, int* width, int* height);
void pcmx_free(void* p);

/* ------------------------------------------------------------- matrix_t (C2) */
typedef struct {
    float** data; /* row pointers into one contiguous, 64-B aligned block (data[0]) */
    int rows;
    int cols;
} matrix_t;

matrix_t* new_matrix(int rows, int cols);
void print_matrix(matrix_t* matrix);
void set_value(matrix_t* matrix, int row, int col, float value);
float get_value(matrix_t* matrix, int row, int col);
/* fraction of zero entries >= threshold (fixed semantics, see B1). */
int is_sparse(matrix_t matrix, float sparse_threshold);
/* reference formula total/zeros >= threshold, kept for the --compat demo (B1). */
int is_sparse_compat(matrix_t matrix, float sparse_threshold);
/* c = a*b; -1 on shape mismatch. Large products go to the registered GPU GEMM backend. */
int matrix_multiply(matrix_t* a, matrix_t* b, matrix_t** c);
void change_size(matrix_t* matrix, int new_rows, int new_cols);
void free_matrix(matrix_t* matrix);

/* GEMM backend hook: row-major C[MxN] = A[MxK] * B[KxN]; returns 0 on success. */
typedef int (*pcmx_gemm_fn)(const float* a, const float* b, float* c, int m, int n, int k);
void pcmx_set_gemm_backend(pcmx_gemm_fn fn, long long min_flops);
/* Multithreaded cache-blocked host SGEMM (the CPU fallback). */
void pcmx_sgemm_host(const float* a, const float* b, float* c, int m, int n, int k);
/* The reference's i-j-k triple loop (for the baseline benchmark only). */
void pcmx_sgemm_naive(const float* a, const float* b, float* c, int m, int n, int k);

/* ------------------------------------------------------------------ SpMV (C5) */
typedef struct {
    int n_row_ptr;
    int* row_ptr;
    int* col_ind;
    int n_values;
    float* values;
} csr_matrix_t;

typedef struct {
    float* values;
    int n, a, b, c, d, e;
} s_matrix_t;

int diag_count(int dim, int n);
csr_matrix_t* create_csr_matrix(int n_rows, int n_cols, int a, int b, int c, int d, int e);
void free_csr_matrix(csr_matrix_t* m);
float* create_vector(int n);
void print_raw_csr_matrix(csr_matrix_t* m);
void print_formated_csr_matrix(csr_matrix_t* m);
void print_vector(float* v, int n, int orientation);
void print_time(struct timeval start, struct timeval end);
void print_time_seconds(double seconds); /* "Time : %f s" for a device-timed product */
void multiply_naive(csr_matrix_t* m, float* v, float* r);
void compare(float* a, float* b, int n);
s_matrix_t* create_s_matrix(int dim, int a, int b, int c, int d, int e);
s_matrix_t* convert_to_s_matrix(csr_matrix_t* csr, int n, int a, int b, int c, int d, int e);
/* banded SpMV with implicit column indices, AVX2 (replaces the SSE kernel of spmv.c:212-329). */
void multiply(s_matrix_t* matrix, float* v, float* r);
/* multithreaded variants */
void pcmx_spmv_csr_omp(int n_rows, const int* row_ptr, const int* col_ind, const float* values,
                       const float* v, float* r);
void pcmx_spmv_banded_omp(const s_matrix_t* matrix, const float* v, float* r);
/* band limits of row i: 5 half-open column ranges [lo[k], hi[k]) (the row's nnz in order). */
void pcmx_band_ranges(int n, int a, int b, int c, int d, int e, int row, int lo[5], int hi[5]);
/* Power-law (Chung–Lu) CSR generator: expected degree ~ (i+1)^(-1/(alpha-1)) scaled to nnz. */
long long pcmx_powerlaw_row_counts(int n_rows, long long target_nnz, double alpha, unsigned long long seed,
                                   long long* row_ptr /* n_rows+1 */);
void pcmx_powerlaw_fill(int n_rows, int n_cols, const long long* row_ptr, unsigned long long seed,
                        int* col_ind, float* values);
/* rows [row0, row1) only (a rank's block; bit-identical to the same rows of pcmx_powerlaw_fill);
 * outputs start at row_ptr[row0]. */
void pcmx_powerlaw_fill_rows(int row0, int row1, int n_cols, const long long* row_ptr, unsigned long long seed,
                             int* col_ind, float* values);

/* -------------------------------------------------- histogram equalization (C6-C8) */
#define PCMX_HIST_BINS 256
/* All three compute out[i] = (uint8)tf[img[i]], tf[v] = sum_{j<=v} fl(255*h[j]) / npix (f32, in order). */
void pcmx_histeq_serial(const unsigned char* img, unsigned char* out, int npix);
void pcmx_histeq_omp(const unsigned char* img, unsigned char* out, int npix, int n_threads);
void pcmx_histeq_pthreads(const unsigned char* img, unsigned char* out, int npix, int n_threads);
void pcmx_histogram_u8(const unsigned char* img, int npix, int* hist /*256*/);
void pcmx_transfer_function(const int* hist, int npix, float* tf /*256*/);

/* ------------------------------------------------------ vector ops (C12, north-star #1) */
void pcmx_vmul_host(const float* a, const float* b, float* r, long long n);
void pcmx_vadd_omp(const float* a, const float* b, float* r, long long n, int n_threads);
double pcmx_dot_omp(const float* a, const float* b, long long n, int n_threads);
double pcmx_sum_omp(const float* a, long long n, int n_threads);
void pcmx_axpy_omp(float alpha, const float* x, float* y, long long n, int n_threads);

/* ------------------------------------------------------------- serial oracles */
/* 2D region growing on a w x h image (4-connectivity, |a-b| < threshold), seeds in (x,y) pairs.
 * region[] gets 1 for region pixels. Returns region size. */
long long pcmx_region2d_serial(const unsigned char* img, int w, int h, const int* seeds_xy, int n_seeds,
                               int threshold, unsigned char* region);
/* 3D flood fill on a dim^3 volume, 6-connectivity, |a-b| < threshold (reference: 1). */
long long pcmx_region3d_serial(const unsigned char* data, int dim, int sx, int sy, int sz, int threshold,
                               unsigned char* region);
/* Reference volume (ref raycast.cu:114-158): glibc rand()%20 background, spheres/boxes on top. */
void pcmx_create_data(unsigned char* data, int dim);
/* Deterministic hash-background variant (same foreground) matching the GPU generator. */
void pcmx_create_data_hash(unsigned char* data, int dim, unsigned int seed);
/* Camera constants shared by every ray caster (ref raycast.cu:216-241). */
typedef struct {
    float camera[3], forward[3], right[3], up[3];
    float pixel_width, step_size;
    int max_steps;
} pcmx_camera_t;
void pcmx_default_camera(int image_dim, pcmx_camera_t* cam);
/* z-slab decomposition (parallel/volume3d.py): planes [z_first, z_first + nplanes) of the hash volume (zeros
 * outside 0..dim-1); slab flood fill over nz owned planes at data/region with read-only halo planes -1 / nz
 * (halos bit 0 / 1), returns the voxels added; slab ray caster: the reference march restricted to samples with
 * z >= z0 (all samples on the bottom slab), carried per pixel in state[6] = {pos xyz, colour (f32 bits), steps,
 * flags}, slab buffers starting at global plane z0 - 1, image written by the bottom slab. */
void pcmx_create_data_hash_slab(unsigned char* data, int dim, int z_first, int nplanes, unsigned int seed);
long long pcmx_region3d_slab_host(const unsigned char* data, unsigned char* region, int dim, int nz, int halos, int thr);
void pcmx_raycast_slab_host(const unsigned char* data, const unsigned char* region, int dim, int z0, int z1,
                            int image_dim, int* state, int init, int bottom, unsigned char* image);
/* Serial software ray caster, bit-compatible with the reference value_at() (swapped weights, B21). */
void pcmx_raycast_serial(const unsigned char* data, const unsigned char* region, int dim, int image_dim,
                         unsigned char* image);

/* ---------------------------------------------------------------- misc */
double pcmx_wtime(void);
int pcmx_omp_max_threads(void);

/* ---------------------------------------------------------------- reference programs (demos.c) */
int pcmx_matrix_demo(int compat);
int pcmx_spmv_demo(int dim, int a, int b, int c, int d, int e);
int pcmx_histogram_demo(const char* image, int n_threads, int method);
int pcmx_vecops_demo(long long n, int n_threads, int reps);

#ifdef __cplusplus
}
#endif
#endif /* PCMX_CPU_H */
