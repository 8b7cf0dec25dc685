/*
 * pcmx_hip.h — C ABI of libpcmx_hip.so: every MI355X (gfx950) kernel of the framework.
 *
 * Conventions
 *  - All pointers are DEVICE pointers unless the name says host. Every launcher is asynchronous on the
 *    given stream, allocates nothing and never synchronises, so a caller may capture it into a hipGraph.
 *    Workspaces are caller-provided; pcmx_*_workspace_bytes() says how much.
 *  - Return value: 0 on success, a hipError_t (> 0), or one of the PCMX_ERR_* codes below (< 0).
 *  - No launcher keeps process-global tuning state: every knob is a per-call argument.
 *  - Element counts are 64-bit: 1e9-element arrays (4 GB) are first-class on a 288 GB MI355X.
 *
 * Reference parity (file:line in anonyomous4/parallel-c-programs):
 *  vmul            6-opencl-region-growing/multiply_opencl.cl:1-4
 *  sgemm           1-introduction/matrix.c:63-81 (matrix_multiply) — fp32 MFMA on gfx950
 *  histeq          4-histogram-equalization-openmp-pthreads/histogram_serial.c:11-42
 *  region2d        2-mpi-region-growing/region.c:493-533 (flood fill, tile + 1-px halo)
 *  region3d_*      5-cuda-region-growing/raycast.cu:534-699 (naive + shared-memory kernels)
 *  raycast_*       5-cuda-region-growing/raycast.cu:321-433 (global-memory + texture kernels)
 *  volume_gen      5-cuda-region-growing/raycast.cu:114-158
 *  spmv_*          3-serial-optimization/spmv.c:170-329
 */
#ifndef PCMX_HIP_H
#define PCMX_HIP_H

#include <stdint.h>
#include <hip/hip_runtime_api.h>

#include "pcmx_errors.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- error codes: pcmx_errors.h */

/* ---------------------------------------------------------------- runtime / device info */
int pcmx_device_count(void);
/* Prints count, name, gcnArchName, CUs, LDS/CU, L2, HBM size, clock (replaces print_properties /
 * printDeviceInfo, ref raycast.cu:99-110, clutil.c:63-122). */
void pcmx_print_device_info(int device);
const char* pcmx_error_string(int err);
/* registers the MFMA SGEMM as matrix_multiply()'s backend (host matrices, copies in/out). */
void pcmx_register_gemm_backend(long long min_flops);
int pcmx_sgemm_host_arrays(const float* a, const float* b, float* c, int m, int n, int k);

/* ---------------------------------------------------------------- element-wise (HBM-bound) */
int pcmx_vmul_f32(const float* a, const float* b, float* r, long long n, hipStream_t s);
int pcmx_vadd_f32(const float* a, const float* b, float* r, long long n, hipStream_t s);
int pcmx_axpy_f32(float alpha, const float* x, float* y, long long n, hipStream_t s);
int pcmx_copy_f32(const float* a, float* r, long long n, hipStream_t s);
// dst[i] = src[idx[i]] (32-bit indices; an index outside [0, n_src) reads 0); idx, dst 16-B aligned
int pcmx_gather_f32(const float* src, long long n_src, const int* idx, float* dst, long long n, hipStream_t s);
int pcmx_fill_f32(float* x, float v, long long n, hipStream_t s);
/* x[i] = uniform[lo,hi) from a counter-based hash of (seed, i): on-device synthetic data */
int pcmx_rand_uniform_f32(float* x, long long n, unsigned long long seed, float lo, float hi, hipStream_t s);

/* ---------------------------------------------------------------- reductions */
enum { PCMX_OP_SUM = 0, PCMX_OP_MIN = 1, PCMX_OP_MAX = 2 };
/* number of first-pass partials the reduce launchers use (workspace = that many elements * 8 B) */
long long pcmx_reduce_workspace_bytes(long long n);
/* out[0] = op(x[0..n)) ; two passes, deterministic (fixed grid, fixed combine order) */
int pcmx_reduce_f32(const float* x, long long n, int op, float* out, void* workspace, hipStream_t s);
int pcmx_reduce_i32(const int32_t* x, long long n, int op, int32_t* out, void* workspace, hipStream_t s);
/* out[0] = sum a*b */
int pcmx_dot_f32(const float* a, const float* b, long long n, float* out, void* workspace, hipStream_t s);

/* ---------------------------------------------------------------- prefix scan */
long long pcmx_scan_workspace_bytes(long long n);
/* out[i] = init + sum_{j<=i} x[j] (inclusive) or init + sum_{j<i} x[j] (exclusive), single pass with
 * decoupled look-back; init is read from device memory (init_dev may be NULL => 0) so a multi-GPU
 * offset can be fed without a host round trip. In-place (out == x) is allowed.
 * A look-back that exceeds its bounded spin (a stalled predecessor) leaves an INVALID result: it is recorded in
 * the workspace (pcmx_scan_check) and OR-ed into *err_flag when err_flag != NULL (device or host-mapped word,
 * sticky: the caller clears it). */
int pcmx_scan_f32(const float* x, float* out, long long n, int exclusive, const float* init_dev, void* workspace,
                  unsigned* err_flag, hipStream_t s);
/* same with an explicit tile shape: rows = f32x4 rows per lane, 16 (8 waves, the default) or 8 (16 waves) */
int pcmx_scan_f32_rows(const float* x, float* out, long long n, int exclusive, const float* init_dev, void* workspace,
                       unsigned* err_flag, int rows, hipStream_t s);
/* schedule A/B entry (csrc/kernels/scan.hip): 0 persistent R16xW8, 1 persistent R8xW16, 2 parked-tile R16xW8,
 * 3 parked-tile R8xW16, 4 parked-tile R16xW8 with early polls (pcmx_scan_f32) */
int pcmx_scan_f32_variant(const float* x, float* out, long long n, int exclusive, const float* init_dev,
                          void* workspace, unsigned* err_flag, int variant, hipStream_t s);
/* synchronises s; PCMX_ERR_TIMEOUT if the last scan on this workspace gave up a look-back, else 0 */
int pcmx_scan_check(const void* workspace, hipStream_t s);

/* ---------------------------------------------------------------- SGEMM (fp32 MFMA) */
/* C = alpha*A*B + beta*C, row-major. Fast path needs M%256==0, N%256==0 (or %128 for the small-tile
 * kernel), K%32==0, 16-B aligned rows; anything else returns -1 (the torch layer pads). */
int pcmx_sgemm_f32(const float* A, const float* B, float* C, int M, int N, int K, int lda, int ldb, int ldc,
                   float alpha, float beta, hipStream_t s);
/* explicit kernel: 16 = register-staged 256x256x32 / 8 waves (large problems), 0 = LDS-DMA 256x256x32 / 8 waves,
 * 1 = LDS-DMA 128x128x32 / 4 waves (the lab variants live in scripts/sgemm_lab.hip) */
int pcmx_sgemm_f32_variant(const float* A, const float* B, float* C, int M, int N, int K, int lda, int ldb,
                           int ldc, float alpha, float beta, int variant, hipStream_t s);
/* fp32 GEMM on the bf16 matrix cores, operands split exactly into 3 bf16 pieces, 6 piece products (fp32
 * accuracy; sgemm_x6.hip). M, N % 256 == 0, K % 32 == 0. Also reachable as pcmx_sgemm_f32_variant(..., 20). */
int pcmx_sgemm_f32_x6(const float* A, const float* B, float* C, int M, int N, int K, int lda, int ldb, int ldc,
                      float alpha, float beta, hipStream_t s);
/* Reference-style f32 VALU GEMM (one thread per output, LDS tiles) for A/B comparisons. */
int pcmx_sgemm_f32_simt(const float* A, const float* B, float* C, int M, int N, int K, hipStream_t s);

/* ---------------------------------------------------------------- histogram equalisation */
/* out = tf[img] (bit-identical to the serial reference). ws: pcmx_histeq_workspace_bytes(), 16-B aligned, ZEROED
 * before the first call and left zeroed by every call (self-cleaning ticket); one call in flight per workspace. */
long long pcmx_histeq_workspace_bytes(void);
int pcmx_histeq_u8(const unsigned char* img, unsigned char* out, long long npix, void* ws, hipStream_t s);

/* ---------------------------------------------------------------- region growing */
long long pcmx_region2d_workspace_bytes(int H, int W);
/* padded (H+2) x ld arrays, interior 1..H x 1..W; halo cells are read-only seeds. Blocks once per batch. */
int pcmx_region2d_grow(const unsigned char* img, unsigned char* region, int H, int W, int ld, int thr, void* ws,
                       int batch, int max_launches, hipStream_t s, int* launches_out);
long long pcmx_region3d_workspace_bytes(int dim);
int pcmx_region3d_grow_tiled(const unsigned char* data, unsigned char* region, int dim, int thr, void* ws, int batch,
                             int max_launches, hipStream_t s, int* launches_out);
/* z-slab of a distributed volume: dim x dim x nz planes at data/region (plane 0 = first owned plane); halos bit 0 /
 * bit 1 = plane -1 / plane nz are readable halo planes (read-only seeds, never grown); dim % 16 == 0 */
long long pcmx_region3d_slab_workspace_bytes(int dim, int nz);
int pcmx_region3d_grow_slab(const unsigned char* data, unsigned char* region, int dim, int nz, int halos, int thr,
                            void* ws, int batch, int max_launches, hipStream_t s, int* launches_out);
/* reference 0/1/2 frontier semantics, one launch per BFS level; flag_ws: 4 device ints (the pipelined fixpoint check's
 * flag ring); region 16-B aligned */
int pcmx_region3d_grow_naive(const unsigned char* data, unsigned char* region, int dim, int thr, int* flag_ws,
                             int max_launches, hipStream_t s, int* launches_out);

/* ---------------------------------------------------------------- volume + ray casting */
int pcmx_volume_gen_u8(unsigned char* data, int dim, unsigned seed, hipStream_t s);
/* planes [z_first, z_first + nplanes) of the same volume (zeros outside 0..dim-1): a z-slab with halo planes */
int pcmx_volume_gen_slab_u8(unsigned char* data, int dim, int z_first, int nplanes, unsigned seed, hipStream_t s);
/* z-slab stage of the distributed reference caster (bit-identical to pcmx_raycast_global with f64 colour):
 * data/region start at global plane z0 - 1 and hold plane z1 when the slab has one above; state = 6 ints per pixel
 * {pos xyz, colour (f32 bits), steps, flags}, initialised by the first (top) slab when init != 0; the bottom slab
 * (bottom != 0) marches to the end and writes the image. */
int pcmx_raycast_slab(const unsigned char* data, const unsigned char* region, int dim, int z0, int* state, int init,
                      int bottom, unsigned char* image, int image_dim, const float* cam12, float pixel_width,
                      float step, int max_steps, hipStream_t s);
int pcmx_raycast_global(const unsigned char* data, const unsigned char* region, int dim, unsigned char* image,
                        int image_dim, const float* cam12, float pixel_width, float step, int max_steps, int f64_color,
                        hipStream_t s);
/* the same with an explicit caster variant (0 = production; 1 = one step in flight, 16x16 tiles; 2 / 3 = 4 / 16 steps
 * in flight): identical images, the lab's A/B (scripts/raycast_global_lab.py) */
int pcmx_raycast_global_variant(const unsigned char* data, const unsigned char* region, int dim, unsigned char* image,
                                int image_dim, const float* cam12, float pixel_width, float step, int max_steps,
                                int f64_color, int variant, hipStream_t s);
long long pcmx_raycast_dr16_bytes(int dim);
int pcmx_raycast_dr16_pack(const unsigned char* data, const unsigned char* region, int dim, void* dr, hipStream_t s);
int pcmx_raycast_global_dr(const void* dr, int dim, unsigned char* image, int image_dim, const float* cam12,
                           float pixel_width, float step, int max_steps, int f64_color, int variant, hipStream_t s);
/* texture path: tex holds dim^3 * 16 + 16 bytes: per-voxel texels with the 2x2x2 footprint of data and region
 * (8-byte texels when every data value < 128, else 16-byte; the format flag is stored behind the texels),
 * dim <= 2048 */
int pcmx_brick_pack(const unsigned char* data, const unsigned char* region, int dim, void* tex, hipStream_t s);
/* texture ray caster; batch = steps per prefetch batch (1, 4, 8, 16; 0 = 16, the measured best); segments = waves
 * marching one ray patch, each a contiguous share of the step range (1, 2, 4; 0 = the measured best) */
int pcmx_raycast_bricked(const void* tex, int dim, unsigned char* image, int image_dim,
                         const float* cam12, float pixel_width, float step, int max_steps, int batch, int segments,
                         hipStream_t s);

/* ---------------------------------------------------------------- stencil */
int pcmx_stencil5_bf16(const void* u, void* out, int rows, int cols, int ld, int r0, int r1, long long global_row0,
                       long long global_rows, float k, hipStream_t s);
/* `steps` (2, 3, 4, 6, 8) fused updates (temporal blocking, bit-identical to single steps) over local rows
 * [r0, r1) of a (rows + 2*halo) x ld slab; cols % 8 == 0; rows within `steps` of a non-global slab edge need
 * halo >= steps. pcmx_stencil5x2_bf16 = steps 2. */
int pcmx_stencil5xT_bf16(const void* u, void* out, int rows, int cols, int ld, int halo, int steps, int r0, int r1,
                         long long global_row0, long long global_rows, float k, hipStream_t s);
/* the same over two row spans [r0a, r1a) and [r0b, r1b) (disjoint, either may be empty) in ONE launch: the
 * distributed step updates both rank-edge bands with one kernel once the halo rows have arrived */
int pcmx_stencil5xT_bf16_spans(const void* u, void* out, int rows, int cols, int ld, int halo, int steps, int r0a,
                               int r1a, int r0b, int r1b, long long global_row0, long long global_rows, float k,
                               hipStream_t s);
/* the same with an explicit launch shape of this launch (0 = production rule; bits 0-7 columns per lane 4 / 8, 8-15 rows
 * per wave, 16-23 prefetch ring depth 3 / 6 / 9): the lab sweeps, no state kept in the library */
int pcmx_stencil5xT_bf16_spans_shape(const void* u, void* out, int rows, int cols, int ld, int halo, int steps, int r0a,
                                     int r1a, int r0b, int r1b, long long global_row0, long long global_rows, float k,
                                     int shape, hipStream_t s);
int pcmx_stencil5x2_bf16(const void* u, void* out, int rows, int cols, int ld, int halo, int r0, int r1,
                         long long global_row0, long long global_rows, float k, hipStream_t s);

/* ---------------------------------------------------------------- SpMV */
long long pcmx_spmv_csr_plan(const long long* row_ptr_host, int n_rows, void* items_host, long long max_items);
/* the same cut with items of at most item_nnz (64..1024, multiple of 64) nonzeros */
long long pcmx_spmv_csr_plan_nnz(const long long* row_ptr_host, int n_rows, void* items_host, long long max_items,
                                 int item_nnz);
int pcmx_spmv_csr(const long long* row_ptr, const int* col, const float* val, const float* x, float* y, int n_rows,
                  const void* items, long long n_items, hipStream_t s);
/* XCD-sliced CSR (ops/sparse.py SlicedCSR): n_slices = 8 * phases <= PCMX_SPMV_MAX_SLICES; per nonzero col, val
 * and lrow (u16 offset of its row inside its item, rows counted among the rows the slice touches); per slice
 * nnz-balanced items over the slice's touched rows (a later piece of a split long row has row1 == row0).
 * Slice s runs on the blocks b with b % 8 == s % 8 (one XCD) and writes one compact partial per touched row to
 * ypart[slice_out0[s] + touched-row index]; a combine pass sums each row's partials into y (row_mask[r] bit s:
 * slice s touches row r; chunk_base[c * n_slices + s]: touched rows of slice s before row 64c) and a fix-up adds
 * extra[fix[k].item] to y[fix[k].row]. slice_nz0 / slice_item0 / slice_out0 are HOST arrays (n_slices,
 * n_slices + 1 and n_slices + 1 entries).
 * mode: bit 1 = items planned with item_nnz 512 (else 1024); bit 0 = skip the x gathers (lab measurement
 * only); mode >> 8 (if nonzero) = resident
 * blocks per CU (default 2). */
#define PCMX_SPMV_MAX_SLICES 32
int pcmx_spmv_sliced(const unsigned short* lrow, const int* col, const float* val, const float* x, float* ypart,
                     float* extra, float* y, int n_rows, int n_cols, int n_slices, const long long* slice_nz0,
                     const long long* slice_item0, const long long* slice_out0, const void* items,
                     const unsigned* row_mask, const int* chunk_base, const void* fix, int n_fix, int mode,
                     const int* slice_colbase, hipStream_t s);
/* the combine + split-row fix-up (+ send-buffer pack: sendbuf[send_slot[p]] = y[r] for p in send_ptr[r] ..
 * send_ptr[r + 1]) of the partials a products-only pcmx_spmv_sliced call (mode bit 4) wrote, in ONE launch.
 * slice_out0: host array of n_slices + 1 partial offsets; fix: int2 {item, row} sorted by row; fix_chunk0: the fix range
 * of every 64-row chunk (n_rows / 64 + 2 ints, or NULL: no split rows); send_ptr (n_rows + 1) / send_slot / sendbuf
 * may be NULL (no pack). Same bits as combine + fix-up. */
/* products only of phases [a_lo, a_lo + a_n) of sliced matrix A and [b_lo, b_lo + b_n) of B (same x) in ONE launch
 * (production packed layout; item_mode 2: 512-nnz items); nz0 / item0 / out0 / colbase: host arrays per matrix */
int pcmx_spmv_sliced_pair(const float* x, int n_cols, int item_mode, int mode, const int* col_a, const float* val_a,
                          const void* items_a, float* ypart_a, float* extra_a, int s_a, const long long* nz0_a,
                          const long long* item0_a, const long long* out0_a, const int* colbase_a, int a_lo, int a_n,
                          const int* col_b, const float* val_b, const void* items_b, float* ypart_b, float* extra_b,
                          int s_b, const long long* nz0_b, const long long* item0_b, const long long* out0_b,
                          const int* colbase_b, int b_lo, int b_n, hipStream_t s);
int pcmx_spmv_sliced_combine(const float* ypart, const unsigned* row_mask, const int* chunk_base,
                             const long long* slice_out0, int n_slices, float* y, int n_rows, const float* extra,
                             const void* fix, const int* fix_chunk0, const int* send_ptr, const int* send_slot,
                             float* sendbuf, hipStream_t s);
int pcmx_spmv_banded(const float* vals, const long long* row_off, int n, int a, int b, int c, int d, int e,
                     const float* x, float* y, hipStream_t s);
/* variant 0: one wave per row (strided band loops, global x); 1: LDS-staged x windows, row blocks, 4-B loads;
 * 2 / 3: the same with 16-B value loads, 2 / 4 rows per wave in flight */
int pcmx_spmv_banded_variant(const float* vals, const long long* row_off, int n, int a, int b, int c, int d, int e,
                             const float* x, float* y, int variant, hipStream_t s);

/* ---------------------------------------------------------------- halo pack/unpack */
int pcmx_pack_edges(const void* tile, int elem_bytes, int H, int W, int ld, void* buf, hipStream_t s);
int pcmx_unpack_halo(void* tile, int elem_bytes, int H, int W, int ld, const void* buf, int mask, hipStream_t s);
/* as pcmx_unpack_halo, and *changed (device int) is set to 1 when any halo cell takes a new value */
int pcmx_unpack_halo_changed(void* tile, int elem_bytes, int H, int W, int ld, const void* buf, int mask, int* changed,
                             hipStream_t s);

/* ---------------------------------------------------------------- grouped exchange on a dedicated RCCL communicator
 * (comm/exchange_rccl.hip): per-peer byte segments send[soff[q] .. + scnt[q]) -> peer q, recv[roff[q] .. + rcnt[q])
 * <- peer q, on the communicator's stream, ordered after `compute` (event) and waited for by pcmx_xcomm_wait. */
int pcmx_xcomm_id_bytes(void);
int pcmx_xcomm_unique_id(void* out);
int pcmx_xcomm_create(const void* id, int world, int rank, int device, void** out);
int pcmx_xcomm_exchange(void* handle, int slot, const void* send, const long long* soff, const long long* scnt,
                        void* recv, const long long* roff, const long long* rcnt, hipStream_t compute);
int pcmx_xcomm_wait(void* handle, int slot, hipStream_t compute);
int pcmx_xcomm_probe(void* handle, int timeout_ms);
int pcmx_xcomm_async_error(void* handle);
int pcmx_xcomm_destroy(void* handle);

#ifdef __cplusplus
}
#endif
#endif /* PCMX_HIP_H */
