/*
 * pcmx_pipeline3d.h — the reference 3-D pipelines' C entry points, with their exact signatures, on MI355X.
 *
 *   ref 5-cuda-region-growing/raycast.cu     print_properties :99, create_data :146, raycast_serial :216,
 *                                            grow_region_serial :281, raycast_gpu :436, raycast_gpu_texture :472,
 *                                            grow_region_gpu :702, grow_region_gpu_shared :759
 *   ref 6-opencl-region-growing/raycast.c    grow_region_gpu :308, raycast_gpu :379 (IMAGE_DIM 64)
 *
 * Every function returns a malloc'd HOST array the caller frees (the reference contract): DATA_DIM^3 region
 * bytes (1 = in region, 0 = outside) or an IMAGE_DIM^2 image. The GPU versions copy the volume to the current
 * HIP device, run the gfx950 kernels of libpcmx_hip and copy the result back:
 *   grow_region_gpu         naive 0/1/2-frontier kernel, one launch per BFS level (ref region_grow_kernel)
 *   grow_region_gpu_shared  bit-parallel LDS/wave-tiled kernel on a device-built tile worklist
 *                           (ref region_grow_kernel_shared)
 *   raycast_gpu             global-memory software-trilinear caster, reference weights, f64 colour update
 *   raycast_gpu_texture     brick-packed texel volume + texture-path caster (gfx950 has no exposed texture
 *                           unit: software trilinear on packed texels; ref raycast_kernel_texture)
 * Any failure prints the pcmx error to stderr and returns NULL.
 *
 * DATA_DIM / IMAGE_DIM default to the CUDA program's 512 / 512. A translation unit that defines IMAGE_DIM (e.g.
 * 64, the OpenCL program) or DATA_DIM before including this header gets the reference names mapped onto the
 * explicit-size entry points below, so the OpenCL program's `raycast_gpu(data, region)` renders 64 x 64.
 * Links against libpcmx_hip (GPU entry points) and libpcmx_cpu (create_data and the serial ones).
 */
#ifndef PCMX_PIPELINE3D_H
#define PCMX_PIPELINE3D_H

#ifdef __cplusplus
extern "C" {
#endif

#define PCMX_DATA_DIM 512
#define PCMX_IMAGE_DIM 512
#define PCMX_SEED_X 50 /* ref raycast.cu:718 */
#define PCMX_SEED_Y 300
#define PCMX_SEED_Z 300

/* ---- explicit sizes (dim^3 volume, image_dim^2 image) */
unsigned char* pcmx_create_data_dim(int dim);
unsigned char* pcmx_raycast_serial_dims(const unsigned char* data, const unsigned char* region, int dim, int image_dim);
unsigned char* pcmx_grow_region_serial_dim(const unsigned char* data, int dim);
unsigned char* pcmx_raycast_gpu_dims(const unsigned char* data, const unsigned char* region, int dim, int image_dim);
unsigned char* pcmx_raycast_gpu_texture_dims(const unsigned char* data, const unsigned char* region, int dim,
                                             int image_dim);
unsigned char* pcmx_grow_region_gpu_dim(const unsigned char* data, int dim);
unsigned char* pcmx_grow_region_gpu_shared_dim(const unsigned char* data, int dim);

/* ---- reference names, 512^3 volume and 512^2 image (the CUDA program) */
void print_properties(void);
unsigned char* create_data(void);
unsigned char* raycast_serial(unsigned char* data, unsigned char* region);
unsigned char* grow_region_serial(unsigned char* data);
unsigned char* raycast_gpu(unsigned char* data, unsigned char* region);
unsigned char* raycast_gpu_texture(unsigned char* data, unsigned char* region);
unsigned char* grow_region_gpu(unsigned char* host_data);
unsigned char* grow_region_gpu_shared(unsigned char* host_data);

#ifdef __cplusplus
}
#endif

/* OpenCL-program sizes (or any other): remap the reference names onto the explicit-size entry points */
#if (defined(IMAGE_DIM) && IMAGE_DIM != PCMX_IMAGE_DIM) || (defined(DATA_DIM) && DATA_DIM != PCMX_DATA_DIM)
#ifndef DATA_DIM
#define DATA_DIM PCMX_DATA_DIM
#endif
#ifndef IMAGE_DIM
#define IMAGE_DIM PCMX_IMAGE_DIM
#endif
#define create_data() pcmx_create_data_dim(DATA_DIM)
#define raycast_serial(d, r) pcmx_raycast_serial_dims((d), (r), DATA_DIM, IMAGE_DIM)
#define grow_region_serial(d) pcmx_grow_region_serial_dim((d), DATA_DIM)
#define raycast_gpu(d, r) pcmx_raycast_gpu_dims((d), (r), DATA_DIM, IMAGE_DIM)
#define raycast_gpu_texture(d, r) pcmx_raycast_gpu_texture_dims((d), (r), DATA_DIM, IMAGE_DIM)
#define grow_region_gpu(d) pcmx_grow_region_gpu_dim((d), DATA_DIM)
#define grow_region_gpu_shared(d) pcmx_grow_region_gpu_shared_dim((d), DATA_DIM)
#endif

#endif /* PCMX_PIPELINE3D_H */
