// GPU entry points of the reference 3-D pipelines (pcmx_pipeline3d.h) with the reference signatures:
// print_properties, grow_region_gpu, grow_region_gpu_shared, raycast_gpu, raycast_gpu_texture
// (ref 5-cuda-region-growing/raycast.cu:99,702,759,436,472; OpenCL twins 6-opencl-region-growing/raycast.c:308,379).
//
// Same host contract as the reference (host volume in, malloc'd host result out), MI355X inside: one stream,
// every HIP call checked, the volume uploaded once, and the gfx950 kernels of libpcmx_hip:
//   naive grow    pcmx_region3d_grow_naive — the reference 0/1/2 frontier semantics, one launch per BFS level
//                 (the host reads the device flag once per launch, like the reference's do/while)
//   shared grow   pcmx_region3d_grow_tiled — bit-parallel 64x8x8 wave tiles on a device-built worklist, the host
//                 reads the flag once per 8 launches (the reference re-launches its LDS kernel per level)
//   global cast   pcmx_raycast_global — the reference value_at weights, f64 colour update (bit-exact with the
//                 serial caster)
//   texture cast  pcmx_brick_pack + pcmx_raycast_bricked — texel volume with the 2x2x2 footprint of data and
//                 region per voxel, one load per sample (gfx950 exposes no texture sampler)
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pcmx_common.h"
#include "pcmx_cpu.h"
#include "pcmx_hip.h"
#include "pcmx_pipeline3d.h"

namespace {
constexpr int kMaxLaunches = 1 << 20;

int report(int rc, const char* what) {
    if (rc) fprintf(stderr, "pcmx %s: %s (%d)\n", what, pcmx_error_string(rc), rc);
    return rc;
}

// owns the device buffers of one call
struct Dev {
    hipStream_t s = nullptr;
    unsigned char *data = nullptr, *region = nullptr, *image = nullptr;
    void* ws = nullptr;
    ~Dev() {
        hipFree(ws);
        hipFree(image);
        hipFree(region);
        hipFree(data);
        if (s) hipStreamDestroy(s);
    }
    int init(const unsigned char* host_data, const unsigned char* host_region, int dim) {
        const size_t n = (size_t)dim * dim * dim;
        PCMX_HIP_RET(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        PCMX_HIP_RET(hipMalloc(&data, n));
        PCMX_HIP_RET(hipMalloc(&region, n));
        PCMX_HIP_RET(hipMemcpyAsync(data, host_data, n, hipMemcpyHostToDevice, s));
        if (host_region) PCMX_HIP_RET(hipMemcpyAsync(region, host_region, n, hipMemcpyHostToDevice, s));
        return 0;
    }
};

unsigned char* grow(const unsigned char* host_data, int dim, bool tiled) {
    if (!host_data || dim <= PCMX_SEED_Y || (tiled && dim % 16)) {
        report(PCMX_ERR_ARG, "grow_region_gpu");
        return nullptr;
    }
    const size_t n = (size_t)dim * dim * dim;
    Dev d;
    unsigned char* out = static_cast<unsigned char*>(malloc(n));
    int rc = out ? d.init(host_data, nullptr, dim) : (int)hipErrorOutOfMemory;
    if (!rc) rc = (int)hipMemsetAsync(d.region, 0, n, d.s);
    // seed (ref raycast.cu:718): the naive kernel's frontier value is 2, the tiled kernel's region value 1
    const unsigned char seed = tiled ? 1 : 2;
    const size_t at = ((size_t)PCMX_SEED_Z * dim + PCMX_SEED_Y) * dim + PCMX_SEED_X;
    if (!rc) rc = (int)hipMemcpyAsync(d.region + at, &seed, 1, hipMemcpyHostToDevice, d.s);
    if (!rc) rc = (int)hipStreamSynchronize(d.s);  // `seed` is a stack temporary
    if (!rc) rc = (int)hipMalloc(&d.ws, tiled ? (size_t)pcmx_region3d_workspace_bytes(dim) : 16);
    int launches = 0;
    if (!rc)
        rc = tiled ? pcmx_region3d_grow_tiled(d.data, d.region, dim, 1, d.ws, 8, kMaxLaunches, d.s, &launches)
                   : pcmx_region3d_grow_naive(d.data, d.region, dim, 1, static_cast<int*>(d.ws), kMaxLaunches, d.s,
                                              &launches);
    if (!rc) rc = (int)hipMemcpyAsync(out, d.region, n, hipMemcpyDeviceToHost, d.s);
    if (!rc) rc = (int)hipStreamSynchronize(d.s);
    if (report(rc, tiled ? "grow_region_gpu_shared" : "grow_region_gpu")) {
        free(out);
        return nullptr;
    }
    for (size_t i = 0; i < n; ++i) out[i] = out[i] != 0;  // 1 = in region (the reference's final value)
    return out;
}

unsigned char* cast(const unsigned char* host_data, const unsigned char* host_region, int dim, int image_dim,
                    bool texture) {
    if (!host_data || !host_region || dim <= 1 || dim > 2048 || image_dim <= 0) {
        report(PCMX_ERR_ARG, "raycast_gpu");
        return nullptr;
    }
    Dev d;
    const size_t npix = (size_t)image_dim * image_dim;
    unsigned char* out = static_cast<unsigned char*>(malloc(npix));
    int rc = out ? d.init(host_data, host_region, dim) : (int)hipErrorOutOfMemory;
    if (!rc) rc = (int)hipMalloc(&d.image, npix);
    pcmx_camera_t cam;
    pcmx_default_camera(image_dim, &cam);
    float cam12[12];
    for (int i = 0; i < 3; ++i)
        cam12[i] = cam.camera[i], cam12[3 + i] = cam.forward[i], cam12[6 + i] = cam.right[i], cam12[9 + i] = cam.up[i];
    if (texture) {
        if (!rc) rc = (int)hipMalloc(&d.ws, (size_t)dim * dim * dim * 16 + 16);
        if (!rc) rc = pcmx_brick_pack(d.data, d.region, dim, d.ws, d.s);
        if (!rc)
            rc = pcmx_raycast_bricked(d.ws, dim, d.image, image_dim, cam12, cam.pixel_width, cam.step_size,
                                      cam.max_steps, 0, 0, d.s);
    } else if (!rc) {
        rc = pcmx_raycast_global(d.data, d.region, dim, d.image, image_dim, cam12, cam.pixel_width, cam.step_size,
                                 cam.max_steps, 1, d.s);
    }
    if (!rc) rc = (int)hipMemcpyAsync(out, d.image, npix, hipMemcpyDeviceToHost, d.s);
    if (!rc) rc = (int)hipStreamSynchronize(d.s);
    if (report(rc, texture ? "raycast_gpu_texture" : "raycast_gpu")) {
        free(out);
        return nullptr;
    }
    return out;
}
}  // namespace

extern "C" {

unsigned char* pcmx_raycast_gpu_dims(const unsigned char* data, const unsigned char* region, int dim, int image_dim) {
    return cast(data, region, dim, image_dim, false);
}
unsigned char* pcmx_raycast_gpu_texture_dims(const unsigned char* data, const unsigned char* region, int dim,
                                             int image_dim) {
    return cast(data, region, dim, image_dim, true);
}
unsigned char* pcmx_grow_region_gpu_dim(const unsigned char* data, int dim) { return grow(data, dim, false); }
unsigned char* pcmx_grow_region_gpu_shared_dim(const unsigned char* data, int dim) { return grow(data, dim, true); }

// ref raycast.cu:99-110 output lines ("Device count", "Compute capability", "Name")
void print_properties(void) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) count = 0;
    printf("Device count: %d\n", count);
    hipDeviceProp_t p;
    if (count > 0 && hipSetDevice(0) == hipSuccess && hipGetDeviceProperties(&p, 0) == hipSuccess) {
        printf("Compute capability: %d.%d\n", p.major, p.minor);
        printf("Name: %s\n", p.name[0] ? p.name : p.gcnArchName);  // marketing name can be empty (no amdgpu.ids)
    }
    printf("\n\n");
}

#undef raycast_gpu
#undef raycast_gpu_texture
#undef grow_region_gpu
#undef grow_region_gpu_shared
unsigned char* raycast_gpu(unsigned char* data, unsigned char* region) {
    return cast(data, region, PCMX_DATA_DIM, PCMX_IMAGE_DIM, false);
}
unsigned char* raycast_gpu_texture(unsigned char* data, unsigned char* region) {
    return cast(data, region, PCMX_DATA_DIM, PCMX_IMAGE_DIM, true);
}
unsigned char* grow_region_gpu(unsigned char* host_data) { return grow(host_data, PCMX_DATA_DIM, false); }
unsigned char* grow_region_gpu_shared(unsigned char* host_data) { return grow(host_data, PCMX_DATA_DIM, true); }

}  // extern "C"
