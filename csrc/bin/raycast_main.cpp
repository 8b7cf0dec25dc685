/* bin/raycast [--image-dim N] [--dim D] [--global] [--naive] [--volume hash|rand]
 *
 * The reference's 3-D pipeline (5-cuda-region-growing/raycast.cu:824-854) on one MI355X:
 * device info, the 512^3 synthetic volume, region growing from (50,300,300) with the LDS-tiled kernel
 * ("Grow time:"), the texture-path ray cast on the brick-packed volume ("Raycast time: "), ./out.bmp.
 * `--image-dim 64 --global --naive` is the OpenCL program (6-opencl-region-growing/raycast.c:439-448): naive
 * frontier kernel, global-memory caster, 64x64 image. --volume rand = the reference's glibc rand() bytes
 * generated on the host; the default hash volume is generated on the GPU. Every HIP call is checked. */
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "pcmx_cpu.h"
#include "pcmx_hip.h"

#define CHECK(x)                                                                                 \
    do {                                                                                         \
        int rc_ = (int)(x);                                                                      \
        if (rc_) {                                                                               \
            fprintf(stderr, "%s:%d: %s failed: %s\n", __FILE__, __LINE__, #x, pcmx_error_string(rc_)); \
            exit(1);                                                                             \
        }                                                                                        \
    } while (0)

static void print_time_s(double s) { printf("Time : %f s\n", s); }

int main(int argc, char** argv) {
    int image_dim = 512, dim = 512, global = 0, naive = 0, rand_volume = 0;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--image-dim") && i + 1 < argc) image_dim = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--dim") && i + 1 < argc) dim = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--global")) global = 1;
        else if (!strcmp(argv[i], "--naive")) naive = 1;
        else if (!strcmp(argv[i], "--volume") && i + 1 < argc) rand_volume = !strcmp(argv[++i], "rand");
        else {
            fprintf(stderr, "usage: raycast [--image-dim N] [--dim D] [--global] [--naive] [--volume hash|rand]\n");
            return 2;
        }
    }
    const int opencl = image_dim == 64 && global && naive;
    if (dim < 64 || dim > 2048 || image_dim < 1 || image_dim > 8192) return 2;
    const int sx = 50, sy = 300, sz = 300;  // ref raycast.cu:718
    if (sx >= dim || sy >= dim || sz >= dim) return 2;
    if (pcmx_device_count() <= 0) {
        fprintf(stderr, "raycast: no GPU visible\n");
        return 1;
    }
    if (!opencl) pcmx_print_device_info(0);
    CHECK(hipSetDevice(0));
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const size_t nvox = (size_t)dim * dim * dim;
    unsigned char *data = nullptr, *region = nullptr, *image = nullptr;
    CHECK(hipMalloc(&data, nvox));
    CHECK(hipMalloc(&region, nvox));
    CHECK(hipMalloc(&image, (size_t)image_dim * image_dim));
    if (rand_volume) {
        std::vector<unsigned char> h(nvox);
        pcmx_create_data(h.data(), dim);
        CHECK(hipMemcpyAsync(data, h.data(), nvox, hipMemcpyHostToDevice, s));
        CHECK(hipStreamSynchronize(s));
    } else {
        CHECK(pcmx_volume_gen_u8(data, dim, 0u, s));
    }

    // ---- region growing
    CHECK(hipMemsetAsync(region, 0, nvox, s));
    const unsigned char seed = naive ? 2 : 1;  // naive kernel: reference 0/1/2 frontier semantics
    CHECK(hipMemcpyAsync(region + ((size_t)sz * dim + sy) * dim + sx, &seed, 1, hipMemcpyHostToDevice, s));
    CHECK(hipStreamSynchronize(s));
    void* ws = nullptr;
    int* flag = nullptr;
    if (naive) CHECK(hipMalloc(&flag, 4 * sizeof(int)));
    else CHECK(hipMalloc(&ws, (size_t)pcmx_region3d_workspace_bytes(dim)));
    int launches = 0;
    double t0 = pcmx_wtime();
    if (naive) CHECK(pcmx_region3d_grow_naive(data, region, dim, 1, flag, 1000000, s, &launches));
    else CHECK(pcmx_region3d_grow_tiled(data, region, dim, 1, ws, 8, 1000000, s, &launches));
    CHECK(hipStreamSynchronize(s));
    double t1 = pcmx_wtime();
    if (!opencl) {
        printf("\nGrow time:\n");
        print_time_s(t1 - t0);
        printf("Errors: %s\n", hipGetErrorString(hipGetLastError()));
    }

    // ---- ray casting
    pcmx_camera_t cam;
    pcmx_default_camera(image_dim, &cam);
    float cam12[12];
    for (int i = 0; i < 3; ++i)
        cam12[i] = cam.camera[i], cam12[3 + i] = cam.forward[i], cam12[6 + i] = cam.right[i], cam12[9 + i] = cam.up[i];
    void* tex = nullptr;  // 16-byte texels (pcmx_brick_pack)
    if (!global) CHECK(hipMalloc(&tex, nvox * 16 + 16));
    t0 = pcmx_wtime();
    if (global) {
        CHECK(pcmx_raycast_global(data, region, dim, image, image_dim, cam12, cam.pixel_width, cam.step_size,
                                  cam.max_steps, 1, s));
    } else {
        CHECK(pcmx_brick_pack(data, region, dim, tex, s));
        CHECK(pcmx_raycast_bricked(tex, dim, image, image_dim, cam12, cam.pixel_width, cam.step_size, cam.max_steps, 0, 0, s));
    }
    CHECK(hipStreamSynchronize(s));
    t1 = pcmx_wtime();
    if (!opencl) {
        printf("\nRaycast time: \n");
        print_time_s(t1 - t0);
        printf("Errors: %s\n", hipGetErrorString(hipGetLastError()));
    }
    std::vector<unsigned char> h_img((size_t)image_dim * image_dim);
    CHECK(hipMemcpy(h_img.data(), image, h_img.size(), hipMemcpyDeviceToHost));
    write_bmp(h_img.data(), image_dim, image_dim);
    hipFree(tex);
    hipFree(ws);
    hipFree(flag);
    hipFree(image);
    hipFree(region);
    hipFree(data);
    hipStreamDestroy(s);
    return 0;
}
