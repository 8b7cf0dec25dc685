/* bin/pipeline3d [--serial] — the reference CUDA program's main (ref 5-cuda-region-growing/raycast.cu:824-854)
 * written ONLY against the reference C entry points (pcmx_pipeline3d.h): print_properties, create_data,
 * grow_region_gpu_shared / grow_region_gpu / grow_region_serial, raycast_gpu_texture / raycast_gpu, and the
 * reference utilities print_time / write_bmp.
 * Prints the reference's "Grow time:" / "Raycast time: " blocks, the region size of every grower (T2:
 * 2,197,899 voxels), the image sums, and writes ./out.bmp (texture path, like the reference).
 * --serial also runs raycast_serial at 512^2 (multi-threaded host oracle; seconds) and checks raycast_gpu
 * against it bit for bit.
 * Built as bin/pipeline3d_opencl with -DPCMX_OPENCL_PROGRAM: IMAGE_DIM 64, naive grow + global caster, the
 * OpenCL program (ref 6-opencl-region-growing/raycast.c:439-448); T5: 64^2 image sum 127,180. */
#ifdef PCMX_OPENCL_PROGRAM
#define IMAGE_DIM 64
#endif
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>

#include "pcmx_cpu.h"
#include "pcmx_pipeline3d.h"

#ifndef IMAGE_DIM
#define IMAGE_DIM PCMX_IMAGE_DIM
#endif
#define DIM PCMX_DATA_DIM

static long long count(const unsigned char* r, long long n) {
    long long c = 0;
    for (long long i = 0; i < n; ++i) c += r[i] != 0;
    return c;
}

static long long sum(const unsigned char* img, long long n) {
    long long s = 0;
    for (long long i = 0; i < n; ++i) s += img[i];
    return s;
}

int main(int argc, char** argv) {
    const int serial = argc > 1 && !strcmp(argv[1], "--serial");
    const long long nvox = (long long)DIM * DIM * DIM, npix = (long long)IMAGE_DIM * IMAGE_DIM;
    struct timeval t0, t1;
#ifndef PCMX_OPENCL_PROGRAM
    print_properties();
#endif
    unsigned char* data = create_data();
    if (!data) return 1;

    gettimeofday(&t0, NULL);
#ifdef PCMX_OPENCL_PROGRAM
    unsigned char* region = grow_region_gpu(data);
#else
    unsigned char* region = grow_region_gpu_shared(data);
#endif
    gettimeofday(&t1, NULL);
    if (!region) return 1;
    printf("\nGrow time:\n");
    print_time(t0, t1);
    const long long n_gpu = count(region, nvox);
    unsigned char* region_ref = grow_region_serial(data);
    const long long n_ref = count(region_ref, nvox);
    int ok = n_gpu == n_ref && memcmp(region, region_ref, (size_t)nvox) == 0;
#ifndef PCMX_OPENCL_PROGRAM
    unsigned char* region_naive = grow_region_gpu(data);
    ok = ok && region_naive && memcmp(region_naive, region_ref, (size_t)nvox) == 0;
    free(region_naive);
#endif
    printf("region voxels: %lld (serial %lld) %s\n", n_gpu, n_ref, ok ? "identical" : "MISMATCH");

    gettimeofday(&t0, NULL);
#ifdef PCMX_OPENCL_PROGRAM
    unsigned char* image = raycast_gpu(data, region);
#else
    unsigned char* image = raycast_gpu_texture(data, region);
#endif
    gettimeofday(&t1, NULL);
    if (!image) return 1;
    printf("\nRaycast time: \n");
    print_time(t0, t1);
    unsigned char* image_global = raycast_gpu(data, region);
    if (!image_global) return 1;
    printf("image sum: %lld (global-memory caster %lld)\n", sum(image, npix), sum(image_global, npix));
#ifdef PCMX_OPENCL_PROGRAM
    const int check_serial = 1;
#else
    const int check_serial = serial;
#endif
    if (check_serial) {
        unsigned char* image_ref = raycast_serial(data, region_ref);
        const int same = memcmp(image_ref, image_global, (size_t)npix) == 0;
        printf("serial caster sum: %lld, global caster %s\n", sum(image_ref, npix), same ? "bit-identical" : "DIFFERS");
        ok = ok && same;
        free(image_ref);
    }
    write_bmp(image, IMAGE_DIM, IMAGE_DIM);
    free(image_global);
    free(image);
    free(region_ref);
    free(region);
    free(data);
    return ok ? 0 : 3;
}
