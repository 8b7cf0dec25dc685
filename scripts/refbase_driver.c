/* Timing driver for the REFERENCE's OpenCL program (ref 6-opencl-region-growing/raycast.c), built from the
 * reference's own unmodified sources by scripts/refbase_build.sh (its main() renamed refbase_main at compile time,
 * never called). Same sequence as the reference main (raycast.c:439-448): create_data, grow_region_gpu, raycast_gpu,
 * write_bmp, with a gettimeofday bracket around each GPU entry point (the reference's print_time idiom) and the
 * results that pin it to our tests: region voxels (T2: 2,197,899) and the 64^2 image sum (T5).
 * Prints one JSON line. */
#include <stdio.h>
#include <stdlib.h>
#include <sys/time.h>

unsigned char* create_data();
unsigned char* grow_region_gpu(unsigned char* data);
unsigned char* raycast_gpu(unsigned char* data, unsigned char* region);
void write_bmp(unsigned char* data, int width, int height);

static double now_s(void) {
    struct timeval t;
    gettimeofday(&t, NULL);
    return t.tv_sec + 1e-6 * t.tv_usec;
}

int main(void) {
    const long long nvox = 512LL * 512 * 512, npix = 64 * 64;
    double t0 = now_s();
    unsigned char* data = create_data();
    double t1 = now_s();
    unsigned char* region = grow_region_gpu(data);
    double t2 = now_s();
    unsigned char* image = raycast_gpu(data, region);
    double t3 = now_s();
    long long vox = 0, sum = 0;
    for (long long i = 0; i < nvox; ++i) vox += region[i] != 0;
    for (long long i = 0; i < npix; ++i) sum += image[i];
    write_bmp(image, 64, 64);
    printf("{\"program\": \"reference 6-opencl-region-growing (OpenCL, built from source)\", \"create_data_s\": %.6f, "
           "\"grow_region_gpu_s\": %.6f, \"raycast_gpu_s\": %.6f, \"region_voxels\": %lld, \"image_dim\": 64, "
           "\"image_sum\": %lld}\n",
           t1 - t0, t2 - t1, t3 - t2, vox, sum);
    return 0;
}
