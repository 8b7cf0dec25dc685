/* Timing driver for the REFERENCE's OpenCL program (ref 6-opencl-region-growing/raycast.c), built from the
 * reference's own sources by scripts/refbase_build.sh (its main() renamed refbase_main at compile time, never called).
 * Same sequence as the reference main (raycast.c:439-448) — create_data, grow_region_gpu, raycast_gpu — with a
 * gettimeofday bracket around each GPU entry point (the reference's print_time idiom) and the results that pin it to
 * our tests: region voxels (T2: 2,197,899) and the 64^2 image sum (T5: 127,180). Then, because the reference's GPU
 * grow may not run as written (see profiles/r5_refbase/), the reference's OWN serial grower (grow_region_serial,
 * raycast.c:269-306) supplies the correct region and raycast_gpu runs again on it: the ray-cast kernel timed on the
 * input it was written for. Prints one JSON line. */
#include <stdio.h>
#include <stdlib.h>
#include <sys/time.h>

unsigned char* create_data();
unsigned char* grow_region_gpu(unsigned char* data);
unsigned char* grow_region_serial(unsigned char* data);
unsigned char* raycast_gpu(unsigned char* data, unsigned char* region);
void write_bmp(unsigned char* data, int width, int height);

static double now_s(void) {
    struct timeval t;
    gettimeofday(&t, NULL);
    return t.tv_sec + 1e-6 * t.tv_usec;
}

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

int main(void) {
    const long long nvox = 512LL * 512 * 512, npix = 64 * 64;
    double t0 = now_s();
    unsigned char* data = create_data();
    double t1 = now_s();
    unsigned char* region = grow_region_gpu(data);
    double t2 = now_s();
    unsigned char* image = raycast_gpu(data, region);
    double t3 = now_s();
    unsigned char* region_ok = grow_region_serial(data);
    double t4 = now_s();
    unsigned char* image_ok = raycast_gpu(data, region_ok);
    double t5 = now_s();
    write_bmp(image, 64, 64);
    printf("{\"program\": \"reference 6-opencl-region-growing (OpenCL, built from source)\", \"create_data_s\": %.6f, "
           "\"grow_region_gpu_s\": %.6f, \"region_voxels\": %lld, \"raycast_gpu_s\": %.6f, \"image_sum\": %lld, "
           "\"grow_region_serial_s\": %.6f, \"serial_region_voxels\": %lld, \"raycast_gpu_on_serial_region_s\": %.6f, "
           "\"image_sum_on_serial_region\": %lld, \"image_dim\": 64}\n",
           t1 - t0, t2 - t1, count(region, nvox), t3 - t2, sum(image, npix), t4 - t3, count(region_ok, nvox), t5 - t4,
           sum(image_ok, npix));
    return 0;
}
