/* Host entry points of the reference 3-D pipelines (pcmx_pipeline3d.h): create_data, raycast_serial and
 * grow_region_serial with the signatures of ref 5-cuda-region-growing/raycast.cu:146,216,281 (and their OpenCL
 * twins, 6-opencl-region-growing/raycast.c:134,204,269), over the serial oracles of oracles.c. Each returns a
 * malloc'd array the caller frees. */
#include <stdio.h>
#include <stdlib.h>

#include "pcmx_cpu.h"
#include "pcmx_pipeline3d.h"

unsigned char* pcmx_create_data_dim(int dim) {
    if (dim <= 0) return NULL;
    unsigned char* d = (unsigned char*)malloc((size_t)dim * dim * dim);
    if (d) pcmx_create_data(d, dim);
    return d;
}

unsigned char* pcmx_raycast_serial_dims(const unsigned char* data, const unsigned char* region, int dim, int image_dim) {
    if (!data || !region || dim <= 1 || image_dim <= 0) return NULL;
    unsigned char* img = (unsigned char*)malloc((size_t)image_dim * image_dim);
    if (img) pcmx_raycast_serial(data, region, dim, image_dim, img);
    return img;
}

unsigned char* pcmx_grow_region_serial_dim(const unsigned char* data, int dim) {
    if (!data || dim <= PCMX_SEED_Y) return NULL;
    unsigned char* reg = (unsigned char*)malloc((size_t)dim * dim * dim);
    if (reg) pcmx_region3d_serial(data, dim, PCMX_SEED_X, PCMX_SEED_Y, PCMX_SEED_Z, 1, reg);
    return reg;
}

/* reference names (512^3 volume, 512^2 image); #undef in case a caller's DATA_DIM/IMAGE_DIM mapped them */
#undef create_data
#undef raycast_serial
#undef grow_region_serial
unsigned char* create_data(void) { return pcmx_create_data_dim(PCMX_DATA_DIM); }
unsigned char* raycast_serial(unsigned char* data, unsigned char* region) {
    return pcmx_raycast_serial_dims(data, region, PCMX_DATA_DIM, PCMX_IMAGE_DIM);
}
unsigned char* grow_region_serial(unsigned char* data) { return pcmx_grow_region_serial_dim(data, PCMX_DATA_DIM); }
