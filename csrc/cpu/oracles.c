/*
 * Serial oracles (CPU reference implementations) for the GPU pipelines.
 *
 *  pcmx_region2d_serial   4-connected seeded flood fill, |a-b| < threshold between ADJACENT pixels —
 *                         the semantics of ref 2-mpi-region-growing/region.c:493-533 (DFS + similar()),
 *                         expressed on the whole image (tiles/halos are an implementation detail).
 *  pcmx_region3d_serial   6-connected flood fill, ref 5-cuda-region-growing/raycast.cu:281-318.
 *  pcmx_create_data       the reference volume, ref raycast.cu:114-158 (rand()%20 background drawn for
 *                         every voxel in z,y,x order, then two spheres and two boxes).
 *  pcmx_raycast_serial    ref raycast.cu:216-267 / 6-opencl-region-growing/raycast.c:204-255 including
 *                         the swapped trilinear weights (B21) and the f64 colour update of the C code
 *                         (`color += value_at(...)*(0.01 + r)` promotes to double).
 *
 * This file is compiled with -ffp-contract=off so float rounding matches the reference build.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include "pcmx_cpu.h"

typedef struct {
    long long* v;
    long long n, cap;
} idx_stack_t;

static int stack_push(idx_stack_t* s, long long x) {
    if (s->n == s->cap) {
        long long nc = s->cap ? s->cap * 2 : 4096;
        long long* nv = (long long*)realloc(s->v, sizeof(long long) * (size_t)nc);
        if (!nv) return -1;
        s->v = nv;
        s->cap = nc;
    }
    s->v[s->n++] = x;
    return 0;
}

long long pcmx_region2d_serial(const unsigned char* img, int w, int h, const int* seeds_xy, int n_seeds,
                               int threshold, unsigned char* region) {
    memset(region, 0, (size_t)w * h);
    idx_stack_t st = {0, 0, 0};
    long long count = 0;
    for (int s = 0; s < n_seeds; ++s) {
        int x = seeds_xy[2 * s], y = seeds_xy[2 * s + 1];
        if (x < 0 || y < 0 || x >= w || y >= h) continue;
        long long p = (long long)y * w + x;
        if (!region[p]) {
            region[p] = 1;
            ++count;
            stack_push(&st, p);
        }
    }
    static const int dx[4] = {0, 0, 1, -1}, dy[4] = {1, -1, 0, 0};
    while (st.n > 0) {
        long long p = st.v[--st.n];
        int x = (int)(p % w), y = (int)(p / w);
        for (int k = 0; k < 4; ++k) {
            int cx = x + dx[k], cy = y + dy[k];
            if (cx < 0 || cy < 0 || cx >= w || cy >= h) continue;
            long long q = (long long)cy * w + cx;
            if (region[q]) continue;
            if (abs((int)img[p] - (int)img[q]) < threshold) {
                region[q] = 1;
                ++count;
                stack_push(&st, q);
            }
        }
    }
    free(st.v);
    return count;
}

long long pcmx_region3d_serial(const unsigned char* data, int dim, int sx, int sy, int sz, int threshold,
                               unsigned char* region) {
    const long long plane = (long long)dim * dim, n = plane * dim;
    memset(region, 0, (size_t)n);
    if (sx < 0 || sy < 0 || sz < 0 || sx >= dim || sy >= dim || sz >= dim) return 0;
    idx_stack_t st = {0, 0, 0};
    long long seed = (long long)sz * plane + (long long)sy * dim + sx;
    region[seed] = 1;
    stack_push(&st, seed);
    long long count = 1;
    while (st.n > 0) {
        long long p = st.v[--st.n];
        int x = (int)(p % dim), y = (int)((p / dim) % dim), z = (int)(p / plane);
        const int nb[6][3] = {{-1, 0, 0}, {1, 0, 0}, {0, -1, 0}, {0, 1, 0}, {0, 0, -1}, {0, 0, 1}};
        for (int k = 0; k < 6; ++k) {
            int cx = x + nb[k][0], cy = y + nb[k][1], cz = z + nb[k][2];
            if (cx < 0 || cy < 0 || cz < 0 || cx >= dim || cy >= dim || cz >= dim) continue;
            long long q = (long long)cz * plane + (long long)cy * dim + cx;
            if (region[q]) continue;
            if (abs((int)data[p] - (int)data[q]) < threshold) {
                region[q] = 1;
                ++count;
                stack_push(&st, q);
            }
        }
    }
    free(st.v);
    return count;
}

/* foreground shapes of the reference volume; returns -1 where the background shows through */
static int volume_shape(int x, int y, int z) {
    int v = -1;
    float d1 = (float)sqrt((double)((x - 300) * (x - 300) + (y - 400) * (y - 400) + (z - 100) * (z - 100)));
    if (d1 < 100) v = 30;
    float d2 = (float)sqrt((double)((x - 100) * (x - 100) + (y - 200) * (y - 200) + (z - 400) * (z - 400)));
    if (d2 < 50) v = 50;
    if (x > 200 && x < 300 && y > 300 && y < 500 && z > 200 && z < 300) v = 45;
    if (x > 0 && x < 100 && y > 250 && y < 400 && z > 250 && z < 400) v = 35;
    return v;
}

void pcmx_create_data(unsigned char* data, int dim) {
    srand(1); /* the reference never seeds: glibc's default sequence is seed 1 */
    for (int z = 0; z < dim; ++z)
        for (int y = 0; y < dim; ++y) {
            unsigned char* row = data + ((size_t)z * dim + y) * dim;
            for (int x = 0; x < dim; ++x) {
                int bg = rand() % 20; /* drawn for every voxel, as the reference does */
                int s = volume_shape(x, y, z);
                row[x] = (unsigned char)(s >= 0 ? s : bg);
            }
        }
}

unsigned int pcmx_hash3(unsigned int x, unsigned int y, unsigned int z, unsigned int seed);
unsigned int pcmx_hash3(unsigned int x, unsigned int y, unsigned int z, unsigned int seed) {
    unsigned int h = seed ^ 0x9E3779B9u;
    h ^= x * 0x85EBCA6Bu;
    h = (h << 13) | (h >> 19);
    h ^= y * 0xC2B2AE35u;
    h = (h << 17) | (h >> 15);
    h ^= z * 0x27D4EB2Fu;
    h ^= h >> 16;
    h *= 0x7FEB352Du;
    h ^= h >> 15;
    h *= 0x846CA68Bu;
    h ^= h >> 16;
    return h;
}

void pcmx_create_data_hash(unsigned char* data, int dim, unsigned int seed) {
#pragma omp parallel for schedule(static)
    for (int z = 0; z < dim; ++z)
        for (int y = 0; y < dim; ++y) {
            unsigned char* row = data + ((size_t)z * dim + y) * dim;
            for (int x = 0; x < dim; ++x) {
                int s = volume_shape(x, y, z);
                row[x] = (unsigned char)(s >= 0 ? s : (int)(pcmx_hash3((unsigned)x, (unsigned)y, (unsigned)z, seed) % 20u));
            }
        }
}

/* ---------------------------------------------------------------------- ray casting */

static void v3_cross(const float* a, const float* b, float* c) {
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}
static void v3_normalize(float* v) {
    float l = (float)sqrt((double)(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]));
    v[0] /= l;
    v[1] /= l;
    v[2] /= l;
}

void pcmx_default_camera(int image_dim, pcmx_camera_t* cam) {
    const float z_axis[3] = {0, 0, 1};
    cam->camera[0] = cam->camera[1] = cam->camera[2] = 1000.0f;
    cam->forward[0] = cam->forward[1] = cam->forward[2] = -1.0f;
    v3_cross(cam->forward, z_axis, cam->right);
    v3_cross(cam->right, cam->forward, cam->up);
    v3_normalize(cam->forward);
    v3_normalize(cam->right);
    v3_normalize(cam->up);
    float fov = (float)(3.14 / 4);
    cam->pixel_width = (float)(tan(fov / 2.0) / (image_dim / 2));
    cam->step_size = 0.5f;
    cam->max_steps = 5000;
}

static inline int inside_f(const float* p, int dim) {
    return p[0] >= 0 && p[0] < dim - 1 && p[1] >= 0 && p[1] < dim - 1 && p[2] >= 0 && p[2] < dim - 1;
}

static float value_at_ref(const float* pos, const unsigned char* d, int dim) {
    if (!inside_f(pos, dim)) return 0;
    int x = (int)floor(pos[0]), y = (int)floor(pos[1]), z = (int)floor(pos[2]);
    int xu = (int)ceil(pos[0]), yu = (int)ceil(pos[1]), zu = (int)ceil(pos[2]);
    float rx = pos[0] - x, ry = pos[1] - y, rz = pos[2] - z;
    const size_t P = (size_t)dim * dim;
#define D(zz, yy, xx) d[(size_t)(zz) * P + (size_t)(yy) * dim + (xx)]
    float a0 = rx * D(z, y, x) + (1 - rx) * D(z, y, xu);
    float a1 = rx * D(z, yu, x) + (1 - rx) * D(z, yu, xu);
    float a2 = rx * D(zu, y, x) + (1 - rx) * D(zu, y, xu);
    float a3 = rx * D(zu, yu, x) + (1 - rx) * D(zu, yu, xu);
#undef D
    float b0 = ry * a0 + (1 - ry) * a1;
    float b1 = ry * a2 + (1 - ry) * a3;
    return rz * b0 + (1 - rz) * b1;
}

void pcmx_raycast_serial(const unsigned char* data, const unsigned char* region, int dim, int image_dim,
                         unsigned char* image) {
    pcmx_camera_t cam;
    pcmx_default_camera(image_dim, &cam);
    const int half = image_dim / 2;
#pragma omp parallel for schedule(dynamic, 1)
    for (int y = -half; y < half; ++y)
        for (int x = -half; x < half; ++x) {
            float ray[3], pos[3];
            for (int k = 0; k < 3; ++k) {
                float sc = cam.camera[k] + cam.forward[k];
                float t = (sc + cam.right[k] * (x * cam.pixel_width)) + cam.up[k] * (y * cam.pixel_width);
                ray[k] = t + cam.camera[k] * -1;
                pos[k] = cam.camera[k];
            }
            v3_normalize(ray);
            int i = 0;
            float color = 0;
            while (color < 255 && i < cam.max_steps) {
                ++i;
                for (int k = 0; k < 3; ++k) pos[k] = pos[k] + ray[k] * cam.step_size;
                int r = (int)value_at_ref(pos, region, dim);
                color = (float)((double)color + (double)value_at_ref(pos, data, dim) * (0.01 + r));
            }
            image[(y + half) * image_dim + (x + half)] = (unsigned char)(color > 255 ? 255 : color);
        }
}

/* ------------------------------------------------------- z-slab decomposition of the 3-D pipeline (host side) */

void pcmx_create_data_hash_slab(unsigned char* data, int dim, int z_first, int nplanes, unsigned int seed) {
#pragma omp parallel for schedule(static)
    for (int k = 0; k < nplanes; ++k) {
        const int z = z_first + k;
        unsigned char* pl = data + (size_t)k * dim * dim;
        if (z < 0 || z >= dim) {
            memset(pl, 0, (size_t)dim * dim);
            continue;
        }
        for (int y = 0; y < dim; ++y)
            for (int x = 0; x < dim; ++x) {
                int s = volume_shape(x, y, z);
                pl[(size_t)y * dim + x] =
                    (unsigned char)(s >= 0 ? s : (int)(pcmx_hash3((unsigned)x, (unsigned)y, (unsigned)z, seed) % 20u));
            }
    }
}

long long pcmx_region3d_slab_host(const unsigned char* data, unsigned char* region, int dim, int nz, int halos, int thr) {
    /* data/region point at the slab's first OWNED plane; planes -1 / nz are readable when halos bit 0 / 1 */
    const long long P = (long long)dim * dim;
    idx_stack_t st = {0, 0, 0};
    const long long lo = (halos & 1) ? -P : 0, hi = (halos & 2) ? (nz + 1) * P : nz * P;
    for (long long i = lo; i < hi; ++i) /* every region voxel (owned or halo) seeds the fill */
        if (region[i]) stack_push(&st, i);
    long long added = 0;
    while (st.n > 0) {
        const long long p = st.v[--st.n];
        const int z = p >= 0 ? (int)(p / P) : -1; /* p in [-P, 0): the halo plane below */
        const long long rem = p - (long long)z * P;
        const int y = (int)(rem / dim), x = (int)(rem % dim);
        const int nb[6][3] = {{-1, 0, 0}, {1, 0, 0}, {0, -1, 0}, {0, 1, 0}, {0, 0, -1}, {0, 0, 1}};
        for (int k = 0; k < 6; ++k) {
            const int cx = x + nb[k][0], cy = y + nb[k][1], cz = z + nb[k][2];
            if (cx < 0 || cy < 0 || cx >= dim || cy >= dim || cz < 0 || cz >= nz) continue; /* grow owned planes only */
            const long long q = (long long)cz * P + (long long)cy * dim + cx;
            if (region[q]) continue;
            if (abs((int)data[p] - (int)data[q]) < thr) {
                region[q] = 1;
                ++added;
                stack_push(&st, q);
            }
        }
    }
    free(st.v);
    return added;
}

/* value_at_ref on a slab whose plane 0 is global plane zoff */
static float value_at_slab(const float* pos, const unsigned char* d, int dim, int zoff) {
    if (!inside_f(pos, dim)) return 0;
    int x = (int)floor(pos[0]), y = (int)floor(pos[1]), z = (int)floor(pos[2]);
    int xu = (int)ceil(pos[0]), yu = (int)ceil(pos[1]), zu = (int)ceil(pos[2]);
    float rx = pos[0] - x, ry = pos[1] - y, rz = pos[2] - z;
    const size_t P = (size_t)dim * dim;
#define D(zz, yy, xx) d[(size_t)((zz) - zoff) * P + (size_t)(yy) * dim + (xx)]
    float a0 = rx * D(z, y, x) + (1 - rx) * D(z, y, xu);
    float a1 = rx * D(z, yu, x) + (1 - rx) * D(z, yu, xu);
    float a2 = rx * D(zu, y, x) + (1 - rx) * D(zu, y, xu);
    float a3 = rx * D(zu, yu, x) + (1 - rx) * D(zu, yu, xu);
#undef D
    float b0 = ry * a0 + (1 - ry) * a1;
    float b1 = ry * a2 + (1 - ry) * a3;
    return rz * b0 + (1 - rz) * b1;
}

void pcmx_raycast_slab_host(const unsigned char* data, const unsigned char* region, int dim, int z0, int z1,
                            int image_dim, int* state, int init, int bottom, unsigned char* image) {
    pcmx_camera_t cam;
    pcmx_default_camera(image_dim, &cam);
    const int half = image_dim / 2;
    const int zoff = z0 - 1; /* the slab buffers start at global plane z0 - 1 (halo below) */
#pragma omp parallel for schedule(dynamic, 1)
    for (int py = 0; py < image_dim; ++py)
        for (int px = 0; px < image_dim; ++px) {
            const int x = px - half, y = py - half;
            int* stp = state + 6 * ((size_t)py * image_dim + px);
            float ray[3], pos[3], color;
            int i, flags;
            for (int k = 0; k < 3; ++k) {
                float sc = cam.camera[k] + cam.forward[k];
                float t = (sc + cam.right[k] * (x * cam.pixel_width)) + cam.up[k] * (y * cam.pixel_width);
                ray[k] = t + cam.camera[k] * -1;
            }
            v3_normalize(ray);
            if (init) {
                pos[0] = cam.camera[0], pos[1] = cam.camera[1], pos[2] = cam.camera[2];
                color = 0, i = 0, flags = 0;
            } else {
                memcpy(pos, stp, 3 * sizeof(float));
                memcpy(&color, stp + 3, sizeof(float));
                i = stp[4], flags = stp[5];
            }
            while (!(flags & 2) && color < 255 && i < cam.max_steps) {
                float nxt[3];
                for (int k = 0; k < 3; ++k) nxt[k] = pos[k] + ray[k] * cam.step_size;
                if (!bottom && nxt[2] < (float)z0) break; /* the next sample belongs to a lower slab */
                ++i;
                pos[0] = nxt[0], pos[1] = nxt[1], pos[2] = nxt[2];
                if (!inside_f(pos, dim)) {
                    if (flags & 1) flags |= 2; /* left the convex volume: every later sample is 0 */
                    continue;
                }
                flags |= 1;
                int r = (int)value_at_slab(pos, region, dim, zoff);
                color = (float)((double)color + (double)value_at_slab(pos, data, dim, zoff) * (0.01 + r));
            }
            memcpy(stp, pos, 3 * sizeof(float));
            memcpy(stp + 3, &color, sizeof(float));
            stp[4] = i, stp[5] = flags;
            if (bottom) image[(size_t)py * image_dim + px] = (unsigned char)(color > 255 ? 255 : color);
        }
}
