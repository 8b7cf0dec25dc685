// Volume generation and ray casting on MI355X (ref 5-cuda-region-growing/raycast.cu:114-158 generator,
// :321-371 global-memory ray caster, :374-433 texture ray caster; OpenCL twin 6-opencl-region-growing/
// raycast.cl:93-137 at IMAGE_DIM 64).
//
//  * raycast_global (mode REF): bit-compatible with the serial C ray caster (swapped trilinear weights
//    of value_at, floor/ceil corner selection, f64 colour update of the C build, no FMA contraction).
//    mode CUDA: the same with the f32 colour update of the CUDA kernel.
//  * raycast_bricked: the reference's hardware-texture path re-designed for CDNA (gfx950 exposes no
//    image/texture sampling to HIP): the volume is pre-packed into 8-byte texels holding the 2x2 (x,y)
//    footprint of data AND region, so one trilinear sample of both volumes costs two 8-byte loads
//    (z and z+1) instead of 16 byte loads; texel-centre addressing, clamp-to-edge and 8-bit fixed-point
//    weights emulate cudaFilterModeLinear + cudaReadModeNormalizedFloat.
//  * Both casters march positions by repeated f32 adds exactly like the reference, but skip sampling
//    while the ray is outside the volume's bounding box (the adds still run, so positions are unchanged)
//    and stop once the ray has left it (a convex box cannot be re-entered): identical images, far fewer
//    loads for rays that miss or exit early.
//  * 16x16 pixel workgroups (4 wave64s of 16x4 pixels): neighbouring rays share cache lines.
#include "pcmx_common.h"
#include "pcmx_hip.h"

namespace {

struct Cam {
    float cam[3], fwd[3], right[3], up[3];
    float pw, step;
    int max_steps;
};

__device__ __forceinline__ unsigned hash3(unsigned x, unsigned y, unsigned z, unsigned seed) {
    unsigned h = seed ^ 0x9E3779B9u;
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

__device__ __forceinline__ int shape_value(int x, int y, int z) {
    // (float)sqrt(n) < 100  <=>  n < 10000 for integer n (sqrt(9999) rounds below 100), likewise for 50:
    // integer tests are exactly the reference predicate and independent of device sqrt rounding.
    int v = -1;
    if ((x - 300) * (x - 300) + (y - 400) * (y - 400) + (z - 100) * (z - 100) < 10000) v = 30;
    if ((x - 100) * (x - 100) + (y - 200) * (y - 200) + (z - 400) * (z - 400) < 2500) v = 50;
    if (x > 200 && x < 300 && y > 300 && y < 500 && z > 200 && z < 300) v = 45;
    if (x > 0 && x < 100 && y > 250 && y < 400 && z > 250 && z < 400) v = 35;
    return v;
}

__global__ __launch_bounds__(256) void volume_gen_kernel(unsigned char* __restrict__ data, int dim, unsigned seed) {
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y, z = blockIdx.z;
    if (x >= dim) return;
    const int s = shape_value(x, y, z);
    data[((size_t)z * dim + y) * dim + x] = (unsigned char)(s >= 0 ? s : (int)(hash3(x, y, z, seed) % 20u));
}

// ---------------------------------------------------------------------------------- reference path
#pragma clang fp contract(off)
__device__ __forceinline__ float value_at_ref(float px, float py, float pz, const unsigned char* __restrict__ d, int dim) {
    if (!(px >= 0 && px < dim - 1 && py >= 0 && py < dim - 1 && pz >= 0 && pz < dim - 1)) return 0.f;
    const int x = (int)floorf(px), y = (int)floorf(py), z = (int)floorf(pz);
    const int xu = (int)ceilf(px), yu = (int)ceilf(py), zu = (int)ceilf(pz);
    const float rx = px - x, ry = py - y, rz = pz - z;
    const size_t P = (size_t)dim * dim;
    const unsigned char* zy = d + (size_t)z * P + (size_t)y * dim;
    const unsigned char* zyu = d + (size_t)z * P + (size_t)yu * dim;
    const unsigned char* zuy = d + (size_t)zu * P + (size_t)y * dim;
    const unsigned char* zuyu = d + (size_t)zu * P + (size_t)yu * dim;
    const float a0 = rx * zy[x] + (1 - rx) * zy[xu];
    const float a1 = rx * zyu[x] + (1 - rx) * zyu[xu];
    const float a2 = rx * zuy[x] + (1 - rx) * zuy[xu];
    const float a3 = rx * zuyu[x] + (1 - rx) * zuyu[xu];
    const float b0 = ry * a0 + (1 - ry) * a1;
    const float b1 = ry * a2 + (1 - ry) * a3;
    return rz * b0 + (1 - rz) * b1;
}

__device__ __forceinline__ bool in_box(float px, float py, float pz, float hi) {
    return px >= 0 && px < hi && py >= 0 && py < hi && pz >= 0 && pz < hi;
}

template <bool F64COLOR>
__global__ __launch_bounds__(256) void raycast_ref_kernel(const unsigned char* __restrict__ data,
                                                         const unsigned char* __restrict__ region, int dim,
                                                         unsigned char* __restrict__ image, int image_dim, Cam c) {
    const int px = blockIdx.x * 16 + (threadIdx.x & 15);
    const int py = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (px >= image_dim || py >= image_dim) return;
    const int half = image_dim / 2;
    const int x = px - half, y = py - half;
    float ray[3], pos[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float sc = c.cam[k] + c.fwd[k];
        const float t = (sc + c.right[k] * (x * c.pw)) + c.up[k] * (y * c.pw);
        ray[k] = t + c.cam[k] * -1;
        pos[k] = c.cam[k];
    }
    // correctly rounded f32 sqrt (as the C reference's (float)sqrt((double)...)); v_sqrt_f32 is not
    const float l = (float)sqrt((double)(ray[0] * ray[0] + ray[1] * ray[1] + ray[2] * ray[2]));
    ray[0] /= l, ray[1] /= l, ray[2] /= l;
    const float sx = ray[0] * c.step, sy = ray[1] * c.step, sz = ray[2] * c.step;
    const float hi = (float)(dim - 1);
    int i = 0;
    float color = 0.f;
    bool entered = false;
    while (color < 255 && i < c.max_steps) {
        ++i;
        pos[0] = pos[0] + sx;
        pos[1] = pos[1] + sy;
        pos[2] = pos[2] + sz;
        if (!in_box(pos[0], pos[1], pos[2], hi)) {
            if (entered) break;  // left the convex volume: every later sample is 0
            continue;
        }
        entered = true;
        const int r = (int)value_at_ref(pos[0], pos[1], pos[2], region, dim);
        const float v = value_at_ref(pos[0], pos[1], pos[2], data, dim);
        if constexpr (F64COLOR)
            color = (float)((double)color + (double)v * (0.01 + r));
        else
            color += v * (0.01f + r);
    }
    image[py * image_dim + px] = (unsigned char)(color > 255 ? 255.f : color);
}
#pragma clang fp contract(on)

// ---------------------------------------------------------------------------------- texture path
// texel(x,y,z) = [d(x,y) d(x+1,y) d(x,y+1) d(x+1,y+1) | r(x,y) r(x+1,y) r(x,y+1) r(x+1,y+1)] at plane z,
// neighbours clamped to the volume edge.
__global__ __launch_bounds__(256) void brick_pack_kernel(const unsigned char* __restrict__ data,
                                                        const unsigned char* __restrict__ region, int dim,
                                                        unsigned long long* __restrict__ tex) {
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y, z = blockIdx.z;
    if (x >= dim) return;
    const int x1 = min(x + 1, dim - 1), y1 = min(y + 1, dim - 1);
    const size_t P = (size_t)dim * dim, r0 = (size_t)z * P + (size_t)y * dim, r1 = (size_t)z * P + (size_t)y1 * dim;
    const unsigned long long lo = (unsigned)data[r0 + x] | ((unsigned)data[r0 + x1] << 8) |
                                  ((unsigned)data[r1 + x] << 16) | ((unsigned)data[r1 + x1] << 24);
    const unsigned long long hi = (unsigned)(region[r0 + x] != 0) | ((unsigned)(region[r0 + x1] != 0) << 8) |
                                  ((unsigned)(region[r1 + x] != 0) << 16) | ((unsigned)(region[r1 + x1] != 0) << 24);
    tex[r0 + x] = lo | (hi << 32);
}

__device__ __forceinline__ float bilerp4(unsigned w, float ax, float ay) {
    const float v00 = (float)(w & 0xff), v10 = (float)((w >> 8) & 0xff);
    const float v01 = (float)((w >> 16) & 0xff), v11 = (float)(w >> 24);
    return (1.f - ay) * ((1.f - ax) * v00 + ax * v10) + ay * ((1.f - ax) * v01 + ax * v11);
}

// hardware-like fractional weight: 8 fractional bits
__device__ __forceinline__ float q8(float f) { return rintf(f * 256.f) * (1.f / 256.f); }

__global__ __launch_bounds__(256) void raycast_tex_kernel(const unsigned long long* __restrict__ tex, int dim,
                                                         unsigned char* __restrict__ image, int image_dim, Cam c) {
    const int px = blockIdx.x * 16 + (threadIdx.x & 15);
    const int py = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (px >= image_dim || py >= image_dim) return;
    const int half = image_dim / 2;
    const int x = px - half, y = py - half;
    float ray[3], pos[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float sc = c.cam[k] + c.fwd[k];
        ray[k] = (sc + c.right[k] * (x * c.pw)) + c.up[k] * (y * c.pw) - c.cam[k];
        pos[k] = c.cam[k];
    }
    const float l = sqrtf(ray[0] * ray[0] + ray[1] * ray[1] + ray[2] * ray[2]);
    const float sx = ray[0] / l * c.step, sy = ray[1] / l * c.step, sz = ray[2] / l * c.step;
    const float hi = (float)(dim - 1);
    const size_t P = (size_t)dim * dim;
    float color = 0.f;
    bool entered = false;
    for (int i = 0; i < c.max_steps && color < 255.f; ++i) {
        pos[0] += sx, pos[1] += sy, pos[2] += sz;
        if (!in_box(pos[0], pos[1], pos[2], hi)) {  // texture fetches outside never add colour
            if (entered) break;
            continue;
        }
        entered = true;
        // texel-centre addressing: sample at p - 0.5, clamp-to-edge
        float fx = pos[0] - 0.5f, fy = pos[1] - 0.5f, fz = pos[2] - 0.5f;
        int x0 = (int)floorf(fx), y0 = (int)floorf(fy), z0 = (int)floorf(fz);
        float ax = q8(fx - x0), ay = q8(fy - y0), az = q8(fz - z0);
        if (x0 < 0) x0 = 0, ax = 0.f;
        if (y0 < 0) y0 = 0, ay = 0.f;
        if (z0 < 0) z0 = 0, az = 0.f;
        const int z1 = min(z0 + 1, dim - 1);
        const size_t o = (size_t)y0 * dim + x0;
        const unsigned long long t0 = tex[(size_t)z0 * P + o];
        const unsigned long long t1 = tex[(size_t)z1 * P + o];
        const float d = (1.f - az) * bilerp4((unsigned)t0, ax, ay) + az * bilerp4((unsigned)t1, ax, ay);
        const float rr = (1.f - az) * bilerp4((unsigned)(t0 >> 32), ax, ay) + az * bilerp4((unsigned)(t1 >> 32), ax, ay);
        const int r = (int)rr;  // 255 * normalised region tap, region voxels hold 1
        color += d * (0.01f + r);
    }
    image[py * image_dim + px] = (unsigned char)(color > 255.f ? 255.f : color);
}

Cam make_cam(const float* cam12, float pw, float step, int max_steps) {
    Cam c;
    for (int k = 0; k < 3; ++k) {
        c.cam[k] = cam12[k];
        c.fwd[k] = cam12[3 + k];
        c.right[k] = cam12[6 + k];
        c.up[k] = cam12[9 + k];
    }
    c.pw = pw;
    c.step = step;
    c.max_steps = max_steps;
    return c;
}
}  // namespace

extern "C" int pcmx_volume_gen_u8(unsigned char* data, int dim, unsigned seed, hipStream_t s) {
    if (dim <= 0) return -1;
    volume_gen_kernel<<<dim3((dim + 255) / 256, dim, dim), 256, 0, s>>>(data, dim, seed);
    return (int)hipGetLastError();
}

// cam12 = camera[3], forward[3], right[3], up[3] (host array; already normalised, see pcmx_default_camera)
extern "C" int pcmx_raycast_global(const unsigned char* data, const unsigned char* region, int dim, unsigned char* image,
                                   int image_dim, const float* cam12, float pixel_width, float step, int max_steps,
                                   int f64_color, hipStream_t s) {
    if (dim <= 1 || image_dim <= 0) return -1;
    const Cam c = make_cam(cam12, pixel_width, step, max_steps);
    dim3 grid((image_dim + 15) / 16, (image_dim + 15) / 16);
    if (f64_color)
        raycast_ref_kernel<true><<<grid, 256, 0, s>>>(data, region, dim, image, image_dim, c);
    else
        raycast_ref_kernel<false><<<grid, 256, 0, s>>>(data, region, dim, image, image_dim, c);
    return (int)hipGetLastError();
}

extern "C" int pcmx_brick_pack(const unsigned char* data, const unsigned char* region, int dim, unsigned long long* tex,
                               hipStream_t s) {
    if (dim <= 0) return -1;
    brick_pack_kernel<<<dim3((dim + 255) / 256, dim, dim), 256, 0, s>>>(data, region, dim, tex);
    return (int)hipGetLastError();
}

extern "C" int pcmx_raycast_bricked(const unsigned long long* tex, int dim, unsigned char* image, int image_dim,
                                    const float* cam12, float pixel_width, float step, int max_steps, hipStream_t s) {
    if (dim <= 1 || image_dim <= 0) return -1;
    const Cam c = make_cam(cam12, pixel_width, step, max_steps);
    dim3 grid((image_dim + 15) / 16, (image_dim + 15) / 16);
    raycast_tex_kernel<<<grid, 256, 0, s>>>(tex, dim, image, image_dim, c);
    return (int)hipGetLastError();
}
