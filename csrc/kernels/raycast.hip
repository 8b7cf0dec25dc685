// Volume generation and ray casting on MI355X (ref 5-cuda-region-growing/raycast.cu:114-158 generator,
// :321-371 global-memory ray caster, :374-433 texture ray caster; OpenCL twin 6-opencl-region-growing/
// raycast.cl:93-137 at IMAGE_DIM 64).
//
//  * raycast_global (mode REF): bit-compatible with the serial C ray caster (swapped trilinear weights
//    of value_at, floor/ceil corner selection, f64 colour update of the C build, no FMA contraction).
//    mode CUDA: the same with the f32 colour update of the CUDA kernel.
//  * raycast_bricked: the reference's hardware-texture path re-designed for CDNA (gfx950 exposes no
//    image/texture sampling to HIP): the volume is pre-packed into texels holding the whole 2x2x2 footprint
//    of data AND region (8 bytes with the region in bit 7 when the data is < 128, else 16 bytes), so one
//    trilinear sample of both volumes is ONE load instead of 16 byte loads; texel-centre addressing,
//    clamp-to-edge and 8-bit fixed-point weights emulate cudaFilterModeLinear + cudaReadModeNormalizedFloat.
//    Rays are clipped analytically to the volume and only the steps inside are visited (prefetched in
//    batches of 16 steps; only the raw texels stay live across a batch) and every 16x4 ray patch is split over
//    4 waves by step range (partial colours composed in ray order). 512^2 image of the 512^3 reference volume:
//    march 2.7 -> 1.16 -> 0.83 ms; frame (pack + march) 3.18 -> 1.66 -> 1.18 -> 1.07 ms.
//  * raycast_global marches positions by repeated f32 adds exactly like the reference, but skips sampling
//    while the ray is outside the volume's bounding box (the adds still run, so positions are unchanged)
//    and stops once the ray has left it (a convex box cannot be re-entered): identical images, far fewer
//    loads for rays that miss or exit early.
//  * 16x16 pixel workgroups (4 wave64s of 16x4 pixels): neighbouring rays share cache lines.
#include "pcmx_common.h"
#include "pcmx_hip.h"

#include <type_traits>

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

// planes [z_first, z_first + gridDim.z) of the volume (zeros outside 0..dim-1): a z-slab with its halo planes
__global__ __launch_bounds__(256) void volume_gen_slab_kernel(unsigned char* __restrict__ data, int dim, int z_first,
                                                             unsigned seed) {
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y, z = z_first + (int)blockIdx.z;
    if (x >= dim) return;
    unsigned char v = 0;
    if (z >= 0 && z < dim) {
        const int s = shape_value(x, y, z);
        v = (unsigned char)(s >= 0 ? s : (int)(hash3(x, y, z, seed) % 20u));
    }
    data[((size_t)blockIdx.z * dim + y) * dim + x] = v;
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

// ---- the same march with the samples of B steps in flight (production global caster, round 5).
// The positions of a ray do not depend on its colour: they are the reference's sequence of f32 adds, so the next B
// positions are computed ahead and ALL their loads (8 byte loads per volume per sample) issued before the colour
// of any of them is accumulated in step order. A step's loads no longer wait for the previous step's, which is what
// bounds a march of ~1000 dependent samples (the reference's raycast kernel on MI355X: 2.95 ms at 64^2; ours with one
// step in flight: 4.74 ms; profiles/r5_refbase/). Same arithmetic in the same order: bit-identical images.
struct Taps {
    float rx, ry, rz;
    unsigned char t[8];  // zy[x], zy[xu], zyu[x], zyu[xu], zuy[x], zuy[xu], zuyu[x], zuyu[xu]
    bool ok;
};
__device__ __forceinline__ void taps_load(float px, float py, float pz, const unsigned char* __restrict__ d, int dim,
                                          Taps& T) {
    T.ok = px >= 0 && px < dim - 1 && py >= 0 && py < dim - 1 && pz >= 0 && pz < dim - 1;
    if (!T.ok) return;  // (a sample outside the volume reads as 0: no loads)
    const int x = (int)floorf(px), y = (int)floorf(py), z = (int)floorf(pz);
    const int xu = (int)ceilf(px), yu = (int)ceilf(py), zu = (int)ceilf(pz);
    T.rx = px - x, T.ry = py - y, T.rz = pz - z;
    const size_t P = (size_t)dim * dim;
    const unsigned char* zy = d + (size_t)z * P + (size_t)y * dim;
    const unsigned char* zyu = d + (size_t)z * P + (size_t)yu * dim;
    const unsigned char* zuy = d + (size_t)zu * P + (size_t)y * dim;
    const unsigned char* zuyu = d + (size_t)zu * P + (size_t)yu * dim;
    T.t[0] = zy[x], T.t[1] = zy[xu], T.t[2] = zyu[x], T.t[3] = zyu[xu];
    T.t[4] = zuy[x], T.t[5] = zuy[xu], T.t[6] = zuyu[x], T.t[7] = zuyu[xu];
}
__device__ __forceinline__ float taps_value(const Taps& T) {  // value_at_ref's arithmetic, operation for operation
    if (!T.ok) return 0.f;
    const float rx = T.rx, ry = T.ry, rz = T.rz;
    const float a0 = rx * T.t[0] + (1 - rx) * T.t[1];
    const float a1 = rx * T.t[2] + (1 - rx) * T.t[3];
    const float a2 = rx * T.t[4] + (1 - rx) * T.t[5];
    const float a3 = rx * T.t[6] + (1 - rx) * T.t[7];
    const float b0 = ry * a0 + (1 - ry) * a1;
    const float b1 = ry * a2 + (1 - ry) * a3;
    return rz * b0 + (1 - rz) * b1;
}

template <bool F64COLOR, int B>
__global__ __launch_bounds__(64) void raycast_ref_batch_kernel(const unsigned char* __restrict__ data,
                                                               const unsigned char* __restrict__ region, int dim,
                                                               unsigned char* __restrict__ image, int image_dim, Cam c) {
    // one wave per 8x8 pixel tile: a small image (the OpenCL program's 64^2: 64 rays per ... 64 waves) spreads over
    // 64 CUs instead of 16, each wave with a CU's load pipeline to itself
    const int px = blockIdx.x * 8 + (threadIdx.x & 7);
    const int py = blockIdx.y * 8 + (threadIdx.x >> 3);
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
    const float l = (float)sqrt((double)(ray[0] * ray[0] + ray[1] * ray[1] + ray[2] * ray[2]));
    ray[0] /= l, ray[1] /= l, ray[2] /= l;
    const float sx = ray[0] * c.step, sy = ray[1] * c.step, sz = ray[2] * c.step;
    const float hi = (float)(dim - 1);
    int i = 0;
    float color = 0.f;
    // outside the volume's box a sample adds exactly 0: walk the positions to the first sample inside (adds only)
    while (i < c.max_steps) {
        const float nx = pos[0] + sx, ny = pos[1] + sy, nz = pos[2] + sz;
        if (in_box(nx, ny, nz, hi)) break;
        ++i;
        pos[0] = nx, pos[1] = ny, pos[2] = nz;
    }
    bool done = i >= c.max_steps;
    while (!done) {
        float q[B][3];
#pragma unroll
        for (int b = 0; b < B; ++b) {
            pos[0] = pos[0] + sx, pos[1] = pos[1] + sy, pos[2] = pos[2] + sz;
            q[b][0] = pos[0], q[b][1] = pos[1], q[b][2] = pos[2];
        }
        Taps R[B], D[B];
#pragma unroll
        for (int b = 0; b < B; ++b) {
            taps_load(q[b][0], q[b][1], q[b][2], region, dim, R[b]);
            taps_load(q[b][0], q[b][1], q[b][2], data, dim, D[b]);
        }
#pragma unroll
        for (int b = 0; b < B; ++b) {
            if (!done) {
                if (!(color < 255 && i < c.max_steps)) {
                    done = true;
                } else {
                    ++i;
                    if (!in_box(q[b][0], q[b][1], q[b][2], hi)) {
                        done = true;  // left the convex volume: every later sample is 0
                    } else {
                        const int r = (int)taps_value(R[b]);
                        const float v = taps_value(D[b]);
                        if constexpr (F64COLOR)
                            color = (float)((double)color + (double)v * (0.01 + r));
                        else
                            color += v * (0.01f + r);
                    }
                }
            }
        }
    }
    image[py * image_dim + px] = (unsigned char)(color > 255 ? 255.f : color);
}

// ---- round 6: PAIR taps and GROUP-PER-RAY marching.
// Pair taps: the two x taps of a row (x and xu = x or x + 1) come from ONE 8-byte buffer load at the 4-byte-aligned
// address below x (bytes x and x + 1 both lie inside it); the descriptor spans the volume, so a load running past its
// end reads 0 instead of faulting. 8 load instructions per sample (4 rows x 2 volumes) instead of 16 byte loads.
struct Taps2 {
    float rx, ry, rz;
    unsigned char t[8];
    bool ok;
};
__device__ __forceinline__ void taps_load2(float px, float py, float pz, __amdgpu_buffer_rsrc_t rs, int dim, Taps2& T) {
    T.ok = px >= 0 && px < dim - 1 && py >= 0 && py < dim - 1 && pz >= 0 && pz < dim - 1;
    if (!T.ok) return;
    const int x = (int)floorf(px), y = (int)floorf(py), z = (int)floorf(pz);
    const int xu = (int)ceilf(px), yu = (int)ceilf(py), zu = (int)ceilf(pz);
    T.rx = px - x, T.ry = py - y, T.rz = pz - z;
    const unsigned P = (unsigned)dim * (unsigned)dim;
    const unsigned rows[4] = {(unsigned)z * P + (unsigned)y * dim, (unsigned)z * P + (unsigned)yu * dim,
                              (unsigned)zu * P + (unsigned)y * dim, (unsigned)zu * P + (unsigned)yu * dim};
    const unsigned sh = (unsigned)(x & 3) * 8u, dx = (unsigned)(xu - x) * 8u;
    unsigned long long w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        w[k] = __builtin_bit_cast(unsigned long long,
                                  __builtin_amdgcn_raw_buffer_load_b64(rs, rows[k] + (unsigned)(x & ~3), 0, 0));
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        T.t[2 * k] = (unsigned char)(w[k] >> sh);
        T.t[2 * k + 1] = (unsigned char)(w[k] >> (sh + dx));
    }
}
__device__ __forceinline__ float taps2_value(const Taps2& T) {  // value_at_ref's arithmetic, operation for operation
    if (!T.ok) return 0.f;
    const float rx = T.rx, ry = T.ry, rz = T.rz;
    const float a0 = rx * T.t[0] + (1 - rx) * T.t[1];
    const float a1 = rx * T.t[2] + (1 - rx) * T.t[3];
    const float a2 = rx * T.t[4] + (1 - rx) * T.t[5];
    const float a3 = rx * T.t[6] + (1 - rx) * T.t[7];
    const float b0 = ry * a0 + (1 - ry) * a1;
    const float b1 = ry * a2 + (1 - ry) * a3;
    return rz * b0 + (1 - rz) * b1;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t volume_rsrc(const unsigned char* d, int dim) {
    const long long bytes = (long long)dim * dim * dim;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(d), (short)0,
                                             (int)(bytes < 0x7fffffffLL ? bytes : 0x7fffffffLL), 0x00020000);
}

// The reference's ray set-up for pixel (px, py), operation for operation (raycast.cu:352-357).
__device__ __forceinline__ void ray_setup(const Cam& c, int px, int py, int image_dim, float (&pos)[3], float& sx,
                                          float& sy, float& sz) {
    const int half = image_dim / 2;
    const int x = px - half, y = py - half;
    float ray[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float sc = c.cam[k] + c.fwd[k];
        const float t = (sc + c.right[k] * (x * c.pw)) + c.up[k] * (y * c.pw);
        ray[k] = t + c.cam[k] * -1;
        pos[k] = c.cam[k];
    }
    const float l = (float)sqrt((double)(ray[0] * ray[0] + ray[1] * ray[1] + ray[2] * ray[2]));
    ray[0] /= l, ray[1] /= l, ray[2] /= l;
    sx = ray[0] * c.step, sy = ray[1] * c.step, sz = ray[2] * c.step;
}

// The batch caster with pair taps (variant 4): otherwise raycast_ref_batch_kernel.
template <bool F64COLOR, int B>
__global__ __launch_bounds__(64) void raycast_ref_batch2_kernel(const unsigned char* __restrict__ data,
                                                                const unsigned char* __restrict__ region, int dim,
                                                                unsigned char* __restrict__ image, int image_dim, Cam c) {
    const int px = blockIdx.x * 8 + (threadIdx.x & 7);
    const int py = blockIdx.y * 8 + (threadIdx.x >> 3);
    if (px >= image_dim || py >= image_dim) return;
    const auto rd = volume_rsrc(data, dim), rr = volume_rsrc(region, dim);
    float pos[3], sx, sy, sz;
    ray_setup(c, px, py, image_dim, pos, sx, sy, sz);
    const float hi = (float)(dim - 1);
    int i = 0;
    float color = 0.f;
    while (i < c.max_steps) {
        const float nx = pos[0] + sx, ny = pos[1] + sy, nz = pos[2] + sz;
        if (in_box(nx, ny, nz, hi)) break;
        ++i;
        pos[0] = nx, pos[1] = ny, pos[2] = nz;
    }
    bool done = i >= c.max_steps;
    while (!done) {
        float q[B][3];
#pragma unroll
        for (int b = 0; b < B; ++b) {
            pos[0] = pos[0] + sx, pos[1] = pos[1] + sy, pos[2] = pos[2] + sz;
            q[b][0] = pos[0], q[b][1] = pos[1], q[b][2] = pos[2];
        }
        Taps2 R[B], D[B];
#pragma unroll
        for (int b = 0; b < B; ++b) {
            taps_load2(q[b][0], q[b][1], q[b][2], rr, dim, R[b]);
            taps_load2(q[b][0], q[b][1], q[b][2], rd, dim, D[b]);
        }
#pragma unroll
        for (int b = 0; b < B; ++b) {
            if (!done) {
                if (!(color < 255 && i < c.max_steps)) {
                    done = true;
                } else {
                    ++i;
                    if (!in_box(q[b][0], q[b][1], q[b][2], hi)) {
                        done = true;
                    } else {
                        const int r = (int)taps2_value(R[b]);
                        const float v = taps2_value(D[b]);
                        if constexpr (F64COLOR)
                            color = (float)((double)color + (double)v * (0.01 + r));
                        else
                            color += v * (0.01f + r);
                    }
                }
            }
        }
    }
    image[py * image_dim + px] = (unsigned char)(color > 255 ? 255.f : color);
}

// DR16 layout: data and region interleaved per voxel (u16 = data | region << 8, dr16_pack_kernel), so ONE 8-byte load
// at the 4-byte-aligned address below voxel x of a row holds voxels x and x + 1 of BOTH volumes: 4 load instructions
// per sample. The same bytes, so the same arithmetic and bit-identical images.
__global__ __launch_bounds__(256) void dr16_pack_kernel(const unsigned char* __restrict__ data,
                                                        const unsigned char* __restrict__ region,
                                                        unsigned* __restrict__ out, long long n4) {
    // 4 voxels per thread: one u32 of each volume in, two u32 of interleaved pairs out
    const long long stride = (long long)gridDim.x * 256;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
        const unsigned d = __builtin_nontemporal_load(reinterpret_cast<const unsigned*>(data) + i);
        const unsigned r = __builtin_nontemporal_load(reinterpret_cast<const unsigned*>(region) + i);
        const unsigned lo = (d & 0xffu) | ((r & 0xffu) << 8) | ((d & 0xff00u) << 8) | ((r & 0xff00u) << 16);
        const unsigned hi = ((d >> 16) & 0xffu) | (((r >> 16) & 0xffu) << 8) | ((d >> 24) << 16) | ((r >> 24) << 24);
        reinterpret_cast<uint2*>(out)[i] = make_uint2(lo, hi);
    }
}

__device__ __forceinline__ void taps_load_dr(float px, float py, float pz, __amdgpu_buffer_rsrc_t rs, int dim,
                                             Taps2& R, Taps2& D) {
    D.ok = px >= 0 && px < dim - 1 && py >= 0 && py < dim - 1 && pz >= 0 && pz < dim - 1;
    R.ok = D.ok;
    if (!D.ok) return;
    const int x = (int)floorf(px), y = (int)floorf(py), z = (int)floorf(pz);
    const int xu = (int)ceilf(px), yu = (int)ceilf(py), zu = (int)ceilf(pz);
    D.rx = R.rx = px - x, D.ry = R.ry = py - y, D.rz = R.rz = pz - z;
    const unsigned P = (unsigned)dim * (unsigned)dim;
    const unsigned rows[4] = {(unsigned)z * P + (unsigned)y * dim, (unsigned)z * P + (unsigned)yu * dim,
                              (unsigned)zu * P + (unsigned)y * dim, (unsigned)zu * P + (unsigned)yu * dim};
    // byte offset of voxel x = 2x; the 4-aligned 8-byte window below it holds voxels x and x + 1
    const unsigned sh = (unsigned)(x & 1) * 16u, dx = (unsigned)(xu - x) * 16u;
    unsigned long long w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        w[k] = __builtin_bit_cast(unsigned long long,
                                  __builtin_amdgcn_raw_buffer_load_b64(rs, 2u * (rows[k] + (unsigned)(x & ~1)), 0, 0));
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const unsigned a = (unsigned)(w[k] >> sh), b = (unsigned)(w[k] >> (sh + dx));
        D.t[2 * k] = (unsigned char)a, R.t[2 * k] = (unsigned char)(a >> 8);
        D.t[2 * k + 1] = (unsigned char)b, R.t[2 * k + 1] = (unsigned char)(b >> 8);
    }
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t dr16_rsrc(const unsigned short* d, int dim) {
    const long long bytes = 2LL * dim * dim * dim;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned short*>(d), (short)0,
                                             (int)(bytes < 0x7fffffffLL ? bytes : 0x7fffffffLL), 0x00020000);
}

// The batch caster on the DR16 layout (variant 9): per-lane rays, B steps' samples in flight.
template <bool F64COLOR, int B>
__global__ __launch_bounds__(64) void raycast_dr_batch_kernel(const unsigned short* __restrict__ dr, int dim,
                                                              unsigned char* __restrict__ image, int image_dim, Cam c) {
    const int px = blockIdx.x * 8 + (threadIdx.x & 7);
    const int py = blockIdx.y * 8 + (threadIdx.x >> 3);
    if (px >= image_dim || py >= image_dim) return;
    const auto rs = dr16_rsrc(dr, dim);
    float pos[3], sx, sy, sz;
    ray_setup(c, px, py, image_dim, pos, sx, sy, sz);
    const float hi = (float)(dim - 1);
    int i = 0;
    float color = 0.f;
    while (i < c.max_steps) {
        const float nx = pos[0] + sx, ny = pos[1] + sy, nz = pos[2] + sz;
        if (in_box(nx, ny, nz, hi)) break;
        ++i;
        pos[0] = nx, pos[1] = ny, pos[2] = nz;
    }
    bool done = i >= c.max_steps;
    while (!done) {
        float q[B][3];
#pragma unroll
        for (int b = 0; b < B; ++b) {
            pos[0] = pos[0] + sx, pos[1] = pos[1] + sy, pos[2] = pos[2] + sz;
            q[b][0] = pos[0], q[b][1] = pos[1], q[b][2] = pos[2];
        }
        Taps2 R[B], D[B];
#pragma unroll
        for (int b = 0; b < B; ++b) taps_load_dr(q[b][0], q[b][1], q[b][2], rs, dim, R[b], D[b]);
#pragma unroll
        for (int b = 0; b < B; ++b) {
            if (!done) {
                if (!(color < 255 && i < c.max_steps)) {
                    done = true;
                } else {
                    ++i;
                    if (!in_box(q[b][0], q[b][1], q[b][2], hi)) {
                        done = true;
                    } else {
                        const int r = (int)taps2_value(R[b]);
                        const float v = taps2_value(D[b]);
                        if constexpr (F64COLOR)
                            color = (float)((double)color + (double)v * (0.01 + r));
                        else
                            color += v * (0.01f + r);
                    }
                }
            }
        }
    }
    image[py * image_dim + px] = (unsigned char)(color > 255 ? 255.f : color);
}

// GROUP-PER-RAY caster (variants 5-7): G consecutive lanes march ONE ray, G steps at a time. Every lane of the group
// replays the ray's f32 position adds (the same sequence as the serial caster, so positions stay bit-exact) and keeps
// the position of ITS step: lane j of the group samples steps k + j + 1 of each round of G. Each lane computes its
// step's term (v * (0.01 + r), in f32 or f64 as the colour mode wants) in parallel; the terms go through LDS and every
// lane of the group adds them to the colour in step order, so the colour's roundings are exactly the serial
// caster's. The loop stops after a round in which the colour reached 255 (later terms are >= 0, and the output clamps
// to 255 either way) or the ray left the volume's box (later samples read 0; adding 0 leaves the colour unchanged).
// A small image then fills the chip: 64^2 rays at G = 64 are 4096 waves instead of 64.
template <bool F64COLOR, int G, bool DR>
__global__ __launch_bounds__(256) void raycast_ref_group_kernel(const unsigned char* __restrict__ data,
                                                                const unsigned char* __restrict__ region,
                                                                const unsigned short* __restrict__ dr, int dim,
                                                                unsigned char* __restrict__ image, int image_dim, Cam c) {
    using Term = typename std::conditional<F64COLOR, double, float>::type;
    __shared__ Term s_term[256];
    const int lane = threadIdx.x & 63, sub = lane & (G - 1);
    const int ray = (int)((blockIdx.x * 256u + threadIdx.x) / G);
    const int n_rays = image_dim * image_dim;
    bool done = ray >= n_rays;  // group-uniform, as everything below that decides control flow
    const int px = done ? 0 : ray % image_dim, py = done ? 0 : ray / image_dim;
    const auto rd = volume_rsrc(data, dim), rr = volume_rsrc(region, dim);
    const auto rs = dr16_rsrc(dr, dim);
    float pos[3], sx, sy, sz;
    ray_setup(c, px, py, image_dim, pos, sx, sy, sz);
    const float hi = (float)(dim - 1);
    int i = 0;
    if (!done) {
        while (i < c.max_steps) {  // outside the box a sample adds exactly 0: adds only up to the first sample inside
            const float nx = pos[0] + sx, ny = pos[1] + sy, nz = pos[2] + sz;
            if (in_box(nx, ny, nz, hi)) break;
            ++i;
            pos[0] = nx, pos[1] = ny, pos[2] = nz;
        }
        done = i >= c.max_steps;
    }
    float color = 0.f;
    const int g0 = threadIdx.x & ~(G - 1);  // the group's first slot in s_term
    const unsigned long long gmask = (G == 64 ? ~0ull : ((1ull << G) - 1ull)) << (lane & ~(G - 1));
    while (__ballot(!done) != 0ull) {
        if (!done) {
            float q0 = 0.f, q1 = 0.f, q2 = 0.f;
#pragma unroll 8
            for (int b = 0; b < G; ++b) {
                pos[0] = pos[0] + sx, pos[1] = pos[1] + sy, pos[2] = pos[2] + sz;
                if (sub == b) q0 = pos[0], q1 = pos[1], q2 = pos[2];
            }
            const bool valid = i + sub + 1 <= c.max_steps;
            Taps2 R, D;
            if (valid) {
                if constexpr (DR) {
                    taps_load_dr(q0, q1, q2, rs, dim, R, D);
                } else {
                    taps_load2(q0, q1, q2, rr, dim, R);
                    taps_load2(q0, q1, q2, rd, dim, D);
                }
            }
            Term t = 0;
            if (valid && D.ok) {
                const int r = (int)taps2_value(R);
                const float v = taps2_value(D);
                if constexpr (F64COLOR)
                    t = (double)v * (0.01 + r);
                else
                    t = v * (0.01f + r);
            }
            s_term[threadIdx.x] = t;
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll 8
            for (int b = 0; b < G; ++b) {
                if constexpr (F64COLOR)
                    color = (float)((double)color + s_term[g0 + b]);
                else
                    color = color + s_term[g0 + b];
            }
            __builtin_amdgcn_wave_barrier();  // the slots are rewritten next round
            const bool left = valid && !in_box(q0, q1, q2, hi);
            i += G;
            done = color >= 255 || i >= c.max_steps || (__ballot(left) & gmask) != 0ull;
        }
    }
    if (ray < n_rays && sub == 0) image[py * image_dim + px] = (unsigned char)(color > 255 ? 255.f : color);
}

// value_at_ref on a z-slab buffer whose plane 0 is global plane zoff (identical arithmetic)
__device__ __forceinline__ float value_at_slab(float px, float py, float pz, const unsigned char* __restrict__ d, int dim,
                                              int zoff) {
    if (!(px >= 0 && px < dim - 1 && py >= 0 && py < dim - 1 && pz >= 0 && pz < dim - 1)) return 0.f;
    const int x = (int)floorf(px), y = (int)floorf(py), z = (int)floorf(pz);
    const int xu = (int)ceilf(px), yu = (int)ceilf(py), zu = (int)ceilf(pz);
    const float rx = px - x, ry = py - y, rz = pz - z;
    const size_t P = (size_t)dim * dim;
    const unsigned char* zy = d + (size_t)(z - zoff) * P + (size_t)y * dim;
    const unsigned char* zyu = d + (size_t)(z - zoff) * P + (size_t)yu * dim;
    const unsigned char* zuy = d + (size_t)(zu - zoff) * P + (size_t)y * dim;
    const unsigned char* zuyu = d + (size_t)(zu - zoff) * P + (size_t)yu * dim;
    const float a0 = rx * zy[x] + (1 - rx) * zy[xu];
    const float a1 = rx * zyu[x] + (1 - rx) * zyu[xu];
    const float a2 = rx * zuy[x] + (1 - rx) * zuy[xu];
    const float a3 = rx * zuyu[x] + (1 - rx) * zuyu[xu];
    const float b0 = ry * a0 + (1 - ry) * a1;
    const float b1 = ry * a2 + (1 - ry) * a3;
    return rz * b0 + (1 - rz) * b1;
}

// z-slab stage of the distributed reference caster (parallel/volume3d.py): the march of raycast_ref_kernel<true>
// restricted to samples with z >= z0 (every sample on the bottom slab). Rays run towards -z for the reference
// camera, so the slabs are visited top to bottom; per pixel the state {pos xyz, colour, steps, flags (1 =
// entered the box, 2 = done)} travels from slab to slab. A slab hands a ray over BEFORE taking a step whose
// position lies below z0, so the next slab recomputes the very same position: the image is bit-identical to
// the single-volume caster. data/region start at global plane z0 - 1 (halo below) and hold plane z1 (halo above).
__global__ __launch_bounds__(256) void raycast_slab_kernel(const unsigned char* __restrict__ data,
                                                          const unsigned char* __restrict__ region, int dim, int z0,
                                                          int* __restrict__ state, int init, int bottom,
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
    const float l = (float)sqrt((double)(ray[0] * ray[0] + ray[1] * ray[1] + ray[2] * ray[2]));
    ray[0] /= l, ray[1] /= l, ray[2] /= l;
    const float sx = ray[0] * c.step, sy = ray[1] * c.step, sz = ray[2] * c.step;
    const float hi = (float)(dim - 1);
    int* st = state + 6 * ((size_t)py * image_dim + px);
    int i = 0, flags = 0;
    float color = 0.f;
    if (!init) {
        pos[0] = __int_as_float(st[0]), pos[1] = __int_as_float(st[1]), pos[2] = __int_as_float(st[2]);
        color = __int_as_float(st[3]), i = st[4], flags = st[5];
    }
    const int zoff = z0 - 1;
    while (!(flags & 2) && color < 255 && i < c.max_steps) {
        const float nx = pos[0] + sx, ny = pos[1] + sy, nz = pos[2] + sz;
        if (!bottom && nz < (float)z0) break;  // the next sample belongs to a lower slab
        ++i;
        pos[0] = nx, pos[1] = ny, pos[2] = nz;
        if (!in_box(pos[0], pos[1], pos[2], hi)) {
            if (flags & 1) flags |= 2;  // left the convex volume: every later sample is 0
            continue;
        }
        flags |= 1;
        const int r = (int)value_at_slab(pos[0], pos[1], pos[2], region, dim, zoff);
        const float v = value_at_slab(pos[0], pos[1], pos[2], data, dim, zoff);
        color = (float)((double)color + (double)v * (0.01 + r));
    }
    st[0] = __float_as_int(pos[0]), st[1] = __float_as_int(pos[1]), st[2] = __float_as_int(pos[2]);
    st[3] = __float_as_int(color), st[4] = i, st[5] = flags;
    if (bottom) image[py * image_dim + px] = (unsigned char)(color > 255 ? 255.f : color);
}
#pragma clang fp contract(on)

// ---------------------------------------------------------------------------------- texture path
// Texel formats (chosen on the device, no host round trip: brick_pack first scans the data for a byte >= 128
// and records the answer in a flag stored behind the texels, which every later kernel reads):
//  * narrow (every data value < 128, e.g. the reference volume, values <= 50): 8 bytes per voxel holding the
//    whole 2x2x2 trilinear footprint, region folded into bit 7 of each data byte:
//      .x = [d|r<<7] at (x,y,z) (x+1,y,z) (x,y+1,z) (x+1,y+1,z)      .y = the same at plane z+1
//  * wide (any value >= 128): 16 bytes per voxel, .x/.y = data at planes z/z+1, .z/.w = region (0/1).
// Neighbours are clamped to the volume edge. One sample of both volumes is ONE load per lane: the march is
// bound by the L2 lane-request rate (~2.6e8 samples per 512^2 image), and the pack by its texel writes.
__global__ __launch_bounds__(256) void data_hibit_kernel(const unsigned char* __restrict__ data, size_t n,
                                                        int* __restrict__ flag) {
    size_t i = ((size_t)blockIdx.x * 256 + threadIdx.x) * 16;
    int hit = 0;
    for (; i < n; i += (size_t)gridDim.x * 256 * 16) {
        if (i + 16 <= n && ((reinterpret_cast<size_t>(data) + i) % 16) == 0) {
            const uint4 v = *reinterpret_cast<const uint4*>(data + i);
            hit |= ((v.x | v.y | v.z | v.w) & 0x80808080u) != 0;
        } else {
            for (size_t j = i; j < n && j < i + 16; ++j) hit |= data[j] >= 128;
        }
    }
    if (__syncthreads_or(hit) && threadIdx.x == 0) atomicOr(flag, 1);
}

__device__ __forceinline__ unsigned rbit(unsigned char v) { return v != 0; }

__global__ __launch_bounds__(256) void brick_pack_kernel(const unsigned char* __restrict__ data,
                                                        const unsigned char* __restrict__ region, int dim,
                                                        void* __restrict__ tex, const int* __restrict__ wide_flag) {
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y, z = blockIdx.z;
    if (x >= dim) return;
    const bool wide = *wide_flag != 0;
    const int x1 = min(x + 1, dim - 1), y1 = min(y + 1, dim - 1), z1 = min(z + 1, dim - 1);
    const size_t P = (size_t)dim * dim, v = (size_t)z * P + (size_t)y * dim + x;
    unsigned w[4];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const size_t zz = (size_t)(q ? z1 : z) * P;
        const size_t r0 = zz + (size_t)y * dim, r1 = zz + (size_t)y1 * dim;
        const unsigned d = (unsigned)data[r0 + x] | ((unsigned)data[r0 + x1] << 8) | ((unsigned)data[r1 + x] << 16) |
                           ((unsigned)data[r1 + x1] << 24);
        const unsigned r = rbit(region[r0 + x]) | (rbit(region[r0 + x1]) << 8) | (rbit(region[r1 + x]) << 16) |
                           (rbit(region[r1 + x1]) << 24);
        w[q] = wide ? d : (d | (r << 7));
        w[2 + q] = r;
    }
    if (wide)
        reinterpret_cast<uint4*>(tex)[v] = make_uint4(w[0], w[1], w[2], w[3]);
    else
        reinterpret_cast<uint2*>(tex)[v] = make_uint2(w[0], w[1]);
}

// 4 voxels per thread (dim % 4 == 0): each of the 8 source rows is read as one aligned u32 (+ the next byte);
// the 4 texels go through LDS so the stores leave fully coalesced (consecutive lanes, consecutive texels).
// (4 rows per thread, re-using the shared source rows, measured slower: 64 KB of LDS halves occupancy. Taking
// the next byte from the neighbour lane (DPP shift) with a guarded load for lane 63 measured 700 vs 510 us at
// 512^3: the 8 divergent guarded loads serialise their waits.)
__device__ __forceinline__ unsigned row5(const unsigned char* __restrict__ p, int x, int dim, unsigned& next) {
    next = p[min(x + 4, dim - 1)];
    return *reinterpret_cast<const unsigned*>(p + x);
}

__device__ __forceinline__ unsigned pair(unsigned a, unsigned an, unsigned b, unsigned bn, int i) {
    // bytes (x+i, x+i+1) of row a then of row b
    const unsigned a0 = (a >> (8 * i)) & 0xff, a1 = i < 3 ? (a >> (8 * i + 8)) & 0xff : an;
    const unsigned b0 = (b >> (8 * i)) & 0xff, b1 = i < 3 ? (b >> (8 * i + 8)) & 0xff : bn;
    return a0 | (a1 << 8) | (b0 << 16) | (b1 << 24);
}

// LDS slot of texel j of the block's 1024: slot = j ^ ((j >> 3) & 3). The write (ds_write_b128: 8-lane groups,
// bank = (a/4) mod 32, i.e. 8 16-B slots) has lane t at texel 4t+i: the XOR makes the 8 lanes of a group hit 8
// distinct slots mod 8 (the unswizzled 4t+i, or the former +j/16 pad, is 2-way: 5.0e7 conflict cycles per pack at
// 512^3). The read-back (texel j by lane j, ds_read_b128 groups of 16 lanes made of aligned 4-lane blocks) only
// permutes slots inside aligned groups of 4, so its groups still cover 16 distinct slots mod 16.
__device__ __forceinline__ int tex_slot(int j) { return j ^ ((j >> 3) & 3); }
// the same for 8 texels per lane (lane t writes 8t+i): XOR with t mod 8 spreads an 8-lane write group over 8
// distinct 16-B slots (t mod 4 left 2-way conflicts: 2.1e7 per 512^3 pack, r2_pmc/raycast.md); the read-back
// still only permutes slots inside aligned groups of 8
__device__ __forceinline__ int tex_slot8(int j) { return j ^ ((j >> 3) & 7); }
// narrow texel pairs: slot of pair p (texels 2p, 2p+1) of the block's 512 — lane t writes pairs 4t..4t+3
// (ds_write_b128, conflict-free: the rotation by p >> 3 spreads an 8-lane group over 8 distinct slots mod 8) and
// lane j reads pair j back (ds_read_b128; only permutes inside aligned groups of 4)
__device__ __forceinline__ int pair_slot(int p) { return 4 * (p >> 2) + (((p & 3) + (p >> 3)) & 3); }
// The 1 GiB of texels is written once and read back only by the later march (more than the 256-MiB Infinity
// Cache holds): nontemporal 16-B stores took the 512^3 pack from ~300 to ~206 us (profiles/r3_raycast/pack_nt.txt;
// the same loads with ordinary 16-B stores: 300 us, so the write-allocate path, not the stores' count, was the cost)
using u32x4_t = unsigned __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store_nt16(uint4 t, uint4* p) {
    __builtin_nontemporal_store(u32x4_t{t.x, t.y, t.z, t.w}, reinterpret_cast<u32x4_t*>(p));
}

// A block covers 1024 consecutive texels of one z-plane in row-major (y, x) order (rows of several y when
// dim < 1024; dim % 4 == 0 keeps a thread's 4 texels in one row), so every thread is busy (one block per row
// left half of each 256-thread block clamped onto duplicate loads at dim 512: 466 -> 392 us). A persistent,
// software-pipelined variant (next unit's loads in flight, double-buffered 32-KiB stage, 4 blocks/CU) measured
// 451 us: occupancy matters more here than the pipelining.
__global__ __launch_bounds__(256) void brick_pack4_kernel(const unsigned char* __restrict__ data,
                                                         const unsigned char* __restrict__ region, int dim,
                                                         void* __restrict__ tex, const int* __restrict__ wide_flag) {
    const size_t plane_texels = (size_t)dim * dim;
    const size_t lin0 = (size_t)blockIdx.x * 1024;  // first texel of this block inside its plane
    const size_t lin = min(lin0 + (size_t)threadIdx.x * 4, plane_texels - 4);
    const int y = (int)(lin / dim), x = (int)(lin % dim), z = blockIdx.y;
    const bool wide = *wide_flag != 0;
    const int y1 = min(y + 1, dim - 1), z1 = min(z + 1, dim - 1);
    const size_t P = (size_t)dim * dim;
    const size_t rows[4] = {(size_t)z * P + (size_t)y * dim, (size_t)z * P + (size_t)y1 * dim,
                            (size_t)z1 * P + (size_t)y * dim, (size_t)z1 * P + (size_t)y1 * dim};
    unsigned d[4], dn[4], r[4], rn[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        d[q] = row5(data + rows[q], x, dim, dn[q]);
        r[q] = row5(region + rows[q], x, dim, rn[q]);
        // region bytes -> 0/1
        r[q] = ((r[q] & 0x000000ff) ? 1u : 0u) | ((r[q] & 0x0000ff00) ? 0x100u : 0u) | ((r[q] & 0x00ff0000) ? 0x10000u : 0u) |
               ((r[q] & 0xff000000) ? 0x1000000u : 0u);
        rn[q] = rn[q] ? 1u : 0u;
    }
    __shared__ uint4 stage[1024];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const unsigned r0 = pair(r[0], rn[0], r[1], rn[1], i), r1 = pair(r[2], rn[2], r[3], rn[3], i);
        const unsigned d0 = pair(d[0], dn[0], d[1], dn[1], i), d1 = pair(d[2], dn[2], d[3], dn[3], i);
        stage[tex_slot(threadIdx.x * 4 + i)] =
            wide ? make_uint4(d0, d1, r0, r1) : make_uint4(d0 | (r0 << 7), d1 | (r1 << 7), 0u, 0u);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int j = i * 256 + threadIdx.x;
        if (lin0 + j >= plane_texels) continue;
        const uint4 t = stage[tex_slot(j)];
        const size_t o = (size_t)z * plane_texels + lin0 + j;
        if (wide)
            reinterpret_cast<uint4*>(tex)[o] = t;
        else
            reinterpret_cast<uint2*>(tex)[o] = make_uint2(t.x, t.y);
    }
}

// 8 texels per thread (dim % 8 == 0): one aligned 8-B load per source row; the byte after it (x + 8) is the
// low byte of the next lane's load (DPP lane shift), and one byte load per row (issued by every lane with the
// others, used by lane 63 only) covers the wave's last lane — 16 loads per 8 texels instead of 32. 128 threads
// x 8 texels = the same 1024-texel unit and 16-KiB stage as brick_pack4_kernel.
__device__ __forceinline__ unsigned pair8(unsigned long long a, unsigned an, unsigned long long b, unsigned bn, int i) {
    const unsigned a0 = (unsigned)(a >> (8 * i)) & 0xff, a1 = i < 7 ? (unsigned)(a >> (8 * i + 8)) & 0xff : an;
    const unsigned b0 = (unsigned)(b >> (8 * i)) & 0xff, b1 = i < 7 ? (unsigned)(b >> (8 * i + 8)) & 0xff : bn;
    return a0 | (a1 << 8) | (b0 << 16) | (b1 << 24);
}

__device__ __forceinline__ unsigned long long nz_bytes64(unsigned long long w) {  // each byte -> 0/1
    const unsigned long long t = (((w & 0x7f7f7f7f7f7f7f7full) + 0x7f7f7f7f7f7f7f7full) | w) & 0x8080808080808080ull;
    return t >> 7;
}

template <int ZP>
__global__ __launch_bounds__(128) void brick_pack8_kernel(const unsigned char* __restrict__ data,
                                                         const unsigned char* __restrict__ region, int dim,
                                                         void* __restrict__ tex, const int* __restrict__ wide_flag) {
    // ZP consecutive output planes per block: their ZP + 1 source planes are loaded once, all up front (ZP times
    // the loads in flight of one plane per block, (ZP+1)/(2 ZP) of the row loads). The pack is latency-bound, not
    // VALU- or bandwidth-bound: 1 GiB of texels took ~370 us with ZP = 1 against a 155-us 1-GiB fill (counters:
    // 130 MB fetched); a byte-transpose (v_perm) assembly and an XCD-contiguous unit order changed nothing.
    // Measured at 512^3: ZP 1 / 2 / 4 / 8 = 367 / 301 / 285 / 283 us (LDS-free direct stores: 537 us); with
    // nontemporal 16-B stores ZP 2 / 4 / 8 = 207 / 206 / 209 us (round 3).
    const int lane = pcmx::lane_id();
    const size_t P = (size_t)dim * dim;
    const size_t lin0 = (size_t)blockIdx.x * 1024;
    const size_t lin = min(lin0 + (size_t)threadIdx.x * 8, P - 8);
    const int y = (int)(lin / dim), x = (int)(lin % dim), zb = blockIdx.y * ZP;
    const bool wide = *wide_flag != 0;
    const int y1 = min(y + 1, dim - 1), xn = min(x + 8, dim - 1);
    unsigned long long d[ZP + 1][2], r[ZP + 1][2];
    unsigned dl[ZP + 1][2], rl[ZP + 1][2];
#pragma unroll
    for (int j = 0; j <= ZP; ++j) {
        const size_t pl = (size_t)min(zb + j, dim - 1) * P;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const size_t row = pl + (size_t)(e ? y1 : y) * dim;
            d[j][e] = *reinterpret_cast<const unsigned long long*>(data + row + x);
            r[j][e] = *reinterpret_cast<const unsigned long long*>(region + row + x);
            dl[j][e] = data[row + xn];
            rl[j][e] = region[row + xn];
        }
    }
    unsigned dn[ZP + 1][2], rn[ZP + 1][2];
    const bool own_next = lane == 63 || x + 8 >= dim;  // the next lane's word is not this row's x + 8
#pragma unroll
    for (int j = 0; j <= ZP; ++j)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const unsigned dnb = (unsigned)__float_as_int(pcmx::wave_from_next(__int_as_float((int)(unsigned)d[j][e]))) & 0xffu;
            const unsigned rnb = (unsigned)__float_as_int(pcmx::wave_from_next(__int_as_float((int)(unsigned)r[j][e]))) & 0xffu;
            dn[j][e] = own_next ? dl[j][e] : dnb;
            rn[j][e] = (own_next ? rl[j][e] : rnb) ? 1u : 0u;
            r[j][e] = nz_bytes64(r[j][e]);
        }
    __shared__ uint4 stage[1024];
#pragma unroll
    for (int k = 0; k < ZP; ++k) {
        const int z = zb + k;
        if (z >= dim) break;  // block-uniform
        if (k) __syncthreads();  // the previous plane's stage has been read back
        unsigned w[8][4];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const unsigned r0 = pair8(r[k][0], rn[k][0], r[k][1], rn[k][1], i);
            const unsigned r1 = pair8(r[k + 1][0], rn[k + 1][0], r[k + 1][1], rn[k + 1][1], i);
            const unsigned d0 = pair8(d[k][0], dn[k][0], d[k][1], dn[k][1], i);
            const unsigned d1 = pair8(d[k + 1][0], dn[k + 1][0], d[k + 1][1], dn[k + 1][1], i);
            w[i][0] = wide ? d0 : d0 | (r0 << 7);
            w[i][1] = wide ? d1 : d1 | (r1 << 7);
            w[i][2] = r0, w[i][3] = r1;
        }
        if (wide) {
#pragma unroll
            for (int i = 0; i < 8; ++i) stage[tex_slot8(threadIdx.x * 8 + i)] = make_uint4(w[i][0], w[i][1], w[i][2], w[i][3]);
            __syncthreads();
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int j = i * 128 + threadIdx.x;
                if (lin0 + j >= P) continue;
                const uint4 t = stage[tex_slot8(j)];
                store_nt16(t, reinterpret_cast<uint4*>(tex) + (size_t)z * P + lin0 + j);
            }
        } else {  // narrow: texel PAIRS (2 x 8 B) per 16-B slot and store
#pragma unroll
            for (int m = 0; m < 4; ++m)
                stage[pair_slot(threadIdx.x * 4 + m)] = make_uint4(w[2 * m][0], w[2 * m][1], w[2 * m + 1][0], w[2 * m + 1][1]);
            __syncthreads();
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int j = i * 128 + threadIdx.x;  // pair j = texels lin0 + 2j, lin0 + 2j + 1 (P is even)
                if (lin0 + 2 * j >= P) continue;
                store_nt16(stage[pair_slot(j)], reinterpret_cast<uint4*>(tex) + ((size_t)z * P + lin0) / 2 + j);
            }
        }
    }
}

// Production pack for 16 <= dim <= 1024, dim % 8 == 0 (round 3). Differences to brick_pack8_kernel:
//  * one 12-B buffer load per source row (bytes x .. x+11: the 8 texel bytes AND the next byte, no byte loads,
//    no lane shift; lanes at a row's right edge load x-4 .. x+7 and clamp the next byte onto x+7);
//  * ZP = 8 planes per block, all 9 source planes' rows loaded up front (152 VGPRs, 3 waves per SIMD): the loads
//    run from cold HBM after the previous frame's march, and the deeper block re-reads 1/8 instead of 1/2 of the
//    planes: cold pack ZP 2 / 4 / 8 / 16 = 245-261 / 232-245 / 225-237 / 271-282 us; a rolling register ring
//    (planes loaded 1-3 ahead, ZP 8-32) 239-400 us (profiles/r3_raycast/pack_cold_zp.txt);
//  * nontemporal 16-B stores of texel pairs;
//  * no format pre-pass: the narrow kernel ORs the data bytes it loads anyway and raises the wide flag itself; a
//    small wide kernel launched behind it returns at once unless the flag is set, and then rewrites every texel
//    in the 16-B format (the data_hibit_kernel scan of the whole volume, 25 us per frame, is gone).
using u32x3_t = unsigned __attribute__((ext_vector_type(3)));
template <int ZP, bool kWide>
__device__ __forceinline__ bool pack12_unit(const unsigned char* __restrict__ data,
                                            const unsigned char* __restrict__ region, int dim, void* __restrict__ tex,
                                            unsigned unit, int zb, uint4* stage) {
    const unsigned P = (unsigned)dim * (unsigned)dim;
    const unsigned lin0 = unit * 1024u;
    const unsigned lin = min(lin0 + threadIdx.x * 8u, P - 8u);
    const int y = (int)(lin / (unsigned)dim), x = (int)(lin % (unsigned)dim);
    const int y1 = min(y + 1, dim - 1);
    const bool edge = x + 8 >= dim;
    const unsigned nbytes = P * (unsigned)dim;
    const auto rd = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(data), (short)0, (int)nbytes, 0x00020000);
    const auto rr = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(region), (short)0, (int)nbytes, 0x00020000);
    u32x3_t dw[ZP + 1][2], rw[ZP + 1][2];
#pragma unroll
    for (int j = 0; j <= ZP; ++j) {
        const unsigned pl = (unsigned)min(zb + j, dim - 1) * P;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const unsigned o = pl + (unsigned)(e ? y1 : y) * (unsigned)dim + (unsigned)x - (edge ? 4u : 0u);
            dw[j][e] = __builtin_amdgcn_raw_buffer_load_b96(rd, o, 0, 0);
            rw[j][e] = __builtin_amdgcn_raw_buffer_load_b96(rr, o, 0, 0);
        }
    }
    unsigned long long d[ZP + 1][2], r[ZP + 1][2], hi = 0;
    unsigned dn[ZP + 1][2], rn[ZP + 1][2];
#pragma unroll
    for (int j = 0; j <= ZP; ++j)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const u32x3_t a = dw[j][e], b = rw[j][e];
            d[j][e] = edge ? ((unsigned long long)a.z << 32 | a.y) : ((unsigned long long)a.y << 32 | a.x);
            hi |= d[j][e];
            const unsigned long long rb = edge ? ((unsigned long long)b.z << 32 | b.y) : ((unsigned long long)b.y << 32 | b.x);
            dn[j][e] = edge ? (a.z >> 24) : (a.z & 0xffu);
            rn[j][e] = (edge ? (b.z >> 24) : (b.z & 0xffu)) ? 1u : 0u;
            r[j][e] = nz_bytes64(rb);
        }
#pragma unroll
    for (int k = 0; k < ZP; ++k) {
        const int z = zb + k;
        if (z >= dim) break;  // block-uniform
        __syncthreads();      // the previous plane's (or unit's) stage has been read back
        unsigned w[8][4];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const unsigned r0 = pair8(r[k][0], rn[k][0], r[k][1], rn[k][1], i);
            const unsigned r1 = pair8(r[k + 1][0], rn[k + 1][0], r[k + 1][1], rn[k + 1][1], i);
            const unsigned d0 = pair8(d[k][0], dn[k][0], d[k][1], dn[k][1], i);
            const unsigned d1 = pair8(d[k + 1][0], dn[k + 1][0], d[k + 1][1], dn[k + 1][1], i);
            w[i][0] = kWide ? d0 : d0 | (r0 << 7);
            w[i][1] = kWide ? d1 : d1 | (r1 << 7);
            w[i][2] = r0, w[i][3] = r1;
        }
        if constexpr (kWide) {
#pragma unroll
            for (int i = 0; i < 8; ++i) stage[tex_slot8(threadIdx.x * 8 + i)] = make_uint4(w[i][0], w[i][1], w[i][2], w[i][3]);
            __syncthreads();
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const unsigned j = i * 128u + threadIdx.x;
                if (lin0 + j >= P) continue;
                store_nt16(stage[tex_slot8(j)], reinterpret_cast<uint4*>(tex) + (size_t)z * P + lin0 + j);
            }
        } else {
#pragma unroll
            for (int m = 0; m < 4; ++m)
                stage[pair_slot(threadIdx.x * 4 + m)] = make_uint4(w[2 * m][0], w[2 * m][1], w[2 * m + 1][0], w[2 * m + 1][1]);
            __syncthreads();
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const unsigned j = i * 128u + threadIdx.x;  // pair j = texels lin0 + 2j, lin0 + 2j + 1 (P is even)
                if (lin0 + 2 * j >= P) continue;
                store_nt16(stage[pair_slot(j)], reinterpret_cast<uint4*>(tex) + ((size_t)z * P + lin0) / 2 + j);
            }
        }
    }
    return (hi & 0x8080808080808080ull) != 0;
}

template <int ZP>
__global__ __launch_bounds__(128) void brick_pack12_narrow_kernel(const unsigned char* __restrict__ data,
                                                                  const unsigned char* __restrict__ region, int dim,
                                                                  void* __restrict__ tex, int* __restrict__ wide_flag) {
    __shared__ uint4 stage[512];
    const bool hi = pack12_unit<ZP, false>(data, region, dim, tex, blockIdx.x, (int)blockIdx.y * ZP, stage);
    if (__syncthreads_or(hi) && threadIdx.x == 0) atomicOr(wide_flag, 1);
}

// grid-stride over (unit, plane group); every block returns at once while the flag is clear (the common case)
template <int ZP>
__global__ __launch_bounds__(128) void brick_pack12_wide_kernel(const unsigned char* __restrict__ data,
                                                                const unsigned char* __restrict__ region, int dim,
                                                                void* __restrict__ tex, const int* __restrict__ wide_flag,
                                                                unsigned units, unsigned groups) {
    if (__hip_atomic_load(wide_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
    __shared__ uint4 stage[1024];
    for (unsigned t = blockIdx.x; t < units * groups; t += gridDim.x)
        pack12_unit<ZP, true>(data, region, dim, tex, t % units, (int)(t / units) * ZP, stage);
}

__device__ __forceinline__ float bilerp4(unsigned w, float ax, float ay) {
    const float v00 = (float)(w & 0xff), v10 = (float)((w >> 8) & 0xff);
    const float v01 = (float)((w >> 16) & 0xff), v11 = (float)(w >> 24);
    return (1.f - ay) * ((1.f - ax) * v00 + ax * v10) + ay * ((1.f - ax) * v01 + ax * v11);
}

// hardware-like fractional weight: 8 fractional bits
__device__ __forceinline__ float q8(float f) { return rintf(f * 256.f) * (1.f / 256.f); }

// Texture march. Profiled on MI355X: ~100k VALU per wave but 2.7 ms, and the time scaled with max_steps even
// below the ~1700 steps a ray needs to REACH the volume (1000 steps, no ray inside: 0.49 ms): the kernel was
// bound by marching empty space (and by the rays that miss the volume, which run all 5000 steps), a serial
// chain of adds, compares and branches at 4 waves per SIMD. Here each ray is clipped analytically against the
// sampled box [0, dim-1)^3 (slab test, one step of margin each side), only the steps inside are visited, and
// position k is computed directly as cam + k * step_vector (so steps are independent); D steps are prefetched
// per batch (2*D texel loads in flight) and consumed in order with the reference's termination tests (stop at
// colour >= 255, stop when the ray leaves the convex box). Positions differ from the reference's repeated
// f32 adds by rounding only (~1e-3 voxel), below the 8-bit weight quantum of the emulated texture filter.
// Ray of pixel (px, py): step vector and the analytic clip of its march against the sampled box [0, dim-1)^3,
// in units of steps with one step of margin each side. k0 > k1 = the ray misses the volume.
struct TexRay {
    float sv[3];
    int k0, k1;
};
__device__ __forceinline__ TexRay tex_ray(int px, int py, int image_dim, int dim, const Cam& c) {
    const int half = image_dim / 2;
    const int x = px - half, y = py - half;
    float ray[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float sc = c.cam[k] + c.fwd[k];
        ray[k] = (sc + c.right[k] * (x * c.pw)) + c.up[k] * (y * c.pw) - c.cam[k];
    }
    const float l = sqrtf(ray[0] * ray[0] + ray[1] * ray[1] + ray[2] * ray[2]);
    TexRay r;
#pragma unroll
    for (int k = 0; k < 3; ++k) r.sv[k] = ray[k] / l * c.step;
    const float hi = (float)(dim - 1);
    // slab clip in units of steps: inside <=> 0 <= cam + k*sv < hi on every axis
    float k_lo = 1.f, k_hi = (float)c.max_steps;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        if (r.sv[a] == 0.f) {
            if (!(c.cam[a] >= 0.f && c.cam[a] < hi)) k_hi = -1.f;
            continue;
        }
        const float t0 = (0.f - c.cam[a]) / r.sv[a], t1 = (hi - c.cam[a]) / r.sv[a];
        k_lo = fmaxf(k_lo, fminf(t0, t1));
        k_hi = fminf(k_hi, fmaxf(t0, t1));
    }
    if (k_lo <= k_hi) {
        r.k0 = max(1, (int)floorf(k_lo) - 1);
        r.k1 = min(c.max_steps, (int)ceilf(k_hi) + 1);
    } else {
        r.k0 = 1, r.k1 = 0;
    }
    return r;
}

// Colour accumulated over steps [k0, k1] of the ray (reference termination tests: stop at colour >= 255, stop
// when the ray leaves the convex box after entering it).
template <int D, bool WIDE>
__device__ __forceinline__ float tex_march(const void* __restrict__ texv, int dim, const Cam& c, const float (&sv)[3],
                                           int k0, int k1) {
    const size_t P = (size_t)dim * dim;
    const float hi = (float)(dim - 1);
    float color = 0.f;
    // texel-centre addressing (sample at p - 0.5), clamp-to-edge, 8-bit fractional weights
    auto tap = [&](int step, float& ax, float& ay, float& az, bool& inb, bool opaque) -> size_t {
        float kk = (float)step;
        if (opaque) asm volatile("" : "+v"(kk));  // recompute at use: keeps the compiler from holding the
                                                 // issue-time values live across the batch
        const float p0 = fmaf(kk, sv[0], c.cam[0]), p1 = fmaf(kk, sv[1], c.cam[1]), p2 = fmaf(kk, sv[2], c.cam[2]);
        inb = in_box(p0, p1, p2, hi);
        const float fx = p0 - 0.5f, fy = p1 - 0.5f, fz = p2 - 0.5f;
        int x0 = (int)floorf(fx), y0 = (int)floorf(fy), z0 = (int)floorf(fz);
        ax = q8(fx - x0), ay = q8(fy - y0), az = q8(fz - z0);
        if (x0 < 0) x0 = 0, ax = 0.f;
        if (y0 < 0) y0 = 0, ay = 0.f;
        if (z0 < 0) z0 = 0, az = 0.f;
        x0 = min(x0, dim - 1), y0 = min(y0, dim - 1), z0 = min(z0, dim - 1);
        return (size_t)z0 * P + ((unsigned)y0 * (unsigned)dim + (unsigned)x0);  // row part < 2^32 (dim <= 2048)
    };
    using Texel = typename std::conditional<WIDE, uint4, uint2>::type;
    bool entered = false, active = true;
    for (int i = k0; active && i <= k1 && color < 255.f; i += D) {
        // only the raw texels stay live across the batch (2 or 4 VGPRs per step in flight); the weights are
        // recomputed at use, so deep batches keep the occupancy
        Texel q[D];
#pragma unroll
        for (int k = 0; k < D; ++k) {
            float ax, ay, az;
            bool inb;
            q[k] = reinterpret_cast<const Texel*>(texv)[tap(i + k, ax, ay, az, inb, false)];  // always in bounds
        }
#pragma unroll
        for (int k = 0; k < D; ++k) {
            const bool live = active && i + k <= k1 && color < 255.f;
            active = live;
            if (!live) continue;
            float ax, ay, az;
            bool inb;
            (void)tap(i + k, ax, ay, az, inb, true);
            if (!inb) {  // texture fetches outside never add colour; a convex box is never re-entered
                if (entered) active = false;
                continue;
            }
            entered = true;
            uint4 t;  // data z, data z+1, region z, region z+1 (4 corners each)
            if constexpr (WIDE)
                t = q[k];
            else
                t = make_uint4(q[k].x & 0x7f7f7f7fu, q[k].y & 0x7f7f7f7fu, (q[k].x >> 7) & 0x01010101u,
                               (q[k].y >> 7) & 0x01010101u);
            const float d = (1.f - az) * bilerp4(t.x, ax, ay) + az * bilerp4(t.y, ax, ay);
            const float rr = (1.f - az) * bilerp4(t.z, ax, ay) + az * bilerp4(t.w, ax, ay);
            const int r = (int)rr;  // 255 * normalised region tap, region voxels hold 1
            color += d * (0.01f + r);
        }
    }
    return color;
}

template <int D, bool WIDE, int SEG>
__device__ __forceinline__ void raycast_tex_march(const void* __restrict__ texv, int dim,
                                                  unsigned char* __restrict__ image, int image_dim, const Cam& c,
                                                  float* s_part) {
    // SEG waves share one 16x4 ray patch, each marching 1/SEG of the clipped step range (see raycast_tex_kernel)
    constexpr int kRows = 16 / SEG;  // pixel rows per 4-wave block
    const int lane = pcmx::lane_id(), wave = threadIdx.x / pcmx::kWave, g = wave / SEG, seg = wave % SEG;
    const int px = blockIdx.x * 16 + (lane & 15);  // (8x8-pixel waves measured no faster)
    const int py = blockIdx.y * kRows + g * 4 + (lane >> 4);
    const bool valid = px < image_dim && py < image_dim;
    if (SEG == 1 && !valid) return;
    const TexRay r = tex_ray(px, py, image_dim, dim, c);
    float color = 0.f;
    if (valid && r.k0 <= r.k1) {
        int k0 = r.k0, k1 = r.k1;
        if (SEG > 1) {  // this wave's share of [k0, k1]; the in-box steps of a convex box are contiguous
            const int len = (k1 - k0 + SEG) / SEG;
            k0 += seg * len;
            k1 = min(k1, k0 + len - 1);
        }
        color = tex_march<D, WIDE>(texv, dim, c, r.sv, k0, k1);
    }
    if (SEG > 1) {  // segment partial colours compose in ray order; a saturated prefix ends the ray
        s_part[threadIdx.x] = color;
        __syncthreads();
        if (seg != 0 || !valid) return;
        color = 0.f;
#pragma unroll
        for (int q = 0; q < SEG; ++q)
            if (color < 255.f) color += s_part[(g * SEG + q) * pcmx::kWave + lane];
    }
    image[py * image_dim + px] = (unsigned char)(color > 255.f ? 255.f : color);
}

// 256-thread blocks of 4 waves. SEG = 1: each wave marches a 16x4 pixel patch (a block covers 16x16). SEG > 1:
// SEG waves take the SAME 16x4 patch and each marches a contiguous 1/SEG of every ray's clipped step range; the
// partial colours are summed in ray order through LDS (a ray whose earlier segments reach 255 is saturated, as
// the sequential march's stop at colour >= 255 gives after the final clamp). A 512^2 image is only 4096 waves,
// 4 per SIMD: splitting the rays gives the march SEG times the waves to hide its texel-load latency.
template <int D, int SEG>
__global__ __launch_bounds__(256) void raycast_tex_kernel(const void* __restrict__ tex, const int* __restrict__ wide,
                                                         int dim, unsigned char* __restrict__ image, int image_dim, Cam c) {
    __shared__ float s_part[SEG > 1 ? 256 : 1];
    if (*wide)
        raycast_tex_march<D, true, SEG>(tex, dim, image, image_dim, c, s_part);
    else
        raycast_tex_march<D, false, SEG>(tex, dim, image, image_dim, c, s_part);
}

constexpr long long kRaycastSmallRays = 1LL << 16;  // production rule of pcmx_raycast_global

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
// Production global caster (round 6): images of up to 2^16 rays march one ray per 16-lane group (variant 6: a 64^2
// image is 1024 waves instead of 64); larger images interleave data and region into the DR16 layout first (one 8-byte
// load per row and sample for both volumes) and march one ray per 4-lane group (variant 11). Measured on one MI355X
// (scripts/raycast_global_lab.py, profiles/r6_raycast/; every image bit-identical to the serial caster's): 64^2
// 1.98 -> 0.47 ms, 512^2 5.2 -> 2.5 ms (pack included). The DR16 buffer comes from the stream-ordered allocator here
// (the torch op passes its own, pcmx_raycast_global_dr); a failed allocation falls back to variant 4.
extern "C" int pcmx_raycast_global(const unsigned char* data, const unsigned char* region, int dim, unsigned char* image,
                                   int image_dim, const float* cam12, float pixel_width, float step, int max_steps,
                                   int f64_color, hipStream_t s) {
    if (dim <= 1 || image_dim <= 0) return -1;
    const long long n_rays = (long long)image_dim * image_dim;
    if (n_rays > kRaycastSmallRays && dim % 4 == 0) {
        static bool pool_kept = false;  // keep freed async allocations in the pool (no OS round trip per frame)
        int dev = 0;
        if (!pool_kept && hipGetDevice(&dev) == hipSuccess) {
            hipMemPool_t pool;
            if (hipDeviceGetDefaultMemPool(&pool, dev) == hipSuccess) {
                unsigned long long keep = ~0ull;
                (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
            }
            pool_kept = true;
        }
        void* dr = nullptr;
        if (hipMallocAsync(&dr, (size_t)pcmx_raycast_dr16_bytes(dim), s) == hipSuccess) {
            int rc = pcmx_raycast_dr16_pack(data, region, dim, dr, s);
            if (rc == 0)
                rc = pcmx_raycast_global_dr(dr, dim, image, image_dim, cam12, pixel_width, step, max_steps, f64_color, 11, s);
            const hipError_t fe = hipFreeAsync(dr, s);
            return rc ? rc : (int)fe;
        }
        (void)hipGetLastError();
        return pcmx_raycast_global_variant(data, region, dim, image, image_dim, cam12, pixel_width, step, max_steps,
                                           f64_color, 4, s);
    }
    return pcmx_raycast_global_variant(data, region, dim, image, image_dim, cam12, pixel_width, step, max_steps,
                                       f64_color, 6, s);
}

// variant 0: the round-5 caster, 8x8-pixel one-wave tiles, the samples of 8 steps in flight (raycast_ref_batch_kernel; 16
// on images of more than 2^16 rays); 1: the round-4 caster (16x16 tiles, one step in flight); 2 / 3: batch kernel with
// 4 / 16 steps in flight; 4: variant 0 with pair taps; 5 / 6 / 7 / 8: one ray per 64 / 16 / 8 / 4-lane group; 9 / 10 /
// 11: DR16 layout (pcmx_raycast_global_dr). Identical images. The production choice is pcmx_raycast_global's.
extern "C" int pcmx_raycast_global_variant(const unsigned char* data, const unsigned char* region, int dim,
                                           unsigned char* image, int image_dim, const float* cam12, float pixel_width,
                                           float step, int max_steps, int f64_color, int variant, hipStream_t s) {
    if (dim <= 1 || image_dim <= 0 || variant < 0 || variant > 11) return -1;
    const Cam c = make_cam(cam12, pixel_width, step, max_steps);
    const long long n_rays = (long long)image_dim * image_dim;
    if (variant >= 5 && variant <= 8) {  // group-per-ray: G lanes per ray, 256 / G rays per block
        const int G = variant == 5 ? 64 : variant == 6 ? 16 : variant == 7 ? 8 : 4;
        const unsigned blocks = (unsigned)((n_rays * G + 255) / 256);
#define PCMX_RAYCAST_G(GG)                                                                                                   \
    (f64_color ? raycast_ref_group_kernel<true, GG, false><<<blocks, 256, 0, s>>>(data, region, nullptr, dim, image,         \
                                                                                 image_dim, c)                             \
               : raycast_ref_group_kernel<false, GG, false><<<blocks, 256, 0, s>>>(data, region, nullptr, dim, image,        \
                                                                                  image_dim, c))
        if (G == 64) PCMX_RAYCAST_G(64);
        else if (G == 16) PCMX_RAYCAST_G(16);
        else if (G == 8) PCMX_RAYCAST_G(8);
        else PCMX_RAYCAST_G(4);
#undef PCMX_RAYCAST_G
        return (int)hipGetLastError();
    }
    if (variant >= 9) return PCMX_ERR_ARG;  // DR16 variants: pcmx_raycast_global_dr
    if (variant == 4) {  // batch caster with pair taps
        const dim3 grid((image_dim + 7) / 8, (image_dim + 7) / 8);
        if (n_rays > (1 << 16))
            f64_color ? raycast_ref_batch2_kernel<true, 16><<<grid, 64, 0, s>>>(data, region, dim, image, image_dim, c)
                      : raycast_ref_batch2_kernel<false, 16><<<grid, 64, 0, s>>>(data, region, dim, image, image_dim, c);
        else
            f64_color ? raycast_ref_batch2_kernel<true, 8><<<grid, 64, 0, s>>>(data, region, dim, image, image_dim, c)
                      : raycast_ref_batch2_kernel<false, 8><<<grid, 64, 0, s>>>(data, region, dim, image, image_dim, c);
        return (int)hipGetLastError();
    }
    if (variant == 1) {
        const dim3 grid((image_dim + 15) / 16, (image_dim + 15) / 16);
        if (f64_color)
            raycast_ref_kernel<true><<<grid, 256, 0, s>>>(data, region, dim, image, image_dim, c);
        else
            raycast_ref_kernel<false><<<grid, 256, 0, s>>>(data, region, dim, image, image_dim, c);
        return (int)hipGetLastError();
    }
    const dim3 grid((image_dim + 7) / 8, (image_dim + 7) / 8);
    // production: 8 steps in flight up to 2^16 rays (64^2: 1.97 ms vs 2.06 with 16 and 3.1 with one step), 16 above
    // (512^2: 5.2 ms vs 7.6 with 4 and 7.1 with one step; scripts/raycast_global_lab.py, profiles/r5_refbase/)
    const int b = variant == 2 ? 4 : variant == 3 ? 16 : (long long)image_dim * image_dim > (1 << 16) ? 16 : 8;
#define PCMX_RAYCAST_B(BB)                                                                                         \
    (f64_color ? raycast_ref_batch_kernel<true, BB><<<grid, 64, 0, s>>>(data, region, dim, image, image_dim, c)     \
               : raycast_ref_batch_kernel<false, BB><<<grid, 64, 0, s>>>(data, region, dim, image, image_dim, c))
    if (b == 4) PCMX_RAYCAST_B(4);
    else if (b == 8) PCMX_RAYCAST_B(8);
    else PCMX_RAYCAST_B(16);
#undef PCMX_RAYCAST_B
    return (int)hipGetLastError();
}

extern "C" long long pcmx_raycast_dr16_bytes(int dim) { return dim > 1 ? 2LL * dim * dim * dim : 0; }

// Interleaves data and region into the DR16 layout (dim^3 u16; dim % 4 == 0 and 4-B aligned volumes).
extern "C" int pcmx_raycast_dr16_pack(const unsigned char* data, const unsigned char* region, int dim, void* dr,
                                      hipStream_t s) {
    if (dim <= 1 || dim % 4 || !dr || ((uintptr_t)data & 3u) || ((uintptr_t)region & 3u) || ((uintptr_t)dr & 7u))
        return PCMX_ERR_ARG;
    const long long n4 = (long long)dim * dim * dim / 4;
    const long long blocks = (n4 + 255) / 256 < 16384 ? (n4 + 255) / 256 : 16384;
    dr16_pack_kernel<<<(int)blocks, 256, 0, s>>>(data, region, reinterpret_cast<unsigned*>(dr), n4);
    return (int)hipGetLastError();
}

// Global caster on a DR16 volume (pcmx_raycast_dr16_pack): variant 9 = per-lane rays (batch), 10 / 11 = group per ray
// with 16 / 4 lanes. Bit-identical to pcmx_raycast_global_variant.
extern "C" int pcmx_raycast_global_dr(const void* dr, int dim, unsigned char* image, int image_dim, const float* cam12,
                                      float pixel_width, float step, int max_steps, int f64_color, int variant,
                                      hipStream_t s) {
    if (dim <= 1 || image_dim <= 0 || !dr || variant < 9 || variant > 11) return PCMX_ERR_ARG;
    const Cam c = make_cam(cam12, pixel_width, step, max_steps);
    const unsigned short* d16 = reinterpret_cast<const unsigned short*>(dr);
    const long long n_rays = (long long)image_dim * image_dim;
    if (variant == 9) {
        const dim3 grid((image_dim + 7) / 8, (image_dim + 7) / 8);
        if (n_rays > (1 << 16))
            f64_color ? raycast_dr_batch_kernel<true, 16><<<grid, 64, 0, s>>>(d16, dim, image, image_dim, c)
                      : raycast_dr_batch_kernel<false, 16><<<grid, 64, 0, s>>>(d16, dim, image, image_dim, c);
        else
            f64_color ? raycast_dr_batch_kernel<true, 8><<<grid, 64, 0, s>>>(d16, dim, image, image_dim, c)
                      : raycast_dr_batch_kernel<false, 8><<<grid, 64, 0, s>>>(d16, dim, image, image_dim, c);
        return (int)hipGetLastError();
    }
    const int G = variant == 10 ? 16 : 4;
    const unsigned blocks = (unsigned)((n_rays * G + 255) / 256);
    if (G == 16)
        f64_color ? raycast_ref_group_kernel<true, 16, true><<<blocks, 256, 0, s>>>(nullptr, nullptr, d16, dim, image, image_dim, c)
                  : raycast_ref_group_kernel<false, 16, true><<<blocks, 256, 0, s>>>(nullptr, nullptr, d16, dim, image, image_dim, c);
    else
        f64_color ? raycast_ref_group_kernel<true, 4, true><<<blocks, 256, 0, s>>>(nullptr, nullptr, d16, dim, image, image_dim, c)
                  : raycast_ref_group_kernel<false, 4, true><<<blocks, 256, 0, s>>>(nullptr, nullptr, d16, dim, image, image_dim, c);
    return (int)hipGetLastError();
}

extern "C" int pcmx_volume_gen_slab_u8(unsigned char* data, int dim, int z_first, int nplanes, unsigned seed,
                                       hipStream_t s) {
    if (dim <= 0 || nplanes <= 0) return PCMX_ERR_ARG;
    volume_gen_slab_kernel<<<dim3((dim + 255) / 256, dim, nplanes), 256, 0, s>>>(data, dim, z_first, seed);
    return (int)hipGetLastError();
}

extern "C" int pcmx_raycast_slab(const unsigned char* data, const unsigned char* region, int dim, int z0,
                                 int* state, int init, int bottom, unsigned char* image, int image_dim,
                                 const float* cam12, float pixel_width, float step, int max_steps, hipStream_t s) {
    if (dim <= 1 || image_dim <= 0 || z0 < 0 || z0 >= dim || !state) return PCMX_ERR_ARG;
    const Cam c = make_cam(cam12, pixel_width, step, max_steps);
    const dim3 grid((image_dim + 15) / 16, (image_dim + 15) / 16);
    raycast_slab_kernel<<<grid, 256, 0, s>>>(data, region, dim, z0, state, init, bottom, image, image_dim, c);
    return (int)hipGetLastError();
}

extern "C" int pcmx_brick_pack(const unsigned char* data, const unsigned char* region, int dim, void* tex,
                               hipStream_t s) {
    if (dim <= 0 || dim > 2048) return -1;
    const size_t nvox = (size_t)dim * dim * dim;
    int* wide = reinterpret_cast<int*>(reinterpret_cast<char*>(tex) + nvox * 16);  // format flag behind the texels
    PCMX_HIP_RET(hipMemsetAsync(wide, 0, sizeof(int), s));
    const dim3 units((unsigned)(((size_t)dim * dim + 1023) / 1024), dim);  // 1024-texel units of each z-plane
    const size_t align = reinterpret_cast<size_t>(data) | reinterpret_cast<size_t>(region);
    if (dim % 8 == 0 && dim >= 16 && dim <= 1024 && align % 4 == 0) {  // 32-bit buffer offsets: dim^3 <= 2^30
        constexpr int ZP = 8, ZPW = 2;  // wide rewrite: 2 planes per unit (its 16-B texels double the stores)
        brick_pack12_narrow_kernel<ZP><<<dim3(units.x, (dim + ZP - 1) / ZP), 128, 0, s>>>(data, region, dim, tex, wide);
        brick_pack12_wide_kernel<ZPW><<<512, 128, 0, s>>>(data, region, dim, tex, wide, units.x, (dim + ZPW - 1) / ZPW);
        return (int)hipGetLastError();
    }
    data_hibit_kernel<<<1024, 256, 0, s>>>(data, nvox, wide);
    if (dim % 8 == 0 && align % 8 == 0)
        brick_pack8_kernel<4><<<dim3(units.x, (dim + 3) / 4), 128, 0, s>>>(data, region, dim, tex, wide);
    else if (dim % 4 == 0 && align % 4 == 0)
        brick_pack4_kernel<<<units, 256, 0, s>>>(data, region, dim, tex, wide);
    else
        brick_pack_kernel<<<dim3((dim + 255) / 256, dim, dim), 256, 0, s>>>(data, region, dim, tex, wide);
    return (int)hipGetLastError();
}

// batch = steps per prefetch batch (1, 4, 8, 16; 0 = 16, the measured best); segments = waves per ray patch
// (1, 2, 4; 0 = the measured best)
template <int D>
void launch_tex(const void* tex, const int* wide, int dim, unsigned char* image, int image_dim, const Cam& c,
                int segments, hipStream_t s) {
    const unsigned gx = (unsigned)(image_dim + 15) / 16;
    switch (segments) {
        case 1: raycast_tex_kernel<D, 1><<<dim3(gx, (image_dim + 15) / 16), 256, 0, s>>>(tex, wide, dim, image, image_dim, c); break;
        case 2: raycast_tex_kernel<D, 2><<<dim3(gx, (image_dim + 7) / 8), 256, 0, s>>>(tex, wide, dim, image, image_dim, c); break;
        default: raycast_tex_kernel<D, 4><<<dim3(gx, (image_dim + 3) / 4), 256, 0, s>>>(tex, wide, dim, image, image_dim, c); break;
    }
}

extern "C" int pcmx_raycast_bricked(const void* tex, int dim, unsigned char* image, int image_dim,
                                    const float* cam12, float pixel_width, float step, int max_steps, int batch,
                                    int segments, hipStream_t s) {
    if (dim <= 1 || dim > 2048 || image_dim <= 0) return PCMX_ERR_ARG;
    if (batch != 0 && batch != 1 && batch != 4 && batch != 8 && batch != 16) return PCMX_ERR_ARG;
    if (segments != 0 && segments != 1 && segments != 2 && segments != 4) return PCMX_ERR_ARG;
    if (segments == 0) segments = 4;
    const Cam c = make_cam(cam12, pixel_width, step, max_steps);
    const int* wide = reinterpret_cast<const int*>(reinterpret_cast<const char*>(tex) + (size_t)dim * dim * dim * 16);
    switch (batch) {
        case 1: launch_tex<1>(tex, wide, dim, image, image_dim, c, segments, s); break;
        case 4: launch_tex<4>(tex, wide, dim, image, image_dim, c, segments, s); break;
        case 8: launch_tex<8>(tex, wide, dim, image, image_dim, c, segments, s); break;
        default: launch_tex<16>(tex, wide, dim, image, image_dim, c, segments, s); break;
    }
    return (int)hipGetLastError();
}

