// Region growing on MI355X: 2-D (ref 2-mpi-region-growing/region.c:493-533, 4-connected, |a-b| < thr
// between ADJACENT pixels, seeded flood fill) and 3-D (ref 5-cuda-region-growing/raycast.cu:534-699,
// 6-connected).
//
// MI355X design
//  * Tiled local fixpoint: a workgroup stages its tile plus a 1-cell halo of image and region in LDS and
//    iterates Gauss-Seidel sweeps until nothing changes inside the tile (`__syncthreads_or`), so one
//    launch advances the front across a whole tile instead of one cell (the naive kernel of
//    raycast.cu:534 needs one launch per BFS level).
//  * Active-tile worklist: a tile only runs if a face neighbour changed in the previous launch. 2-D:
//    act_in -> act_out flags over the tile grid. 3-D (65k tiles at 512^3): a compacted device-built list
//    walked by a persistent grid, so a launch costs the frontier, not a full-volume dispatch.
//  * Halo cells are read-only inputs. That makes the same kernel the compute step of the distributed
//    version: a rank's halo holds its neighbours' boundary after an RCCL exchange (parallel/region2d.py).
//  * Region state is 0/1 (a cell never leaves the region), so races between tiles are benign and the
//    fixpoint equals the serial flood fill.
#include "pcmx_common.h"
#include "pcmx_hip.h"

namespace {

// ----------------------------------------------------------------------------------------------- 2-D
constexpr int kT2 = 64;            // tile interior edge
constexpr int kE2 = kT2 + 2;       // with halo
constexpr int kThreads2 = 256;

// Arrays are padded: interior rows/cols 1..H / 1..W, pitch `ld` >= W+2.
__global__ __launch_bounds__(kThreads2) void region2d_tile_kernel(const unsigned char* __restrict__ img,
                                                                 unsigned char* __restrict__ region, int H, int W,
                                                                 int ld, int thr, const int* __restrict__ act_in,
                                                                 int* __restrict__ act_out, int* __restrict__ flag) {
    const int tx = blockIdx.x, ty = blockIdx.y;
    const int ntx = gridDim.x, nty = gridDim.y;
    if (act_in && act_in[ty * ntx + tx] == 0) return;
    __shared__ unsigned char simg[kE2][kE2 + 2];
    __shared__ unsigned char sreg[kE2][kE2 + 2];
    const int x0 = tx * kT2, y0 = ty * kT2;  // padded coords of the halo corner
    for (int i = threadIdx.x; i < kE2 * kE2; i += kThreads2) {
        const int ly = i / kE2, lx = i % kE2;
        const int gy = y0 + ly, gx = x0 + lx;
        const bool ok = gy <= H + 1 && gx <= W + 1;
        simg[ly][lx] = ok ? img[(size_t)gy * ld + gx] : 0;
        sreg[ly][lx] = ok ? region[(size_t)gy * ld + gx] : 0;
    }
    __syncthreads();
    const int lx = 1 + (threadIdx.x & 63);
    const int rowgrp = threadIdx.x >> 6;  // 4 row groups, 16 rows each
    const bool col_in = x0 + lx <= W;
    unsigned long long mine = 0;  // bit k: this thread set row 1 + rowgrp + 4k
    bool any_block = false;
    while (true) {
        int changed = 0;
#pragma unroll
        for (int k = 0; k < kT2 / 4; ++k) {
            const int ly = 1 + rowgrp + 4 * k;
            if (!col_in || y0 + ly > H || sreg[ly][lx]) continue;
            const int v = simg[ly][lx];
            const bool grow = (sreg[ly - 1][lx] && abs(v - (int)simg[ly - 1][lx]) < thr) ||
                              (sreg[ly + 1][lx] && abs(v - (int)simg[ly + 1][lx]) < thr) ||
                              (sreg[ly][lx - 1] && abs(v - (int)simg[ly][lx - 1]) < thr) ||
                              (sreg[ly][lx + 1] && abs(v - (int)simg[ly][lx + 1]) < thr);
            if (grow) {
                sreg[ly][lx] = 1;
                mine |= 1ull << k;
                changed = 1;
            }
        }
        if (!__syncthreads_or(changed)) break;
        any_block = true;
    }
    if (mine) {
#pragma unroll
        for (int k = 0; k < kT2 / 4; ++k)
            if (mine & (1ull << k)) region[(size_t)(y0 + 1 + rowgrp + 4 * k) * ld + x0 + lx] = 1;
    }
    if (any_block && threadIdx.x == 0) {
        *flag = 1;
        act_out[ty * ntx + tx] = 1;
        if (tx > 0) act_out[ty * ntx + tx - 1] = 1;
        if (tx + 1 < ntx) act_out[ty * ntx + tx + 1] = 1;
        if (ty > 0) act_out[(ty - 1) * ntx + tx] = 1;
        if (ty + 1 < nty) act_out[(ty + 1) * ntx + tx] = 1;
    }
}

// ----------------------------------------------------------------------------------------------- 3-D
// Tile interior 32(x) x 8(y) x 8(z); one thread per (x,y) column of the tile walks 8 z-slices.
// Work is a COMPACTED tile list: launch e processes list[e%2] (count[e%3]) with a persistent grid and
// appends the tiles to visit next (changed tiles and their face neighbours) to list[(e+1)%2], deduplicated
// by stamping mark[tile] = e+1 with an atomic exchange. A 512^3 grow touches ~1-2k of the 65k tiles per
// launch, so a launch costs what the frontier costs, not a full-volume dispatch. The first list holds the
// tiles that contain any region voxel (one scan of the region). Counters rotate over 3 slots: launch e
// zeroes slot (e+2)%3, the output slot of launch e+1, so no memset sits between launches.
constexpr int kTX = 32, kTY = 8, kTZ = 8;
constexpr int kThreads3 = kTX * kTY;
constexpr int kListGrid = 2048;  // persistent grid of the list kernel (8 workgroups per CU)

struct Grow3dWs {
    int flag;
    int count[3];
    // followed by: int mark[ntiles]; int list[2][ntiles]
};

__device__ __forceinline__ void push_tile(int t, int stamp, int* __restrict__ mark, int* __restrict__ list,
                                          int* __restrict__ count) {
    if (atomicExch(&mark[t], stamp) != stamp) list[atomicAdd(count, 1)] = t;
}

// Grows one tile to its local fixpoint; returns (block-uniform) whether any voxel of the tile changed.
__device__ bool grow_tile3d(const unsigned char* __restrict__ data, unsigned char* __restrict__ region, int dim, int thr,
                            int bx, int by, int bz, unsigned char (*sd)[kTY + 2][kTX + 2],
                            unsigned char (*sr)[kTY + 2][kTX + 2]) {
    const int x0 = bx * kTX - 1, y0 = by * kTY - 1, z0 = bz * kTZ - 1;
    const size_t plane = (size_t)dim * dim;
    constexpr int kE = (kTZ + 2) * (kTY + 2) * (kTX + 2);
    for (int i = threadIdx.x; i < kE; i += kThreads3) {
        const int lx = i % (kTX + 2), ly = (i / (kTX + 2)) % (kTY + 2), lz = i / ((kTX + 2) * (kTY + 2));
        const int gx = x0 + lx, gy = y0 + ly, gz = z0 + lz;
        const bool ok = gx >= 0 && gy >= 0 && gz >= 0 && gx < dim && gy < dim && gz < dim;
        const size_t g = (size_t)gz * plane + (size_t)gy * dim + gx;
        sd[lz][ly][lx] = ok ? data[g] : 0;
        sr[lz][ly][lx] = ok ? (region[g] != 0) : 0;
    }
    __syncthreads();
    const int lx = 1 + threadIdx.x % kTX, ly = 1 + threadIdx.x / kTX;
    const bool col_in = x0 + lx < dim && y0 + ly < dim;
    unsigned mine = 0;
    bool any_block = false;
    while (true) {
        int changed = 0;
#pragma unroll
        for (int lz = 1; lz <= kTZ; ++lz) {
            if (!col_in || z0 + lz >= dim || sr[lz][ly][lx]) continue;
            const int v = sd[lz][ly][lx];
            const bool grow = (sr[lz][ly][lx - 1] && abs(v - (int)sd[lz][ly][lx - 1]) < thr) ||
                              (sr[lz][ly][lx + 1] && abs(v - (int)sd[lz][ly][lx + 1]) < thr) ||
                              (sr[lz][ly - 1][lx] && abs(v - (int)sd[lz][ly - 1][lx]) < thr) ||
                              (sr[lz][ly + 1][lx] && abs(v - (int)sd[lz][ly + 1][lx]) < thr) ||
                              (sr[lz - 1][ly][lx] && abs(v - (int)sd[lz - 1][ly][lx]) < thr) ||
                              (sr[lz + 1][ly][lx] && abs(v - (int)sd[lz + 1][ly][lx]) < thr);
            if (grow) {
                sr[lz][ly][lx] = 1;
                mine |= 1u << lz;
                changed = 1;
            }
        }
        if (!__syncthreads_or(changed)) break;
        any_block = true;
    }
    if (mine) {
#pragma unroll
        for (int lz = 1; lz <= kTZ; ++lz)
            if (mine & (1u << lz)) region[(size_t)(z0 + lz) * plane + (size_t)(y0 + ly) * dim + x0 + lx] = 1;
    }
    return any_block;
}

__global__ __launch_bounds__(kThreads3) void region3d_list_kernel(const unsigned char* __restrict__ data,
                                                                 unsigned char* __restrict__ region, int dim, int thr,
                                                                 int nbx, int nby, int nbz, int epoch,
                                                                 Grow3dWs* __restrict__ ws, int* __restrict__ mark,
                                                                 int* __restrict__ lists, int ntiles) {
    __shared__ unsigned char sd[kTZ + 2][kTY + 2][kTX + 2];
    __shared__ unsigned char sr[kTZ + 2][kTY + 2][kTX + 2];
    const int* list_in = lists + (epoch & 1) * ntiles;
    int* list_out = lists + ((epoch + 1) & 1) * ntiles;
    int* count_out = &ws->count[(epoch + 1) % 3];
    if (blockIdx.x == 0 && threadIdx.x == 0) ws->count[(epoch + 2) % 3] = 0;
    const int n = __hip_atomic_load(&ws->count[epoch % 3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int idx = blockIdx.x; idx < n; idx += gridDim.x) {
        const int t = list_in[idx];
        const int bx = t % nbx, by = (t / nbx) % nby, bz = t / (nbx * nby);
        const bool changed = grow_tile3d(data, region, dim, thr, bx, by, bz, sd, sr);
        // a changed tile reached its local fixpoint; its 6 face neighbours see new halo cells next launch
        // (the tile itself is re-queued only if a neighbour changes in turn)
        if (changed && threadIdx.x < 7) {
            const int d = threadIdx.x;
            if (d == 0) {
                ws->flag = 1;
            } else {
                const int nx = bx + (d == 1) - (d == 2), ny = by + (d == 3) - (d == 4), nz = bz + (d == 5) - (d == 6);
                if (nx >= 0 && ny >= 0 && nz >= 0 && nx < nbx && ny < nby && nz < nbz)
                    push_tile((nz * nby + ny) * nbx + nx, epoch + 1, mark, list_out, count_out);
            }
        }
        __syncthreads();  // LDS tile buffers are reused by the next tile of this workgroup
    }
}

// First work list: every tile holding a region voxel (16 B per thread loads of the region).
__global__ __launch_bounds__(kThreads3) void region3d_seed_tiles_kernel(const unsigned char* __restrict__ region, int dim,
                                                                       int nbx, int nby, Grow3dWs* __restrict__ ws,
                                                                       int* __restrict__ mark, int* __restrict__ list0) {
    // one workgroup per (y-row of tiles, z-slab of tiles): 8 x 8 voxel rows of the full x extent
    const int by = blockIdx.x % nby, bz = blockIdx.x / nby;
    const size_t plane = (size_t)dim * dim;
    __shared__ int hit[64];
    if (threadIdx.x < 64) hit[threadIdx.x] = 0;
    __syncthreads();
    const int vecs_per_row = dim / 16;  // dim % 16 == 0 on this path
    for (int i = threadIdx.x; i < kTY * kTZ * vecs_per_row; i += kThreads3) {
        const int v = i % vecs_per_row, yz = i / vecs_per_row;
        const int y = by * kTY + yz % kTY, z = bz * kTZ + yz / kTY;
        if (y >= dim || z >= dim) continue;
        const pcmx::i32x4 w = *reinterpret_cast<const pcmx::i32x4*>(region + (size_t)z * plane + (size_t)y * dim + v * 16);
        if ((w.x | w.y | w.z | w.w) != 0) hit[(v * 16) / kTX] = 1;
    }
    __syncthreads();
    if (threadIdx.x < nbx && hit[threadIdx.x]) {
        const int t = (bz * nby + by) * nbx + threadIdx.x;
        push_tile(t, 0, mark, list0, &ws->count[0]);
    }
}

// Naive frontier kernel with the reference's 0/1/2 states (raycast.cu:534-574, region.cl:34-73):
// a voxel holding 2 becomes 1 and marks its similar 0-neighbours 2. Bounds-checked (B19 fixed).
__global__ __launch_bounds__(256) void region3d_step_kernel(const unsigned char* __restrict__ data,
                                                           unsigned char* __restrict__ region, int dim, int thr,
                                                           int* __restrict__ unfinished) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    const int z = blockIdx.z;
    if (x >= dim || y >= dim || z >= dim) return;
    const size_t plane = (size_t)dim * dim;
    const size_t i = (size_t)z * plane + (size_t)y * dim + x;
    if (region[i] != 2) return;
    *unfinished = 1;
    region[i] = 1;
    const int v = data[i];
    const int dx[6] = {-1, 1, 0, 0, 0, 0}, dy[6] = {0, 0, -1, 1, 0, 0}, dz[6] = {0, 0, 0, 0, -1, 1};
#pragma unroll
    for (int n = 0; n < 6; ++n) {
        const int cx = x + dx[n], cy = y + dy[n], cz = z + dz[n];
        if (cx < 0 || cy < 0 || cz < 0 || cx >= dim || cy >= dim || cz >= dim) continue;
        const size_t j = (size_t)cz * plane + (size_t)cy * dim + cx;
        if (region[j] == 0 && abs(v - (int)data[j]) < thr) region[j] = 2;
    }
}

struct ActWs {
    int flag;
    int pad[3];
};

// Runs tile launches until a batch of `batch` launches changes nothing. Blocks the host once per batch.
template <class Launch>
int run_active_loop(Launch launch, long long ntiles, void* ws, int batch, int max_launches, hipStream_t s,
                    int* launches_out) {
    int* flag = reinterpret_cast<int*>(ws);
    int* act[2] = {flag + 4, flag + 4 + ntiles};
    PCMX_HIP_RET(hipMemsetAsync(act[0], 0xff, ntiles * sizeof(int), s));  // every tile active at first
    int launches = 0, cur = 0;
    while (launches < max_launches) {
        PCMX_HIP_RET(hipMemsetAsync(flag, 0, sizeof(int), s));
        for (int b = 0; b < batch && launches < max_launches; ++b, ++launches) {
            PCMX_HIP_RET(hipMemsetAsync(act[cur ^ 1], 0, ntiles * sizeof(int), s));
            launch(act[cur], act[cur ^ 1], flag);
            PCMX_HIP_RET(hipGetLastError());
            cur ^= 1;
        }
        int h = 0;
        PCMX_HIP_RET(hipMemcpyAsync(&h, flag, sizeof(int), hipMemcpyDeviceToHost, s));
        PCMX_HIP_RET(hipStreamSynchronize(s));
        if (!h) break;
    }
    if (launches_out) *launches_out = launches;
    return 0;
}
}  // namespace

extern "C" long long pcmx_region2d_workspace_bytes(int H, int W) {
    const long long nt = (long long)((W + kT2 - 1) / kT2) * ((H + kT2 - 1) / kT2);
    return 16 + 2 * nt * 4;
}

extern "C" int pcmx_region2d_grow(const unsigned char* img, unsigned char* region, int H, int W, int ld, int thr,
                                  void* ws, int batch, int max_launches, hipStream_t s, int* launches_out) {
    if (H <= 0 || W <= 0 || ld < W + 2 || !ws) return -1;
    dim3 grid((W + kT2 - 1) / kT2, (H + kT2 - 1) / kT2);
    const long long nt = (long long)grid.x * grid.y;
    auto launch = [&](const int* ain, int* aout, int* flag) {
        region2d_tile_kernel<<<grid, kThreads2, 0, s>>>(img, region, H, W, ld, thr, ain, aout, flag);
    };
    return run_active_loop(launch, nt, ws, batch < 1 ? 4 : batch, max_launches, s, launches_out);
}

extern "C" long long pcmx_region3d_workspace_bytes(int dim) {
    const long long nt = (long long)((dim + kTX - 1) / kTX) * ((dim + kTY - 1) / kTY) * ((dim + kTZ - 1) / kTZ);
    return (long long)sizeof(Grow3dWs) + 3 * nt * 4;
}

// Grows `region` (0 = outside, nonzero = inside) to the 6-connected fixpoint. Host syncs once per `batch`
// launches (a changed-flag read back); launches run on the device-built tile lists in between.
extern "C" int pcmx_region3d_grow_tiled(const unsigned char* data, unsigned char* region, int dim, int thr, void* ws,
                                        int batch, int max_launches, hipStream_t s, int* launches_out) {
    if (dim <= 0 || !ws) return -1;
    if (dim % 16 || (((uintptr_t)region) & 15)) return -1;  // seed scan reads 16-B vectors
    const int nbx = (dim + kTX - 1) / kTX, nby = (dim + kTY - 1) / kTY, nbz = (dim + kTZ - 1) / kTZ;
    if (nbx > 64) return -1;  // seed scan keeps one hit flag per x-tile in a 64-entry LDS array
    const long long nt = (long long)nbx * nby * nbz;
    if (nt > 0x3fffffff) return -1;
    Grow3dWs* w = reinterpret_cast<Grow3dWs*>(ws);
    int* mark = reinterpret_cast<int*>(w + 1);
    int* lists = mark + nt;
    // marks = -1 (no epoch), counters = 0, then the seed tiles (epoch 0) go to list 0
    PCMX_HIP_RET(hipMemsetAsync(w, 0, sizeof(Grow3dWs), s));
    PCMX_HIP_RET(hipMemsetAsync(mark, 0xff, (size_t)nt * 4, s));
    region3d_seed_tiles_kernel<<<nby * nbz, kThreads3, 0, s>>>(region, dim, nbx, nby, w, mark, lists);
    PCMX_HIP_RET(hipGetLastError());
    const int b = batch < 1 ? 8 : batch;
    int launches = 0;
    while (launches < max_launches) {
        PCMX_HIP_RET(hipMemsetAsync(&w->flag, 0, sizeof(int), s));
        for (int i = 0; i < b && launches < max_launches; ++i, ++launches) {
            region3d_list_kernel<<<kListGrid, kThreads3, 0, s>>>(data, region, dim, thr, nbx, nby, nbz, launches, w, mark,
                                                               lists, (int)nt);
            PCMX_HIP_RET(hipGetLastError());
        }
        int h = 0;
        PCMX_HIP_RET(hipMemcpyAsync(&h, &w->flag, sizeof(int), hipMemcpyDeviceToHost, s));
        PCMX_HIP_RET(hipStreamSynchronize(s));
        if (!h) break;
    }
    if (launches_out) *launches_out = launches;
    return 0;
}

extern "C" int pcmx_region3d_grow_naive(const unsigned char* data, unsigned char* region, int dim, int thr, int* flag_ws,
                                        int max_launches, hipStream_t s, int* launches_out) {
    if (dim <= 0 || !flag_ws) return -1;
    dim3 grid((dim + 63) / 64, (dim + 3) / 4, dim);
    int launches = 0;
    while (launches < max_launches) {
        PCMX_HIP_RET(hipMemsetAsync(flag_ws, 0, sizeof(int), s));
        region3d_step_kernel<<<grid, 256, 0, s>>>(data, region, dim, thr, flag_ws);
        PCMX_HIP_RET(hipGetLastError());
        ++launches;
        int h = 0;
        PCMX_HIP_RET(hipMemcpyAsync(&h, flag_ws, sizeof(int), hipMemcpyDeviceToHost, s));
        PCMX_HIP_RET(hipStreamSynchronize(s));
        if (!h) break;
    }
    if (launches_out) *launches_out = launches;
    return 0;
}
