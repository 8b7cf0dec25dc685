// Region growing on MI355X: 2-D (ref 2-mpi-region-growing/region.c:493-533, 4-connected, |a-b| < thr
// between ADJACENT pixels, seeded flood fill) and 3-D (ref 5-cuda-region-growing/raycast.cu:534-699,
// 6-connected).
//
// MI355X design
//  * Tiled local fixpoint, so one launch advances the front across a whole tile instead of one cell (the
//    naive kernel of raycast.cu:534 needs one launch per BFS level: 249 launches, 61 ms at 512^3).
//    2-D: a workgroup stages its tile plus a 1-cell halo in LDS and iterates Gauss-Seidel sweeps
//    (`__syncthreads_or`). 3-D: BIT-PARALLEL one-wave tiles of 64x8x8 — a lane holds one 64-voxel row as
//    a 64-bit mask, similarity to the x / y / z neighbours as link masks, and a sweep is a few 64-bit ops
//    plus cross-lane shuffles (a front crosses a whole row per sweep; no LDS, no barriers): 0.73 ms per
//    512^3 grow (the 32x8x8 LDS-tile version took 1.47 ms).
//  * Active-tile worklist: a tile only runs if a face neighbour changed in the previous launch. 2-D:
//    act_in -> act_out flags over the tile grid. 3-D (32k tiles at 512^3): a compacted device-built list
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
// Work is a COMPACTED tile list: launch e processes list[e%2] (count[e%3]) with a persistent grid and
// appends the tiles to visit next (neighbours across faces whose voxels changed) to list[(e+1)%2],
// deduplicated by stamping mark[tile] = e+1 with an atomic exchange. A 512^3 grow touches ~1-2k of the 32k
// tiles per launch, so a launch costs what the frontier costs, not a full-volume dispatch. The first list
// holds the tiles that contain any region voxel (one scan of the region); in that first launch a tile's
// faces holding region voxels push their neighbours too (a seed on a tile face whose own tile cannot grow
// must still reach the next tile). Counters rotate over 3 slots: launch e zeroes slot (e+2)%3, the output
// slot of launch e+1, so no memset sits between launches.
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

// --------------------------------------------------------------------------- 3-D, bit-parallel tiles
// Tile 64(x) x 8(y) x 8(z), ONE WAVE per tile, one 64-voxel x-row per lane (lane = y + 8 z): the row's region
// membership is a 64-bit mask R, and similarity to the neighbour along x / y+1 / z+1 is a link mask per row,
// computed once from the data (SWAR byte compares). A sweep is then a handful of 64-bit ops per lane:
//   R |= (R of lane y+-1 & y-links) | (R of lane z+-1 & z-links) | external seeds (halo rows / halo bits)
//   R  = flood of R along the x-links of the row (log-step doubling: any distance in 6 steps each way)
// iterated (wave ballot) until no lane changes: a front crosses a whole row in ONE sweep and the tile in
// ~y+z sweeps, with no LDS and no block barriers (the 32x8x8 LDS tiles needed up to ~40 barrier-separated
// Gauss-Seidel sweeps per tile; measured 1.47 -> 0.78 ms per 512^3 grow). Only faces whose voxels changed
// push their neighbour tile.
constexpr int kBX = 64, kBY = 8, kBZ = 8;

__device__ __forceinline__ unsigned long long shfl64(unsigned long long v, int src) {
    const int lo = __shfl((int)(unsigned)v, src, 64), hi = __shfl((int)(unsigned)(v >> 32), src, 64);
    return ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo;
}

// bit b of the result (0..15) = |a_byte[b] - b_byte[b]| < thr for two 16-byte vectors
__device__ __forceinline__ unsigned similar16(pcmx::i32x4 a, pcmx::i32x4 b, int thr) {
    unsigned m = 0;
    if (thr == 1) {  // equality: exact SWAR zero-byte test of a ^ b
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const unsigned x = (unsigned)a[k] ^ (unsigned)b[k];
            const unsigned t = ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x | 0x7f7f7f7fu);  // bit 7 of zero bytes
            m |= (((t >> 7) & 1u) | ((t >> 14) & 2u) | ((t >> 21) & 4u) | ((t >> 28) & 8u)) << (4 * k);
        }
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int va = ((unsigned)a[k >> 2] >> (8 * (k & 3))) & 0xff, vb = ((unsigned)b[k >> 2] >> (8 * (k & 3))) & 0xff;
            m |= (unsigned)(abs(va - vb) < thr) << k;
        }
    }
    return m;
}

struct Row64 {
    pcmx::i32x4 v[4];
};

__device__ __forceinline__ Row64 load_row(const unsigned char* __restrict__ p) {
    Row64 r;
#pragma unroll
    for (int c = 0; c < 4; ++c) r.v[c] = reinterpret_cast<const pcmx::i32x4*>(p)[c];
    return r;
}

__device__ __forceinline__ unsigned long long similar64(const Row64& a, const Row64& b, int thr) {
    unsigned long long m = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) m |= (unsigned long long)similar16(a.v[c], b.v[c], thr) << (16 * c);
    return m;
}

__device__ __forceinline__ unsigned long long nonzero64(const Row64& a) {
    unsigned long long m = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const unsigned x = (unsigned)a.v[c][k];
            const unsigned t = (((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;  // bit 7 of nonzero bytes
            m |= (unsigned long long)(((t >> 7) & 1u) | ((t >> 14) & 2u) | ((t >> 21) & 4u) | ((t >> 28) & 8u))
                 << (16 * c + 4 * k);
        }
    return m;
}

// x-flood of R along links L (bit i: voxel i ~ voxel i+1), both directions, log-step doubling
__device__ __forceinline__ unsigned long long xflood(unsigned long long R, unsigned long long L) {
    unsigned long long M = L;
#pragma unroll
    for (int s = 1; s < 64; s <<= 1) {
        R |= (R & M) << s;
        M &= M >> s;
    }
    M = L;
#pragma unroll
    for (int s = 1; s < 64; s <<= 1) {
        R |= (R >> s) & M;
        M &= M >> s;
    }
    return R;
}

// Grows one tile (one wave) to its local fixpoint. Returns the face-change mask of the wave (bit f set if
// face f = x-, x+, y-, y+, z-, z+ has changed voxels; with seed_faces, voxels already in the region count).
__device__ unsigned grow_tile3d_bits(const unsigned char* __restrict__ data, unsigned char* __restrict__ region,
                                     int dim, int thr, int bx, int by, int bz, bool seed_faces) {
    const int lane = pcmx::lane_id(), ly = lane & 7, lz = lane >> 3;
    const int x0 = bx * kBX, y = by * kBY + ly, z = bz * kBZ + lz;
    const size_t P = (size_t)dim * dim;
    const bool row_ok = y < dim && z < dim;
    const unsigned long long valid = !row_ok ? 0ull : (dim - x0 >= 64 ? ~0ull : ((1ull << (dim - x0)) - 1));
    unsigned long long R0 = 0, Lx = 0, Lyu = 0, Lzu = 0, ext = 0;
    if (row_ok) {
        const size_t o = (size_t)z * P + (size_t)y * dim + x0;
        const Row64 d = load_row(data + o), r = load_row(region + o);
        R0 = nonzero64(r) & valid;
        // x links: byte i vs byte i+1 (the byte after the row is the x+ halo voxel, or none at the volume edge)
        Row64 sh;
        const int nxt = x0 + 64 < dim ? data[o + 64] : 0;
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const unsigned cur = (unsigned)d.v[c][k];
                const unsigned after = (k < 3) ? (unsigned)d.v[c][k + 1] : (c < 3 ? (unsigned)d.v[c + 1][0] : (unsigned)nxt);
                sh.v[c][k] = (int)((cur >> 8) | (after << 24));
            }
        Lx = similar64(d, sh, thr);  // bit 63 = link to the x+ halo voxel
        if (x0 + 64 < dim && (Lx >> 63) && region[o + 64]) ext |= 1ull << 63;
        Lx &= valid & (valid >> 1);
        if (x0 > 0 && region[o - 1] && abs((int)data[o - 1] - (int)(((unsigned)d.v[0][0]) & 0xff)) < thr) ext |= 1ull;
        // y / z links to the next row (inside the tile or the halo row), and halo rows as external seeds
        if (y + 1 < dim) {
            const Row64 dn = load_row(data + o + dim);
            Lyu = similar64(d, dn, thr) & valid;
            if (ly == kBY - 1) ext |= Lyu & nonzero64(load_row(region + o + dim));
        }
        if (z + 1 < dim) {
            const Row64 dn = load_row(data + o + P);
            Lzu = similar64(d, dn, thr) & valid;
            if (lz == kBZ - 1) ext |= Lzu & nonzero64(load_row(region + o + P));
        }
        if (ly == 0 && y > 0)
            ext |= similar64(d, load_row(data + o - dim), thr) & nonzero64(load_row(region + o - dim)) & valid;
        if (lz == 0 && z > 0)
            ext |= similar64(d, load_row(data + o - P), thr) & nonzero64(load_row(region + o - P)) & valid;
    }
    // links seen from the other side (rows y-1 / z-1 of this tile). The shuffles run on ALL lanes (a lane
    // that is inactive in a cross-lane read does not supply its value), then the edge rows are masked off.
    const unsigned long long Lyd = shfl64(Lyu, (lane + 63) & 63) & (ly > 0 ? ~0ull : 0ull);
    const unsigned long long Lzd = shfl64(Lzu, (lane + 64 - kBY) & 63) & (lz > 0 ? ~0ull : 0ull);
    const unsigned long long Lyi = ly < kBY - 1 ? Lyu : 0ull, Lzi = lz < kBZ - 1 ? Lzu : 0ull;
    unsigned long long R = R0;
    while (true) {
        const unsigned long long old = R;
        const unsigned long long up_y = shfl64(R, (lane + 1) & 63), dn_y = shfl64(R, (lane + 63) & 63);
        const unsigned long long up_z = shfl64(R, (lane + kBY) & 63), dn_z = shfl64(R, (lane + 64 - kBY) & 63);
        R |= ext | (up_y & Lyi) | (dn_y & Lyd) | (up_z & Lzi) | (dn_z & Lzd);
        R = xflood(R, Lx) & valid;
        if (!__any(R != old)) break;
    }
    const unsigned long long mine = R & ~R0;
    if (mine) {  // OR 0x01 bytes into the region row (new voxels were 0 there)
        const size_t o = (size_t)z * P + (size_t)y * dim + x0;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const unsigned b = (unsigned)(mine >> (16 * c)) & 0xffffu;
            if (!b) continue;
            pcmx::i32x4 w;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const unsigned n = b >> (4 * k);
                w[k] = (int)((n & 1u) | ((n & 2u) << 7) | ((n & 4u) << 14) | ((n & 8u) << 21));
            }
            pcmx::i32x4* dst = reinterpret_cast<pcmx::i32x4*>(region + o) + c;
            const pcmx::i32x4 old = *dst;
            *dst = old | w;
        }
    }
    const unsigned long long face = seed_faces ? R : mine;
    unsigned f = 0;
    f |= __any((face & 1ull) != 0) ? 1u : 0u;
    f |= __any((face >> 63) != 0) ? 2u : 0u;
    f |= __any(ly == 0 && face != 0) ? 4u : 0u;
    f |= __any(ly == kBY - 1 && face != 0) ? 8u : 0u;
    f |= __any(lz == 0 && face != 0) ? 16u : 0u;
    f |= __any(lz == kBZ - 1 && face != 0) ? 32u : 0u;
    return f | (__any(mine != 0) ? 64u : 0u);
}

__global__ __launch_bounds__(256) void region3d_bits_kernel(const unsigned char* __restrict__ data,
                                                           unsigned char* __restrict__ region, int dim, int thr,
                                                           int nbx, int nby, int nbz, int epoch,
                                                           Grow3dWs* __restrict__ ws, int* __restrict__ mark,
                                                           int* __restrict__ lists, int ntiles) {
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / 64), lane = pcmx::lane_id();
    const int* list_in = lists + (epoch & 1) * ntiles;
    int* list_out = lists + ((epoch + 1) & 1) * ntiles;
    int* count_out = &ws->count[(epoch + 1) % 3];
    if (blockIdx.x == 0 && threadIdx.x == 0) ws->count[(epoch + 2) % 3] = 0;
    const int n = __hip_atomic_load(&ws->count[epoch % 3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int idx = blockIdx.x * 4 + w; idx < n; idx += gridDim.x * 4) {
        const int t = list_in[idx];
        const int bx = t % nbx, by = (t / nbx) % nby, bz = t / (nbx * nby);
        const unsigned f = grow_tile3d_bits(data, region, dim, thr, bx, by, bz, epoch == 0);
        if ((f & 64u) && lane == 0) ws->flag = 1;
        // faces whose voxels changed: the neighbour across sees new halo voxels next launch
        if (lane >= 1 && lane <= 6 && ((f >> (lane - 1)) & 1u)) {
            const int d = lane;
            const int nx = bx - (d == 1) + (d == 2), ny = by - (d == 3) + (d == 4), nz = bz - (d == 5) + (d == 6);
            if (nx >= 0 && ny >= 0 && nz >= 0 && nx < nbx && ny < nby && nz < nbz)
                push_tile((nz * nby + ny) * nbx + nx, epoch + 1, mark, list_out, count_out);
        }
    }
}

// First work list: every tile holding a region voxel (16 B per thread loads of the region).
constexpr int kSeedThreads = 256;
template <int TX, int TY, int TZ>
__global__ __launch_bounds__(kSeedThreads) void region3d_seed_tiles_kernel(const unsigned char* __restrict__ region, int dim,
                                                                       int nbx, int nby, Grow3dWs* __restrict__ ws,
                                                                       int* __restrict__ mark, int* __restrict__ list0) {
    // one workgroup per (y-row of tiles, z-slab of tiles): 8 x 8 voxel rows of the full x extent
    const int by = blockIdx.x % nby, bz = blockIdx.x / nby;
    const size_t plane = (size_t)dim * dim;
    __shared__ int hit[64];
    if (threadIdx.x < 64) hit[threadIdx.x] = 0;
    __syncthreads();
    const int vecs_per_row = dim / 16;  // dim % 16 == 0 on this path
    for (int i = threadIdx.x; i < TY * TZ * vecs_per_row; i += kSeedThreads) {
        const int v = i % vecs_per_row, yz = i / vecs_per_row;
        const int y = by * TY + yz % TY, z = bz * TZ + yz / TY;
        if (y >= dim || z >= dim) continue;
        const pcmx::i32x4 w = *reinterpret_cast<const pcmx::i32x4*>(region + (size_t)z * plane + (size_t)y * dim + v * 16);
        if ((w.x | w.y | w.z | w.w) != 0) hit[(v * 16) / TX] = 1;
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
    const long long nt = (long long)((dim + kBX - 1) / kBX) * ((dim + kBY - 1) / kBY) * ((dim + kBZ - 1) / kBZ);
    return (long long)sizeof(Grow3dWs) + 3 * nt * 4;
}

// Grows `region` (0 = outside, nonzero = inside) to the 6-connected fixpoint. Host syncs once per `batch`
// launches (a changed-flag read back); launches run on the device-built tile lists in between.
extern "C" int pcmx_region3d_grow_tiled(const unsigned char* data, unsigned char* region, int dim, int thr, void* ws,
                                        int batch, int max_launches, hipStream_t s, int* launches_out) {
    if (dim <= 0 || !ws) return -1;
    if (dim % 16 || (((uintptr_t)region) & 15)) return -1;  // seed scan reads 16-B vectors
    const int nbx = (dim + kBX - 1) / kBX, nby = (dim + kBY - 1) / kBY, nbz = (dim + kBZ - 1) / kBZ;
    if (nbx > 64) return -1;  // seed scan keeps one hit flag per x-tile in a 64-entry LDS array
    const long long nt = (long long)nbx * nby * nbz;
    if (nt > 0x3fffffff) return -1;
    Grow3dWs* w = reinterpret_cast<Grow3dWs*>(ws);
    int* mark = reinterpret_cast<int*>(w + 1);
    int* lists = mark + nt;
    // marks = -1 (no epoch), counters = 0, then the seed tiles (epoch 0) go to list 0
    PCMX_HIP_RET(hipMemsetAsync(w, 0, sizeof(Grow3dWs), s));
    PCMX_HIP_RET(hipMemsetAsync(mark, 0xff, (size_t)nt * 4, s));
    region3d_seed_tiles_kernel<kBX, kBY, kBZ><<<nby * nbz, kSeedThreads, 0, s>>>(region, dim, nbx, nby, w, mark, lists);
    PCMX_HIP_RET(hipGetLastError());
    const int b = batch < 1 ? 8 : batch;
    int launches = 0;
    while (launches < max_launches) {
        PCMX_HIP_RET(hipMemsetAsync(&w->flag, 0, sizeof(int), s));
        for (int i = 0; i < b && launches < max_launches; ++i, ++launches) {
            region3d_bits_kernel<<<kListGrid, 256, 0, s>>>(data, region, dim, thr, nbx, nby, nbz, launches, w, mark,
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
