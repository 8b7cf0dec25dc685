// Region growing on MI355X: 2-D (ref 2-mpi-region-growing/region.c:493-533, 4-connected, |a-b| < thr
// between ADJACENT pixels, seeded flood fill) and 3-D (ref 5-cuda-region-growing/raycast.cu:534-699,
// 6-connected).
//
// MI355X design
//  * Tiled local fixpoint, so one launch advances the front across a whole tile instead of one cell (the
//    naive kernel of raycast.cu:534 needs one launch per BFS level: 249 launches, 61 ms at 512^3).
//    2-D: BIT-PARALLEL one-wave 64x64 tiles (a lane holds a 64-pixel row word; Kogge-Stone closures along
//    rows and, by shuffles, along columns), 4x4 tiles per workgroup exchanging borders through LDS. 3-D:
//    BIT-PARALLEL one-wave tiles of 64x8x8 — a lane holds one 64-voxel row as
//    a 64-bit mask, similarity to the x / y / z neighbours as link masks, and a sweep is a few 64-bit ops
//    plus cross-lane shuffles (a front crosses a whole row per sweep; no LDS, no barriers): 0.52 ms of
//    kernels per 512^3 grow (the 32x8x8 LDS-tile version took 1.47 ms), 0.63 ms with the host loop
//    (fixpoint_pipelined: the changed-flag check of a batch overlaps the next batch).
//  * Active-tile worklist: a tile only runs if a face neighbour changed in the previous launch. 2-D:
//    act_in -> act_out flags over the block grid (self-cleaning, no memset between launches). 3-D (32k tiles at 512^3): a compacted device-built list
//    walked by a persistent grid, so a launch costs the frontier, not a full-volume dispatch.
//  * Halo cells are read-only inputs. That makes the same kernel the compute step of the distributed
//    version: a rank's halo holds its neighbours' boundary after an RCCL exchange (parallel/region2d.py).
//  * Region state is 0/1 (a cell never leaves the region), so races between tiles are benign and the
//    fixpoint equals the serial flood fill.
#include "pcmx_common.h"
#include "pcmx_hip.h"

namespace {

// ----------------------------------------------------------------------------------------------- 2-D
// Bit-parallel: the padded (H+2) x (W+2) grid is held as 64-bit words (row y, word x = columns 64x..64x+63):
// rb = region bits, hl = "pixel c is similar to c+1" links, vl = "pixel (y,c) is similar to (y+1,c)" links
// (built once per grow by region2d_bits_prep_kernel). A wave owns a 64-row x 1-word tile (lane = row); a
// 16-wave workgroup owns a 4 x 4 block of tiles (256 x 256 pixels) whose words it keeps in LDS. A sweep is a
// Kogge-Stone closure along the row (6 shift/and steps each way: a front crosses any horizontal run in one
// sweep) and along the column across lanes (6 shuffle steps each way), repeated to the tile fixpoint (wave
// ballot, no barrier), then tiles exchange borders through LDS until the block is stable (one barrier per
// round). Blocks exchange borders between launches; a block runs only if a neighbour's border changed.
// Halo cells (row 0 / H+1, column 0 / W+1) are read-only seeds: nothing propagates INTO or THROUGH them.
constexpr int kB2 = 4;                   // tiles per block edge
constexpr int kWaves2 = kB2 * kB2;       // one wave per tile
constexpr int kThreads2 = kWaves2 * 64;  // 1024

typedef unsigned long long u64;

__device__ __forceinline__ u64 shfl_up64(u64 v, int k) {
    const int l = pcmx::lane_id();
    const u64 t = __shfl_up(v, (unsigned)k, 64);
    return l >= k ? t : 0ull;
}
__device__ __forceinline__ u64 shfl_down64(u64 v, int k) {
    const int l = pcmx::lane_id();
    const u64 t = __shfl_down(v, (unsigned)k, 64);
    return l + k < 64 ? t : 0ull;
}

// interior bits of word x in row y: columns 1..W of rows 1..H
__device__ __forceinline__ u64 interior_mask(int y, int x, int H, int W) {
    if (y < 1 || y > H) return 0ull;
    const int c0 = 64 * x, lo = c0 < 1 ? 1 - c0 : 0, hi = W - c0;  // bits lo..hi
    if (hi < lo) return 0ull;
    const u64 upto = hi >= 63 ? ~0ull : ((1ull << (hi + 1)) - 1);
    return upto & (~0ull << lo);
}

// One wave per (row y, word x): lane = column bit. Builds rb/hl/vl with ballots.
__global__ __launch_bounds__(256) void region2d_bits_prep_kernel(const unsigned char* __restrict__ img,
                                                                const unsigned char* __restrict__ region, int R, int C,
                                                                int ld, int nw, int thr, u64* __restrict__ rb,
                                                                u64* __restrict__ hl, u64* __restrict__ vl) {
    const long long wid = ((long long)blockIdx.x * 256 + threadIdx.x) >> 6;
    if (wid >= (long long)R * nw) return;
    const int y = (int)(wid / nw), x = (int)(wid % nw);
    const int c = 64 * x + pcmx::lane_id();
    bool r = false, h = false, v = false;
    if (c < C) {
        const int a = img[(size_t)y * ld + c];
        r = region[(size_t)y * ld + c] != 0;
        if (c + 1 < C) h = abs(a - (int)img[(size_t)y * ld + c + 1]) < thr;
        if (y + 1 < R) v = abs(a - (int)img[(size_t)(y + 1) * ld + c]) < thr;
    }
    const u64 br = __ballot(r), bh = __ballot(h), bv = __ballot(v);
    if (pcmx::lane_id() == 0) rb[wid] = br, hl[wid] = bh, vl[wid] = bv;
}

// New interior bits back to the byte region (only 0 -> 1 writes).
__global__ __launch_bounds__(256) void region2d_bits_store_kernel(unsigned char* __restrict__ region, int H, int W,
                                                                 int ld, int nw, const u64* __restrict__ rb) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= (long long)H * W) return;
    const int y = 1 + (int)(i / W), c = 1 + (int)(i % W);
    if ((rb[(size_t)y * nw + (c >> 6)] >> (c & 63)) & 1ull) {
        unsigned char* p = region + (size_t)y * ld + c;
        if (!*p) *p = 1;
    }
}

__global__ __launch_bounds__(kThreads2) void region2d_bits_kernel(u64* __restrict__ rb, const u64* __restrict__ hl,
                                                                 const u64* __restrict__ vl, int R, int H, int W,
                                                                 int nw, int* __restrict__ act_in,
                                                                 int* __restrict__ act_out, int* __restrict__ flag) {
    const int nbx = gridDim.x, bxi = blockIdx.x, byi = blockIdx.y, bid = byi * nbx + bxi;
    if (act_in[bid] == 0) return;
    __shared__ u64 sr[kB2 * 64][kB2];  // the block's region words, [row][word]
    __shared__ int any_change;
    const int lane = pcmx::lane_id(), wave = threadIdx.x >> 6;
    const int wy = wave / kB2, wx = wave % kB2;
    const int y = (byi * kB2 + wy) * 64 + lane, x = bxi * kB2 + wx;
    const int ly = wy * 64 + lane;
    const bool valid = y < R && x < nw;
    const size_t at = (size_t)y * nw + x;
    const u64 im = valid ? interior_mask(y, x, H, W) : 0ull;
    const u64 h = valid ? hl[at] : 0ull;
    const u64 v = valid ? vl[at] : 0ull;                                  // row y <-> y+1
    u64 vup = shfl_up64(v, 1);                                              // row y-1 <-> y
    if (lane == 0 && valid && y > 0) vup = vl[at - nw];
    const u64 hleft = (valid && x > 0) ? hl[at - 1] : 0ull;                 // bit 63: column 64x-1 <-> 64x
    // receive masks (only interior cells receive)
    const u64 E = (h << 1) & im;                                            // x <- x-1
    const u64 Wm = h & im;                                                  // x <- x+1 (bit 63: from next word)
    const u64 D = vup & im;                                                 // from the row above
    const u64 U = v & im;                                                   // from the row below
    const bool in_l = (hleft >> 63) & im & 1ull, in_r = (h >> 63) & (im >> 63) & 1ull;
    // words outside the block (fixed during this launch): left/right neighbours per row, rows above/below
    const bool bl = wx == 0, br = wx == kB2 - 1, bt = wy == 0, bb = wy == kB2 - 1;
    const u64 ext_l = (bl && valid && x > 0) ? rb[at - 1] : 0ull;
    const u64 ext_r = (br && valid && x + 1 < nw) ? rb[at + 1] : 0ull;
    const u64 ext_t = (bt && lane == 0 && valid && y > 0) ? rb[at - nw] : 0ull;
    const u64 ext_b = (bb && lane == 63 && x < nw && y + 1 < R) ? rb[at + nw] : 0ull;
    const u64 r0 = valid ? rb[at] : 0ull;
    u64 r = r0;
    sr[ly][wx] = r;
    __syncthreads();
    for (;;) {
        // seeds from the 4 neighbour tiles (LDS inside the block, launch-start values outside)
        const u64 nl = bl ? ext_l : sr[ly][wx - 1];
        const u64 nr = br ? ext_r : sr[ly][wx + 1];
        u64 nt = 0ull, nb = 0ull;
        if (lane == 0) nt = bt ? ext_t : sr[ly - 1][wx];
        if (lane == 63) nb = bb ? ext_b : sr[ly + 1][wx];
        u64 g = r | (in_l && (nl >> 63) ? 1ull : 0ull) | (in_r && (nr & 1ull) ? (1ull << 63) : 0ull) | (nt & D) | (nb & U);
        const u64 start = r;
        for (;;) {
            const u64 before = g;
            u64 p = E;  // along the row, towards higher bits
            g |= (g << 1) & p, p &= p << 1;
            g |= (g << 2) & p, p &= p << 2;
            g |= (g << 4) & p, p &= p << 4;
            g |= (g << 8) & p, p &= p << 8;
            g |= (g << 16) & p, p &= p << 16;
            g |= (g << 32) & p;
            p = Wm & ~(1ull << 63);  // towards lower bits (bit 63's link leads out of the word)
            g |= (g >> 1) & p, p &= p >> 1;
            g |= (g >> 2) & p, p &= p >> 2;
            g |= (g >> 4) & p, p &= p >> 4;
            g |= (g >> 8) & p, p &= p >> 8;
            g |= (g >> 16) & p, p &= p >> 16;
            g |= (g >> 32) & p;
            p = D;  // down the column (across lanes)
#pragma unroll
            for (int k = 1; k < 64; k <<= 1) {
                g |= shfl_up64(g, k) & p;
                p &= shfl_up64(p, k);
            }
            p = U;  // up the column
#pragma unroll
            for (int k = 1; k < 64; k <<= 1) {
                g |= shfl_down64(g, k) & p;
                p &= shfl_down64(p, k);
            }
            if (!__any(g != before)) break;
        }
        r = g;
        const int changed = r != start;
        __syncthreads();  // everyone has read the neighbours' words of this round
        sr[ly][wx] = r;
        if (!__syncthreads_or(changed)) break;
    }
    // publish: changed words, then activate the neighbour blocks whose shared border changed
    const u64 diff = r ^ r0;
    if (valid && diff) rb[at] = r;
    const bool cl = bl && __any(diff & 1ull), cr = br && __any(diff >> 63), ct = bt && __any(lane == 0 && diff),
               cb = bb && __any(lane == 63 && diff), cany = __any(diff != 0ull);
    if (threadIdx.x == 0) any_change = 0;
    __syncthreads();
    if (lane == 0) {
        if (cany) atomicOr(&any_change, 1);
        if (cl && bxi > 0) act_out[bid - 1] = 1;
        if (cr && bxi + 1 < nbx) act_out[bid + 1] = 1;
        if (ct && byi > 0) act_out[bid - nbx] = 1;
        if (cb && byi + 1 < (int)gridDim.y) act_out[bid + nbx] = 1;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        act_in[bid] = 0;  // self-cleaning: this array is the next-but-one launch's act_out
        if (any_change) *flag = 1;  // (the block itself is at its fixpoint: only neighbours re-activate it)
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
    int flags[4];  // "a tile changed" flag of each batch in flight (fixpoint_pipelined ring)
    int count[3];
    int pad;
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
// Volume = dim (x) x dim (y) x nz (z) planes; with halo_lo / halo_hi the planes -1 / nz are readable (a z-slab's
// halo planes: read-only external seeds, never grown).
__device__ unsigned grow_tile3d_bits(const unsigned char* __restrict__ data, unsigned char* __restrict__ region,
                                     int dim, int nz, bool halo_lo, bool halo_hi, int thr, int bx, int by, int bz,
                                     bool seed_faces) {
    const int lane = pcmx::lane_id(), ly = lane & 7, lz = lane >> 3;
    const int x0 = bx * kBX, y = by * kBY + ly, z = bz * kBZ + lz;
    const size_t P = (size_t)dim * dim;
    const bool row_ok = y < dim && z < nz;
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
        if (z + 1 < nz || (halo_hi && z + 1 == nz)) {
            const Row64 dn = load_row(data + o + P);
            Lzu = similar64(d, dn, thr) & valid;
            if (lz == kBZ - 1 || z + 1 == nz) ext |= Lzu & nonzero64(load_row(region + o + P));
        }
        if (ly == 0 && y > 0)
            ext |= similar64(d, load_row(data + o - dim), thr) & nonzero64(load_row(region + o - dim)) & valid;
        if (lz == 0 && (z > 0 || halo_lo))
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
                                                           unsigned char* __restrict__ region, int dim, int nz,
                                                           int halos, int thr, int nbx, int nby, int nbz, int epoch,
                                                           Grow3dWs* __restrict__ ws, int* __restrict__ mark,
                                                           int* __restrict__ lists, int ntiles, int* __restrict__ flag) {
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / 64), lane = pcmx::lane_id();
    const int* list_in = lists + (epoch & 1) * ntiles;
    int* list_out = lists + ((epoch + 1) & 1) * ntiles;
    int* count_out = &ws->count[(epoch + 1) % 3];
    if (blockIdx.x == 0 && threadIdx.x == 0) ws->count[(epoch + 2) % 3] = 0;
    const int n = __hip_atomic_load(&ws->count[epoch % 3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int idx = blockIdx.x * 4 + w; idx < n; idx += gridDim.x * 4) {
        const int t = list_in[idx];
        const int bx = t % nbx, by = (t / nbx) % nby, bz = t / (nbx * nby);
        const unsigned f = grow_tile3d_bits(data, region, dim, nz, halos & 1, halos & 2, thr, bx, by, bz, epoch == 0);
        if ((f & 64u) && lane == 0) *flag = 1;
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
// With halo planes, a tile of the first / last z-layer also scans the halo plane next to it (its region voxels
// seed that tile); every tile also scans one plane beyond each of its z-faces, which at worst seeds a neighbour
// of a region tile (harmless extra work).
template <int TX, int TY, int TZ>
__global__ __launch_bounds__(kSeedThreads) void region3d_seed_tiles_kernel(const unsigned char* __restrict__ region, int dim,
                                                                       int nz, int halos, int nbx, int nby,
                                                                       Grow3dWs* __restrict__ ws,
                                                                       int* __restrict__ mark, int* __restrict__ list0) {
    // one workgroup per (y-row of tiles, z-slab of tiles): 8 x (8 + 2) voxel rows of the full x extent
    const int by = blockIdx.x % nby, bz = blockIdx.x / nby;
    const size_t plane = (size_t)dim * dim;
    __shared__ int hit[64];
    if (threadIdx.x < 64) hit[threadIdx.x] = 0;
    __syncthreads();
    const int vecs_per_row = dim / 16;  // dim % 16 == 0 on this path
    const int zmin = (halos & 1) ? -1 : 0, zmax = (halos & 2) ? nz : nz - 1;
    for (int i = threadIdx.x; i < TY * (TZ + 2) * vecs_per_row; i += kSeedThreads) {
        const int v = i % vecs_per_row, yz = i / vecs_per_row;
        const int y = by * TY + yz % TY, z = bz * TZ - 1 + yz / TY;
        if (y >= dim || z < zmin || z > zmax) continue;
        const pcmx::i32x4 w = *reinterpret_cast<const pcmx::i32x4*>(region + (long long)z * (long long)plane +
                                                                    (size_t)y * dim + v * 16);
        if ((w.x | w.y | w.z | w.w) != 0) hit[(v * 16) / TX] = 1;
    }
    __syncthreads();
    if (threadIdx.x < nbx && hit[threadIdx.x]) {
        const int t = (bz * nby + by) * nbx + threadIdx.x;
        push_tile(t, 0, mark, list0, &ws->count[0]);
    }
}

// Naive frontier kernel with the reference's 0/1/2 states (raycast.cu:534-574, region.cl:34-73): a voxel holding 2
// becomes 1 and marks its similar 0-neighbours 2 (benign races, as in the reference: writes are monotone 0 -> 2 -> 1
// and the flag is idempotent). Bounds-checked (B19 fixed). A lane owns 16 consecutive voxels and reads their region
// bytes as ONE 16-B load; a lane without a 2 among them (all but the few on the frontier) is done, so a launch streams
// the 128 MiB region once at HBM speed instead of issuing one byte load per voxel (the reference's one work-item per
// voxel: 177 us per launch at 512^3 through the AMD OpenCL runtime on MI355X, profiles/r5_refbase/; our earlier
// one-lane-per-voxel form 225 us).
constexpr int kNaiveVox = 16;
__device__ __forceinline__ bool has_byte2(unsigned v) {
    v ^= 0x02020202u;  // a byte equal to 2 becomes 0
    return ((v - 0x01010101u) & ~v & 0x80808080u) != 0;
}
__global__ __launch_bounds__(256) void region3d_step_kernel(const unsigned char* __restrict__ data,
                                                           unsigned char* __restrict__ region, int dim, int thr,
                                                           int* __restrict__ unfinished) {
    const long long plane = (long long)dim * dim, total = plane * dim;
    const long long i0 = ((long long)blockIdx.x * 256 + threadIdx.x) * kNaiveVox;
    if (i0 >= total) return;
    unsigned w[4] = {0u, 0u, 0u, 0u};
    if (i0 + kNaiveVox <= total) {  // (region is 16-B aligned: checked by the launcher)
        const uint4 q = *reinterpret_cast<const uint4*>(region + i0);
        w[0] = q.x, w[1] = q.y, w[2] = q.z, w[3] = q.w;
    } else {
        for (int b = 0; b < (int)(total - i0); ++b) w[b >> 2] |= (unsigned)region[i0 + b] << (8 * (b & 3));
    }
    if (!(has_byte2(w[0]) || has_byte2(w[1]) || has_byte2(w[2]) || has_byte2(w[3]))) return;
    const int dx[6] = {-1, 1, 0, 0, 0, 0}, dy[6] = {0, 0, -1, 1, 0, 0}, dz[6] = {0, 0, 0, 0, -1, 1};
    for (int b = 0; b < kNaiveVox; ++b) {
        if (((w[b >> 2] >> (8 * (b & 3))) & 0xffu) != 2u) continue;
        const long long i = i0 + b;
        const int z = (int)(i / plane), y = (int)((i / dim) % dim), x = (int)(i % dim);
        *unfinished = 1;
        region[i] = 1;
        const int v = data[i];
#pragma unroll
        for (int n = 0; n < 6; ++n) {
            const int cx = x + dx[n], cy = y + dy[n], cz = z + dz[n];
            if (cx < 0 || cy < 0 || cz < 0 || cx >= dim || cy >= dim || cz >= dim) continue;
            const long long j = (long long)cz * plane + (long long)cy * dim + cx;
            if (region[j] == 0 && abs(v - (int)data[j]) < thr) region[j] = 2;
        }
    }
}

}  // namespace

namespace {

// Host side of the iterate-to-fixpoint loops. A batch of launches sets a device flag when anything changed; the
// fixpoint is the first batch that changed nothing. Instead of a blocking read-back per batch (the GPU idled
// ~40 us per batch behind the host's copy + sync round trip), the NEXT batch is enqueued before the host waits
// for the current one's flag: each batch owns a flag slot (ring of kFixRing), its flag is copied into pinned
// host memory and an event is recorded; the GPU always has the next batch queued, and after convergence at most
// one speculative batch runs, whose launches find an empty worklist and exit.
constexpr int kFixRing = 4;
struct FixpointHost {
    int* pinned = nullptr;
    hipEvent_t ev[kFixRing] = {};
    unsigned pending = 0;  // slots whose copy may still be in flight from an earlier call
    bool ready = false;
};
FixpointHost* fixpoint_host() {
    constexpr int kMaxDev = 64;
    thread_local FixpointHost hosts[kMaxDev];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return nullptr;
    FixpointHost& h = hosts[dev];
    if (!h.ready) {
        if (hipHostMalloc(reinterpret_cast<void**>(&h.pinned), kFixRing * sizeof(int), hipHostMallocPortable) != hipSuccess)
            return nullptr;
        for (int i = 0; i < kFixRing; ++i)
            if (hipEventCreateWithFlags(&h.ev[i], hipEventDisableTiming) != hipSuccess) return nullptr;
        h.ready = true;
    }
    for (int i = 0; i < kFixRing; ++i)  // a speculative batch of the previous call may still be copying
        if (h.pending & (1u << i)) (void)hipEventSynchronize(h.ev[i]);
    h.pending = 0;
    return &h;
}

// launch(n, dflag, first) enqueues n launches (global launch indices first..first+n-1) that raise *dflag on a
// change; dflags: kFixRing device ints. Returns 0 at the fixpoint, PCMX_ERR_NOT_CONVERGED when max_launches ran
// out with the last batch still changing; *launches_out = launches up to the confirming batch.
template <class Launch>
int fixpoint_pipelined(hipStream_t s, int* dflags, int batch, int max_launches, Launch&& launch, int* launches_out) {
    FixpointHost* H = fixpoint_host();
    if (!H) return PCMX_ERR_ARG;
    int launched = 0, confirmed = 0, head = 0, tail = 0, len[kFixRing] = {};
    bool converged = false;
    while (true) {
        while (head - tail < 2 && launched < max_launches) {  // keep two batches queued
            const int slot = head % kFixRing, n = batch < max_launches - launched ? batch : max_launches - launched;
            PCMX_HIP_RET(hipMemsetAsync(&dflags[slot], 0, sizeof(int), s));
            if (const int lrc = launch(n, &dflags[slot], launched)) return lrc;
            PCMX_HIP_RET(hipMemcpyAsync(&H->pinned[slot], &dflags[slot], sizeof(int), hipMemcpyDeviceToHost, s));
            PCMX_HIP_RET(hipEventRecord(H->ev[slot], s));
            H->pending |= 1u << slot;
            launched += n, len[slot] = n, ++head;
        }
        if (tail == head) break;
        const int slot = tail % kFixRing;
        PCMX_HIP_RET(hipEventSynchronize(H->ev[slot]));
        H->pending &= ~(1u << slot);
        confirmed += len[slot], ++tail;
        if (H->pinned[slot] == 0) {
            converged = true;
            break;
        }
    }
    if (launches_out) *launches_out = confirmed;
    return converged ? 0 : PCMX_ERR_NOT_CONVERGED;
}

struct Region2dGeom {
    int R, C, nw, nbx, nby;
    long long words, nblocks;
};
Region2dGeom region2d_geom(int H, int W) {
    Region2dGeom g;
    g.R = H + 2, g.C = W + 2, g.nw = (g.C + 63) / 64;
    g.nbx = (g.nw + kB2 - 1) / kB2, g.nby = ((g.R + 63) / 64 + kB2 - 1) / kB2;
    g.words = (long long)g.R * g.nw, g.nblocks = (long long)g.nbx * g.nby;
    return g;
}
}  // namespace

extern "C" long long pcmx_region2d_workspace_bytes(int H, int W) {
    const Region2dGeom g = region2d_geom(H, W);
    return 64 + ((2 * g.nblocks * 4 + 7) / 8) * 8 + 3 * g.words * 8;
}

// ws: [flag ring (16 ints) | act0 | act1 | rb | hl | vl]. Batches of `batch` launches, pipelined fixpoint check.
extern "C" int pcmx_region2d_grow(const unsigned char* img, unsigned char* region, int H, int W, int ld, int thr,
                                  void* ws, int batch, int max_launches, hipStream_t s, int* launches_out) {
    if (H <= 0 || W <= 0 || ld < W + 2 || !ws || ((uintptr_t)ws & 7)) return PCMX_ERR_ARG;
    const Region2dGeom g = region2d_geom(H, W);
    int* flag = reinterpret_cast<int*>(ws);
    int* act[2] = {flag + 16, flag + 16 + g.nblocks};
    u64* rb = reinterpret_cast<u64*>((char*)ws + 64 + ((2 * g.nblocks * 4 + 7) / 8) * 8);
    u64* hl = rb + g.words;
    u64* vl = hl + g.words;
    const long long prep_threads = g.words * 64;
    region2d_bits_prep_kernel<<<(unsigned)((prep_threads + 255) / 256), 256, 0, s>>>(img, region, g.R, g.C, ld, g.nw,
                                                                                    thr, rb, hl, vl);
    PCMX_HIP_RET(hipGetLastError());
    PCMX_HIP_RET(hipMemsetAsync(act[0], 0x01, g.nblocks * sizeof(int), s));  // every block runs first (nonzero)
    PCMX_HIP_RET(hipMemsetAsync(act[1], 0, g.nblocks * sizeof(int), s));
    const dim3 grid(g.nbx, g.nby);
    if (batch < 1) batch = 4;
    const int rc = fixpoint_pipelined(
        s, flag, batch, max_launches,
        [&](int n, int* f, int first) {
            for (int b = 0; b < n; ++b) {  // act lists alternate by global launch index
                const int cur = (first + b) & 1;
                region2d_bits_kernel<<<grid, kThreads2, 0, s>>>(rb, hl, vl, g.R, H, W, g.nw, act[cur], act[cur ^ 1], f);
            }
            return (int)hipGetLastError();
        },
        launches_out);
    if (rc != 0 && rc != PCMX_ERR_NOT_CONVERGED) return rc;
    region2d_bits_store_kernel<<<(unsigned)(((long long)H * W + 255) / 256), 256, 0, s>>>(region, H, W, ld, g.nw, rb);
    PCMX_HIP_RET(hipGetLastError());
    // NOT_CONVERGED: the last batch still changed something, the fixpoint was not confirmed (the region is partial)
    return rc;
}

extern "C" long long pcmx_region3d_slab_workspace_bytes(int dim, int nz) {
    const long long nt = (long long)((dim + kBX - 1) / kBX) * ((dim + kBY - 1) / kBY) * ((nz + kBZ - 1) / kBZ);
    return (long long)sizeof(Grow3dWs) + 3 * nt * 4;
}

extern "C" long long pcmx_region3d_workspace_bytes(int dim) { return pcmx_region3d_slab_workspace_bytes(dim, dim); }

// Grows `region` (0 = outside, nonzero = inside) to the 6-connected fixpoint over dim x dim x nz planes. halos bit 0
// / bit 1: plane -1 / plane nz exist (read-only seeds of a z-slab). Launches run on the device-built tile lists
// in batches of `batch`; the changed-flag check of batch k overlaps batch k+1 (fixpoint_pipelined).
extern "C" int pcmx_region3d_grow_slab(const unsigned char* data, unsigned char* region, int dim, int nz, int halos,
                                       int thr, void* ws, int batch, int max_launches, hipStream_t s,
                                       int* launches_out) {
    if (dim <= 0 || nz <= 0 || !ws || halos < 0 || halos > 3) return PCMX_ERR_ARG;
    if (dim % 16 || (((uintptr_t)region) & 15) || (((size_t)dim * dim) & 15)) return PCMX_ERR_ARG;  // 16-B seed scan
    const int nbx = (dim + kBX - 1) / kBX, nby = (dim + kBY - 1) / kBY, nbz = (nz + kBZ - 1) / kBZ;
    if (nbx > 64) return PCMX_ERR_ARG;  // seed scan keeps one hit flag per x-tile in a 64-entry LDS array
    const long long nt = (long long)nbx * nby * nbz;
    if (nt > 0x3fffffff) return PCMX_ERR_ARG;
    Grow3dWs* w = reinterpret_cast<Grow3dWs*>(ws);
    int* mark = reinterpret_cast<int*>(w + 1);
    int* lists = mark + nt;
    // marks = -1 (no epoch), counters = 0, then the seed tiles (epoch 0) go to list 0
    PCMX_HIP_RET(hipMemsetAsync(w, 0, sizeof(Grow3dWs), s));
    PCMX_HIP_RET(hipMemsetAsync(mark, 0xff, (size_t)nt * 4, s));
    region3d_seed_tiles_kernel<kBX, kBY, kBZ><<<nby * nbz, kSeedThreads, 0, s>>>(region, dim, nz, halos, nbx, nby, w,
                                                                                mark, lists);
    PCMX_HIP_RET(hipGetLastError());
    const int b = batch < 1 ? 8 : batch;
    return fixpoint_pipelined(
        s, w->flags, b, max_launches,
        [&](int n, int* f, int first) {
            for (int i = 0; i < n; ++i)  // launch index = list epoch
                region3d_bits_kernel<<<kListGrid, 256, 0, s>>>(data, region, dim, nz, halos, thr, nbx, nby, nbz,
                                                             first + i, w, mark, lists, (int)nt, f);
            return (int)hipGetLastError();
        },
        launches_out);
}

extern "C" int pcmx_region3d_grow_tiled(const unsigned char* data, unsigned char* region, int dim, int thr, void* ws,
                                        int batch, int max_launches, hipStream_t s, int* launches_out) {
    return pcmx_region3d_grow_slab(data, region, dim, dim, 0, thr, ws, batch, max_launches, s, launches_out);
}

extern "C" int pcmx_region3d_grow_naive(const unsigned char* data, unsigned char* region, int dim, int thr, int* flag_ws,
                                        int max_launches, hipStream_t s, int* launches_out) {
    if (dim <= 0 || !flag_ws || ((uintptr_t)region & 15)) return PCMX_ERR_ARG;
    const long long groups = ((long long)dim * dim * dim + kNaiveVox - 1) / kNaiveVox;
    const unsigned grid = (unsigned)((groups + 255) / 256);
    // one launch per BFS level as in the reference, but the host checks the changed flag once per batch of 8 launches
    // with the next batch already queued (fixpoint_pipelined; flag_ws holds its kFixRing = 4 flag slots) instead of a
    // blocking read-back after every launch (the reference's clFinish + read per level)
    return fixpoint_pipelined(
        s, flag_ws, 8, max_launches,
        [&](int n, int* f, int) {
            for (int i = 0; i < n; ++i) region3d_step_kernel<<<grid, 256, 0, s>>>(data, region, dim, thr, f);
            return (int)hipGetLastError();
        },
        launches_out);
}
