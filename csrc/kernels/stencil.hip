// 2-D 5-point stencil (explicit heat/Jacobi step) on bf16 grids — north-star config "16384^2 bf16, 8 GPUs
// with halo exchange". Reference ancestor: the 4-neighbour update + 1-cell halo of the distributed region
// growing (ref 2-mpi-region-growing/region.c:250-353, 499-527), promoted to a numeric stencil.
//
//   u'[i][j] = c + k * (((n + s) + (w + e)) - 4c)     c = u[i][j], computed in f32 (no contraction),
//                                                    rounded to bf16 (RNE) on store
// Rows 0 and H-1 of the GLOBAL grid and columns 0 and W-1 are Dirichlet (copied unchanged).
//
// MI355X design (HBM-bound: 2 B read + 2 B write per cell and step):
//  * a wave owns a 512-column strip (8 bf16 = one 16-B load per lane) and marches down 64 rows keeping
//    north/centre/south rows in registers, so every row is fetched from memory once per strip;
//    west/east neighbours come from the adjacent lanes (__shfl), only lanes 0/63 touch the next strip.
//  * workgroup = 4 waves = 512 columns x 256 rows; grid covers the local slab.
//  * the slab layout [halo row | rows | halo row] lets the distributed driver run the same kernel after
//    an RCCL halo exchange, and a row range [r0, r1) lets it split interior and boundary rows so the
//    interior update overlaps the exchange.
#include <hip/hip_bf16.h>
#include "pcmx_common.h"
#include "pcmx_hip.h"

namespace {
constexpr int kStripCols = 512;
constexpr int kRowsPerWave = 64;
constexpr int kWaves = 4;

__device__ __forceinline__ float bf2f(unsigned short h) { return __uint_as_float((unsigned)h << 16); }
__device__ __forceinline__ unsigned short f2bf(float f) {
    unsigned u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (unsigned short)((u >> 16) | 0x40);  // quiet NaN
    u += 0x7fffu + ((u >> 16) & 1u);
    return (unsigned short)(u >> 16);
}

// One fetched row segment: 8 bf16 (one 16-B load) plus, for the strip-edge lanes, the bf16 just outside
// the strip (lane 0: west neighbour, lane 63: east neighbour), fetched together so no load sits on the
// per-row critical path.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
struct RowRaw {
    u32x4 w;
    unsigned short edge;
};

__device__ __forceinline__ float lo(unsigned x) { return __uint_as_float(x << 16); }
__device__ __forceinline__ float hi(unsigned x) { return __uint_as_float(x & 0xffff0000u); }

#pragma clang fp contract(off)
// u, out: [(rows + 2) x ld] slabs; slab row 1+r is local row r; global row of local row r is grow0 + r.
// Each wave marches down its rows keeping north/centre in registers and a ring of kAhead prefetched rows
// in flight (Little's law: one outstanding 16-B load per wave cannot cover HBM latency).
template <int kAhead>
__global__ __launch_bounds__(kWaves * 64) void stencil5_kernel(const unsigned short* __restrict__ u,
                                                               unsigned short* __restrict__ out, int rows, int cols,
                                                               int ld, int r0, int r1, long long grow0,
                                                               long long grows, float k) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int c0 = blockIdx.x * kStripCols + lane * 8;  // first column of this lane
    const int rs = max(r0, (int)(blockIdx.y * (kWaves * kRowsPerWave) + wave * kRowsPerWave));
    const int re = min(r1, (int)(blockIdx.y * (kWaves * kRowsPerWave) + (wave + 1) * kRowsPerWave));
    if (rs >= re) return;
    const bool full = c0 + 8 <= cols;
    const bool has_w = lane == 0 && c0 > 0, has_e = lane == 63 && c0 + 8 < cols;
    if (!full) {  // ragged right edge (cols % 512 != 0): plain per-element path
        for (int r = rs; r < re; ++r) {
            const long long g = grow0 + r;
            const bool fixed_row = g == 0 || g == grows - 1;
            for (int i = 0; i < 8 && c0 + i < cols; ++i) {
                const int col = c0 + i;
                const size_t at = (size_t)(r + 1) * ld + col;
                const float c = bf2f(u[at]);
                float res = c;
                if (!(fixed_row || col == 0 || col == cols - 1)) {
                    const float n = bf2f(u[at - ld]), s = bf2f(u[at + ld]);
                    const float w = bf2f(u[at - 1]), e = bf2f(u[at + 1]);
                    res = c + k * (((n + s) + (w + e)) - 4.0f * c);
                }
                out[at] = f2bf(res);
            }
        }
        return;
    }
    const unsigned short* base = u + c0;
    const int eoff = has_w ? -1 : 8;
    auto fetch = [&](int r) __attribute__((always_inline)) {
        RowRaw x;
        const unsigned short* p = base + (size_t)(r + 1) * ld;
        x.w = *reinterpret_cast<const u32x4*>(p);
        x.edge = (has_w || has_e) ? p[eoff] : (unsigned short)0;
        return x;
    };
    RowRaw north = fetch(rs - 1), cen = fetch(rs);
    RowRaw q[kAhead];
#pragma unroll
    for (int j = 0; j < kAhead; ++j) q[j] = fetch(min(rs + 1 + j, re));
    for (int rb = rs; rb < re; rb += kAhead) {
#pragma unroll
        for (int j = 0; j < kAhead; ++j) {
            const int r = rb + j;
            if (r < re) {
                const RowRaw south = q[j];
                q[j] = fetch(min(r + 1 + kAhead, re));
                float cv[8], nv[8], sv[8];
                const unsigned cw[4] = {cen.w.x, cen.w.y, cen.w.z, cen.w.w};
                const unsigned nw[4] = {north.w.x, north.w.y, north.w.z, north.w.w};
                const unsigned sw[4] = {south.w.x, south.w.y, south.w.z, south.w.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    cv[2 * i] = lo(cw[i]), cv[2 * i + 1] = hi(cw[i]);
                    nv[2 * i] = lo(nw[i]), nv[2 * i + 1] = hi(nw[i]);
                    sv[2 * i] = lo(sw[i]), sv[2 * i + 1] = hi(sw[i]);
                }
                // neighbours across lanes: west of element 0 is the previous lane's element 7
                float west = __shfl_up(cv[7], 1, 64);
                float east = __shfl_down(cv[0], 1, 64);
                if (has_w) west = bf2f(cen.edge);
                if (has_e) east = bf2f(cen.edge);
                const long long g = grow0 + r;
                const bool fixed_row = g == 0 || g == grows - 1;
                unsigned short o[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const float c = cv[i];
                    const float w = i == 0 ? west : cv[i - 1];
                    const float e = i == 7 ? east : cv[i + 1];
                    const int col = c0 + i;
                    float res = c + k * (((nv[i] + sv[i]) + (w + e)) - 4.0f * c);
                    if (fixed_row || col == 0 || col == cols - 1) res = c;
                    o[i] = f2bf(res);
                }
                u32x4 pk;
                pk.x = o[0] | ((unsigned)o[1] << 16);
                pk.y = o[2] | ((unsigned)o[3] << 16);
                pk.z = o[4] | ((unsigned)o[5] << 16);
                pk.w = o[6] | ((unsigned)o[7] << 16);
                __builtin_nontemporal_store(pk, reinterpret_cast<u32x4*>(out + (size_t)(r + 1) * ld + c0));
                north = cen;
                cen = south;
            }
        }
    }
}
#pragma clang fp contract(on)
}  // namespace

// One step over local rows [r0, r1) of a slab with `rows` local rows (slab has rows+2 rows of pitch ld).
extern "C" int pcmx_stencil5_bf16(const void* u, void* out, int rows, int cols, int ld, int r0, int r1,
                                  long long global_row0, long long global_rows, float k, hipStream_t s) {
    if (rows <= 0 || cols <= 0 || ld < cols || (ld & 7) || (cols & 7) || (((uintptr_t)u | (uintptr_t)out) & 15))
        return -1;
    r0 = max(r0, 0);
    r1 = min(r1, rows);
    if (r0 >= r1) return 0;
    dim3 grid((cols + kStripCols - 1) / kStripCols, (rows + kWaves * kRowsPerWave - 1) / (kWaves * kRowsPerWave));
    stencil5_kernel<8><<<grid, kWaves * 64, 0, s>>>((const unsigned short*)u, (unsigned short*)out, rows, cols, ld, r0, r1,
                                                  global_row0, global_rows, k);
    return (int)hipGetLastError();
}
