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
//    west/east neighbours come from the adjacent lanes (DPP wave shifts), only lanes 0/63 touch the next strip.
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
// f32 -> bf16 round-to-nearest-even on the gfx950 converter (v_cvt_pk_bf16_f32: two values per instruction,
// no branches; bit-identical to the RNE rounding of torch's .to(bfloat16) for finite values)
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned pack2bf(float a, float b) {
    const f32x2 v = {a, b};
    return __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2));
}
__device__ __forceinline__ unsigned short f2bf(float f) { return (unsigned short)(pack2bf(f, 0.f) & 0xffffu); }

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
                float west = pcmx::wave_from_prev(cv[7]);
                float east = pcmx::wave_from_next(cv[0]);
                if (has_w) west = bf2f(cen.edge);
                if (has_e) east = bf2f(cen.edge);
                const long long g = grow0 + r;
                const bool fixed_row = g == 0 || g == grows - 1;
                float o[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const float c = cv[i];
                    const float w = i == 0 ? west : cv[i - 1];
                    const float e = i == 7 ? east : cv[i + 1];
                    const int col = c0 + i;
                    const float res = c + k * (((nv[i] + sv[i]) + (w + e)) - 4.0f * c);
                    o[i] = (fixed_row || col == 0 || col == cols - 1) ? c : res;
                }
                u32x4 pk;
                pk.x = pack2bf(o[0], o[1]);
                pk.y = pack2bf(o[2], o[3]);
                pk.z = pack2bf(o[4], o[5]);
                pk.w = pack2bf(o[6], o[7]);
                __builtin_nontemporal_store(pk, reinterpret_cast<u32x4*>(out + (size_t)(r + 1) * ld + c0));
                north = cen;
                cen = south;
            }
        }
    }
}
// ---------------------------------------------------------------- T fused time steps (temporal blocking)
// u -> s1 -> ... -> sT in one pass: every cell is read and written once per T updates (2 B + 2 B per cell
// instead of 4T B), bit-identical to T single steps because every intermediate level is rounded to bf16
// exactly as a stored step would be.
//  * OVERLAPPING STRIPS: a wave loads 512 columns starting 8 columns left of its strip and keeps a T-level
//    register pipeline; the values of lane 0 / lane 63 go stale one column per level (their outer neighbour
//    is not loaded), so after T <= 8 levels lanes 1..62 are exact and only they store: a 496-column output
//    strip per wave, 3% redundant loads, no per-edge special cases.
//  * ROW PIPELINE: each new u row i feeds level 1 row i-1, level 2 row i-2, ..., level T row i-T (stored).
//    Level t keeps its last two rows as floats (already bf16-rounded); rows below the needed range are
//    computed from zero-initialised windows and never reach a stored value.
//  * Slab: (rows + 2*halo) x ld, local row r at slab row r + halo. Rows within T of a rank boundary read T
//    halo rows (halo >= T, checked by the launcher); at a GLOBAL edge the clamped rows only feed Dirichlet rows.
constexpr int kOutCols = kStripCols - 16;  // 496 output columns per wave strip

__device__ __forceinline__ void unpack8(const u32x4& w, float (&v)[8]) {
    v[0] = lo(w.x), v[1] = hi(w.x), v[2] = lo(w.y), v[3] = hi(w.y);
    v[4] = lo(w.z), v[5] = hi(w.z), v[6] = lo(w.w), v[7] = hi(w.w);
}

// one update of a lane's 8 columns (rounded to bf16, returned packed and as floats). Dirichlet handling:
// `fixed_row` is wave-uniform (a scalar branch, taken on 2 rows of the whole grid); columns 0 / cols-1 can
// only be element 0 / 7 of a lane (cols % 8 == 0), so they are per-lane flags.
// ---- packed-f32 row arithmetic (the fused kernel is VALU-bound: one wave64 VALU op per 4 cycles per SIMD)
// A lane's 8 columns live as 4 PAIRS p[k] = (e_k, e_{k+4}), so every v_pk_* op works on aligned register
// pairs: the west neighbours of pair k are pair k-1 and the east neighbours pair k+1; only pair 0's west
// and pair 3's east need a lane shift (DPP). Per 8 cells: 24 packed flops, 4 shifts/moves, 12 ops of
// bf16 rounding (v_cvt_pk_bf16_f32 + unpack) — ~40 VALU ops instead of ~100 for the scalar form.
typedef float f2 __attribute__((ext_vector_type(2)));
struct Row8 {
    f2 p[4];
};
__device__ __forceinline__ Row8 unpack_pairs(const u32x4& w) {  // words: (e0|e1) (e2|e3) (e4|e5) (e6|e7)
    Row8 r;
    r.p[0] = f2{lo(w.x), lo(w.z)};
    r.p[1] = f2{hi(w.x), hi(w.z)};
    r.p[2] = f2{lo(w.y), lo(w.w)};
    r.p[3] = f2{hi(w.y), hi(w.w)};
    return r;
}
__device__ __forceinline__ u32x4 pack_pairs(const Row8& r) {
    u32x4 w;
    w.x = pack2bf(r.p[0].x, r.p[1].x);
    w.y = pack2bf(r.p[2].x, r.p[3].x);
    w.z = pack2bf(r.p[0].y, r.p[1].y);
    w.w = pack2bf(r.p[2].y, r.p[3].y);
    return w;
}

// One update of a lane's 8 columns in pair layout; returns the bf16 row (packed) and, via nx, its exact float
// values for the next level. fixed_row is wave-uniform (a scalar branch, taken on 2 rows of the grid);
// columns 0 / cols-1 can only be element 0 / 7 of a lane (cols % 8 == 0): per-lane flags.
__device__ __forceinline__ u32x4 update_pairs(const Row8& n, const Row8& c, const Row8& s, bool fixed_row, bool fix0,
                                              bool fix7, float k, Row8& nx) {
    u32x4 pk;
    if (fixed_row) {
        pk = pack_pairs(c);
    } else {
        // west pair of pair 0 = (e_{-1}, e_3), east pair of pair 3 = (e_4, e_8)
        const f2 w0 = f2{pcmx::wave_from_prev(c.p[3].y), c.p[3].x};
        const f2 e3 = f2{c.p[0].y, pcmx::wave_from_next(c.p[0].x)};
        const f2 kk = f2{k, k}, m4 = f2{-4.f, -4.f};
        Row8 o;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const f2 w = q == 0 ? w0 : c.p[q - 1];
            const f2 e = q == 3 ? e3 : c.p[q + 1];
            const f2 t3 = (n.p[q] + s.p[q]) + (w + e);
            // t3 - 4c with 4c exact == fma(c, -4, t3): one rounding, bit-identical to the reference
            const f2 lap = __builtin_elementwise_fma(c.p[q], m4, t3);
            o.p[q] = c.p[q] + kk * lap;
        }
        o.p[0].x = fix0 ? c.p[0].x : o.p[0].x;
        o.p[3].y = fix7 ? c.p[3].y : o.p[3].y;
        pk = pack_pairs(o);
    }
    nx = unpack_pairs(pk);
    return pk;
}

// kAhead must be a multiple of 3: level windows are 3-slot rings indexed by (row - first row) % 3, which the
// fully unrolled prefetch loop turns into compile-time register names (no window-shifting moves). Rings hold
// PACKED bf16 rows (4 VGPRs each): the kernel is latency-bound, so unpacking a row per use (ALU) is cheaper
// than the occupancy lost to 8-VGPR float rows (T=4: 187 -> ~110 VGPRs, 2 -> 4 waves per SIMD).
template <int T, int kAhead, int RPW = kRowsPerWave>
__global__ __launch_bounds__(kWaves * 64) void stencil5xT_kernel(const unsigned short* __restrict__ u,
                                                                 unsigned short* __restrict__ out, int rows, int cols,
                                                                 int ld, int halo, int r0, int r1, long long grow0,
                                                                 long long grows, float k) {
    static_assert(T >= 1 && T <= 8, "lanes 1..62 stay exact for at most 8 levels");
    static_assert(kAhead % 3 == 0, "ring slots must be compile-time");
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int c0 = (int)blockIdx.x * kOutCols - 8 + lane * 8;  // first column of this lane (may be < 0)
    const int rs = max(r0, (int)(blockIdx.y * (kWaves * RPW) + wave * RPW));
    const int re = min(r1, (int)(blockIdx.y * (kWaves * RPW) + (wave + 1) * RPW));
    if (rs >= re) return;
    const bool in_grid = c0 >= 0 && c0 + 8 <= cols;  // cols % 8 == 0
    const bool store_lane = in_grid && lane >= 1 && lane <= 62;
    const bool fix0 = c0 == 0, fix7 = c0 + 8 == cols;
    const int slab_rows = rows + 2 * halo;
    const unsigned short* base = u + (in_grid ? c0 : 0);
    auto fetch = [&](int r) __attribute__((always_inline)) {  // local row r, clamped into the slab
        const int sr = min(max(r + halo, 0), slab_rows - 1);
        u32x4 w = *reinterpret_cast<const u32x4*>(base + (size_t)sr * ld);
        if (!in_grid) w = u32x4{0u, 0u, 0u, 0u};
        return w;
    };
    // ring[t][slot]: level t (0 = u) row with (row index - first) % 3 == slot, as exact floats in pair layout
    Row8 ring[T][3];
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int q = 0; q < 3; ++q)
#pragma unroll
            for (int p = 0; p < 4; ++p) ring[t][q].p[p] = f2{0.f, 0.f};
    const int i0 = rs - T, i1 = re + T;  // u rows consumed: [i0, i1)
    u32x4 pre[kAhead];
#pragma unroll
    for (int j = 0; j < kAhead; ++j) pre[j] = fetch(min(i0 + j, i1 - 1));
    for (int ib = i0; ib < i1; ib += kAhead) {
#pragma unroll
        for (int j = 0; j < kAhead; ++j) {
            const int i = ib + j;
            if (i < i1) {
                const int m0 = j % 3, m1 = (j + 2) % 3, m2 = (j + 1) % 3;  // slots of rows i, i-1, i-2
                ring[0][m0] = unpack_pairs(pre[j]);
                pre[j] = fetch(min(i + kAhead, i1 - 1));
                // level t+1 row i-t-1 from level t rows (i-t-2, i-t-1, i-t): slots (m2, m1, m0) of level t;
                // it lands in slot m0 of level t+1 (its row index i-t-1 is "newest" for that level)
#pragma unroll
                for (int t = 0; t < T; ++t) {
                    const int r = i - t - 1;
                    const long long g = grow0 + r;
                    Row8 nx;
                    const u32x4 pk = update_pairs(ring[t][m2], ring[t][m1], ring[t][m0], g == 0 || g == grows - 1,
                                                  fix0, fix7, k, nx);
                    if (t + 1 < T) {
                        ring[t + 1 < T ? t + 1 : 0][m0] = nx;
                    } else if (r >= rs && store_lane) {
                        __builtin_nontemporal_store(pk, reinterpret_cast<u32x4*>(out + (size_t)(r + halo) * ld + c0));
                    }
                }
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

// T fused updates over local rows [r0, r1) of a slab with `halo` rows above and below (T = 2, 3, 4, 6, 8).
extern "C" int pcmx_stencil5xT_bf16(const void* u, void* out, int rows, int cols, int ld, int halo, int steps, int r0,
                                    int r1, long long global_row0, long long global_rows, float k, hipStream_t s) {
    if (rows <= 0 || cols <= 0 || ld < cols || (ld & 7) || (cols & 7) || halo < 1 || steps < 1 ||
        (((uintptr_t)u | (uintptr_t)out) & 15))
        return -1;
    r0 = max(r0, 0);
    r1 = min(r1, rows);
    if (r0 >= r1) return 0;
    // rows that read `steps` rows beyond the local range need that deep a halo unless the side is a global edge
    const bool top_global = global_row0 == 0, bot_global = global_row0 + rows == global_rows;
    if (halo < steps && ((r0 < steps && !top_global) || (r1 > rows - steps && !bot_global))) return -1;
    dim3 grid((cols + kOutCols - 1) / kOutCols, (rows + kWaves * kRowsPerWave - 1) / (kWaves * kRowsPerWave));
    const unsigned short* ui = (const unsigned short*)u;
    unsigned short* uo = (unsigned short*)out;
    switch (steps) {
        case 2: stencil5xT_kernel<2, 6><<<grid, kWaves * 64, 0, s>>>(ui, uo, rows, cols, ld, halo, r0, r1, global_row0, global_rows, k); break;
        case 3: stencil5xT_kernel<3, 6><<<grid, kWaves * 64, 0, s>>>(ui, uo, rows, cols, ld, halo, r0, r1, global_row0, global_rows, k); break;
        case 4: stencil5xT_kernel<4, 6><<<grid, kWaves * 64, 0, s>>>(ui, uo, rows, cols, ld, halo, r0, r1, global_row0, global_rows, k); break;
        case 6: stencil5xT_kernel<6, 6><<<grid, kWaves * 64, 0, s>>>(ui, uo, rows, cols, ld, halo, r0, r1, global_row0, global_rows, k); break;
        case 8: stencil5xT_kernel<8, 6><<<grid, kWaves * 64, 0, s>>>(ui, uo, rows, cols, ld, halo, r0, r1, global_row0, global_rows, k); break;
        default: return -1;
    }
    return (int)hipGetLastError();
}

// Two fused updates (kept as the named entry point of the fuse=2 path).
extern "C" int pcmx_stencil5x2_bf16(const void* u, void* out, int rows, int cols, int ld, int halo, int r0, int r1,
                                    long long global_row0, long long global_rows, float k, hipStream_t s) {
    return pcmx_stencil5xT_bf16(u, out, rows, cols, ld, halo, 2, r0, r1, global_row0, global_rows, k, s);
}
