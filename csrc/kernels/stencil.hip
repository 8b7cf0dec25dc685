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
                float west = __shfl_up(cv[7], 1, 64);
                float east = __shfl_down(cv[0], 1, 64);
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
// ---------------------------------------------------------------- two fused time steps (temporal blocking)
// u -> s1 -> s2 in one pass: every cell is read and written once per TWO updates (2 B + 2 B per cell instead
// of 4 + 4), bit-identical to two single steps because the intermediate s1 is rounded to bf16 exactly as a
// stored step would be. A wave marches down its rows with a 3-row window of u (packed bf16) and a 3-row
// window of s1; s1 of the column just outside the strip (lane 0: c0-1, lane 63: c0+8) is computed from a
// 4-byte pair of u fetched next to the strip, so the strip needs no neighbour strip's registers.
// Slab: (rows + 2*halo) x ld, local row r at slab row r + halo; rows within 2 of a rank boundary need
// halo >= 2 (checked by the launcher); at a GLOBAL edge the extra rows are never used (Dirichlet rows).
struct RowPair {
    u32x4 w;         // 8 bf16 of the strip
    unsigned edge2;  // lane 0: u[c0-2] | u[c0-1] << 16 ; lane 63: u[c0+8] | u[c0+9] << 16
};
struct RowEdge {
    u32x4 w;               // 8 bf16 of s1
    unsigned short edge;   // s1 just outside the strip (lane 0: c0-1, lane 63: c0+8)
};

__device__ __forceinline__ void unpack8(const u32x4& w, float (&v)[8]) {
    v[0] = lo(w.x), v[1] = hi(w.x), v[2] = lo(w.y), v[3] = hi(w.y);
    v[4] = lo(w.z), v[5] = hi(w.z), v[6] = lo(w.w), v[7] = hi(w.w);
}

// one update of the strip's 8 columns; west/east = the neighbours of elements 0 and 7
__device__ __forceinline__ u32x4 update8(const float (&nv)[8], const float (&cv)[8], const float (&sv)[8], float west,
                                         float east, bool fixed_row, int c0, int cols, float k) {
    float o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const float c = cv[i];
        const float w = i == 0 ? west : cv[i - 1];
        const float e = i == 7 ? east : cv[i + 1];
        const float res = c + k * (((nv[i] + sv[i]) + (w + e)) - 4.0f * c);
        const int col = c0 + i;
        o[i] = (fixed_row || col == 0 || col == cols - 1) ? c : res;
    }
    u32x4 pk;
    pk.x = pack2bf(o[0], o[1]);
    pk.y = pack2bf(o[2], o[3]);
    pk.z = pack2bf(o[4], o[5]);
    pk.w = pack2bf(o[6], o[7]);
    return pk;
}

template <int kAhead>
__global__ __launch_bounds__(kWaves * 64) void stencil5x2_kernel(const unsigned short* __restrict__ u,
                                                                 unsigned short* __restrict__ out, int rows, int cols,
                                                                 int ld, int halo, int r0, int r1, long long grow0,
                                                                 long long grows, float k) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int c0 = blockIdx.x * kStripCols + lane * 8;
    const int rs = max(r0, (int)(blockIdx.y * (kWaves * kRowsPerWave) + wave * kRowsPerWave));
    const int re = min(r1, (int)(blockIdx.y * (kWaves * kRowsPerWave) + (wave + 1) * kRowsPerWave));
    if (rs >= re || c0 >= cols) return;  // the launcher guarantees cols % 512 == 0
    const bool is_w = lane == 0 && c0 > 0, is_e = lane == 63 && c0 + 8 < cols;
    const int slab_rows = rows + 2 * halo;
    const unsigned short* base = u + c0;
    const int eoff = is_w ? -2 : 8;
    auto fetch = [&](int r) __attribute__((always_inline)) {  // local row r, clamped into the slab
        RowPair x;
        const int sr = min(max(r + halo, 0), slab_rows - 1);
        const unsigned short* p = base + (size_t)sr * ld;
        x.w = *reinterpret_cast<const u32x4*>(p);
        x.edge2 = (is_w || is_e) ? *reinterpret_cast<const unsigned*>(p + eoff) : 0u;
        return x;
    };
    // first update of local row r from u rows r-1, r, r+1 (+ the out-of-strip column for the edge lanes)
    auto step1 = [&](const RowPair& n, const RowPair& c, const RowPair& s, int r) __attribute__((always_inline)) {
        float nv[8], cv[8], sv[8];
        unpack8(n.w, nv), unpack8(c.w, cv), unpack8(s.w, sv);
        float west = __shfl_up(cv[7], 1, 64);
        float east = __shfl_down(cv[0], 1, 64);
        // the pair next to the strip: lane 0 holds (c0-2, c0-1), lane 63 holds (c0+8, c0+9)
        const float pn_in = is_w ? hi(n.edge2) : lo(n.edge2), ps_in = is_w ? hi(s.edge2) : lo(s.edge2);
        const float pc_in = is_w ? hi(c.edge2) : lo(c.edge2), pc_out = is_w ? lo(c.edge2) : hi(c.edge2);
        if (is_w) west = pc_in;
        if (is_e) east = pc_in;
        const long long g = grow0 + r;
        const bool fixed_row = g == 0 || g == grows - 1;
        RowEdge o;
        o.w = update8(nv, cv, sv, west, east, fixed_row, c0, cols, k);
        // s1 at the out-of-strip column: never a Dirichlet column (cols % 8 == 0, strip interior edge)
        const float adj = is_w ? cv[0] : cv[7];
        const float ev = pc_in + k * (((pn_in + ps_in) + (is_w ? (pc_out + adj) : (adj + pc_out))) - 4.0f * pc_in);
        o.edge = f2bf(fixed_row ? pc_in : ev);
        return o;
    };
    // second update of local row r from s1 rows r-1, r, r+1
    auto step2 = [&](const RowEdge& n, const RowEdge& c, const RowEdge& s, int r) __attribute__((always_inline)) {
        float nv[8], cv[8], sv[8];
        unpack8(n.w, nv), unpack8(c.w, cv), unpack8(s.w, sv);
        float west = __shfl_up(cv[7], 1, 64);
        float east = __shfl_down(cv[0], 1, 64);
        if (is_w) west = bf2f(c.edge);
        if (is_e) east = bf2f(c.edge);
        const long long g = grow0 + r;
        return update8(nv, cv, sv, west, east, g == 0 || g == grows - 1, c0, cols, k);
    };

    RowPair ua = fetch(rs - 2), ub = fetch(rs - 1), uN = fetch(rs), uC = fetch(rs + 1);
    RowEdge s1P = step1(ua, ub, uN, rs - 1);
    RowEdge s1C = step1(ub, uN, uC, rs);
    RowPair q[kAhead];
#pragma unroll
    for (int j = 0; j < kAhead; ++j) q[j] = fetch(min(rs + 2 + j, re + 1));
    for (int rb = rs; rb < re; rb += kAhead) {
#pragma unroll
        for (int j = 0; j < kAhead; ++j) {
            const int r = rb + j;
            if (r < re) {
                const RowPair uS = q[j];  // u row r+2
                q[j] = fetch(min(r + 2 + kAhead, re + 1));
                const RowEdge s1N = step1(uN, uC, uS, r + 1);
                const u32x4 pk = step2(s1P, s1C, s1N, r);
                __builtin_nontemporal_store(pk, reinterpret_cast<u32x4*>(out + (size_t)(r + halo) * ld + c0));
                uN = uC, uC = uS, s1P = s1C, s1C = s1N;
            }
        }
    }
}
#pragma clang fp contract(on)
}  // namespace

// Two fused updates over local rows [r0, r1) of a slab with `halo` rows above and below.
extern "C" int pcmx_stencil5x2_bf16(const void* u, void* out, int rows, int cols, int ld, int halo, int r0, int r1,
                                    long long global_row0, long long global_rows, float k, hipStream_t s) {
    if (rows <= 0 || cols <= 0 || ld < cols || (ld & 7) || (cols % kStripCols) || halo < 1 ||
        (((uintptr_t)u | (uintptr_t)out) & 15))
        return -1;
    r0 = max(r0, 0);
    r1 = min(r1, rows);
    if (r0 >= r1) return 0;
    // rows that read two rows beyond the local range need a depth-2 halo unless that side is a global edge
    const bool top_global = global_row0 == 0, bot_global = global_row0 + rows == global_rows;
    if (halo < 2 && ((r0 < 2 && !top_global) || (r1 > rows - 2 && !bot_global))) return -1;
    dim3 grid(cols / kStripCols, (rows + kWaves * kRowsPerWave - 1) / (kWaves * kRowsPerWave));
    stencil5x2_kernel<8><<<grid, kWaves * 64, 0, s>>>((const unsigned short*)u, (unsigned short*)out, rows, cols, ld,
                                                    halo, r0, r1, global_row0, global_rows, k);
    return (int)hipGetLastError();
}

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
