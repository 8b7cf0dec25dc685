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
// LANE GEOMETRY. A lane holds CPL consecutive columns (8: one 16-B row load, as above; 4: one 8-B load, twice the
// waves and half the registers per wave, for short slabs that fill the chip with too few waves). The values of the
// first / last L = ceil(T / CPL) lanes of a strip go stale (one column per level from the strip edge), so lanes
// L .. 63-L store: a strip loads 64*CPL columns and stores OUT = (64 - 2L)*CPL. Strip x loads
// [x*OUT, x*OUT + 64*CPL). At a GLOBAL edge column (Dirichlet, never changes) nothing goes stale: strip 0 stores its
// lanes 0 .. L-1 and the strip holding column cols-1 its lanes beyond 63-L. 8 columns, T <= 8: 16384 columns =
// 504 + 31 x 496 + 504, 33 strips.
template <int CPL, int T>
struct Geo {
    static constexpr int NP = CPL / 2;  // column pairs per lane
    static constexpr int L = (T + CPL - 1) / CPL;
    static constexpr int OUT = (64 - 2 * L) * CPL;
    static_assert(CPL == 4 || CPL == 8, "4 or 8 columns per lane");
    static_assert(L >= 1 && 2 * L < 64, "stale lanes");
    __device__ static int c0(int lane) { return (int)blockIdx.x * OUT + lane * CPL; }
    __device__ static bool store_lane(int lane, int cols, bool in_grid) {
        const int x0 = (int)blockIdx.x * OUT;
        return in_grid && (lane >= L || x0 == 0) && (lane <= 63 - L || x0 + 64 * CPL >= cols);
    }
};
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
template <int NP>
struct RawT;
template <>
struct RawT<2> {
    typedef u32x2 type;
};
template <>
struct RawT<4> {
    typedef u32x4 type;
};

// ---- packed-f32 row arithmetic (the fused kernel is VALU-bound: one wave64 VALU op per 4 cycles per SIMD)
// A lane's CPL columns live as NP = CPL/2 PAIRS p[q] = (e_q, e_{q+NP}), so every v_pk_* op works on aligned register
// pairs: the west neighbours of pair q are pair q-1 and the east neighbours pair q+1; only pair 0's west and pair
// NP-1's east need a lane shift (DPP). Per 8 cells: 24 packed flops, 4 shifts/moves, 12 ops of bf16 rounding
// (v_cvt_pk_bf16_f32 + unpack) — ~40 VALU ops instead of ~100 for the scalar form.
typedef float f2 __attribute__((ext_vector_type(2)));
template <int NP>
struct RowP {
    f2 p[NP];
};
using Row8 = RowP<4>;
// raw words w[d] = (e_2d | e_2d+1) <-> pairs
template <int NP>
__device__ __forceinline__ RowP<NP> unpack_pairs(const typename RawT<NP>::type& w) {
    auto elem = [&](int i) { return (i & 1) ? hi(w[i >> 1]) : lo(w[i >> 1]); };
    RowP<NP> r;
#pragma unroll
    for (int q = 0; q < NP; ++q) r.p[q] = f2{elem(q), elem(q + NP)};
    return r;
}
template <int NP>
__device__ __forceinline__ typename RawT<NP>::type pack_pairs(const RowP<NP>& r) {
    auto elem = [&](int i) { return i < NP ? r.p[i].x : r.p[i - NP].y; };
    typename RawT<NP>::type w;
#pragma unroll
    for (int d = 0; d < NP; ++d) w[d] = pack2bf(elem(2 * d), elem(2 * d + 1));
    return w;
}

// One update of a lane's columns in pair layout; returns the bf16 row (packed) and, via nx, its exact float values
// for the next level. fixed_row is wave-uniform (a scalar branch, taken on 2 rows of the grid); columns 0 / cols-1
// can only be the first / last element of a lane (cols % 8 == 0): per-lane flags.
template <int NP>
__device__ __forceinline__ typename RawT<NP>::type update_pairs(const RowP<NP>& n, const RowP<NP>& c,
                                                                const RowP<NP>& s, bool fixed_row, bool fix0,
                                                                bool fixl, float k, RowP<NP>& nx) {
    typename RawT<NP>::type pk;
    if (fixed_row) {
        pk = pack_pairs<NP>(c);
    } else {
        // west pair of pair 0 = (e_{-1}, e_{NP-1}), east pair of pair NP-1 = (e_NP, e_{2NP})
        const f2 w0 = f2{pcmx::wave_from_prev(c.p[NP - 1].y), c.p[NP - 1].x};
        const f2 eL = f2{c.p[0].y, pcmx::wave_from_next(c.p[0].x)};
        const f2 kk = f2{k, k}, m4 = f2{-4.f, -4.f};
        RowP<NP> o;
#pragma unroll
        for (int q = 0; q < NP; ++q) {
            const f2 w = q == 0 ? w0 : c.p[q - 1];
            const f2 e = q == NP - 1 ? eL : c.p[q + 1];
            const f2 t3 = (n.p[q] + s.p[q]) + (w + e);
            // t3 - 4c with 4c exact == fma(c, -4, t3): one rounding, bit-identical to the reference
            const f2 lap = __builtin_elementwise_fma(c.p[q], m4, t3);
            o.p[q] = c.p[q] + kk * lap;
        }
        o.p[0].x = fix0 ? c.p[0].x : o.p[0].x;
        o.p[NP - 1].y = fixl ? c.p[NP - 1].y : o.p[NP - 1].y;
        pk = pack_pairs<NP>(o);
    }
    nx = unpack_pairs<NP>(pk);
    return pk;
}

// kAhead must be a multiple of 3: level windows are 3-slot rings indexed by (row - first row) % 3, which the
// fully unrolled prefetch loop turns into compile-time register names (no window-shifting moves). Rings hold
// PACKED bf16 rows (4 VGPRs each): the kernel is latency-bound, so unpacking a row per use (ALU) is cheaper
// than the occupancy lost to 8-VGPR float rows (T=4: 187 -> ~110 VGPRs, 2 -> 4 waves per SIMD).
// Row spans of one launch: blocks [0, nby_a) of grid.y cover local rows [a0, a1), the rest [b0, b1) (empty when
// b0 == b1). A distributed step updates both rank-edge row bands in ONE launch after the halo arrives, and a
// launch covers only its rows (no grid over the whole slab with idle blocks).
// rpw: rows per wave, a launch parameter (not a template argument): the host picks it per launch by the launched row
// count and fusion depth (the rule in pcmx_stencil5xT_bf16_spans_shape), or an explicit launch shape overrides it.
struct RowSpans {
    int a0, a1, b0, b1, nby_a, rpw;
};
// The rows [rs, re) of this wave (rs >= re: none).
__device__ __forceinline__ void wave_rows(const RowSpans& sp, int wave, int& rs, int& re) {
    int by = (int)blockIdx.y, base = sp.a0, lim = sp.a1;
    if (by >= sp.nby_a) by -= sp.nby_a, base = sp.b0, lim = sp.b1;
    rs = base + by * (kWaves * sp.rpw) + wave * sp.rpw;
    re = min(lim, rs + sp.rpw);
}

template <int T, int kAhead, int CPL = 8>
__device__ __forceinline__ void stencil5xT_body(const unsigned short* __restrict__ u, unsigned short* __restrict__ out,
                                                int rows, int cols, int ld, int halo, int rs, int re, long long grow0,
                                                long long grows, float k) {
    using G = Geo<CPL, T>;
    constexpr int NP = G::NP;
    using W = typename RawT<NP>::type;
    static_assert(kAhead % 3 == 0, "ring slots must be compile-time");
    const int lane = threadIdx.x & 63;
    const int c0 = G::c0(lane);  // first column of this lane
    if (rs >= re) return;
    const bool in_grid = c0 + CPL <= cols;  // cols % 8 == 0
    const bool store_lane = G::store_lane(lane, cols, in_grid);
    const bool fix0 = c0 == 0, fixl = c0 + CPL == cols;
    const int slab_rows = rows + 2 * halo;
    const unsigned short* base = u + (in_grid ? c0 : 0);
    auto fetch = [&](int r) __attribute__((always_inline)) {  // local row r, clamped into the slab
        const int sr = min(max(r + halo, 0), slab_rows - 1);
        W w = *reinterpret_cast<const W*>(base + (size_t)sr * ld);
        if (!in_grid) w = W{0u};
        return w;
    };
    // ring[t][slot]: level t (0 = u) row with (row index - first) % 3 == slot, as exact floats in pair layout
    RowP<NP> ring[T][3];
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int q = 0; q < 3; ++q)
#pragma unroll
            for (int p = 0; p < NP; ++p) ring[t][q].p[p] = f2{0.f, 0.f};
    const int i0 = rs - T, i1 = re + T;  // u rows consumed: [i0, i1)
    W pre[kAhead];
#pragma unroll
    for (int j = 0; j < kAhead; ++j) pre[j] = fetch(min(i0 + j, i1 - 1));
    for (int ib = i0; ib < i1; ib += kAhead) {
#pragma unroll
        for (int j = 0; j < kAhead; ++j) {
            const int i = ib + j;
            if (i < i1) {
                const int m0 = j % 3, m1 = (j + 2) % 3, m2 = (j + 1) % 3;  // slots of rows i, i-1, i-2
                ring[0][m0] = unpack_pairs<NP>(pre[j]);
                pre[j] = fetch(min(i + kAhead, i1 - 1));
                // level t+1 row i-t-1 from level t rows (i-t-2, i-t-1, i-t): slots (m2, m1, m0) of level t;
                // it lands in slot m0 of level t+1 (its row index i-t-1 is "newest" for that level)
#pragma unroll
                for (int t = 0; t < T; ++t) {
                    const int r = i - t - 1;
                    // level t+1 row r feeds a stored row only if r >= rs - (T - t - 1): the first 2t+2 rows of
                    // every level lie outside the wave's trapezoid (level T: rows above rs; same results)
                    if (i - i0 <= 2 * t + 1) continue;
                    const long long g = grow0 + r;
                    RowP<NP> nx;
                    const W pk = update_pairs<NP>(ring[t][m2], ring[t][m1], ring[t][m0], g == 0 || g == grows - 1,
                                                  fix0, fixl, k, nx);
                    if (t + 1 < T) {
                        ring[t + 1 < T ? t + 1 : 0][m0] = nx;
                    } else if (r >= rs && store_lane) {
                        __builtin_nontemporal_store(pk, reinterpret_cast<W*>(out + (size_t)(r + halo) * ld + c0));
                    }
                }
            }
        }
    }
}
template <int T, int kAhead>
__global__ __launch_bounds__(kWaves * 64) void stencil5xT_kernel(const unsigned short* __restrict__ u,
                                                                 unsigned short* __restrict__ out, int rows, int cols,
                                                                 int ld, int halo, RowSpans sp, long long grow0,
                                                                 long long grows, float k) {
    int rs, re;
    wave_rows(sp, (int)threadIdx.x >> 6, rs, re);
    stencil5xT_body<T, kAhead>(u, out, rows, cols, ld, halo, rs, re, grow0, grows, k);
}

// ---- v2: the same T-level row pipeline with ~30% fewer VALU ops per level (the kernel is VALU-issue bound):
//  * wave-uniform row bookkeeping: the wave index is read as a scalar, so the Dirichlet-row test, row clamps
//    and addressing are SALU work and `fixed_row` is a scalar branch (v1 spent ~4 VALU ops + exec-mask
//    juggling per level on 64-bit row compares);
//  * buffer loads/stores with a per-wave descriptor: the row offset is an SGPR soffset, a lane's column offset
//    a constant voffset, and lanes outside the grid get an out-of-range voffset, so the hardware returns 0 /
//    drops the store (no per-row address VALU, no select);
//  * the two lane-edge neighbours enter as DPP-sourced scalar adds (w + e of pair 0 and pair NP-1 built directly
//    in their packed registers: no DPP move + pair-forming moves + packed add);
//  * an intermediate level is rounded to bf16 AS FLOATS with one v_cvt_pk_bf16_f32 per value (low half 0),
//    instead of pack + unpack; only the stored last level is packed;
//  * no Dirichlet handling on the fast path: the few waves that hold column 0 / cols-1 or compute a level row on
//    global row 0 / grows-1 (a block column at each side, a wave or two at the top and bottom of the grid) run
//    the v1 pipeline instead (kept as a separate loop: one kernel, two code paths chosen per wave).
// Same arithmetic, same order: bit-identical to v1 and to T single steps. Measured (scripts/stencil_lab.hip,
// 16384^2): T=4 0.29-0.35 -> 0.235-0.24 ms, T=6 0.43-0.49 -> 0.31-0.32 ms (5.1 TGLUP/s).
__device__ __forceinline__ float round_bf16(float x) {  // x rounded to bf16 (RNE), kept as f32
    const f32x2 v = {0.f, x};
    return __uint_as_float(__builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2)));
}

// Sum of a lane-edge neighbour and an own-lane value as ONE scalar add: keeps the SLP vectoriser from forming a
// pair (DPP move + pair move + packed add) so the DPP move can fold into the add (v_add_f32_dpp).
__device__ __forceinline__ float add_scalar(float a, float b) {
    float r = a + b;
    asm volatile("" : "+v"(r));
    return r;
}

template <bool kLast, int NP>
__device__ __forceinline__ void level_pairs(const RowP<NP>& n, const RowP<NP>& c, const RowP<NP>& s, float k,
                                            RowP<NP>& nx, typename RawT<NP>::type& pk) {
    const f2 kk = f2{k, k}, m4 = f2{-4.f, -4.f};
    f2 we[NP];
#ifndef PCMX_FAULT_INJECT
    const float em1 = pcmx::wave_from_prev(c.p[NP - 1].y);  // e_{-1}: previous lane's last element
#else
    // test-only build (libpcmx_faultinj.so): lane 17 of every strip takes its EAST neighbour e_1 as the west neighbour
    // of its first column, a one-lane neighbour swap that is invisible on a constant grid (tests/test_gpu_errors.py:
    // the bench's timed-grid check must catch it on the random grid)
    float em1 = pcmx::wave_from_prev(c.p[NP - 1].y);
    if (pcmx::lane_id() == 17) em1 = c.p[1].x;
#endif
    const float eL = pcmx::wave_from_next(c.p[0].x);  // e_{2NP}: next lane's first element
    // pair 0: (e_{-1} + e_1, e_{NP-1} + e_{NP+1}); pair NP-1: (e_{NP-2} + e_NP, e_{2NP-2} + e_{2NP})
    we[0] = f2{add_scalar(em1, c.p[1].x), add_scalar(c.p[NP - 1].x, c.p[1].y)};
#pragma unroll
    for (int q = 1; q < NP - 1; ++q) we[q] = c.p[q - 1] + c.p[q + 1];
    we[NP - 1] = f2{add_scalar(c.p[NP - 2].x, c.p[0].y), add_scalar(c.p[NP - 2].y, eL)};
    RowP<NP> o;
#pragma unroll
    for (int q = 0; q < NP; ++q) {
        const f2 t3 = (n.p[q] + s.p[q]) + we[q];
        const f2 lap = __builtin_elementwise_fma(c.p[q], m4, t3);
        o.p[q] = c.p[q] + kk * lap;
    }
    if constexpr (kLast) {
        pk = pack_pairs<NP>(o);
    } else {
#pragma unroll
        for (int q = 0; q < NP; ++q) nx.p[q] = f2{round_bf16(o.p[q].x), round_bf16(o.p[q].y)};
    }
}

template <int NP>
__device__ __forceinline__ typename RawT<NP>::type buffer_load_row(__amdgpu_buffer_rsrc_t r, unsigned vo, int so) {
    if constexpr (NP == 4)
        return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, vo, so, 0));
    else
        return __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(r, vo, so, 0));
}
template <int NP>
__device__ __forceinline__ void buffer_store_row(const typename RawT<NP>::type& w, __amdgpu_buffer_rsrc_t r, unsigned vo,
                                                 int so) {
    if constexpr (NP == 4)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(pcmx::i32x4, w), r, vo, so, 2);
    else
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, w), r, vo, so, 2);
}

// The row pipeline of one interior wave (no Dirichlet row or column in reach).
template <int T, int kAhead, int NP>
__device__ __forceinline__ void pipeline_v2(const __amdgpu_buffer_rsrc_t ru, const __amdgpu_buffer_rsrc_t ro, unsigned vld,
                                            unsigned vst, int sr0, int pitch, int slab_rows, int halo, int rs, int i0,
                                            int i1, float k) {
    using W = typename RawT<NP>::type;
    auto fetch = [&](int r) __attribute__((always_inline)) {  // local row r, clamped into the slab
        const int sr = min(max(r + halo, 0), slab_rows - 1);
        return buffer_load_row<NP>(ru, vld, (sr - sr0) * pitch);
    };
    // ring[t][slot]: level t (0 = u) row with (row index - first) % 3 == slot, as exact floats in pair layout
    RowP<NP> ring[T][3];
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int q = 0; q < 3; ++q)
#pragma unroll
            for (int p = 0; p < NP; ++p) ring[t][q].p[p] = f2{0.f, 0.f};
    W pre[kAhead];
#pragma unroll
    for (int j = 0; j < kAhead; ++j) pre[j] = fetch(min(i0 + j, i1 - 1));
    // (a branch-free main loop — the per-level trapezoid / store tests peeled into the first 2T rows — measured no
    // faster at any shape and spilled at 8 columns per lane: profiles/r4_stencil/peel_rpw128_rejected.txt. Round 5,
    // profiles/r5_stencil/README.md: a steady-state turn with no guard at all raised the 8-column kernels to 256
    // VGPRs, 33% slower, and still carried the vmcnt(0) at the loop head; a compile-time row count per wave (the loop
    // fully unrolled, exact per-load waits) was bit-exact and no faster; a skewed schedule (level t+1 two rows behind
    // level t, so the T level updates of one iteration are independent) was bit-exact and 2-12% slower)
    for (int ib = i0; ib < i1; ib += kAhead) {
#pragma unroll
        for (int j = 0; j < kAhead; ++j) {
            const int i = ib + j;
            if (i < i1) {
                const int m0 = j % 3, m1 = (j + 2) % 3, m2 = (j + 1) % 3;  // slots of rows i, i-1, i-2
                ring[0][m0] = unpack_pairs<NP>(pre[j]);
                pre[j] = fetch(min(i + kAhead, i1 - 1));
#pragma unroll
                for (int t = 0; t < T; ++t) {
                    const int r = i - t - 1;
                    if (t + 1 < T) {
                        if (i - i0 <= 2 * t + 1) continue;  // outside the wave's trapezoid (see stencil5xT_body)
                        W unused;
                        level_pairs<false, NP>(ring[t][m2], ring[t][m1], ring[t][m0], k,
                                               ring[t + 1 < T ? t + 1 : 0][m0], unused);
                    } else if (r >= rs) {
                        W pk;
                        RowP<NP> unused;
                        level_pairs<true, NP>(ring[t][m2], ring[t][m1], ring[t][m0], k, unused, pk);
                        buffer_store_row<NP>(pk, ro, vst, (r + halo - sr0) * pitch);
                    }
                }
            }
        }
    }
}

// ---- PAIRED waves (round 6): two vertically adjacent waves of a workgroup share their common trapezoid.
// An unpaired wave of rows [rs, re) also computes the level rows its T-step cone reaches beyond both ends: T(T-1)
// level rows per wave (28% extra work at 18 rows per wave, T = 6: the short slab of an N = 8 rank). In a pair the
// upper wave marches DOWN its rows [rs, R) and the lower one UP its rows [R, re), so both reach the common boundary R
// at the END of their march, at the same time. There the T - 1 "drain" steps trade one boundary row per level
// through LDS instead of recomputing the other's rows: at drain step d (d = 1 .. T-1) each wave takes the partner's
// level-d row next to R (computed at the partner's step d - 1) and publishes its own level-(d+1) row; a barrier closes
// every drain step but the last. The outer ends keep their trapezoids (they border other workgroups). Same arithmetic
// from the same inputs (the update is symmetric in north / south), so bit-identical. Every wave of a paired block
// executes exactly T - 1 barriers (unpaired and empty waves execute them idly).
template <int NP>
struct PairXch {
    RowP<NP> v[2][2][2][64];  // [pair][writer: 0 down, 1 up][parity of the level written][lane]
};

template <int T, int kAhead, int NP, bool UP>
__device__ __forceinline__ void pipeline_v2_pair(const __amdgpu_buffer_rsrc_t ru, const __amdgpu_buffer_rsrc_t ro,
                                                 unsigned vld, unsigned vst, int sr0, int pitch, int slab_rows, int halo,
                                                 int rs, int re, float k, RowP<NP> (*mine)[64],
                                                 const RowP<NP> (*other)[64]) {
    using W = typename RawT<NP>::type;
    const int lane = threadIdx.x & 63;
    // DOWN: own rows [rs, R = re), input rows i0 = rs - T ascending to R + T - 1 (steps past R are the drain);
    // UP:   own rows [R = rs, re), input rows i0 = re - 1 + T descending to R - T
    const int R = UP ? rs : re;
    const int i0 = UP ? re - 1 + T : rs - T;
    const int nsteps = (re - rs) + 2 * T;
    const int ilast = UP ? R - 1 : R;  // the last real input row (drain step 0)
    auto fetch = [&](int r) __attribute__((always_inline)) {
        const int sr = min(max(r + halo, 0), slab_rows - 1);
        return buffer_load_row<NP>(ru, vld, (sr - sr0) * pitch);
    };
    RowP<NP> ring[T][3];
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int q = 0; q < 3; ++q)
#pragma unroll
            for (int p = 0; p < NP; ++p) ring[t][q].p[p] = f2{0.f, 0.f};
    W pre[kAhead];
#pragma unroll
    for (int j = 0; j < kAhead; ++j) pre[j] = fetch(UP ? max(i0 - j, ilast) : min(i0 + j, ilast));
    for (int sb = 0; sb < nsteps; sb += kAhead) {
#pragma unroll
        for (int j = 0; j < kAhead; ++j) {
            const int s = sb + j;  // step index: slots are (s % 3), compile-time within the unrolled body
            if (s < nsteps) {
                const int i = UP ? i0 - s : i0 + s;
                const int d = UP ? (R - 1) - i : i - R;  // drain step (>= 0)
                const int m0 = j % 3, m1 = (j + 2) % 3, m2 = (j + 1) % 3;  // slots of the steps s, s-1, s-2
                if (d <= 0) {
                    ring[0][m0] = unpack_pairs<NP>(pre[j]);
                    pre[j] = fetch(UP ? max(i - kAhead, ilast) : min(i + kAhead, ilast));
                }
#pragma unroll
                for (int t = 0; t < T; ++t) {
                    const int r = UP ? i + t + 1 : i - t - 1;  // the level t+1 row of this step
                    if (t + 1 < T) {
                        if (s <= 2 * t + 1) continue;  // outside the wave's outer trapezoid
                        if (UP ? r < R : r >= R) {     // the partner's row: its value arrives through LDS
                            if (t == d - 1) ring[t + 1][m0] = other[d & 1][lane];
                            continue;
                        }
                        W unused;
                        level_pairs<false, NP>(ring[t][m2], ring[t][m1], ring[t][m0], k, ring[t + 1][m0], unused);
                        if (d >= 0 && t == d) mine[(d + 1) & 1][lane] = ring[t + 1][m0];  // own row next to R
                    } else if (UP ? r < re : r >= rs) {
                        W pk;
                        RowP<NP> unused;
                        level_pairs<true, NP>(ring[t][m2], ring[t][m1], ring[t][m0], k, unused, pk);
                        buffer_store_row<NP>(pk, ro, vst, (r + halo - sr0) * pitch);
                    }
                }
                if (d >= 0 && d <= T - 2) __syncthreads();
            }
        }
    }
}

// MINW: minimum waves per SIMD the register allocation must allow (__launch_bounds__'s second argument): a short
// slab has few waves, so fitting one more per SIMD (T=4: 138 -> <= 128 VGPRs, 3 -> 4 waves) can matter more than
// the few rematerialised values it costs.
template <int T, int kAhead, int MINW = 1, int CPL = 8>
__global__ __launch_bounds__(kWaves * 64, MINW) void stencil5xT2_kernel(const unsigned short* __restrict__ u,
                                                                  unsigned short* __restrict__ out, int rows, int cols,
                                                                  int ld, int halo, RowSpans sp, long long grow0,
                                                                  long long grows, float k) {
    using G = Geo<CPL, T>;
    static_assert(kAhead % 3 == 0, "ring slots must be compile-time");
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int c0 = G::c0(lane);  // first column of this lane
    int rs, re;
    wave_rows(sp, wave, rs, re);
    if (rs >= re) return;
    const bool in_grid = c0 + CPL <= cols;  // cols % 8 == 0
    const bool store_lane = G::store_lane(lane, cols, in_grid);
    const bool fix0 = c0 == 0, fixl = c0 + CPL == cols;
    const int slab_rows = rows + 2 * halo;
    const int i0 = rs - T, i1 = re + T;  // u rows consumed: [i0, i1); level rows computed: [i0 - T, i1 - 1)
    // the wave's slab rows [sr0, sr1) (clamped like the fetch); one descriptor per buffer over exactly them
    const int sr0 = min(max(i0 + halo, 0), slab_rows - 1), sr1 = min(max(i1 - 1 + halo, 0), slab_rows - 1) + 1;
    const int pitch = ld * 2;
    const unsigned bytes = (unsigned)((size_t)(sr1 - sr0) * (size_t)pitch);
    const auto ru = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned short*>(u) + (size_t)sr0 * ld, (short)0,
                                                      (int)bytes, 0x00020000);
    const auto ro = __builtin_amdgcn_make_buffer_rsrc(out + (size_t)sr0 * ld, (short)0, (int)bytes, 0x00020000);
    const unsigned vld = in_grid ? (unsigned)c0 * 2 : 0x80000000u;     // out of range: the load returns 0
    const unsigned vst = store_lane ? (unsigned)c0 * 2 : 0x80000000u;  // out of range: the store is dropped
    const long long g0 = grow0 + i0 - T, g1 = grow0 + i1 - 2;          // global rows of computed level rows
    const bool edge_rows = (g0 <= 0 && 0 <= g1) || (g0 <= grows - 1 && grows - 1 <= g1);
    const bool slow = edge_rows || __builtin_amdgcn_ballot_w64(fix0 || fixl) != 0;
    if (slow)  // a few waves per grid: the v1 pipeline (per-column selects, per-row Dirichlet test; same results)
        stencil5xT_body<T, kAhead, CPL>(u, out, rows, cols, ld, halo, rs, re, grow0, grows, k);
    else
        pipeline_v2<T, kAhead, G::NP>(ru, ro, vld, vst, sr0, pitch, slab_rows, halo, rs, i0, i1, k);
}

// The block's rows [brs, bre) (all waves of a block lie in one span).
__device__ __forceinline__ void block_rows(const RowSpans& sp, int& brs, int& bre) {
    int by = (int)blockIdx.y, base = sp.a0, lim = sp.a1;
    if (by >= sp.nby_a) by -= sp.nby_a, base = sp.b0, lim = sp.b1;
    brs = base + by * (kWaves * sp.rpw);
    bre = min(lim, brs + kWaves * sp.rpw);
}

// The paired form of stencil5xT2_kernel (see pipeline_v2_pair): waves 2p / 2p+1 march down / up and meet. A block
// that holds a Dirichlet row or column anywhere in reach runs the unpaired per-wave paths (no barriers at all);
// otherwise every wave executes exactly T - 1 barriers.
template <int T, int kAhead, int MINW = 1, int CPL = 8>
__global__ __launch_bounds__(kWaves * 64, MINW) void stencil5xT2p_kernel(const unsigned short* __restrict__ u,
                                                                   unsigned short* __restrict__ out, int rows, int cols,
                                                                   int ld, int halo, RowSpans sp, long long grow0,
                                                                   long long grows, float k) {
    using G = Geo<CPL, T>;
    constexpr int NP = G::NP;
    static_assert(kAhead % 3 == 0, "ring slots must be compile-time");
    __shared__ PairXch<NP> xch;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int c0 = G::c0(lane);
    int rs, re, brs, bre;
    wave_rows(sp, wave, rs, re);
    block_rows(sp, brs, bre);
    const bool in_grid = c0 + CPL <= cols;
    const bool store_lane = G::store_lane(lane, cols, in_grid);
    const bool fix0 = c0 == 0, fixl = c0 + CPL == cols;
    const int slab_rows = rows + 2 * halo;
    const int pitch = ld * 2;
    const unsigned vld = in_grid ? (unsigned)c0 * 2 : 0x80000000u;
    const unsigned vst = store_lane ? (unsigned)c0 * 2 : 0x80000000u;
    // block-uniform: the strip's columns are the same for every wave, the row test covers the block's whole reach
    const long long g0 = grow0 + brs - 2 * T, g1 = grow0 + bre + 2 * T;
    const bool block_slow = (g0 <= 0 && 0 <= g1) || (g0 <= grows - 1 && grows - 1 <= g1) ||
                            __builtin_amdgcn_ballot_w64(fix0 || fixl) != 0;
    auto descriptors = [&](int lo, int hi, __amdgpu_buffer_rsrc_t& ru, __amdgpu_buffer_rsrc_t& ro, int& sr0) {
        sr0 = min(max(lo + halo, 0), slab_rows - 1);
        const int sr1 = min(max(hi + halo, 0), slab_rows - 1) + 1;
        const unsigned bytes = (unsigned)((size_t)(sr1 - sr0) * (size_t)pitch);
        ru = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned short*>(u) + (size_t)sr0 * ld, (short)0, (int)bytes,
                                               0x00020000);
        ro = __builtin_amdgcn_make_buffer_rsrc(out + (size_t)sr0 * ld, (short)0, (int)bytes, 0x00020000);
    };
    if (block_slow) {  // exactly the unpaired kernel's per-wave paths
        if (rs >= re) return;
        const long long w0 = grow0 + rs - 2 * T, w1 = grow0 + re + T - 2;
        const bool edge_rows = (w0 <= 0 && 0 <= w1) || (w0 <= grows - 1 && grows - 1 <= w1);
        if (edge_rows || __builtin_amdgcn_ballot_w64(fix0 || fixl) != 0) {
            stencil5xT_body<T, kAhead, CPL>(u, out, rows, cols, ld, halo, rs, re, grow0, grows, k);
        } else {
            __amdgpu_buffer_rsrc_t ru, ro;
            int sr0;
            descriptors(rs - T, re + T - 1, ru, ro, sr0);
            pipeline_v2<T, kAhead, NP>(ru, ro, vld, vst, sr0, pitch, slab_rows, halo, rs, rs - T, re + T, k);
        }
        return;
    }
    const int pair = wave >> 1;
    const bool up = (wave & 1) != 0;
    int prs, pre;  // the partner's rows
    wave_rows(sp, wave ^ 1, prs, pre);
    const bool paired = up ? rs < re : prs < pre;  // the pair exists iff its lower (up) wave has rows
    if (!paired) {
        if (rs < re) {  // an upper wave whose partner is empty: the unpaired pipeline (both trapezoids)
            __amdgpu_buffer_rsrc_t ru, ro;
            int sr0;
            descriptors(rs - T, re + T - 1, ru, ro, sr0);
            pipeline_v2<T, kAhead, NP>(ru, ro, vld, vst, sr0, pitch, slab_rows, halo, rs, rs - T, re + T, k);
        }
        for (int b = 0; b < T - 1; ++b) __syncthreads();  // the paired waves' drain barriers
        return;
    }
    __amdgpu_buffer_rsrc_t ru, ro;
    int sr0;
    if (up) {
        descriptors(rs - 1, re - 1 + T, ru, ro, sr0);
        pipeline_v2_pair<T, kAhead, NP, true>(ru, ro, vld, vst, sr0, pitch, slab_rows, halo, rs, re, k, xch.v[pair][1],
                                              xch.v[pair][0]);
    } else {
        descriptors(rs - T, re, ru, ro, sr0);
        pipeline_v2_pair<T, kAhead, NP, false>(ru, ro, vld, vst, sr0, pitch, slab_rows, halo, rs, re, k,
                                               xch.v[pair][0], xch.v[pair][1]);
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

namespace {
// The production choice of paired waves (stencil5xT2p_kernel) for a launch: see pcmx_stencil5xT_bf16_spans_shape.
bool PairedDefault(int steps, bool edge, int rpw) {
    (void)steps, (void)edge, (void)rpw;
    return false;  // measured, not adopted (see the launch rule)
}

// strips covering `cols` columns (see Geo): the first strip whose loaded range [x*OUT, x*OUT + 64*CPL) reaches cols
// is the last one
int strips_for(int cols, int cpl, int steps) {
    const int L = (steps + cpl - 1) / cpl, out = (64 - 2 * L) * cpl;
    return cols <= 64 * cpl ? 1 : 1 + (cols - 64 * cpl + out - 1) / out;
}
// the halo rule of one row range: a row r reads rows r - steps .. r + steps, which must lie in the slab on a side
// with a neighbour (at a GLOBAL edge the clamped reads only feed Dirichlet rows)
bool halo_ok(int rows, int halo, int steps, int r0, int r1, long long global_row0, long long global_rows) {
    const bool top_global = global_row0 == 0, bot_global = global_row0 + rows == global_rows;
    return r0 >= r1 || ((top_global || r0 - steps >= -halo) && (bot_global || r1 + steps <= rows + halo));
}
}  // namespace

// T fused updates over local rows [r0a, r1a) and [r0b, r1b) (either may be empty) of a slab with `halo` rows
// above and below (T = 2, 3, 4, 6, 8), in one launch. On a side with a neighbour a span may reach into the halo
// region (local rows -(halo - T) .. rows + halo - T): the deep-halo schedule of the distributed stencil computes
// those rows redundantly so the next step needs no exchange (parallel/stencil.py); at a global edge spans are
// clamped to [0, rows).
// shape: an EXPLICIT launch-shape override of this one launch (0 = the production rule below): bits 0-7 columns per
// lane (4 / 8), bits 8-15 rows per wave (1 .. 255), bits 16-23 prefetch ring depth (3 / 6 / 9); each field 0 keeps the
// rule's value. The lab scripts sweep shapes through it (scripts/stencil_*_lab.py); no launch state lives in the library.
extern "C" int pcmx_stencil5xT_bf16_spans_shape(const void* u, void* out, int rows, int cols, int ld, int halo,
                                                int steps, int r0a, int r1a, int r0b, int r1b, long long global_row0,
                                                long long global_rows, float k, int shape, hipStream_t s) {
    if (rows <= 0 || cols <= 0 || ld < cols || (ld & 7) || (cols & 7) || halo < 1 || steps < 1 ||
        (((uintptr_t)u | (uintptr_t)out) & 15))
        return -1;
    const int o_cpl = shape & 0xff, o_rpw = (shape >> 8) & 0xff, o_ahead = (shape >> 16) & 0xff;
    const int o_pair = (shape >> 24) & 0x3;  // 1: paired waves, 2: unpaired, 0: the rule below
    if ((o_cpl != 0 && o_cpl != 4 && o_cpl != 8) || (o_ahead != 0 && o_ahead != 3 && o_ahead != 6 && o_ahead != 9) ||
        (shape >> 26) != 0 || o_pair == 3)
        return -1;
    const bool top_global = global_row0 == 0, bot_global = global_row0 + rows == global_rows;
    const int lo_lim = top_global ? 0 : -max(0, halo - steps), hi_lim = bot_global ? rows : rows + max(0, halo - steps);
    r0a = max(r0a, lo_lim), r1a = min(r1a, hi_lim), r0b = max(r0b, lo_lim), r1b = min(r1b, hi_lim);
    const bool ea = r0a >= r1a, eb = r0b >= r1b;
    if (ea) r0a = r1a = 0;
    if (eb) r0b = r1b = 0;
    if (ea && eb) return 0;
    if (!ea && !eb && r1a > r0b && r1b > r0a) return -1;  // overlapping spans would race (two waves storing one row)
    if (!halo_ok(rows, halo, steps, r0a, r1a, global_row0, global_rows) ||
        !halo_ok(rows, halo, steps, r0b, r1b, global_row0, global_rows))
        return -1;
    const unsigned short* ui = (const unsigned short*)u;
    unsigned short* uo = (unsigned short*)out;
    // Prefetch ring: 9 rows ahead at T >= 6 on 64-row waves (2 waves per SIMD there, so deeper per-wave prefetch
    // hides more load latency: T=8 0.390-0.403 -> 0.383 ms, T=6 0.305-0.320 -> 0.302 ms at 16384^2; 12 rows spill
    // at T=8; on the 24-row waves of a 4096-row slab 9 rows measured ~7% slower; profiles/r2_stencil/
    // prefetch_depth_ab.txt), 6 otherwise.
    // T = 2 is HBM-bound: the v1 kernel. T >= 3 is VALU-bound: v2, rows per wave by the launched row count (each
    // wave recomputes the T-row trapezoid overlap with its neighbours, so short waves trade redundant level rows for
    // more waves; scripts/stencil_lab.hip sweep after the trapezoid skip, profiles/r2_stencil/rpw_sweep_trapezoid.txt,
    // 16384 columns, GLUP/s of the best RPW: 2048 rows T=4 24 (3.9k), T=6/8 16 (3.6k/3.4k); 4096 rows 24 (4.4-4.5k);
    // 8192 rows 24-32 (4.9-5.1k); 16384 rows T=6/8 64 (5.4k/5.5k), T=4 24 (4.8k))
    // Round 3 (profiles/r3_stencil/short_slab_sweep.txt, counters short_slab_pmc.txt): on a 2048-row slab (one rank
    // at N = 8) T = 4 with an 18-row wave and a 3-row prefetch ring (126 VGPRs: 4 waves per SIMD, 3828 waves in
    // one round) runs 3.9-4.0k against 3.6-3.9k for 24 rows / 6-row ring (138 VGPRs, 3 waves per SIMD); the waves
    // are VALU-busy only ~20% of the time, split between load waits and the level-to-level dependency chain.
    const int span_rows = (r1a - r0a) + (r1b - r0b);
    // Lanes and rows per wave (round 3, scripts/stencil_lanes_lab.py, profiles/r3_stencil/lanes_*.txt): 4 columns per
    // lane (twice the waves, half the registers) pays at T >= 6 below 12288 rows; an EDGE launch (the two halo
    // bands of a distributed step, <= 2T rows) is a few waves whose row pipeline is the whole cost, so it runs
    // 2-row waves of 4 columns per lane (shorter dependency chains, 8-16x the waves).
    // Short slabs at T = 6 (one N = 8 rank, 2048 rows): 18 rows per wave with the 3-row ring. Round 4 sized the grid to
    // one residency round (29 rows per wave: 0.0526 against 0.0567 ms for a full launch, rpw_sweep.txt); round 5's
    // interleaved A/B (profiles/r5_stencil/rpw_deep_ab.txt, 6 alternations in one process) finds the full launch equal
    // at 18 / 24 / 29 (0.0531 / 0.0532 / 0.0533 ms) and the deep-halo steps the production schedule runs faster at 18
    // (m = 5: 0.0539 / 0.0547 / 0.0558 ms per step).
    const bool edge = span_rows <= 64;
    int cpl, rpw;
    if (edge)
        cpl = 4, rpw = 2;
    else if (span_rows < 3072)
        cpl = steps >= 6 ? 4 : 8, rpw = steps == 6 ? 18 : 24;
    else if (span_rows < 6144)
        cpl = steps >= 6 ? 4 : 8, rpw = steps == 8 ? 32 : 24;
    else if (span_rows < 12288)
        cpl = steps == 8 ? 4 : 8, rpw = 32;
    else
        cpl = 8, rpw = steps <= 4 ? 24 : 64;
    if (o_cpl) cpl = o_cpl;
    if (o_rpw) rpw = o_rpw;
    if (steps == 2) cpl = 8, rpw = kRowsPerWave;  // T = 2: the HBM-bound v1 kernel, one shape
    if (steps == 3) cpl = 8;                      // T = 3: 8-column lanes only
    // prefetch ring depth (rows in flight per wave; a multiple of 3, see stencil5xT_body)
    int ahead = (steps >= 6 && rpw >= 64) ? 9 : (rpw <= 4 || (rpw > 16 && rpw <= 20)) ? 3 : 6;
    if (o_ahead) ahead = o_ahead;
    // paired waves (stencil5xT2p_kernel): the two waves of a pair share their common trapezoid through LDS. A lab
    // shape only (T = 6 with 4 columns per lane, the N = 8 short slab; any other paired shape is refused): bit-exact,
    // but no faster — the pair's T - 1 drain hand-offs keep the wave's critical path, and the extra code raises the
    // kernel from 88 to 110 VGPRs (5 -> 4 waves per SIMD; forcing 5 spills and runs 1.8x slower):
    // profiles/r6_stencil/README.md.
    bool paired = PairedDefault(steps, edge, rpw);
    if (o_pair) paired = o_pair == 1;
    if (steps < 3 || rpw < steps) paired = false;
    const int per = kWaves * rpw;
    const RowSpans sp{r0a, r1a, r0b, r1b, (r1a - r0a + per - 1) / per, rpw};
    const dim3 g(strips_for(cols, steps == 2 ? 8 : cpl, steps), sp.nby_a + (r1b - r0b + per - 1) / per);
#define PCMX_STENCIL_V2_KA(T, KA, C)                                                                                \
    case KA:                                                                                                        \
        if (paired) {                                                                                               \
            if constexpr (T == 6 && C == 4)                                                                         \
                stencil5xT2p_kernel<T, KA, 1, C><<<g, kWaves * 64, 0, s>>>(ui, uo, rows, cols, ld, halo, sp,        \
                                                                            global_row0, global_rows, k);           \
            else                                                                                                    \
                return -1;                                                                                          \
        } else {                                                                                                    \
            stencil5xT2_kernel<T, KA, 1, C><<<g, kWaves * 64, 0, s>>>(ui, uo, rows, cols, ld, halo, sp, global_row0, \
                                                                       global_rows, k);                             \
        }                                                                                                           \
        break;
#define PCMX_STENCIL_V2C(T, C)                                                                                      \
    switch (ahead) {                                                                                                \
        PCMX_STENCIL_V2_KA(T, 3, C)                                                                                 \
        PCMX_STENCIL_V2_KA(T, 6, C)                                                                                 \
        PCMX_STENCIL_V2_KA(T, 9, C)                                                                                 \
        default: return -1;                                                                                         \
    }
#define PCMX_STENCIL_V2(T)                                                                                          \
    if (cpl == 4) {                                                                                                 \
        PCMX_STENCIL_V2C(T, 4)                                                                                      \
    } else {                                                                                                        \
        PCMX_STENCIL_V2C(T, 8)                                                                                      \
    }
    switch (steps) {
        case 2:
            stencil5xT_kernel<2, 6><<<g, kWaves * 64, 0, s>>>(ui, uo, rows, cols, ld, halo, sp, global_row0, global_rows, k);
            break;
        case 3: PCMX_STENCIL_V2C(3, 8) break;
        case 4: PCMX_STENCIL_V2(4) break;
        case 5: PCMX_STENCIL_V2(5) break;
        case 6: PCMX_STENCIL_V2(6) break;
        case 8: PCMX_STENCIL_V2(8) break;
        default: return -1;
    }
#undef PCMX_STENCIL_V2
#undef PCMX_STENCIL_V2C
#undef PCMX_STENCIL_V2_KA
    return (int)hipGetLastError();
}

extern "C" int pcmx_stencil5xT_bf16_spans(const void* u, void* out, int rows, int cols, int ld, int halo, int steps,
                                          int r0a, int r1a, int r0b, int r1b, long long global_row0,
                                          long long global_rows, float k, hipStream_t s) {
    return pcmx_stencil5xT_bf16_spans_shape(u, out, rows, cols, ld, halo, steps, r0a, r1a, r0b, r1b, global_row0,
                                            global_rows, k, 0, s);
}

// T fused updates over local rows [r0, r1) of a slab with `halo` rows above and below (T = 2, 3, 4, 5, 6, 8).
extern "C" int pcmx_stencil5xT_bf16(const void* u, void* out, int rows, int cols, int ld, int halo, int steps, int r0,
                                    int r1, long long global_row0, long long global_rows, float k, hipStream_t s) {
    return pcmx_stencil5xT_bf16_spans(u, out, rows, cols, ld, halo, steps, r0, r1, 0, 0, global_row0, global_rows, k, s);
}

// Two fused updates (kept as the named entry point of the fuse=2 path).
extern "C" int pcmx_stencil5x2_bf16(const void* u, void* out, int rows, int cols, int ld, int halo, int r0, int r1,
                                    long long global_row0, long long global_rows, float k, hipStream_t s) {
    return pcmx_stencil5xT_bf16(u, out, rows, cols, ld, halo, 2, r0, r1, global_row0, global_rows, k, s);
}
