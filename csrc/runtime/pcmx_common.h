// Shared device-side helpers for the gfx950 kernels (wave64 collectives, vector types, checks).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define PCMX_HIP_RET(expr)                                  \
    do {                                                    \
        hipError_t _e = (expr);                             \
        if (_e != hipSuccess) return (int)_e;               \
    } while (0)

#define PCMX_HIP_CHECK(expr)                                                                       \
    do {                                                                                           \
        hipError_t _e = (expr);                                                                    \
        if (_e != hipSuccess) {                                                                    \
            fprintf(stderr, "HIP error %s at %s:%d: %s\n", hipGetErrorString(_e), __FILE__, __LINE__, #expr); \
            abort();                                                                               \
        }                                                                                          \
    } while (0)

namespace pcmx {

// Native clang vectors (HIP's float4 is a struct the nontemporal builtins reject).
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
template <class V>
__device__ __forceinline__ V ld_nt(const V* p) { return __builtin_nontemporal_load(p); }
template <class V>
__device__ __forceinline__ void st_nt(V* p, V v) { __builtin_nontemporal_store(v, p); }

constexpr int kWave = 64;  // CDNA wavefront: 64 lanes (never 32)
constexpr int kNumXcd = 8;

__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }

template <class T>
__device__ __forceinline__ T op_apply(int op, T a, T b) {
    return op == 0 ? a + b : (op == 1 ? (a < b ? a : b) : (a > b ? a : b));
}

// Full-wave butterfly reduction (DPP/permute lowered by the compiler); result in every lane.
template <class T, int OP>
__device__ __forceinline__ T wave_reduce(T v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        T o = __shfl_xor(v, off, kWave);
        v = OP == 0 ? v + o : (OP == 1 ? (o < v ? o : v) : (o > v ? o : v));
    }
    return v;
}

// Sum over the 64 lanes on the DPP path (no LDS round trip): quad swaps and row rotations leave every lane of a
// 16-lane row holding its row sum, then row_bcast:15 / row_bcast:31 fold the rows upward. The total is in lane 63
// (other lanes hold partial sums).
template <int kCtrl, int kRowMask>
__device__ __forceinline__ float dpp_add(float v) {
    return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), kCtrl, kRowMask, 0xf, false));
}
__device__ __forceinline__ float wave_sum_to_lane63(float v) {
    v = dpp_add<0xb1, 0xf>(v);   // quad_perm [1,0,3,2]
    v = dpp_add<0x4e, 0xf>(v);   // quad_perm [2,3,0,1]
    v = dpp_add<0x124, 0xf>(v);  // row_ror:4
    v = dpp_add<0x128, 0xf>(v);  // row_ror:8
    v = dpp_add<0x142, 0xa>(v);  // row_bcast:15 into rows 1 and 3
    v = dpp_add<0x143, 0xc>(v);  // row_bcast:31 into rows 2 and 3
    return v;
}

// Whole-wave lane shifts on the DPP path (GFX9 wave_shr:1 / wave_shl:1): a VALU modifier, no LDS round trip
// like __shfl_up/__shfl_down (ds_bpermute). wave_from_prev: lane l gets lane l-1's value; wave_from_next: lane
// l gets lane l+1's value. The end lane (0 / 63) receives 0.
__device__ __forceinline__ float wave_from_prev(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float wave_from_next(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x130, 0xf, 0xf, true));
}

// Inclusive wave scan (Hillis-Steele over 64 lanes).
__device__ __forceinline__ float wave_inclusive_scan(float v) {
    const int l = lane_id();
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
        float o = __shfl_up(v, off, kWave);
        if (l >= off) v += o;
    }
    return v;
}

// Bijective XCD-aware remap of a linear workgroup id (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): blocks that the dispatcher deals to one XCD (b, b+8, b+16, ...) get consecutive ids.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    const int q = nwg / kNumXcd, r = nwg % kNumXcd;
    const int xcd = bid % kNumXcd, slot = bid / kNumXcd;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
}

// Streaming grid cap (256 CUs x 64 blocks, then grid-stride): at 1e9 f32 a 16384-block grid streams 5.5 TB/s for
// vadd / copy / fill against 4.8-5.1 with 2048 (scripts/stream_bw_lab.hip, profiles/r4_bench/stream_bw_lab.txt)
inline int grid_cap_streaming() { return 256 * 64; }

}  // namespace pcmx
