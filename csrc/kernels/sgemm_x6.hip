// FP32 GEMM on the gfx950 BF16 matrix cores by exact 3-way operand splitting ("x6") — an fp32-accurate
// alternative to the native f32 MFMA kernel of sgemm.hip. Reference ancestor: matrix_multiply,
// ref 1-introduction/matrix.c:63-81.
//
// Why: v_mfma_f32_32x32x2_f32 runs at 64 FLOP/clk/SIMD (157 TF, the headline kernel sits at 99% of it), while
// v_mfma_f32_32x32x16_bf16 runs at 1024 FLOP/clk/SIMD (2.5 PF): 16x the rate for 8-bit significands.
//  * Every fp32 operand x is split on the fly, in registers, into three bf16 values x = x0 + x1 + x2 EXACTLY
//    (round-to-nearest split: x0 = bf16(x), x1 = bf16(x - x0), x2 = x - x0 - x1, which has <= 8 significant bits
//    and so is a bf16; the two subtractions are exact). Holds for finite |x| >= 2^-110 (residuals stay normal);
//    Inf/NaN operands produce NaN.
//  * a*b = sum over the 9 piece products; the 6 with i + j <= 2 are computed (a0b0, a0b1, a1b0, a0b2, a1b1,
//    a2b0), the dropped three are below 2^-24 |a||b| (RNE pieces: |x1| <= 2^-8 |x|, |x2| <= 2^-16 |x|), i.e.
//    below the rounding of one fp32 product. Each bf16 x bf16 product is exact in the f32 accumulator and the
//    accumulation is an f32 chain like the native kernel's: the result has fp32 accuracy (bench field
//    sgemm_x6_max_rel_err_vs_fp64 vs sgemm_max_rel_err_vs_fp64).
//  * 6 bf16 MFMAs per 16 k at 32 cycles = 192 cycles vs 8 f32 MFMAs (k 2 each) at 64 = 512 cycles: 2.67x
//    the native f32 peak in MFMA time.
// Layout (MI355X_MICROARCH.md "Matrix cores"; operand maps cdna_hip_programming.md §3):
//  * 4 waves (one per SIMD, 512 registers), block tile 256x256, wave tile 128x128 = 4x4 32x32 MFMA tiles
//    (256 f32 accumulators), like sgemm.hip variant 17: operands straight from L2 into registers, no LDS.
//  * k step of 16: lane (l32, h) needs A[row l32][k0 + 8h + e] and B[k0 + 8h + e][col] for e = 0..7:
//    A = two 16-B loads of its row; B = eight 16-B loads of B[k0 + 8h + e][c0 + 4 l32 .. +3], i.e. N-tile j owns
//    columns c0 + 4c + j (one 16-B load feeds 4 N-tiles; the epilogue stores 16 B per lane).
//  * Split cost: 11 VALU ops per pair of elements (3 v_cvt_pk_bf16_f32, 4 unpacks, 4 subtractions), 352 per wave
//    per 16-k step against 96 MFMAs (3072 cycles): 3-4 ops in every MFMA gap (sched_group_barrier pattern), issued
//    in the MFMA shadow. Raw A is loaded one step ahead of its split, raw B two (2-slot ring); each M-tile's region
//    splits the next A tile and one k-word of all four B tiles for the next step (B planes double-buffered).
//  * Measured (profiles/r3_sgemm_x6/): 8192^3 in 4.11-4.15 ms = 265-267 TFLOPS, 1.73x hipBLASLt's fp32 GEMM, MFMA
//    busy 89% of the active cycles; the 6x bf16 work runs at 1.60 PF, above hipBLASLt's own bf16 GEMM on the box
//    (1.41 PF): the kernel is bound by the power-limited clock under dense bf16 MFMA, not by issue.
#include "pcmx_common.h"
#include "pcmx_hip.h"
#include <type_traits>

namespace {
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
using pcmx::f32x4;

struct Planes {  // one bf16x8 MFMA operand per split level
    u32x4 p[3];
};

__device__ __forceinline__ unsigned cvt2(float a, float b) {
    const f32x2 v = {a, b};
    return __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2));
}
__device__ __forceinline__ float lo16(unsigned w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi16(unsigned w) { return __uint_as_float(w & 0xffff0000u); }

// Split of 8 elements (k order) into three bf16x8 planes, x == p0 + p1 + p2: per pair of elements 3
// v_cvt_pk_bf16_f32, 2 unpacks and 2 residual subtractions for each of 2 levels (f32x2 arithmetic; the compiler
// unpacks v_pk_add_f32 in the MFMA shadow). A tile: r[q] holds k = 4q .. 4q+3; words d = 2q, 2q+1 of each level come from r[q].
// FAKE (lab only, wrong results): one conversion per pair and no residuals, to price the split's VALU work.
template <bool FAKE = false>
__device__ __forceinline__ void split_a4(f32x4 (&r)[2], Planes& o) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        f32x2 x0 = {r[q][0], r[q][1]}, x1 = {r[q][2], r[q][3]};
#pragma unroll
        for (int l = 0; l < 3; ++l) {
            if (FAKE && l > 0) {
                o.p[l][2 * q] = o.p[0][2 * q], o.p[l][2 * q + 1] = o.p[0][2 * q + 1];
                continue;
            }
            const unsigned w0 = cvt2(x0[0], x0[1]), w1 = cvt2(x1[0], x1[1]);
            o.p[l][2 * q] = w0, o.p[l][2 * q + 1] = w1;
            if (!FAKE && l < 2) x0 -= f32x2{lo16(w0), hi16(w0)}, x1 -= f32x2{lo16(w1), hi16(w1)};
        }
    }
}
// B: word d (k rows 2d, 2d+1) of every level for all 4 N-tiles; r[e] holds k row e of the 4 N-tiles' columns.
template <bool FAKE = false>
__device__ __forceinline__ void split_b_word(const f32x4 (&r)[8], int d, Planes (&o)[4]) {
    f32x2 x[2][2];  // [row 2d / 2d+1][N-tile pair]
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) x[e][jp] = f32x2{r[2 * d + e][2 * jp], r[2 * d + e][2 * jp + 1]};
#pragma unroll
    for (int l = 0; l < 3; ++l) {
        unsigned w[4];
        if (FAKE && l > 0) {
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j].p[l][d] = o[j].p[0][d];
            continue;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j].p[l][d] = w[j] = cvt2(x[0][j >> 1][j & 1], x[1][j >> 1][j & 1]);
        if (!FAKE && l < 2) {
#pragma unroll
            for (int jp = 0; jp < 2; ++jp) {
                x[0][jp] -= f32x2{lo16(w[2 * jp]), lo16(w[2 * jp + 1])};
                x[1][jp] -= f32x2{hi16(w[2 * jp]), hi16(w[2 * jp + 1])};
            }
        }
    }
}

// products (level of A, level of B), smallest first
constexpr int kPA[6] = {2, 1, 0, 1, 0, 0};
constexpr int kPB[6] = {0, 1, 2, 0, 1, 0};

__device__ __forceinline__ f32x16 mfma(const u32x4& a, const u32x4& b, const f32x16& c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                   0, 0);
}

template <bool BETA, int VPM>
__global__ __launch_bounds__(256, 1) void sgemm_x6_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                          float* __restrict__ C, int M, int N, int K, int lda, int ldb,
                                                          int ldc, float alpha, float beta) {
    const int lane = pcmx::lane_id();
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int h = lane >> 5, l32 = lane & 31;
    // tile of this block: XCD remap, then column strips 8 tile-rows tall (as sgemm.hip tile_coords)
    const int tiles_m = M / 256, tiles_n = N / 256;
    const int t = pcmx::xcd_remap((int)blockIdx.x, tiles_m * tiles_n);
    const int per_group = 8 * tiles_n, first_m = (t / per_group) * 8;
    const int gsz = min(tiles_m - first_m, 8);
    const int m0 = __builtin_amdgcn_readfirstlane((first_m + (t % per_group) % gsz) * 256);
    const int n0 = __builtin_amdgcn_readfirstlane(((t % per_group) / gsz) * 256);

    const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rC = __builtin_amdgcn_make_buffer_rsrc((void*)C, (short)0, 0x7fffffff, 0x00020000);
    int voA[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) voA[i] = ((32 * i + l32) * lda + 8 * h) * 4;
    const int voB = (8 * h * ldb + 4 * l32) * 4;
    const int voC = (4 * h * ldc + 4 * l32) * 4;
    const int ab = __builtin_amdgcn_readfirstlane((m0 + wm * 128) * lda * 4);
    const int bb = __builtin_amdgcn_readfirstlane((n0 + wn * 128) * 4);
    const int ns = K / 16, last = ns - 1;
    const int bstep = ldb * 64;  // bytes per 16 k-rows of B
    auto ld = [](__amdgpu_buffer_rsrc_t r, int vo, int so) {
        return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, vo, so, 0));
    };
    auto load_a = [&](f32x4 (&dst)[2], int i, int s) __attribute__((always_inline)) {
        const int so = ab + min(s, last) * 64;
        dst[0] = ld(rA, voA[i], so);
        dst[1] = ld(rA, voA[i] + 16, so);
    };
    auto load_b = [&](f32x4 (&dst)[8], int s) __attribute__((always_inline)) {
        const int so = bb + min(s, last) * bstep;
#pragma unroll
        for (int e = 0; e < 8; ++e) dst[e] = ld(rB, voB, so + e * ldb * 4);
    };

    f32x4 ra[4][2];     // raw A of each M-tile, one step ahead of its split
    f32x4 rb[2][8];     // raw B: [step parity][k row e]
    Planes pa[2];       // A planes of the current / next M-tile
    Planes pb[2][4];    // B planes: [step parity][N-tile]
    f32x16 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x16{0};

    // Prologue. Per step s the loop issues A1(s+1) A2(s+1) A3(s+1) A0(s+2) B(s+3); the prologue leaves the same
    // sequence in flight (B(1) | A1(0) A2(0) A3(0) A0(1) B(2)), so the waits the compiler derives at the loop
    // header (merged over the prologue and the back edge) count only loads issued after the awaited one.
    load_a(ra[0], 0, 0);
    load_b(rb[0], 0);
#pragma unroll
    for (int d = 0; d < 4; ++d) split_b_word(rb[0], d, pb[0]);
    split_a4(ra[0], pa[0]);
    __builtin_amdgcn_sched_barrier(0);
    load_b(rb[1], 1);
#pragma unroll
    for (int i = 1; i < 4; ++i) load_a(ra[i], i, 0);
    load_a(ra[0], 0, 1);
    load_b(rb[0], 2);
    __builtin_amdgcn_sched_barrier(0);

    // One 16-k step with compile-time parity P. Region i (one per M-tile) runs tile i's 24 MFMAs and, in their
    // shadow, the split of the next A tile and of word i of the B planes for step s+1 (72 VALU ops: 3 per MFMA,
    // interleaved by sched_group_barrier when VPM > 0).
    auto step = [&](int s, auto P_) __attribute__((always_inline)) {
        constexpr int P = decltype(P_)::value;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            __builtin_amdgcn_sched_barrier(0);  // one scheduling region per M-tile: loads stay in issue order
            const Planes& cur = pa[i & 1];
            const int in = (i + 1) & 3;  // next A tile: i+1 of this step, or tile 0 of step s+1
            split_a4<(VPM >= 10)>(ra[in], pa[in & 1]);
            load_a(ra[in], in, i < 3 ? s + 1 : s + 2);
            split_b_word<(VPM >= 10)>(rb[P ^ 1], i, pb[P ^ 1]);  // word i of every N-tile's planes for step s+1
            if (i == 3) load_b(rb[P ^ 1], s + 3);
#pragma unroll
            for (int p = 0; p < 6; ++p)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = mfma(cur.p[kPA[p]], pb[P][j].p[kPB[p]], acc[i][j]);
            if constexpr (VPM % 10 > 0) {
#pragma unroll
                for (int m = 0; m < 24; ++m) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);    // 1 MFMA
                    __builtin_amdgcn_sched_group_barrier(0x002, VPM % 10, 0);  // VPM VALU
                }
            }
        }
    };
    for (int s = 0; s < ns; s += 2) {  // ns even (K % 32 == 0)
        step(s, std::integral_constant<int, 0>{});
        step(s + 1, std::integral_constant<int, 1>{});
    }

    // epilogue: lane (l32, h) holds column c0 + 4 l32 + j of N-tile j and rows 4h + (r & 3) + 8 (r >> 2) of each
    // 32x32 tile: the 4 N-tiles form one 16-B store
    const int r0 = m0 + wm * 128, c0 = n0 + wn * 128;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int so = ((r0 + i * 32 + (r & 3) + 8 * (r >> 2)) * ldc + c0) * 4;
            f32x4 v{alpha * acc[i][0][r], alpha * acc[i][1][r], alpha * acc[i][2][r], alpha * acc[i][3][r]};
            if constexpr (BETA) v += beta * ld(rC, voC, so);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rC, voC, so, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
}
}  // namespace

namespace {
template <class F>
int launch_x6(const float* A, const float* B, float* C, int M, int N, int K, int lda, int ldb, int ldc, F&& go) {
    if (M <= 0 || N <= 0 || K <= 0 || M % 256 || N % 256 || K % 32) return PCMX_ERR_ARG;
    if ((lda | ldb | ldc) & 3 || (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) & 15)) return PCMX_ERR_ARG;
    if ((long long)M * lda * 4 >= (1LL << 31) || (long long)K * ldb * 4 >= (1LL << 31) ||
        (long long)M * ldc * 4 >= (1LL << 31))
        return PCMX_ERR_ARG;
    go((M / 256) * (N / 256));
    return (int)hipGetLastError();
}
}  // namespace

// Lab knob: 0 = production schedule (3 VALU per MFMA), 2 / 4 = 2 / 4 VALU per MFMA in the interleave pattern,
// 5 = compiler-scheduled regions. Measured at 8192^3 (profiles/r3_sgemm_x6/ab_schedules.log): 4.15 / 4.35 / 4.20 /
// 4.49 ms; the first form (B planes rebuilt only in the last M-tile's region, compiler-scheduled) 4.73 ms.
extern "C" int pcmx_sgemm_f32_x6_variant(const float* A, const float* B, float* C, int M, int N, int K, int lda,
                                         int ldb, int ldc, float alpha, float beta, int v, hipStream_t s) {
    return launch_x6(A, B, C, M, N, K, lda, ldb, ldc, [&](int tiles) {
#define PCMX_X6(VPM)                                                                                                  \
    (beta != 0.f                                                                                                      \
         ? sgemm_x6_kernel<true, VPM><<<tiles, 256, 0, s>>>(A, B, C, M, N, K, lda, ldb, ldc, alpha, beta)             \
         : sgemm_x6_kernel<false, VPM><<<tiles, 256, 0, s>>>(A, B, C, M, N, K, lda, ldb, ldc, alpha, beta))
        switch (v) {
            case 2: PCMX_X6(2); break;
            case 4: PCMX_X6(4); break;
            case 5: PCMX_X6(0); break;
            case 13: PCMX_X6(13); break;  // lab: split VALU priced out (wrong results)
            default: PCMX_X6(3); break;
        }
#undef PCMX_X6
    });
}

// C = alpha * A @ B + beta * C, fp32 operands and result, computed on the bf16 matrix cores with exact 3-way
// operand splitting (fp32 accuracy). M, N % 256 == 0, K % 32 == 0, 16-B aligned rows, 32-bit byte offsets.
extern "C" int pcmx_sgemm_f32_x6(const float* A, const float* B, float* C, int M, int N, int K, int lda, int ldb,
                                 int ldc, float alpha, float beta, hipStream_t s) {
    return pcmx_sgemm_f32_x6_variant(A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, 0, s);
}
