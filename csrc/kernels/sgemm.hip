// FP32 SGEMM on the gfx950 matrix cores — the headline "TFLOPS SGEMM 8192^2" kernel.
// Reference ancestor: matrix_multiply, ref 1-introduction/matrix.c:63-81 (naive i-j-k on float**).
//
// Production kernels only (experimental variants and tuning knobs live in scripts/sgemm_lab.hip and
// scripts/sgemm_dr_lab.hip):
//   variant 17  persistent LDS-free "direct register" kernel, 4 waves (one per SIMD, 128x128 wave tiles) —
//               large problems (round 3; 8192^3: 153.7-154.0 TFLOPS vs hipBLASLt 153.3-153.8 on the same box,
//               both ~99% of the 155 TF measured f32 MFMA peak; scripts/sgemm_dr_ab.py)
//   variant 18  variant 17 with the grid capped at 7 blocks (tests: many tiles per block, uneven split)
//   variant 16  register-staged 256x256x32 tile, 8 waves (2 per SIMD, 64x128 wave tiles) — round-2 production
//   variant 0   LDS-DMA 256x256x32 tile, 8 waves — fallback when buffer offsets would exceed 2 GiB
//   variant 1   LDS-DMA 128x128x32 tile, 4 waves — problems with fewer than 192 256x256 tiles (fills 256 CUs)
//   variant 20  fp32 GEMM on the BF16 matrix cores by exact 3-way operand splitting (sgemm_x6.hip): fp32
//               accuracy, not the f32 MFMA; reported beside the headline, never as it
//   simt        reference-style f32 VALU GEMM (the "CUDA port recompiled" baseline), any shape
//
// Why this shape (MI355X_MICROARCH.md "Matrix cores", cdna_hip_programming.md §3/§5):
//  * v_mfma_f32_32x32x2_f32 is exact f32 (a k-ordered fmaf chain) at 64 FLOP/clk/SIMD = the f32 peak
//    (157 TF); one VGPR per operand per lane, so operand traffic is tiny and the kernel is MFMA-bound as long
//    as the issue stream stays clean.
//  * K-permutation: the MFMA's two k-slots (h = lane>>5) are fed k = 8c+4h+s at step s, so ONE ds_read_b128
//    delivers a lane's A operands for 4 MFMA steps. A and B agree on the permutation, so the sum is the full
//    K sum.
//  * A-tile bank conflicts: the LDS-DMA kernels swizzle 16-B chunks (slot = chunk ^ ((row>>1)&7)); the
//    register-staged kernel pads A rows instead (see variant 16).
//  * XCD-aware bijective block remap + grouped tile order (8 tile-rows per column strip): the blocks resident
//    on one XCD share A/B panels in that XCD's L2.
#include "pcmx_common.h"
#include "pcmx_hip.h"

namespace {
using pcmx::kWave;
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) float lds_float;
typedef __attribute__((address_space(3))) pcmx::f32x4 lds_f4;

template <int BM_, int BN_, int WM_, int WN_>
struct Cfg {
    static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, BK = 32;
    static constexpr int kWaves = WM * WN;
    static constexpr int kThreads = kWaves * kWave;
    static constexpr int kWaveM = BM / WM, kWaveN = BN / WN;
    static constexpr int MT = kWaveM / 32, NT = kWaveN / 32;
    static constexpr int kAFloats = BM * BK, kBFloats = BK * BN;
    static constexpr int kStage = kAFloats + kBFloats;
    static constexpr int kAPieces = kAFloats / 256, kBPieces = kBFloats / 256;  // 1-KiB DMA pieces
    static constexpr int kBLanesPerRow = BN / 4;                               // 16-B chunks per B k-row
    static_assert(kAPieces % kWaves == 0 && kBPieces % kWaves == 0, "DMA pieces must split over waves");
    static_assert(BN <= 256 && 256 % BN == 0, "a B piece holds whole k-rows");
    static_assert(MT >= 1 && NT >= 1, "wave tile must hold a 32x32 MFMA tile");
};
using Big = Cfg<256, 256, 2, 4>;
using Small = Cfg<128, 128, 2, 2>;

// Tile of block blockIdx.x: XCD remap (blocks dealt to one XCD get consecutive ids), then column strips 8
// tile-rows tall (any bijection is correct; this order keeps an XCD's concurrent tiles on shared panels).
template <int BM, int BN>
__device__ __forceinline__ void tile_coords(int M, int N, int& m0, int& n0) {
    constexpr int kGroupM = 8;
    const int tiles_m = M / BM, tiles_n = N / BN;
    const int t = pcmx::xcd_remap((int)blockIdx.x, tiles_m * tiles_n);
    const int per_group = kGroupM * tiles_n;
    const int first_m = (t / per_group) * kGroupM;
    const int gsz = min(tiles_m - first_m, kGroupM);
    m0 = (first_m + (t % per_group) % gsz) * BM;
    n0 = ((t % per_group) / gsz) * BN;
}

// 16-B global->LDS DMA issued from inline asm: hipcc does not count asm memory ops, so it cannot insert the
// conservative `s_waitcnt vmcnt(0)` it emits before every ds_read that *might* alias an in-flight builtin
// LDS-DMA. The kernel waits for the DMA itself (vmcnt(0) + barrier) once per K-step. M0 is set and restored
// inside the same statement (cdna_hip_programming.md §5.7).
__device__ __forceinline__ void glds16(const float* gsrc, lds_float* lds_base) {
    const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds_base);
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(gsrc), "s"(dst)
        : "memory");
}

// One K-step stage of A (swizzle applied to the SOURCE chunk, the LDS image is lane-linear) and B.
template <class C>
__device__ __forceinline__ void stage_load(const float* __restrict__ A, const float* __restrict__ B, int lda, int ldb,
                                           int m0, int n0, int k0, lds_float* sA, lds_float* sB, int wave, int lane) {
#pragma unroll
    for (int i = 0; i < C::kAPieces / C::kWaves; ++i) {
        const int p = wave * (C::kAPieces / C::kWaves) + i;  // rows 8p .. 8p+7
        const int r = p * 8 + (lane >> 3);
        const int chunk = (lane & 7) ^ ((r >> 1) & 7);
        glds16(A + (size_t)(m0 + r) * lda + k0 + chunk * 4, sA + p * 256);
    }
#pragma unroll
    for (int i = 0; i < C::kBPieces / C::kWaves; ++i) {
        const int p = wave * (C::kBPieces / C::kWaves) + i;
        const int kr = p * (256 / C::BN) + lane / C::kBLanesPerRow;
        const int col = (lane % C::kBLanesPerRow) * 4;
        glds16(B + (size_t)(k0 + kr) * ldb + n0 + col, sB + p * 256);
    }
}

// ---------------------------------------------------------------------------------------------------
// Variants 0 / 1: LDS-DMA staging (global_load_lds_dwordx4, 1 KiB per wave instruction, no VGPR round trip),
// two LDS stages, rotated schedule: fragments of step kc+1 are read while the MFMAs of step kc run; the barrier
// that publishes stage t+1 sits between the LAST fragment reads of stage t and the first reads of stage t+1.
template <class C, bool BETA>
__global__ __launch_bounds__(C::kThreads) void sgemm_dma_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                               float* __restrict__ Cmat, int M, int N, int K, int lda,
                                                               int ldb, int ldc, float alpha, float beta) {
    __shared__ __attribute__((aligned(16))) float smem[2 * C::kStage];
    lds_float* lds = (lds_float*)smem;
    const int lane = pcmx::lane_id();
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int wm = wave / C::WN, wn = wave % C::WN;
    const int h = lane >> 5, l32 = lane & 31;
    int m0, n0;
    tile_coords<C::BM, C::BN>(M, N, m0, n0);

    f32x16 acc[C::MT][C::NT];
#pragma unroll
    for (int i = 0; i < C::MT; ++i)
#pragma unroll
        for (int j = 0; j < C::NT; ++j) acc[i][j] = f32x16{0};
    int a_row_off[C::MT], a_swz[C::MT];
#pragma unroll
    for (int i = 0; i < C::MT; ++i) {
        const int r = wm * C::kWaveM + i * 32 + l32;
        a_row_off[i] = r * C::BK;
        a_swz[i] = (r >> 1) & 7;
    }
    const int b_col = wn * C::kWaveN + l32;

    const int nk = K / C::BK;
    stage_load<C>(A, B, lda, ldb, m0, n0, 0, lds, lds + C::kAFloats, wave, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    pcmx::f32x4 fa0[C::MT], fa1[C::MT];
    float fb0[C::NT][4], fb1[C::NT][4];
    auto read = [&](const lds_float* stage, int kc, pcmx::f32x4(&a)[C::MT], float(&b)[C::NT][4]) {
        const lds_float* sB = stage + C::kAFloats;
#pragma unroll
        for (int i = 0; i < C::MT; ++i) a[i] = *(const lds_f4*)(stage + a_row_off[i] + ((2 * kc + h) ^ a_swz[i]) * 4);
#pragma unroll
        for (int j = 0; j < C::NT; ++j)
#pragma unroll
            for (int s = 0; s < 4; ++s) b[j][s] = sB[(kc * 8 + 4 * h + s) * C::BN + b_col + j * 32];
    };
    auto mma = [&](const pcmx::f32x4(&a)[C::MT], const float(&b)[C::NT][4]) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int i = 0; i < C::MT; ++i)
#pragma unroll
                for (int j = 0; j < C::NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][s], b[j][s], acc[i][j], 0, 0, 0);
    };
    read(lds, 0, fa0, fb0);
    for (int t = 0; t < nk; ++t) {
        lds_float* cur = lds + (t & 1) * C::kStage;
        lds_float* nxt = lds + ((t + 1) & 1) * C::kStage;
        if (t + 1 < nk) stage_load<C>(A, B, lda, ldb, m0, n0, (t + 1) * C::BK, nxt, nxt + C::kAFloats, wave, lane);
        read(cur, 1, fa1, fb1);
        mma(fa0, fb0);
        read(cur, 2, fa0, fb0);
        mma(fa1, fb1);
        read(cur, 3, fa1, fb1);
        mma(fa0, fb0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t + 1 < nk) read(nxt, 0, fa0, fb0);
        mma(fa1, fb1);
    }

    // epilogue: lane holds column l32 and rows (r&3) + 8*(r>>2) + 4*h of each 32x32 tile
#pragma unroll
    for (int i = 0; i < C::MT; ++i)
#pragma unroll
        for (int j = 0; j < C::NT; ++j) {
            const int col = n0 + wn * C::kWaveN + j * 32 + l32;
            const int rbase = m0 + wm * C::kWaveM + i * 32 + 4 * h;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                float* p = Cmat + (size_t)(rbase + (r & 3) + 8 * (r >> 2)) * ldc + col;
                const float v = alpha * acc[i][j][r];
                *p = BETA ? v + beta * (*p) : v;
            }
        }
}

// ---------------------------------------------------------------------------------------------------
// Variant 16 (production for large problems): register-staged, 8 waves (2 per SIMD) as 4(M) x 2(N), wave tile
// 64x128 = 2x4 MFMA tiles (128 accumulators in VGPRs): the second wave of a SIMD issues MFMAs while the other
// waits at the per-stage barrier. Every LDS access is 16 B wide.
//  * Staging: buffer_load_dwordx4 (one SRD per operand, 32-bit voffset + scalar soffset) into 8 x 16-B
//    registers, ds_write_b128 into the other LDS stage. Loads run TWO stages ahead (the registers holding
//    stage t+1 are written to LDS during stage t and immediately reloaded with stage t+2), so HBM/L2 latency
//    never reaches the MFMA stream. (The LDS-DMA form of the same kernel loses ~5% to DMA issue cost.)
//  * B columns are interleaved across the wave's 4 N-tiles (tile j owns columns 4c+j), so ONE ds_read_b128 of a
//    B row yields the operands of all 4 tiles for one k (no transpose, conflict-free) and the epilogue stores
//    16 B per lane (512 contiguous bytes per row).
//  * Padded A rows (BK + 4 = 36 floats, 144 B): the 16 rows of a ds_read_b128 lane group start 36 dwords apart,
//    which covers all 64 banks exactly once (conflict-free without a swizzle), so the k-chunk enters the read
//    address as a compile-time offset instead of a lane-dependent XOR. Measured at 8192^3 (interleaved A/B,
//    scripts/sgemm_ab.py): 149.2-149.8 TFLOPS with the XOR swizzle -> 151.2-151.4 padded (lab variant 19).
//  * Each staging piece (ds_write + buffer load) is pinned between MFMA groups (sched_barrier) in chunks 0-1
//    of the stage, so it issues in the MFMA shadow. (Spreading them over all 4 chunks is a race: chunk 3 runs
//    after the barrier while other waves already read `nxt`.)
struct CfgRS8 {
    static constexpr int BM = 256, BN = 256, BK = 32, WM = 4, WN = 2;
    static constexpr int kWaves = WM * WN, kThreads = kWaves * kWave;
    static constexpr int kWaveM = BM / WM, kWaveN = BN / WN;
    static constexpr int MT = kWaveM / 32, NT = kWaveN / 32;
    static constexpr int kAStride = BK + 4;  // padded A row (floats)
    static constexpr int kAFloats = BM * kAStride, kBFloats = BK * BN;
    static constexpr int kStage = kAFloats + kBFloats;  // 2 stages = 136 KiB of the 160 KiB LDS
    static constexpr int kAPW = BM / 8 / kWaves;  // A pieces (8 rows x 128 B) per wave
    static constexpr int kBPW = BK / kWaves;      // B pieces (one 1-KiB k-row) per wave
    static_assert(NT == 4, "interleaved-column B read assumes 4 N-tiles per wave");
};

template <bool BETA>
__global__ __launch_bounds__(CfgRS8::kThreads, 1) void sgemm_rs_kernel(const float* __restrict__ A,
                                                                      const float* __restrict__ B,
                                                                      float* __restrict__ Cmat, int M, int N, int K,
                                                                      int lda, int ldb, int ldc, float alpha, float beta) {
    using C = CfgRS8;
    __shared__ __attribute__((aligned(16))) float smem[2 * C::kStage];
    lds_float* lds = (lds_float*)smem;
    const int lane = pcmx::lane_id();
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int wm = wave / C::WN, wn = wave % C::WN;
    const int h = lane >> 5, l32 = lane & 31;
    int m0, n0;
    tile_coords<C::BM, C::BN>(M, N, m0, n0);

    // buffer resources: A rows of this block, B columns of this block (bounds = whole K extent)
    const __amdgpu_buffer_rsrc_t rA =
        __builtin_amdgcn_make_buffer_rsrc((void*)(A + (size_t)m0 * lda), (short)0, C::BM * lda * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)(B + n0), (short)0, K * ldb * 4, 0x00020000);
    const int voA = ((lane >> 3) * lda + (lane & 7) * 4) * 4;
    const int voB = lane * 16;
    int lwA[C::kAPW];  // LDS byte addresses of this lane's A pieces (identical every stage up to the stage base)
#pragma unroll
    for (int i = 0; i < C::kAPW; ++i) {
        const int r = (wave * C::kAPW + i) * 8 + (lane >> 3);
        lwA[i] = r * C::kAStride * 4 + (lane & 7) * 16;
    }
    const int lwB = (C::kAFloats + wave * C::kBPW * C::BN) * 4 + lane * 16;

    pcmx::f32x4 R[C::kAPW + C::kBPW];
    auto gload = [&](int q, int k0) {  // piece q (A pieces first, then B) of the stage starting at k0
        if (q < C::kAPW) {
            const int so = ((wave * C::kAPW + q) * 8 * lda + k0) * 4;
            R[q] = __builtin_bit_cast(pcmx::f32x4, __builtin_amdgcn_raw_buffer_load_b128(rA, voA, so, 0));
        } else {
            const int so = (k0 + wave * C::kBPW + (q - C::kAPW)) * ldb * 4;
            R[q] = __builtin_bit_cast(pcmx::f32x4, __builtin_amdgcn_raw_buffer_load_b128(rB, voB, so, 0));
        }
    };
    typedef __attribute__((address_space(3))) char lds_char;
    auto lwrite = [&](int q, lds_float* stage) {
        lds_char* base = (lds_char*)stage;
        if (q < C::kAPW)
            *(lds_f4*)(base + lwA[q]) = R[q];
        else
            *(lds_f4*)(base + lwB + (q - C::kAPW) * C::BN * 4) = R[q];
    };

    f32x16 acc[C::MT][C::NT];
#pragma unroll
    for (int i = 0; i < C::MT; ++i)
#pragma unroll
        for (int j = 0; j < C::NT; ++j) acc[i][j] = f32x16{0};
    int a_off[C::MT];  // lane's A row, k offset 4h (the K-permutation); chunk kc adds 8 kc floats
#pragma unroll
    for (int i = 0; i < C::MT; ++i) a_off[i] = (wm * C::kWaveM + i * 32 + l32) * C::kAStride + 4 * h;
    const int b_off = C::kAFloats + wn * C::kWaveN + 4 * l32;

    auto read = [&](const lds_float* stage, int kc, pcmx::f32x4(&a)[C::MT], pcmx::f32x4(&b)[4]) {
#pragma unroll
        for (int i = 0; i < C::MT; ++i) a[i] = *(const lds_f4*)(stage + a_off[i] + 8 * kc);
#pragma unroll
        for (int s = 0; s < 4; ++s) b[s] = *(const lds_f4*)(stage + b_off + (kc * 8 + 4 * h + s) * C::BN);
    };
    // filler(slot) runs after every NT MFMAs (slot = s * MT + i)
    auto mma = [&](const pcmx::f32x4(&a)[C::MT], const pcmx::f32x4(&b)[4], auto&& filler) __attribute__((always_inline)) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int i = 0; i < C::MT; ++i) {
#pragma unroll
                for (int j = 0; j < C::NT; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][s], b[s][j], acc[i][j], 0, 0, 0);
                filler(s * C::MT + i);
            }
    };
    auto pin = [](auto&& f) {
        __builtin_amdgcn_sched_barrier(0);
        f();
        __builtin_amdgcn_sched_barrier(0);
    };

    const int nk = K / C::BK;
    // prologue: stage 0 -> LDS buffer 0, stage 1 -> registers
#pragma unroll
    for (int q = 0; q < C::kAPW + C::kBPW; ++q) gload(q, 0);
#pragma unroll
    for (int q = 0; q < C::kAPW + C::kBPW; ++q) lwrite(q, lds);
    if (nk > 1) {
#pragma unroll
        for (int q = 0; q < C::kAPW + C::kBPW; ++q) gload(q, C::BK);
    }
    __syncthreads();

    pcmx::f32x4 fa0[C::MT], fa1[C::MT], fb0[4], fb1[4];
    read(lds, 0, fa0, fb0);
    auto stage = [&](int t, auto write_c, auto load_c) {
        constexpr bool WRITE = decltype(write_c)::value;  // registers hold stage t+1
        constexpr bool LOAD = decltype(load_c)::value;    // stage t+2 exists
        lds_float* cur = lds + (t & 1) * C::kStage;
        lds_float* nxt = lds + ((t + 1) & 1) * C::kStage;
        const int k2 = (t + 2) * C::BK;
        // the stage's P = kAPW + kBPW pieces spread evenly over chunks 0-1, one per kEvery filler slots
        auto chunk_filler = [&](int chunk) __attribute__((always_inline)) {
            return [&, chunk](int slot) __attribute__((always_inline)) {
                if constexpr (!WRITE) return;
                constexpr int P = C::kAPW + C::kBPW, kSlots = 4 * C::MT;
                constexpr int kChunks = 2, kPer = P / kChunks, kEvery = kSlots / kPer;
                static_assert(P % kChunks == 0 && kSlots % kPer == 0, "even piece spread");
                if (chunk < kChunks && (slot + 1) % kEvery == 0) {
                    const int qq = chunk * kPer + slot / kEvery;
                    pin([&] {
                        lwrite(qq, nxt);
                        if constexpr (LOAD) gload(qq, k2);
                    });
                }
            };
        };
        read(cur, 1, fa1, fb1);
        mma(fa0, fb0, chunk_filler(0));
        read(cur, 2, fa0, fb0);
        mma(fa1, fb1, chunk_filler(1));
        read(cur, 3, fa1, fb1);
        mma(fa0, fb0, chunk_filler(2));
        __syncthreads();
        if constexpr (WRITE) read(nxt, 0, fa0, fb0);
        mma(fa1, fb1, chunk_filler(3));
    };
    int t = 0;
    for (; t + 2 < nk; ++t) stage(t, std::true_type{}, std::true_type{});
    if (t + 1 < nk) stage(t++, std::true_type{}, std::false_type{});
    stage(t, std::false_type{}, std::false_type{});

    // epilogue: tile j holds columns 4c+j, so a lane's 4 tiles form one contiguous 16-B store
#pragma unroll
    for (int i = 0; i < C::MT; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = m0 + wm * C::kWaveM + i * 32 + 4 * h + (r & 3) + 8 * (r >> 2);
            pcmx::f32x4* p = reinterpret_cast<pcmx::f32x4*>(Cmat + (size_t)row * ldc + n0 + wn * C::kWaveN + 4 * l32);
            pcmx::f32x4 v{alpha * acc[i][0][r], alpha * acc[i][1][r], alpha * acc[i][2][r], alpha * acc[i][3][r]};
            if constexpr (BETA) v += beta * (*p);
            *p = v;
        }
}

// ---------------------------------------------------------------------------------------------------
// Variant 17 (production for large problems): persistent, LDS-free "direct register" kernel.
// v_mfma_f32_32x32x2_f32 needs ONE operand VGPR per 2048 MACs, so a 128x128 wave tile (4x4 MFMA tiles, 256
// accumulators) consumes only 8 operand VGPRs per 16 MFMAs (1024 SIMD cycles). That is few enough to load the
// operands straight from L2 into the MFMA operand registers: no LDS stage, no ds_write/ds_read, no workgroup
// barrier. Each of the 4 waves (one per SIMD, 512 registers) is an independent MFMA stream whose loads are
// issued ~8k cycles ahead. Counters (profiles/r3_sgemm/): 98.3-98.5% of the kernel's cycles are MFMA-busy
// against 96.4% for variant 16 (barrier stalls of its 8-wave LDS pipeline) and 97.9% for hipBLASLt.
//  * MFMA step t of a 32-k chunk feeds k-slot h (= lane >> 5) with k = k0 + 16h + t.
//  * A: lane (l32, h) loads A[row l32][k0 + 16h + 4q .. +3] (q = 0..3, issued back to back: the four loads share
//    each row's 128-B line); component s is the operand of step 4q + s. Double-buffered per chunk.
//  * B: lane (l32, h) loads B[k0 + 16h + t][c0 + 4 l32 .. +3]: N-tile j owns columns c0 + 4c + j, so one 16-B load
//    holds the operands of the wave's 4 N-tiles (two 512-B row segments per instruction). 8-step register ring.
//  * Persistent: grid = min(tiles, CUs); block b runs tiles j * grid + xcd_remap(b). In a tile's last iteration
//    the look-ahead loads already fetch the next tile's chunk 0 / steps 0-7 (every tile-dependent address is a
//    scalar soffset over one buffer resource per operand), so the next tile starts with its operands in flight
//    and the epilogue's C stores drain under its MFMAs.
//  * The prologue's B loads are pinned in step order so the loop-top wait (merged over the prologue and the back
//    edge) stays vmcnt(7); the epilogue issues one store at a time (bounded live registers, no spills).
template <bool BETA>
__global__ __launch_bounds__(256, 1) void sgemm_direct_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                              float* __restrict__ C, int M, int N, int K, int lda,
                                                              int ldb, int ldc, float alpha, float beta) {
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const int lane = pcmx::lane_id();
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int h = lane >> 5, l32 = lane & 31;
    const int ntiles = (M / 256) * (N / 256), grid = (int)gridDim.x;
    const int xid = pcmx::xcd_remap((int)blockIdx.x, grid);

    const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rC = __builtin_amdgcn_make_buffer_rsrc((void*)C, (short)0, 0x7fffffff, 0x00020000);
    int voA[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) voA[i] = ((32 * i + l32) * lda + 16 * h) * 4;
    const int voB = (16 * h * ldb + 4 * l32) * 4;
    const int voC = (4 * h * ldc + 4 * l32) * 4;
    const int nk = K / 32;
    const int ldb128 = ldb * 128;  // bytes per 32 k-rows of B
    auto bload = [](__amdgpu_buffer_rsrc_t r, int vo, int so) {
        return __builtin_bit_cast(pcmx::f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, vo, so, 0));
    };

    // scalar byte bases of the block's tile j (past the end: the block's last tile, loaded and never used)
    auto bases = [&](int j, int& ab, int& bb, int& m0, int& n0) {
        int T = j * grid + xid;
        if (T >= ntiles) T = ((ntiles - 1 - xid) / grid) * grid + xid;
        const int tiles_n = N / 256, per_group = 8 * tiles_n, first_m = (T / per_group) * 8;
        const int gsz = min(M / 256 - first_m, 8);
        m0 = __builtin_amdgcn_readfirstlane((first_m + (T % per_group) % gsz) * 256);
        n0 = __builtin_amdgcn_readfirstlane(((T % per_group) / gsz) * 256);
        ab = __builtin_amdgcn_readfirstlane((m0 + wm * 128) * lda * 4);
        bb = __builtin_amdgcn_readfirstlane((n0 + wn * 128) * 4);
    };

    pcmx::f32x4 a[2][4][4];  // [chunk parity][M-tile i][q]
    pcmx::f32x4 b[8];        // ring: step t's B operands in slot t % 8
    f32x16 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x16{0};
    auto pin = [](auto&& f) __attribute__((always_inline)) {
        __builtin_amdgcn_sched_barrier(0);
        f();
        __builtin_amdgcn_sched_barrier(0);
    };

    int ab, bb, m0, n0;
    bases(0, ab, bb, m0, n0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) a[0][i][q] = bload(rA, voA[i] + 16 * q, ab);
#pragma unroll
    for (int t = 0; t < 8; ++t) pin([&] { b[t] = bload(rB, voB, bb + t * ldb * 4); });

    int jt = 0;
    do {  // grid <= tiles: every block has a tile; nk >= 2 (K % 64 == 0)
        int abn, bbn, m0n, n0n;
        bases(jt + 1, abn, bbn, m0n, n0n);
        int kc = 0;
        do {
            const bool last = kc + 2 == nk;
            // chunk p = 0: every look-ahead load stays inside the tile
#pragma unroll
            for (int t = 0; t < 16; ++t) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[0][i][t >> 2][t & 3], b[t & 7][j], acc[i][j], 0, 0, 0);
                    if (i == 3)  // after the step's last read of slot t % 8
                        pin([&] {
                            const int so = t + 8 < 16 ? kc * ldb128 + (t + 8) * ldb * 4 : (kc + 1) * ldb128 + (t - 8) * ldb * 4;
                            b[t & 7] = bload(rB, voB, bb + so);
                        });
                    if (t < 4) pin([&] { a[1][t][i] = bload(rA, voA[t] + 16 * i, ab + (kc + 1) * 128); });
                }
            }
            // chunk p = 1: in the tile's last iteration the look-ahead crosses into the next tile
            const int aso = last ? abn : ab + (kc + 2) * 128;
            const int bso = last ? bbn : bb + (kc + 2) * ldb128;
#pragma unroll
            for (int t = 0; t < 16; ++t) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[1][i][t >> 2][t & 3], b[t & 7][j], acc[i][j], 0, 0, 0);
                    if (i == 3)
                        pin([&] {
                            const int so = t + 8 < 16 ? bb + (kc + 1) * ldb128 + (t + 8) * ldb * 4 : bso + (t - 8) * ldb * 4;
                            b[t & 7] = bload(rB, voB, so);
                        });
                    if (t < 4) pin([&] { a[0][t][i] = bload(rA, voA[t] + 16 * i, aso); });
                }
            }
            kc += 2;
        } while (kc < nk);
        // epilogue of tile jt: lane (l32, h) holds column l32 of each N-tile j (= c0 + 4 l32 + j) and rows
        // 4h + (r & 3) + 8 (r >> 2) of each 32x32 tile, so the 4 N-tiles form one 16-B store; the row goes in soffset
        const int r0 = m0 + wm * 128, c0 = n0 + wn * 128;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int so = ((r0 + i * 32 + (r & 3) + 8 * (r >> 2)) * ldc + c0) * 4;
                pcmx::f32x4 v{alpha * acc[i][0][r], alpha * acc[i][1][r], alpha * acc[i][2][r], alpha * acc[i][3][r]};
                if constexpr (BETA) v += beta * bload(rC, voC, so);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rC, voC, so, 0);
                __builtin_amdgcn_sched_barrier(0);  // one store at a time: bounded live registers
            }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = f32x16{0};
        ab = abn, bb = bbn, m0 = m0n, n0 = n0n;
        ++jt;
    } while (xid + jt * grid < ntiles);
}

// ---------------------------------------------------------------------------------------------------
// Reference-style SIMT kernel (f32 VALU FMAs, 64x64 LDS tiles, 4x4 outputs per thread) — the "CUDA port
// recompiled" baseline the MFMA kernel is compared against. Any shape.
constexpr int kSimtT = 64;
__global__ __launch_bounds__(256) void sgemm_simt_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                         float* __restrict__ C, int M, int N, int K) {
    __shared__ float sA[16][kSimtT + 1];
    __shared__ float sB[16][kSimtT + 1];
    const int tx = threadIdx.x % 16, ty = threadIdx.x / 16;
    const int row0 = blockIdx.y * kSimtT, col0 = blockIdx.x * kSimtT;
    float acc[4][4] = {};
    for (int k0 = 0; k0 < K; k0 += 16) {
        for (int e = threadIdx.x; e < 16 * kSimtT; e += 256) {
            const int kk = e % 16, rr = e / 16;
            const int ar = row0 + rr, ak = k0 + kk;
            sA[kk][rr] = (ar < M && ak < K) ? A[(size_t)ar * K + ak] : 0.f;
            const int bk = k0 + e / kSimtT, bc = col0 + e % kSimtT;
            sB[e / kSimtT][e % kSimtT] = (bk < K && bc < N) ? B[(size_t)bk * N + bc] : 0.f;
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) {
            float av[4], bv[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) av[i] = sA[kk][ty * 4 + i], bv[i] = sB[kk][tx * 4 + i];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(av[i], bv[j], acc[i][j]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int r = row0 + ty * 4 + i, c = col0 + tx * 4 + j;
            if (r < M && c < N) C[(size_t)r * N + c] = acc[i][j];
        }
}

template <class C>
bool tile_aligned(int M, int N, int K) {
    return M > 0 && N > 0 && K > 0 && M % C::BM == 0 && N % C::BN == 0 && K % C::BK == 0;
}

template <class C>
int launch_dma(const float* A, const float* B, float* Cm, int M, int N, int K, int lda, int ldb, int ldc, float alpha,
               float beta, hipStream_t s) {
    if (!tile_aligned<C>(M, N, K)) return PCMX_ERR_ARG;
    if ((lda | ldb) & 3 || (((uintptr_t)A | (uintptr_t)B) & 15)) return PCMX_ERR_ARG;
    const int grid = (M / C::BM) * (N / C::BN);
    if (beta != 0.f)
        sgemm_dma_kernel<C, true><<<grid, C::kThreads, 0, s>>>(A, B, Cm, M, N, K, lda, ldb, ldc, alpha, beta);
    else
        sgemm_dma_kernel<C, false><<<grid, C::kThreads, 0, s>>>(A, B, Cm, M, N, K, lda, ldb, ldc, alpha, beta);
    return (int)hipGetLastError();
}

int launch_rs(const float* A, const float* B, float* Cm, int M, int N, int K, int lda, int ldb, int ldc, float alpha,
              float beta, hipStream_t s) {
    using C = CfgRS8;
    if (!tile_aligned<C>(M, N, K)) return PCMX_ERR_ARG;
    if ((lda | ldb | ldc) & 3 || (((uintptr_t)A | (uintptr_t)B | (uintptr_t)Cm) & 15)) return PCMX_ERR_ARG;
    // 32-bit buffer offsets: the block's A rows and the whole B panel must stay below 2 GiB
    if ((long long)C::BM * lda * 4 >= (1LL << 31) || (long long)K * ldb * 4 >= (1LL << 31)) return PCMX_ERR_ARG;
    const int grid = (M / C::BM) * (N / C::BN);
    if (beta != 0.f)
        sgemm_rs_kernel<true><<<grid, C::kThreads, 0, s>>>(A, B, Cm, M, N, K, lda, ldb, ldc, alpha, beta);
    else
        sgemm_rs_kernel<false><<<grid, C::kThreads, 0, s>>>(A, B, Cm, M, N, K, lda, ldb, ldc, alpha, beta);
    return (int)hipGetLastError();
}
int device_cus() {
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cus[dev] && hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus[dev] = 256;
    return cus[dev] > 0 ? cus[dev] : 256;
}

// max_blocks <= 0: one block per CU
int launch_direct(const float* A, const float* B, float* Cm, int M, int N, int K, int lda, int ldb, int ldc, float alpha,
                  float beta, int max_blocks, hipStream_t s) {
    if (M <= 0 || N <= 0 || K <= 0 || M % 256 || N % 256 || K % 64) return PCMX_ERR_ARG;
    if ((lda | ldb | ldc) & 3 || (((uintptr_t)A | (uintptr_t)B | (uintptr_t)Cm) & 15)) return PCMX_ERR_ARG;
    // every scalar byte offset (A row base + k, B k-row + column, C row + column) must stay below 2^31
    if ((long long)M * lda * 4 >= (1LL << 31) || (long long)K * ldb * 4 >= (1LL << 31) ||
        (long long)M * ldc * 4 >= (1LL << 31))
        return PCMX_ERR_ARG;
    const int tiles = (M / 256) * (N / 256);
    int grid = max_blocks > 0 ? max_blocks : device_cus();
    if (grid > tiles) grid = tiles;
    if (beta != 0.f)
        sgemm_direct_kernel<true><<<grid, 256, 0, s>>>(A, B, Cm, M, N, K, lda, ldb, ldc, alpha, beta);
    else
        sgemm_direct_kernel<false><<<grid, 256, 0, s>>>(A, B, Cm, M, N, K, lda, ldb, ldc, alpha, beta);
    return (int)hipGetLastError();
}
}  // namespace

extern "C" int pcmx_sgemm_f32_variant(const float* A, const float* B, float* C, int M, int N, int K, int lda, int ldb,
                                      int ldc, float alpha, float beta, int variant, hipStream_t s) {
    switch (variant) {
        case 0: return launch_dma<Big>(A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, s);
        case 1: return launch_dma<Small>(A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, s);
        case 16: return launch_rs(A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, s);
        case 17: return launch_direct(A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, 0, s);
        case 18: return launch_direct(A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, 7, s);
        case 20: return pcmx_sgemm_f32_x6(A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, s);
        default: return PCMX_ERR_ARG;
    }
}

extern "C" int pcmx_sgemm_f32(const float* A, const float* B, float* C, int M, int N, int K, int lda, int ldb, int ldc,
                              float alpha, float beta, hipStream_t s) {
    // 256x256 tiles when the grid fills the 256 CUs: the persistent direct-register variant 17 (K % 64 == 0 and
    // 32-bit scalar offsets), else register-staged variant 16, else the LDS-DMA variant 0; otherwise the 128x128
    // kernel (4x more tiles).
    const bool big_ok = tile_aligned<Big>(M, N, K) && (long long)(M / 256) * (N / 256) >= 192;
    if (big_ok) {
        int rc = launch_direct(A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, 0, s);
        if (rc != PCMX_ERR_ARG) return rc;
        rc = launch_rs(A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, s);
        return rc == PCMX_ERR_ARG ? launch_dma<Big>(A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, s) : rc;
    }
    return launch_dma<Small>(A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, s);
}

extern "C" int pcmx_sgemm_f32_simt(const float* A, const float* B, float* C, int M, int N, int K, hipStream_t s) {
    if (M <= 0 || N <= 0 || K <= 0) return PCMX_ERR_ARG;
    dim3 grid((N + kSimtT - 1) / kSimtT, (M + kSimtT - 1) / kSimtT);
    sgemm_simt_kernel<<<grid, 256, 0, s>>>(A, B, C, M, N, K);
    return (int)hipGetLastError();
}
