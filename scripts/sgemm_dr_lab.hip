// SGEMM LAB, round 3: LDS-free "direct register" f32 MFMA kernels (one wave per SIMD, 128x128 wave tiles).
// Built on demand by scripts/_lab.py (dr_lab()) into build/lab/libpcmx_sgemm_dr_lab.so.
//
// Idea: v_mfma_f32_32x32x2_f32 needs ONE operand VGPR per 2048 MACs, so a 128x128 wave tile consumes only
// 8 operand VGPRs (4 A + 4 B) per 16 MFMAs (1024 SIMD cycles). That is few enough to load the operands straight
// from global memory (L2) into the MFMA operand registers, with no LDS stage, no ds_write/ds_read and no
// workgroup barrier: each wave is an independent MFMA stream whose loads are issued ~8k cycles ahead.
//  * A (row-major M x K): lane (l32, h) loads 16 B = A[row l32][k0 + 16h + 4q .. +3]; component s feeds MFMA
//    step t = 4q + s with k = k0 + 16h + t (the MFMA's k-slot h = lane >> 5).
//  * B (row-major K x N): lane (l32, h) loads 16 B = B[k0 + 16h + t][c0 + 4 l32 .. +3]: the 4 components are the
//    operands of the wave's 4 N-tiles (tile j owns columns c0 + 4c + j), so a B load is two 512-B row segments.
//  * Epilogue: lane's 4 N-tiles form one contiguous 16-B store.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned pcmx_v4u __attribute__((ext_vector_type(4)));

constexpr int kNumXcd = 8;
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    const int q = nwg / kNumXcd, r = nwg % kNumXcd;
    const int xcd = bid % kNumXcd, slot = bid / kNumXcd;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
}

template <int BM, int BN, int GM>
__device__ __forceinline__ void tile_coords(int t, int M, int N, int& m0, int& n0) {
    const int tiles_m = M / BM, tiles_n = N / BN;
    const int per_group = GM * tiles_n;
    const int first_m = (t / per_group) * GM;
    const int gsz = min(tiles_m - first_m, GM);
    m0 = (first_m + (t % per_group) % gsz) * BM;
    n0 = ((t % per_group) / gsz) * BN;
}

__device__ __forceinline__ f32x4 bload(__amdgpu_buffer_rsrc_t r, int vo, int so) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, vo, so, 0));
}

// ASCHED 0: the next chunk's 16 A loads in steps 0-3 (one tile row per step, its 4 q-loads back to back: the 4
// loads share every 128-B line). ASCHED 1: one A load per step.
template <bool BETA, int ASCHED, int GM>
__global__ __launch_bounds__(256, 1) void sgemm_dr_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                          float* __restrict__ C, int M, int N, int K, int lda, int ldb,
                                                          int ldc, float alpha, float beta) {
    const int lane = (int)__lane_id();
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int h = lane >> 5, l32 = lane & 31;
    int m0, n0;
    tile_coords<256, 256, GM>(xcd_remap((int)blockIdx.x, (M / 256) * (N / 256)), M, N, m0, n0);
    const int r0 = m0 + wm * 128, c0 = n0 + wn * 128;

    const __amdgpu_buffer_rsrc_t rA =
        __builtin_amdgcn_make_buffer_rsrc((void*)(A + (size_t)r0 * lda), (short)0, 128 * lda * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t rB =
        __builtin_amdgcn_make_buffer_rsrc((void*)(B + c0), (short)0, (K - 1) * ldb * 4 + 512, 0x00020000);
    int voA[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) voA[i] = ((32 * i + l32) * lda + 16 * h) * 4;
    const int voB = (16 * h * ldb + 4 * l32) * 4;

    f32x4 a[2][4][4];  // [chunk parity][tile i][q]
    f32x4 b[8];        // ring: step t's B operands in slot t % 8
    f32x16 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x16{0};

    // Look-ahead loads past the end of K are clamped to the last chunk (loaded, never used): the scalar offset
    // is not part of the buffer range check, so it must stay inside the operands.
    const int nk = K / 32;
    auto loadA = [&](int p, int i, int q, int kc) {  // chunk kc (32 k) into parity p
        a[p][i][q] = bload(rA, voA[i] + 16 * q, min(kc, nk - 1) * 128);
    };
    auto loadB = [&](int slot, int gstep) {  // global step gstep: k row 32*(gstep/16) + gstep%16 (+16h in voB)
        b[slot] = bload(rB, voB, min((gstep >> 4) * 32 + (gstep & 15), K - 32 + 15) * ldb * 4);
    };
    auto pin = [](auto&& f) __attribute__((always_inline)) {
        __builtin_amdgcn_sched_barrier(0);
        f();
        __builtin_amdgcn_sched_barrier(0);
    };

    // prologue: chunk 0's A, steps 0..7 of B
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) loadA(0, i, q, 0);
#pragma unroll
    for (int t = 0; t < 8; ++t) pin([&] { loadB(t, t); });  // in step order (loop-top wait stays vmcnt(7))

    // one chunk of 16 steps; p = chunk parity (compile time), kc = chunk index
    auto chunk = [&](auto pc, int kc) __attribute__((always_inline)) {
        constexpr int p = decltype(pc)::value;
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const int gs = kc * 16 + t;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[p][i][t >> 2][t & 3], b[t & 7][j], acc[i][j], 0, 0, 0);
                if (i == 3) pin([&] { loadB(t & 7, gs + 8); });  // after the step's last read of slot t%8
                if constexpr (ASCHED == 0) {
                    if (t < 4) pin([&] { loadA(p ^ 1, t, i, kc + 1); });
                } else {
                    if (i == 2) pin([&] { loadA(p ^ 1, t >> 2, t & 3, kc + 1); });
                }
            }
        }
    };
    for (int kc = 0; kc < nk; kc += 2) {
        chunk(std::integral_constant<int, 0>{}, kc);
        chunk(std::integral_constant<int, 1>{}, kc + 1);
    }

#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = r0 + i * 32 + 4 * h + (r & 3) + 8 * (r >> 2);
            f32x4* ptr = reinterpret_cast<f32x4*>(C + (size_t)row * ldc + c0 + 4 * l32);
            f32x4 v{alpha * acc[i][0][r], alpha * acc[i][1][r], alpha * acc[i][2][r], alpha * acc[i][3][r]};
            if constexpr (BETA) v += beta * (*ptr);
            *ptr = v;
        }
}

template <int ASCHED, int GM>
int launch_dr(const float* A, const float* B, float* Cm, int M, int N, int K, int lda, int ldb, int ldc, float alpha,
              float beta, hipStream_t s) {
    if (M <= 0 || N <= 0 || K <= 0 || M % 256 || N % 256 || K % 64) return 1;
    if ((lda | ldb | ldc) & 3 || (((uintptr_t)A | (uintptr_t)B | (uintptr_t)Cm) & 15)) return 1;
    if (128LL * lda * 4 >= (1LL << 31) || (long long)(K + 64) * ldb * 4 >= (1LL << 31)) return 1;
    const int grid = (M / 256) * (N / 256);
    if (beta != 0.f)
        sgemm_dr_kernel<true, ASCHED, GM><<<grid, 256, 0, s>>>(A, B, Cm, M, N, K, lda, ldb, ldc, alpha, beta);
    else
        sgemm_dr_kernel<false, ASCHED, GM><<<grid, 256, 0, s>>>(A, B, Cm, M, N, K, lda, ldb, ldc, alpha, beta);
    return (int)hipGetLastError();
}

// Persistent form: grid = min(tiles, CUs); block b runs tiles j*grid + xcd_remap(b) (j = 0, 1, ...), and the load
// stream runs ACROSS tile boundaries: in the last iteration of a tile, the look-ahead loads already fetch the next
// tile's chunk 0 / steps 0-7, so the next tile starts with its operands in flight and the epilogue's C stores drain
// under the next tile's MFMAs (no per-tile prologue latency, no chip-wide synchronous store burst). Every
// tile-dependent address is a scalar byte offset (soffset) over one buffer resource per operand.
template <bool BETA, int GM, int DIAG = 0, int STAGGER = 0>  // DIAG 1: no C stores (diagnostic only: wrong results)
__global__ __launch_bounds__(256, 1) void sgemm_drp_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                           float* __restrict__ C, int M, int N, int K, int lda, int ldb,
                                                           int ldc, float alpha, float beta) {
    const int lane = (int)__lane_id();
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int h = lane >> 5, l32 = lane & 31;
    const int ntiles = (M / 256) * (N / 256), grid = (int)gridDim.x;
    const int xid = xcd_remap((int)blockIdx.x, grid);

    const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, 0x7fffffff, 0x00020000);
    int voA[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) voA[i] = ((32 * i + l32) * lda + 16 * h) * 4;
    const int voB = (16 * h * ldb + 4 * l32) * 4;
    const __amdgpu_buffer_rsrc_t rC = __builtin_amdgcn_make_buffer_rsrc((void*)C, (short)0, 0x7fffffff, 0x00020000);
    const int voC = (4 * h * ldc + 4 * l32) * 4;
    const int nk = K / 32;
    const int ldb128 = ldb * 128;  // bytes per 32 k-rows of B

    // scalar byte bases of tile j (a tile past the end maps to the block's last tile: loaded, never used)
    auto bases = [&](int j, int& ab, int& bb, int& m0, int& n0) {
        int T = j * grid + xid;
        if (T >= ntiles) T = ((ntiles - 1 - xid) / grid) * grid + xid;
        tile_coords<256, 256, GM>(T, M, N, m0, n0);
        m0 = __builtin_amdgcn_readfirstlane(m0);
        n0 = __builtin_amdgcn_readfirstlane(n0);
        ab = __builtin_amdgcn_readfirstlane((m0 + wm * 128) * lda * 4);
        bb = __builtin_amdgcn_readfirstlane((n0 + wn * 128) * 4);
    };

    f32x4 a[2][4][4];
    f32x4 b[8];
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

    // STAGGER: waves (wm, wn) start (wm + wn) * STAGGER * 64 cycles late, so the two waves sharing an A row panel
    // (same wm) or a B column panel (same wn) issue their identical loads one offset apart (L1 hits, not two L2
    // requests in flight for the same line)
    if constexpr (STAGGER > 0) {
        for (int z = 0; z < wm + wn; ++z) __builtin_amdgcn_s_sleep(STAGGER);
    }
    int ab, bb, m0, n0;
    bases(0, ab, bb, m0, n0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) a[0][i][q] = bload(rA, voA[i] + 16 * q, ab);
#pragma unroll
    for (int t = 0; t < 8; ++t) pin([&] { b[t] = bload(rB, voB, bb + t * ldb * 4); });  // in step order: the
    // loop-top wait (merged over the prologue and the back edge) stays vmcnt(7)

    int j = 0;
    do {  // grid <= tiles: every block has a tile; nk >= 2 (K % 64 == 0)
        int abn, bbn, m0n, n0n;
        bases(j + 1, abn, bbn, m0n, n0n);
        int kc = 0;
        do {
            const bool last = kc + 2 == nk;
            // chunk p=0: loads stay inside the tile
#pragma unroll
            for (int t = 0; t < 16; ++t) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj)
                        acc[i][jj] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[0][i][t >> 2][t & 3], b[t & 7][jj], acc[i][jj], 0, 0, 0);
                    if (i == 3)
                        pin([&] {
                            const int so = t + 8 < 16 ? kc * ldb128 + (t + 8) * ldb * 4 : (kc + 1) * ldb128 + (t - 8) * ldb * 4;
                            b[t & 7] = bload(rB, voB, bb + so);
                        });
                    if (t < 4) pin([&] { a[1][t][i] = bload(rA, voA[t] + 16 * i, ab + (kc + 1) * 128); });
                }
            }
            // chunk p=1: the look-ahead crosses into the next tile in the tile's last iteration
            const int aso = last ? abn : ab + (kc + 2) * 128;
            const int bso = last ? bbn : bb + (kc + 2) * ldb128;
#pragma unroll
            for (int t = 0; t < 16; ++t) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj)
                        acc[i][jj] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[1][i][t >> 2][t & 3], b[t & 7][jj], acc[i][jj], 0, 0, 0);
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
        // epilogue of tile j (its stores drain under tile j+1's MFMAs): buffer stores, the row in soffset
        const int r0 = m0 + wm * 128, c0 = n0 + wn * 128;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int so = ((r0 + i * 32 + (r & 3) + 8 * (r >> 2)) * ldc + c0) * 4;
                f32x4 v{alpha * acc[i][0][r], alpha * acc[i][1][r], alpha * acc[i][2][r], alpha * acc[i][3][r]};
                if constexpr (BETA) v += beta * bload(rC, voC, so);
                if constexpr (DIAG == 1) {
                    if (v[0] == 1234.5f && v[1] == -1.f) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(pcmx_v4u, v), rC, voC, so, 0);
                } else {
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(pcmx_v4u, v), rC, voC, so, 0);
                }
                __builtin_amdgcn_sched_barrier(0);  // one store at a time: bounded live VGPRs (no spills)
            }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) acc[i][jj] = f32x16{0};
        ab = abn, bb = bbn, m0 = m0n, n0 = n0n;
        ++j;
    } while (xid + j * grid < ntiles);
}

template <int GM, int DIAG = 0, int STAGGER = 0>
int launch_drp(const float* A, const float* B, float* Cm, int M, int N, int K, int lda, int ldb, int ldc, float alpha,
               float beta, hipStream_t s) {
    if (M <= 0 || N <= 0 || K <= 0 || M % 256 || N % 256 || K % 64) return 1;
    if ((lda | ldb | ldc) & 3 || (((uintptr_t)A | (uintptr_t)B | (uintptr_t)Cm) & 15)) return 1;
    // every scalar byte offset (A row base + k, B k-row + column) must stay below 2^31
    if ((long long)M * lda * 4 >= (1LL << 31) || (long long)K * ldb * 4 >= (1LL << 31)) return 1;
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int tiles = (M / 256) * (N / 256);
    const int grid = tiles < cus ? tiles : cus;
    if (beta != 0.f)
        sgemm_drp_kernel<true, GM, DIAG, STAGGER><<<grid, 256, 0, s>>>(A, B, Cm, M, N, K, lda, ldb, ldc, alpha, beta);
    else
        sgemm_drp_kernel<false, GM, DIAG, STAGGER><<<grid, 256, 0, s>>>(A, B, Cm, M, N, K, lda, ldb, ldc, alpha, beta);
    return (int)hipGetLastError();
}
// Persistent, v_mfma_f32_16x16x4_f32 form (the shape hipBLASLt's fp32 kernel uses): 8x8 MFMA tiles of 16x16 per
// 128x128 wave tile (256 accumulators). MFMA step t of a 32-k chunk feeds k-slot g (= lane >> 4) with
// k = k0 + 8g + t.
//  * A: lane (l, g) loads A[row l][k0 + 8g + 4q .. +3] (q = 0, 1): one 16-row instruction covers half of each row's
//    128-B chunk line, the q = 1 load the other half.
//  * B: N-tile j < 4 owns columns c0 + 4c + j, tile j >= 4 owns c0 + 64 + 4c + (j - 4) (c = lane & 15), so a lane's
//    two 16-B loads per k-row are 256 contiguous bytes per k-slot each, and the epilogue stores 16 B per lane.
template <bool BETA, int GM>
__global__ __launch_bounds__(256, 1) void sgemm_drp16_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                             float* __restrict__ C, int M, int N, int K, int lda, int ldb,
                                                             int ldc, float alpha, float beta) {
    const int lane = (int)__lane_id();
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int g = lane >> 4, l = lane & 15;
    const int ntiles = (M / 256) * (N / 256), grid = (int)gridDim.x;
    const int xid = xcd_remap((int)blockIdx.x, grid);

    const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rC = __builtin_amdgcn_make_buffer_rsrc((void*)C, (short)0, 0x7fffffff, 0x00020000);
    const int voA = (l * lda + 8 * g) * 4;        // + tile i: 16 i lda * 4 (SGPR), + q: 16 q (imm)
    const int voB = (8 * g * ldb + 4 * l) * 4;    // + half: 256 B (imm)
    const int voC = (4 * g * ldc + 4 * l) * 4;
    const int nk = K / 32;
    const int ldb128 = ldb * 128, lda64 = lda * 64;

    auto bases = [&](int j, int& ab, int& bb, int& m0, int& n0) {
        int T = j * grid + xid;
        if (T >= ntiles) T = ((ntiles - 1 - xid) / grid) * grid + xid;
        tile_coords<256, 256, GM>(T, M, N, m0, n0);
        m0 = __builtin_amdgcn_readfirstlane(m0);
        n0 = __builtin_amdgcn_readfirstlane(n0);
        ab = __builtin_amdgcn_readfirstlane((m0 + wm * 128) * lda * 4);
        bb = __builtin_amdgcn_readfirstlane((n0 + wn * 128) * 4);
    };

    f32x4 a[2][8][2];  // [chunk parity][tile i][q]
    f32x4 b[4][2];     // ring: step t's B operands (columns c0+4l.., c0+64+4l..) in slot t % 4
    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0};
    auto pin = [](auto&& f) __attribute__((always_inline)) {
        __builtin_amdgcn_sched_barrier(0);
        f();
        __builtin_amdgcn_sched_barrier(0);
    };
    auto ldA = [&](int i, int q, int so) { return bload(rA, voA + 16 * q, so + i * lda64); };
    auto ldB = [&](int half, int so) { return bload(rB, voB + 256 * half, so); };

    int ab, bb, m0, n0;
    bases(0, ab, bb, m0, n0);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int q = 0; q < 2; ++q) a[0][i][q] = ldA(i, q, ab);
#pragma unroll
    for (int t = 0; t < 4; ++t)
        pin([&] {
            b[t][0] = ldB(0, bb + t * ldb * 4);
            b[t][1] = ldB(1, bb + t * ldb * 4);
        });

    int jt = 0;
    do {
        int abn, bbn, m0n, n0n;
        bases(jt + 1, abn, bbn, m0n, n0n);
        int kc = 0;
        do {
            const bool last = kc + 2 == nk;
            const int aso1 = last ? abn : ab + (kc + 2) * 128;
            const int bso1 = last ? bbn : bb + (kc + 2) * ldb128;
            auto chunk = [&](auto pc) __attribute__((always_inline)) {
                constexpr int p = decltype(pc)::value;
                // look-ahead targets: A of the next chunk; B of step t + 4
                const int aso = p == 0 ? ab + (kc + 1) * 128 : aso1;
                const int bcur = bb + (kc + p) * ldb128, bnext = p == 0 ? bb + (kc + 1) * ldb128 : bso1;
#pragma unroll
                for (int t = 0; t < 8; ++t) {
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
#pragma unroll
                        for (int j = 0; j < 8; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[p][i][t >> 2][t & 3], b[t & 3][j >> 2][j & 3],
                                                                             acc[i][j], 0, 0, 0);
                        if (t < 4 && (i == 1 || i == 4))  // next chunk's A in steps 0-3: >= 4 steps ahead
                            pin([&] {
                                const int ti = 2 * t + (i == 4);
                                a[p ^ 1][ti][0] = ldA(ti, 0, aso);
                                a[p ^ 1][ti][1] = ldA(ti, 1, aso);
                            });
                        if (i == 7)
                            pin([&] {
                                const int so = t + 4 < 8 ? bcur + (t + 4) * ldb * 4 : bnext + (t - 4) * ldb * 4;
                                b[t & 3][0] = ldB(0, so);
                                b[t & 3][1] = ldB(1, so);
                            });
                    }
                }
            };
            chunk(std::integral_constant<int, 0>{});
            chunk(std::integral_constant<int, 1>{});
            kc += 2;
        } while (kc < nk);
        // epilogue: tile (i, j) lane (l, g) holds column col(j, l), rows 16 i + 4 g + r
        const int r0 = m0 + wm * 128, c0 = n0 + wn * 128;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int hf = 0; hf < 2; ++hf) {
                    const int so = ((r0 + 16 * i + r) * ldc + c0 + 64 * hf) * 4;
                    f32x4 v{alpha * acc[i][4 * hf][r], alpha * acc[i][4 * hf + 1][r], alpha * acc[i][4 * hf + 2][r],
                            alpha * acc[i][4 * hf + 3][r]};
                    if constexpr (BETA) v += beta * bload(rC, voC, so);
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(pcmx_v4u, v), rC, voC, so, 0);
                    __builtin_amdgcn_sched_barrier(0);
                }
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0};
        ab = abn, bb = bbn, m0 = m0n, n0 = n0n;
        ++jt;
    } while (xid + jt * grid < ntiles);
}

template <int GM>
int launch_drp16(const float* A, const float* B, float* Cm, int M, int N, int K, int lda, int ldb, int ldc, float alpha,
                 float beta, hipStream_t s) {
    if (M <= 0 || N <= 0 || K <= 0 || M % 256 || N % 256 || K % 64) return 1;
    if ((lda | ldb | ldc) & 3 || (((uintptr_t)A | (uintptr_t)B | (uintptr_t)Cm) & 15)) return 1;
    if ((long long)M * lda * 4 >= (1LL << 31) || (long long)K * ldb * 4 >= (1LL << 31) ||
        (long long)M * ldc * 4 >= (1LL << 31))
        return 1;
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int tiles = (M / 256) * (N / 256);
    const int grid = tiles < cus ? tiles : cus;
    if (beta != 0.f)
        sgemm_drp16_kernel<true, GM><<<grid, 256, 0, s>>>(A, B, Cm, M, N, K, lda, ldb, ldc, alpha, beta);
    else
        sgemm_drp16_kernel<false, GM><<<grid, 256, 0, s>>>(A, B, Cm, M, N, K, lda, ldb, ldc, alpha, beta);
    return (int)hipGetLastError();
}
}  // namespace

extern "C" int pcmx_sgemm_dr_lab_variant(const float* A, const float* B, float* C, int M, int N, int K, int lda,
                                         int ldb, int ldc, float alpha, float beta, int variant, hipStream_t s) {
    switch (variant) {
        case 30: return launch_dr<0, 8>(A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, s);
        case 31: return launch_dr<1, 8>(A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, s);
        case 32: return launch_dr<0, 4>(A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, s);
        case 33: return launch_dr<0, 16>(A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, s);
        case 34: return launch_drp<8>(A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, s);
        case 35: return launch_drp<8, 1>(A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, s);
        case 37: return launch_drp<8, 0, 8>(A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, s);
        case 38: return launch_drp<8, 0, 16>(A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, s);
        case 39: return launch_drp<8, 0, 40>(A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, s);
        case 40: return launch_drp<4, 0, 0>(A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, s);
        case 41: return launch_drp<16, 0, 0>(A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, s);
        case 36: return launch_drp16<8>(A, B, C, M, N, K, lda, ldb, ldc, alpha, beta, s);
        default: return 1;
    }
}
