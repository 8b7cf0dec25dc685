// MFMA f32 issue-rate microbenchmark: v_mfma_f32_32x32x2_f32 vs v_mfma_f32_16x16x4_f32, 1 or 2 waves per
// SIMD, independent accumulator chains. Prints TFLOP/s (device time via hipEvents).
// build: hipcc -O3 --offload-arch=gfx950 scripts/mfma_peak.hip -o build/mfma_peak
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void k32(float* out, int iters, float a, float b) {
    f32x16 acc[NACC];
    for (int i = 0; i < NACC; ++i) acc[i] = f32x16{0};
    float x = a + threadIdx.x, y = b - threadIdx.x;
    for (int it = 0; it < iters; ++it)
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, acc[i], 0, 0, 0);
    float s = 0;
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][15];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NACC>
__global__ __launch_bounds__(256) void k16(float* out, int iters, float a, float b) {
    f32x4 acc[NACC];
    for (int i = 0; i < NACC; ++i) acc[i] = f32x4{0};
    float x = a + threadIdx.x, y = b - threadIdx.x;
    for (int it = 0; it < iters; ++it)
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(x, y, acc[i], 0, 0, 0);
    float s = 0;
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// Random operands (8 A and 8 B registers per lane, hashed from the lane id) for the DVFS comparison: on random data
// the chip may hold a different clock per MFMA shape (MI355X_MICROARCH.md 'DVFS give-back' item 7).
__device__ __forceinline__ float rnd(unsigned v) {
    v ^= v >> 16; v *= 0x7feb352du; v ^= v >> 15; v *= 0x846ca68bu; v ^= v >> 16;
    return (float)(v & 0xffffff) * (1.f / 16777216.f) - 0.5f;
}
template <int NACC>
__global__ __launch_bounds__(256) void k32r(float* out, int iters) {
    f32x16 acc[NACC];
    float xs[8], ys[8];
    for (int i = 0; i < 8; ++i) xs[i] = rnd(threadIdx.x * 131 + blockIdx.x * 7919 + i), ys[i] = rnd(threadIdx.x * 977 + i * 31 + 5);
    for (int i = 0; i < NACC; ++i) acc[i] = f32x16{0};
    for (int it = 0; it < iters; ++it)
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(xs[i & 7], ys[(i * 3 + 1) & 7], acc[i], 0, 0, 0);
    float s = 0;
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][15];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int NACC>
__global__ __launch_bounds__(256) void k16r(float* out, int iters) {
    f32x4 acc[NACC];
    float xs[8], ys[8];
    for (int i = 0; i < 8; ++i) xs[i] = rnd(threadIdx.x * 131 + blockIdx.x * 7919 + i), ys[i] = rnd(threadIdx.x * 977 + i * 31 + 5);
    for (int i = 0; i < NACC; ++i) acc[i] = f32x4{0};
    for (int it = 0; it < iters; ++it)
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(xs[i & 7], ys[(i * 3 + 1) & 7], acc[i], 0, 0, 0);
    float s = 0;
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <class F>
double run(F launch, double flop) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    launch();
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return 5 * flop / (ms * 1e-3) / 1e12;
}

int main() {
    float* out;
    hipMalloc(&out, 1 << 24);
    const int cus = 256, iters = 20000;
    for (int wps = 1; wps <= 2; ++wps) {
        const int blocks = cus * wps;  // 256 threads = 4 waves = 1 per SIMD per block
        const double f32 = (double)blocks * 4 * iters * 16 * 32 * 32 * 2 * 2;
        const double f16 = (double)blocks * 4 * iters * 16 * 16 * 16 * 4 * 2;
        printf("waves/SIMD=%d  32x32x2 (16 acc): %7.1f TF   16x16x4 (16 acc): %7.1f TF   16x16x4 (64 acc): %7.1f TF\n",
               wps, run([&] { k32<16><<<blocks, 256>>>(out, iters, 1.f, 2.f); }, f32),
               run([&] { k16<16><<<blocks, 256>>>(out, iters, 1.f, 2.f); }, f16),
               run([&] { k16<64><<<blocks, 256>>>(out, iters / 4, 1.f, 2.f); }, f16 / 4 * 4));
    }
    for (int rep = 0; rep < 3; ++rep) {
        const int blocks = cus;
        const double f32 = (double)blocks * 4 * iters * 16 * 32 * 32 * 2 * 2;
        const double f16 = (double)blocks * 4 * iters * 64 * 16 * 16 * 4 * 2;
        printf("random operands, 1 wave/SIMD: 32x32x2 (16 acc): %7.1f TF   16x16x4 (64 acc): %7.1f TF\n",
               run([&] { k32r<16><<<blocks, 256>>>(out, iters); }, f32),
               run([&] { k16r<64><<<blocks, 256>>>(out, iters); }, f16));
    }
    hipFree(out);
    return 0;
}
