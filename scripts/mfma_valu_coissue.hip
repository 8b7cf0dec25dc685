// Lab: can the f32 VALU add GEMM flops beside the f32 MFMA on gfx950? One wave per SIMD runs 16 independent
// v_mfma_f32_32x32x2_f32 accumulator chains on random operands (the SGEMM's issue pattern) and, between every two
// MFMAs, V independent v_pk_fma_f32 (2 FMAs per lane) on VALU accumulators. If the VALU issues in the MFMA's shadow
// and the clock holds, the combined rate exceeds the MFMA-only rate by up to V * 256 / 4096 flops per MFMA.
// build: hipcc -O3 --offload-arch=gfx950 scripts/mfma_valu_coissue.hip -o build/mfma_valu_coissue
// run:   build/mfma_valu_coissue        (prints one line per V: MFMA-only, VALU-only and combined TFLOP/s)
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float rnd(unsigned v) {
    v ^= v >> 16; v *= 0x7feb352du; v ^= v >> 15; v *= 0x846ca68bu; v ^= v >> 16;
    return (float)(v & 0xffffff) * (1.f / 16777216.f) - 0.5f;
}

__device__ __forceinline__ void pk_fma(f2& acc, const f2& a, const f2& b) {
    asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}

// MF: MFMAs per iteration (0 = none), V: v_pk_fma_f32 per MFMA slot (VALU-only runs use 16 slots)
template <int MF, int V>
__global__ __launch_bounds__(256, 1) void coissue(float* out, int iters) {
    f32x16 acc[16];
    f2 vacc[16];
    float xs[8], ys[8];
    f2 va[4], vb[4];
    for (int i = 0; i < 8; ++i) xs[i] = rnd(threadIdx.x * 131 + blockIdx.x * 7919 + i), ys[i] = rnd(threadIdx.x * 977 + i * 31 + 5);
    for (int i = 0; i < 4; ++i) va[i] = f2{rnd(threadIdx.x + 17 * i), rnd(threadIdx.x + 19 * i + 3)}, vb[i] = f2{rnd(i + 7), rnd(i + 11)};
    for (int i = 0; i < 16; ++i) acc[i] = f32x16{0}, vacc[i] = f2{0.f, 0.f};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            if constexpr (MF > 0) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(xs[i & 7], ys[(i * 3 + 1) & 7], acc[i], 0, 0, 0);
#pragma unroll
            for (int v = 0; v < V; ++v) pk_fma(vacc[(i * V + v) & 15], va[v & 3], vb[(v + i) & 3]);
        }
    }
    float s = 0;
    for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][15] + vacc[i][0] + vacc[i][1];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <class K>
double time_ms(K kern, float* out, int iters, int blocks) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0), hipEventCreate(&e1);
    kern<<<blocks, 256>>>(out, iters);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 10; ++r) kern<<<blocks, 256>>>(out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / 10;
}

template <int V>
void row(float* out, int iters, int blocks) {
    const double waves = blocks * 4.0, slots = waves * iters * 16.0;
    const double mf = slots * 4096.0, vf = slots * V * 256.0;
    const double t_m = time_ms(coissue<1, 0>, out, iters, blocks);
    const double t_v = time_ms(coissue<0, V>, out, iters, blocks);
    const double t_b = time_ms(coissue<1, V>, out, iters, blocks);
    printf("V=%d  mfma-only %.1f TF (%.3f ms)  valu-only %.1f TF (%.3f ms)  both %.1f TF = mfma %.1f + valu %.1f (%.3f ms)\n", V,
           mf / t_m / 1e9, t_m, vf / t_v / 1e9, t_v, (mf + vf) / t_b / 1e9, mf / t_b / 1e9, vf / t_b / 1e9, t_b);
}

int main() {
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float* out;
    hipMalloc(&out, sizeof(float) * 256 * cus);
    const int iters = 4000;
    row<2>(out, iters, cus);
    row<4>(out, iters, cus);
    row<6>(out, iters, cus);
    row<8>(out, iters, cus);
    hipFree(out);
    return 0;
}
