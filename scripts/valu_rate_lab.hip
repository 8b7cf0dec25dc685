// VALU issue-rate / latency lab (round 4, stencil VALU question): for a handful of gfx950 VALU instructions, the
// time one wave64 needs per instruction (a) over 8 INDEPENDENT register chains (issue rate) and (b) over ONE dependent
// chain (latency), with 1 or 2 waves per SIMD (grid = 256 CUs x 4 SIMDs x waves). Reported as ns per instruction per
// wave and as a ratio to v_add_f32 measured the same way: v_cvt_pk_bf16_f32 at half rate would show 2.0 (independent).
// Every op is inline asm on VGPRs (vector instructions only); results are summed and stored so nothing is dead.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/valu_rate_lab.hip -o bin_lab/valu_rate_lab
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                                \
    do {                                                                     \
        hipError_t e_ = (x);                                                 \
        if (e_ != hipSuccess) {                                              \
            printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
            return 1;                                                        \
        }                                                                    \
    } while (0)

constexpr int kIters = 4096;

typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float first(float v) { return v; }
__device__ __forceinline__ float first(f2 v) { return v.x; }
// ASM: one instruction updating %0 from %0 and %1 (one VGPR, or a register pair for the packed forms)
#define DEF_KERNEL(NAME, ASM, DT)                                                                     \
    template <bool kDep>                                                                              \
    __global__ __launch_bounds__(256) void NAME(float* out, float seed) {                             \
        DT r0 = (DT)(seed + threadIdx.x), r1 = r0 + (DT)1, r2 = r0 + (DT)2, r3 = r0 + (DT)3;            \
        DT r4 = r0 + (DT)4, r5 = r0 + (DT)5, r6 = r0 + (DT)6, r7 = r0 + (DT)7;                          \
        const DT a = (DT)(seed * 0.5f);                                                               \
        for (int i = 0; i < kIters; ++i) {                                                            \
            if constexpr (kDep) {                                                                     \
                asm volatile(ASM : "+v"(r0) : "v"(a));                                                \
                asm volatile(ASM : "+v"(r0) : "v"(a));                                                \
                asm volatile(ASM : "+v"(r0) : "v"(a));                                                \
                asm volatile(ASM : "+v"(r0) : "v"(a));                                                \
                asm volatile(ASM : "+v"(r0) : "v"(a));                                                \
                asm volatile(ASM : "+v"(r0) : "v"(a));                                                \
                asm volatile(ASM : "+v"(r0) : "v"(a));                                                \
                asm volatile(ASM : "+v"(r0) : "v"(a));                                                \
            } else {                                                                                  \
                asm volatile(ASM : "+v"(r0) : "v"(a));                                                \
                asm volatile(ASM : "+v"(r1) : "v"(a));                                                \
                asm volatile(ASM : "+v"(r2) : "v"(a));                                                \
                asm volatile(ASM : "+v"(r3) : "v"(a));                                                \
                asm volatile(ASM : "+v"(r4) : "v"(a));                                                \
                asm volatile(ASM : "+v"(r5) : "v"(a));                                                \
                asm volatile(ASM : "+v"(r6) : "v"(a));                                                \
                asm volatile(ASM : "+v"(r7) : "v"(a));                                                \
            }                                                                                         \
        }                                                                                             \
        const DT s = r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7;                                           \
        out[blockIdx.x * 256 + threadIdx.x] = first(s);                                               \
    }

typedef float f1;
DEF_KERNEL(k_add_f32, "v_add_f32 %0, %0, %1", f1)
DEF_KERNEL(k_pk_add_f32, "v_pk_add_f32 %0, %0, %1", f2)
DEF_KERNEL(k_pk_fma_f32, "v_pk_fma_f32 %0, %0, %1, %0", f2)
DEF_KERNEL(k_cvt_pk_bf16, "v_cvt_pk_bf16_f32 %0, %0, %1", f1)
DEF_KERNEL(k_add_dpp, "v_add_f32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf", f1)
DEF_KERNEL(k_and_b32, "v_and_b32 %0, %0, %1", f1)
DEF_KERNEL(k_lshl_b32, "v_lshlrev_b32 %0, 16, %0", f1)
DEF_KERNEL(k_fma_f32, "v_fma_f32 %0, %0, %1, %0", f1)

int main() {
    float* out;
    CK(hipMalloc(&out, 256 * 8 * 256 * sizeof(float)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto kind, auto kdep) {
        double ns[2][2];
        for (int dep = 0; dep < 2; ++dep)
            for (int w = 1; w <= 2; ++w) {
                const int blocks = 256 * w;  // 4 waves per block, one per SIMD: w waves per SIMD
                auto launch = [&] {
                    if (dep) kdep<<<blocks, 256>>>(out, 1.0f);
                    else kind<<<blocks, 256>>>(out, 1.0f);
                };
                launch();
                hipEventRecord(e0);
                for (int r = 0; r < 5; ++r) launch();
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms = 0;
                hipEventElapsedTime(&ms, e0, e1);
                // per wave: kIters * 8 instructions; w waves share one SIMD
                ns[dep][w - 1] = ms * 1e6 / 5 / ((double)kIters * 8);
            }
        printf("%-20s indep 1w %.3f ns/instr  2w %.3f ns/instr/SIMD-pair   dep 1w %.3f  2w %.3f\n", name, ns[0][0],
               ns[0][1] / 2, ns[1][0], ns[1][1] / 2);
        fflush(stdout);
        return ns[0][1] / 2;
    };
    run("v_add_f32", k_add_f32<false>, k_add_f32<true>);
    run("v_fma_f32", k_fma_f32<false>, k_fma_f32<true>);
    run("v_pk_add_f32", k_pk_add_f32<false>, k_pk_add_f32<true>);
    run("v_pk_fma_f32", k_pk_fma_f32<false>, k_pk_fma_f32<true>);
    run("v_cvt_pk_bf16_f32", k_cvt_pk_bf16<false>, k_cvt_pk_bf16<true>);
    run("v_add_f32_dpp", k_add_dpp<false>, k_add_dpp<true>);
    run("v_and_b32", k_and_b32<false>, k_and_b32<true>);
    run("v_lshlrev_b32", k_lshl_b32<false>, k_lshl_b32<true>);
    return 0;
}
