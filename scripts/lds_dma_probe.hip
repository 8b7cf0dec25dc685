// LDS-DMA layout probe (round 4): where does `buffer_load_dwordx4 ... lds` put lane l's 16 bytes? One wave loads
// src[4 l + k] = 1000 l + k (lane l's float4 = {1000 l, 1000 l + 1, 1000 l + 2, 1000 l + 3}) into LDS at M0 = 0,
// waits vmcnt(0), and copies the first 256 LDS dwords out; the host prints where lanes 0, 1, 63 landed.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/lds_dma_probe.hip -o bin_lab/lds_dma_probe
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ __launch_bounds__(64) void probe(const float* src, float* dst) {
    __shared__ __attribute__((aligned(16))) float lds[512];
    for (int i = threadIdx.x; i < 512; i += 64) lds[i] = -1.f;
    __syncthreads();
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), (short)0, 64 * 16, 0x00020000);
    const unsigned vo = threadIdx.x * 16u;
    const unsigned base = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
                 "s_mov_b32 m0, %0\n\ts_waitcnt vmcnt(0)"
                 : "=&s"(keep)
                 : "v"(vo), "s"(rsrc), "s"(base)
                 : "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 512; i += 64) dst[i] = lds[i];
}

int main() {
    float h[256], *src, *dst, out[512];
    for (int l = 0; l < 64; ++l)
        for (int k = 0; k < 4; ++k) h[4 * l + k] = 1000.f * l + k;
    if (hipMalloc(&src, sizeof h) != hipSuccess || hipMalloc(&dst, sizeof out) != hipSuccess) return 1;
    if (hipMemcpy(src, h, sizeof h, hipMemcpyHostToDevice) != hipSuccess) return 1;
    probe<<<1, 64>>>(src, dst);
    if (hipMemcpy(out, dst, sizeof out, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    printf("lds[0..7]:");
    for (int i = 0; i < 8; ++i) printf(" %g", out[i]);
    printf("\nlds[60..67]:");
    for (int i = 60; i < 68; ++i) printf(" %g", out[i]);
    printf("\nlds[252..259]:");
    for (int i = 252; i < 260; ++i) printf(" %g", out[i]);
    int lane_major = 1, comp_major = 1;
    for (int l = 0; l < 64; ++l)
        for (int k = 0; k < 4; ++k) {
            lane_major &= out[4 * l + k] == 1000.f * l + k;
            comp_major &= out[64 * k + l] == 1000.f * l + k;
        }
    printf("\nlane-major (lane l at 16 l): %s   component-major (dword k of lane l at 256 k + 4 l): %s\n",
           lane_major ? "yes" : "no", comp_major ? "yes" : "no");
    return 0;
}
