// Read-bandwidth lab for the 1e9-f32 reduction (standalone, not part of the library): the library kernel
// against grid-stride / contiguous-chunk variants with different unroll depths, block counts and load kinds.
// build: hipcc -O3 --offload-arch=gfx950 -Icsrc/include -Icsrc/runtime scripts/reduce_lab.hip -o build/reduce_lab
#include "../csrc/kernels/reduce.hip"

#include <cstdio>

namespace lab {
using pcmx::f32x4;

template <int U, bool NT>
__global__ __launch_bounds__(256) void stride_sum(const f32x4* __restrict__ x, long long n4, float* __restrict__ part) {
    float acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = 0.f;
    const long long step = (long long)gridDim.x * 256 * U;
    for (long long i = (long long)blockIdx.x * 256 * U + threadIdx.x; i + (U - 1) * 256 < n4; i += step) {
        f32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(x + i + u * 256) : x[i + u * 256];
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] += (v[u].x + v[u].y) + (v[u].z + v[u].w);
    }
#pragma unroll
    for (int u = 1; u < U; ++u) acc[0] += acc[u];
    float r = pcmx::wave_reduce<float, 0>(acc[0]);
    if (pcmx::lane_id() == 0) atomicAdd(part + (blockIdx.x & 1023), r);
}

// contiguous chunk per block (n4 divisible by blocks*256*U assumed by the caller)
template <int U, bool NT>
__global__ __launch_bounds__(256) void chunk_sum(const f32x4* __restrict__ x, long long per_block, float* __restrict__ part) {
    float acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = 0.f;
    const f32x4* p = x + (long long)blockIdx.x * per_block;
    for (long long i = threadIdx.x; i + (U - 1) * 256 < per_block; i += 256 * U) {  // tail ignored (lab)
        f32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(p + i + u * 256) : p[i + u * 256];
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] += (v[u].x + v[u].y) + (v[u].z + v[u].w);
    }
#pragma unroll
    for (int u = 1; u < U; ++u) acc[0] += acc[u];
    float r = pcmx::wave_reduce<float, 0>(acc[0]);
    if (pcmx::lane_id() == 0) atomicAdd(part + (blockIdx.x & 1023), r);
}
}  // namespace lab

template <class F>
float time_ms(F f, int iters = 20) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a), (void)hipEventCreate(&b);
    for (int i = 0; i < 3; ++i) f();
    (void)hipEventRecord(a);
    for (int i = 0; i < iters; ++i) f();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / iters;
}

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    const long long n = 1000000000LL, n4 = n / 4;
    float *x, *out, *part;
    void* ws;
    if (hipMalloc(&x, n * 4) || hipMalloc(&out, 64) || hipMalloc(&part, 4096 * 4) || hipMalloc(&ws, 1 << 20)) return 1;
    (void)hipMemset(x, 0, n * 4);
    const double gb = n * 4.0 / 1e9;
    auto rep = [&](const char* name, float ms) { printf("%-34s %7.4f ms %7.0f GB/s\n", name, ms, gb / ms * 1e3); };
    rep("library pcmx_reduce_f32", time_ms([&] { pcmx_reduce_f32(x, n, 0, out, ws, 0); }));
    for (int nb : {256, 512, 768, 1024, 1536, 2048, 3072}) {
        char nm[64];
        snprintf(nm, 64, "library pass1+2 blocks %d", nb);
        rep(nm, time_ms([&] {
            reduce_pass1<float, 0, false><<<nb, kThreads>>>(x, x, n, (float*)ws);
            reduce_pass2<float, 0><<<1, kThreads>>>((float*)ws, nb, out);
        }));
    }
    for (int blocks : {1024, 2048}) {
        char nm[64];
        snprintf(nm, 64, "stride U8 nt  blocks %d", blocks);
        rep(nm, time_ms([&] { lab::stride_sum<8, true><<<blocks, 256>>>((const pcmx::f32x4*)x, n4, part); }));
        snprintf(nm, 64, "stride U8     blocks %d", blocks);
        rep(nm, time_ms([&] { lab::stride_sum<8, false><<<blocks, 256>>>((const pcmx::f32x4*)x, n4, part); }));
        snprintf(nm, 64, "stride U16 nt blocks %d", blocks);
        rep(nm, time_ms([&] { lab::stride_sum<16, true><<<blocks, 256>>>((const pcmx::f32x4*)x, n4, part); }));
        snprintf(nm, 64, "stride U4 nt  blocks %d", blocks);
        rep(nm, time_ms([&] { lab::stride_sum<4, true><<<blocks, 256>>>((const pcmx::f32x4*)x, n4, part); }));
    }
    for (int blocks : {1000, 2000}) {   // 2.5e8 f32x4 divisible by blocks * 256 * U? per-block tail ok
        const long long per = n4 / blocks;
        char nm[64];
        snprintf(nm, 64, "chunk U8 nt   blocks %d", blocks);
        rep(nm, time_ms([&] { lab::chunk_sum<8, true><<<blocks, 256>>>((const pcmx::f32x4*)x, per, part); }));
        snprintf(nm, 64, "chunk U4 nt   blocks %d", blocks);
        rep(nm, time_ms([&] { lab::chunk_sum<4, true><<<blocks, 256>>>((const pcmx::f32x4*)x, per, part); }));
    }
    return 0;
}
