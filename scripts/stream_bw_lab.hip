// Streaming-bandwidth lab (NS1 follow-up): where the write side of an HBM stream tops out on MI355X. Kernels over
// n f32 (default 1e9: 4 GB per array): read-only reduce-style sum, write-only fill, copy (1R + 1W), vadd (2R + 1W),
// each with plain or non-temporal stores and several grid caps (blocks of 256 threads, grid-stride, 16-B per lane,
// U independent 16-B accesses per lane per iteration). Prints ms and GB/s (bytes actually moved) per variant.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/stream_bw_lab.hip -o bin_lab/stream_bw_lab
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);         \
            return 1;                                                                \
        }                                                                            \
    } while (0)

template <bool NT>
__device__ __forceinline__ void st(f32x4* p, f32x4 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

template <int U>
__global__ __launch_bounds__(256) void sum_kernel(const f32x4* a, long long n4, float* out) {
    f32x4 acc = {0, 0, 0, 0};
    const long long stride = (long long)gridDim.x * 256 * U;
    for (long long i = (long long)blockIdx.x * 256 * U + threadIdx.x; i < n4; i += stride) {
        f32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = i + u * 256 < n4 ? __builtin_nontemporal_load(a + i + u * 256) : f32x4{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u];
    }
    if (acc.x + acc.y + acc.z + acc.w == 12345.f) out[0] = 1.f;  // keep the loads
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void fill_kernel(f32x4* r, long long n4) {
    const long long stride = (long long)gridDim.x * 256 * U;
    for (long long i = (long long)blockIdx.x * 256 * U + threadIdx.x; i < n4; i += stride) {
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * 256 < n4) st<NT>(r + i + u * 256, f32x4{1, 2, 3, 4});
    }
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_kernel(const f32x4* a, f32x4* r, long long n4) {
    const long long stride = (long long)gridDim.x * 256 * U;
    for (long long i = (long long)blockIdx.x * 256 * U + threadIdx.x; i < n4; i += stride) {
        f32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = i + u * 256 < n4 ? __builtin_nontemporal_load(a + i + u * 256) : f32x4{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * 256 < n4) st<NT>(r + i + u * 256, v[u]);
    }
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void vadd_kernel(const f32x4* a, const f32x4* b, f32x4* r, long long n4) {
    const long long stride = (long long)gridDim.x * 256 * U;
    for (long long i = (long long)blockIdx.x * 256 * U + threadIdx.x; i < n4; i += stride) {
        f32x4 va[U], vb[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool in = i + u * 256 < n4;
            va[u] = in ? __builtin_nontemporal_load(a + i + u * 256) : f32x4{0, 0, 0, 0};
            vb[u] = in ? __builtin_nontemporal_load(b + i + u * 256) : f32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * 256 < n4) st<NT>(r + i + u * 256, va[u] + vb[u]);
    }
}

// CHUNKED variants: block b streams one contiguous chunk [b * chunk, (b + 1) * chunk) of float4s (U x 256 per
// iteration) instead of striding over the whole array with the grid (the scan kernel's tile order, which moves
// 8 B/element at 6.3 TB/s against 5.5 for the grid-stride copy)
template <int U>
__global__ __launch_bounds__(256) void sum_chunk_kernel(const f32x4* a, long long n4, long long chunk, float* out) {
    f32x4 acc = {0, 0, 0, 0};
    const long long b0 = (long long)blockIdx.x * chunk, b1 = b0 + chunk < n4 ? b0 + chunk : n4;
    for (long long i = b0 + threadIdx.x; i < b1; i += 256 * U) {
        f32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = i + u * 256 < b1 ? __builtin_nontemporal_load(a + i + u * 256) : f32x4{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u];
    }
    if (acc.x + acc.y + acc.z + acc.w == 12345.f) out[0] = 1.f;
}
template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_chunk_kernel(const f32x4* a, f32x4* r, long long n4, long long chunk) {
    const long long b0 = (long long)blockIdx.x * chunk, b1 = b0 + chunk < n4 ? b0 + chunk : n4;
    for (long long i = b0 + threadIdx.x; i < b1; i += 256 * U) {
        f32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = i + u * 256 < b1 ? __builtin_nontemporal_load(a + i + u * 256) : f32x4{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * 256 < b1) st<NT>(r + i + u * 256, v[u]);
    }
}
template <int U, bool NT>
__global__ __launch_bounds__(256) void vadd_chunk_kernel(const f32x4* a, const f32x4* b, f32x4* r, long long n4,
                                                         long long chunk) {
    const long long b0 = (long long)blockIdx.x * chunk, b1 = b0 + chunk < n4 ? b0 + chunk : n4;
    for (long long i = b0 + threadIdx.x; i < b1; i += 256 * U) {
        f32x4 va[U], vb[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool in = i + u * 256 < b1;
            va[u] = in ? __builtin_nontemporal_load(a + i + u * 256) : f32x4{0, 0, 0, 0};
            vb[u] = in ? __builtin_nontemporal_load(b + i + u * 256) : f32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * 256 < b1) st<NT>(r + i + u * 256, va[u] + vb[u]);
    }
}

int main(int argc, char** argv) {
    const long long n = argc > 1 ? (long long)atof(argv[1]) : 1000000000LL;
    const long long n4 = n / 4;
    f32x4 *a, *b, *r;
    float* out;
    CK(hipMalloc(&a, n4 * 16));
    CK(hipMalloc(&b, n4 * 16));
    CK(hipMalloc(&r, n4 * 16));
    CK(hipMalloc(&out, 16));
    CK(hipMemset(a, 0, n4 * 16));
    CK(hipMemset(b, 0, n4 * 16));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto time = [&](const char* name, double bytes, auto fn) {
        for (int i = 0; i < 2; ++i) fn();
        hipEventRecord(e0);
        for (int i = 0; i < 10; ++i) fn();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= 10;
        printf("%-28s %.4f ms %7.1f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    const double B = (double)n4 * 16;
    if (argc > 2) {  // chunked-only sweep: grid sizes x chunked kernels
        for (int grid : {1024, 2048, 4096, 8192, 16384, 32768}) {
            const long long chunk = (n4 + grid - 1) / grid;
            char nm[64];
#define RUNC(LABEL, BYTES, ...)                                      \
    snprintf(nm, sizeof nm, "%s g%d", LABEL, grid);                 \
    time(nm, BYTES, [&] { __VA_ARGS__; });
            RUNC("chunk sum U4", B, sum_chunk_kernel<4><<<grid, 256>>>(a, n4, chunk, out))
            RUNC("chunk copy U4 nt", 2 * B, (copy_chunk_kernel<4, true><<<grid, 256>>>(a, r, n4, chunk)))
            RUNC("chunk copy U4 plain", 2 * B, (copy_chunk_kernel<4, false><<<grid, 256>>>(a, r, n4, chunk)))
            RUNC("chunk vadd U4 nt", 3 * B, (vadd_chunk_kernel<4, true><<<grid, 256>>>(a, b, r, n4, chunk)))
            RUNC("chunk vadd U2 nt", 3 * B, (vadd_chunk_kernel<2, true><<<grid, 256>>>(a, b, r, n4, chunk)))
#undef RUNC
        }
        return 0;
    }
    for (int grid : {2048, 4096, 8192, 16384}) {
        char nm[64];
#define RUN(LABEL, BYTES, ...)                                      \
    snprintf(nm, sizeof nm, "%s g%d", LABEL, grid);                 \
    time(nm, BYTES, [&] { __VA_ARGS__; });
        RUN("sum U4", B, sum_kernel<4><<<grid, 256>>>(a, n4, out))
        RUN("fill U1 plain", B, (fill_kernel<1, false><<<grid, 256>>>(r, n4)))
        RUN("fill U1 nt", B, (fill_kernel<1, true><<<grid, 256>>>(r, n4)))
        RUN("fill U4 nt", B, (fill_kernel<4, true><<<grid, 256>>>(r, n4)))
        RUN("copy U4 plain", 2 * B, (copy_kernel<4, false><<<grid, 256>>>(a, r, n4)))
        RUN("copy U4 nt", 2 * B, (copy_kernel<4, true><<<grid, 256>>>(a, r, n4)))
        RUN("vadd U4 plain", 3 * B, (vadd_kernel<4, false><<<grid, 256>>>(a, b, r, n4)))
        RUN("vadd U4 nt", 3 * B, (vadd_kernel<4, true><<<grid, 256>>>(a, b, r, n4)))
        RUN("vadd U2 nt", 3 * B, (vadd_kernel<2, true><<<grid, 256>>>(a, b, r, n4)))
#undef RUN
    }
    return 0;
}
