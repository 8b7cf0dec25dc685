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

// ROUND 6: the SCAN's streaming structure applied to copy / vadd / axpy. scan_parked_kernel moves 1R + 1W at
// 6.29 TB/s; these isolate which of its traits matter: W waves x R f32x4 rows per lane (tile = W*R KiB per input),
// a PERSISTENT grid of `per_cu` blocks per CU, tiles handed out in time order (atomic ticket, TICKET) or statically
// (tile = block + k * grid), and the next tile's loads issued BEFORE the current tile's stores (double buffer).
// NIN = 1: copy (r = a); NIN = 2: r = a + b (vadd; axpy is the same traffic with r aliasing b).
template <int R, int NIN>
struct TileRegs {
    f32x4 a[R], b[NIN == 2 ? R : 1];
};

template <int R, int W, int NIN>
__device__ __forceinline__ void tl_load(const f32x4* a, const f32x4* b, long long t, TileRegs<R, NIN>& v) {
    const long long base = t * (W * 64 * R) + (long long)(threadIdx.x / 64) * (64 * R) + (threadIdx.x & 63);
#pragma unroll
    for (int r = 0; r < R; ++r) v.a[r] = __builtin_nontemporal_load(a + base + r * 64);
    if constexpr (NIN == 2) {
#pragma unroll
        for (int r = 0; r < R; ++r) v.b[r] = __builtin_nontemporal_load(b + base + r * 64);
    }
}
template <int R, int W, int NIN>
__device__ __forceinline__ void tl_store(f32x4* out, long long t, const TileRegs<R, NIN>& v) {
    const long long base = t * (W * 64 * R) + (long long)(threadIdx.x / 64) * (64 * R) + (threadIdx.x & 63);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if constexpr (NIN == 2) __builtin_nontemporal_store(v.a[r] + v.b[r], out + base + r * 64);
        else __builtin_nontemporal_store(v.a[r], out + base + r * 64);
    }
}

template <int R, int W, int NIN, bool TICKET>
__global__ __launch_bounds__(W * 64) void tiled_kernel(const f32x4* a, const f32x4* b, f32x4* r, long long ntiles,
                                                       unsigned* ticket) {
    __shared__ unsigned s_t[2];
    TileRegs<R, NIN> va, vb;
    auto next_tile = [&](long long cur, int slot) -> long long {
        if constexpr (TICKET) {
            if (threadIdx.x == 0) s_t[slot] = atomicAdd(ticket, 1u);
            __syncthreads();
            return (long long)s_t[slot];
        } else {
            return cur + gridDim.x;
        }
    };
    long long ta = TICKET ? next_tile(0, 0) : (long long)blockIdx.x;
    if (ta >= ntiles) return;
    tl_load<R, W, NIN>(a, b, ta, va);
    while (true) {
        const long long tb = next_tile(ta, 1);
        if (tb < ntiles) tl_load<R, W, NIN>(a, b, tb, vb);
        tl_store<R, W, NIN>(r, ta, va);
        if (tb >= ntiles) break;
        ta = next_tile(tb, 0);
        if (ta < ntiles) tl_load<R, W, NIN>(a, b, ta, va);
        tl_store<R, W, NIN>(r, tb, vb);
        if (ta >= ntiles) break;
    }
}

// ONE-SHOT: one tile per block, grid = number of tiles: the hardware dispatcher hands tiles out in launch order (the
// ticket order, with no counter to reset); no double buffer, several resident blocks per CU overlap instead.
template <int R, int W, int NIN>
__global__ __launch_bounds__(W * 64) void oneshot_kernel(const f32x4* a, const f32x4* b, f32x4* r) {
    TileRegs<R, NIN> v;
    tl_load<R, W, NIN>(a, b, blockIdx.x, v);
    tl_store<R, W, NIN>(r, blockIdx.x, v);
}

// SELF-RESETTING TICKET: as tiled_kernel<TICKET> but the counter needs no memset: the last block to finish zeroes it
// (ticket[0] = next tile, ticket[1] = finished blocks); stream order makes the next launch see zeros.
template <int R, int W, int NIN>
__global__ __launch_bounds__(W * 64) void tiled_selfreset_kernel(const f32x4* a, const f32x4* b, f32x4* r,
                                                                 long long ntiles, unsigned* ticket) {
    __shared__ unsigned s_t[2];
    TileRegs<R, NIN> va, vb;
    auto take = [&](int slot) -> long long {
        if (threadIdx.x == 0) s_t[slot] = atomicAdd(ticket, 1u);
        __syncthreads();
        return (long long)s_t[slot];
    };
    long long ta = take(0);
    if (ta < ntiles) {
        tl_load<R, W, NIN>(a, b, ta, va);
        while (true) {
            const long long tb = take(1);
            if (tb < ntiles) tl_load<R, W, NIN>(a, b, tb, vb);
            tl_store<R, W, NIN>(r, ta, va);
            if (tb >= ntiles) break;
            ta = take(0);
            if (ta < ntiles) tl_load<R, W, NIN>(a, b, ta, va);
            tl_store<R, W, NIN>(r, tb, vb);
            if (ta >= ntiles) break;
        }
    }
    if (threadIdx.x == 0) {
        __threadfence();
        if (atomicAdd(ticket + 1, 1u) == gridDim.x - 1) {
            atomicExch(ticket, 0u);
            atomicExch(ticket + 1, 0u);
        }
    }
}

// Ticket-ordered READ-ONLY stream (the reduce's traffic): persistent, next tile's loads in flight while the current
// tile is summed; per-lane partial kept (written once so the loads stay live).
template <int R, int W>
__global__ __launch_bounds__(W * 64) void tsum_kernel(const f32x4* a, long long ntiles, unsigned* ticket, float* out) {
    __shared__ unsigned s_t[2];
    TileRegs<R, 1> va, vb;
    f32x4 acc = {0, 0, 0, 0};
    auto take = [&](int slot) -> long long {
        if (threadIdx.x == 0) s_t[slot] = atomicAdd(ticket, 1u);
        __syncthreads();
        return (long long)s_t[slot];
    };
    long long ta = take(0);
    if (ta < ntiles) {
        tl_load<R, W, 1>(a, a, ta, va);
        while (true) {
            const long long tb = take(1);
            if (tb < ntiles) tl_load<R, W, 1>(a, a, tb, vb);
#pragma unroll
            for (int r = 0; r < R; ++r) acc += va.a[r];
            if (tb >= ntiles) break;
            ta = take(0);
            if (ta < ntiles) tl_load<R, W, 1>(a, a, ta, va);
#pragma unroll
            for (int r = 0; r < R; ++r) acc += vb.a[r];
            if (ta >= ntiles) break;
        }
    }
    if (acc.x + acc.y + acc.z + acc.w == 12345.f) out[0] = 1.f;
}

int tiled_sweep(f32x4* a, f32x4* b, f32x4* r, long long n4, unsigned* ticket, hipEvent_t e0, hipEvent_t e1) {
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const double B = (double)n4 * 16;
    auto time = [&](const char* name, double bytes, auto fn) {
        for (int i = 0; i < 2; ++i) fn();
        hipEventRecord(e0);
        for (int i = 0; i < 10; ++i) fn();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= 10;
        printf("%-36s %.4f ms %7.1f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    char nm[96];
#define TL(R, W, NIN, TK, PERCU)                                                                               \
    {                                                                                                          \
        const long long tile4 = (long long)W * 64 * R, nt = n4 / tile4;                                        \
        const int grid = (int)(nt < (long long)cus * PERCU ? nt : (long long)cus * PERCU);                     \
        snprintf(nm, sizeof nm, "%s R%d W%d %s x%d", NIN == 1 ? "copy" : "vadd", R, W, TK ? "ticket" : "static", \
                 PERCU);                                                                                       \
        time(nm, (NIN + 1) * (double)nt * tile4 * 16, [&] {                                                    \
            if (TK) hipMemsetAsync(ticket, 0, 4);                                                              \
            tiled_kernel<R, W, NIN, TK><<<grid, W * 64>>>(a, b, r, nt, ticket);                                \
        });                                                                                                    \
    }
    TL(16, 8, 1, true, 1)
    TL(16, 8, 1, false, 1)
    TL(16, 8, 1, true, 2)
    TL(16, 8, 1, false, 2)
    TL(8, 8, 1, true, 2)
    TL(8, 8, 1, false, 2)
    TL(8, 16, 1, true, 1)
    TL(8, 4, 1, false, 4)
    TL(16, 4, 1, false, 2)
    TL(8, 8, 2, true, 1)
    TL(8, 8, 2, false, 1)
    TL(8, 8, 2, true, 2)
    TL(8, 8, 2, false, 2)
    TL(16, 8, 2, false, 1)
    TL(8, 16, 2, true, 1)
    TL(8, 4, 2, false, 4)
    TL(4, 8, 2, false, 4)
#undef TL
    (void)B;
    return 0;
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
    if (argc > 2 && argv[2][0] == 't') {  // persistent tiled (scan-structure) sweep
        unsigned* ticket;
        CK(hipMalloc(&ticket, 16));
        return tiled_sweep(a, b, r, n4, ticket, e0, e1);
    }
    if (argc > 2 && argv[2][0] == 'a') {  // interleaved A/B: grid-stride vs ticket-tiled, 6 alternations
        unsigned* ticket;
        CK(hipMalloc(&ticket, 16));
        int cus = 256;
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
        const long long ntc = n4 / (8 * 64 * 16), ntv = n4 / (8 * 64 * 8);
        for (int rep = 0; rep < 6; ++rep) {
            printf("-- alternation %d\n", rep);
            time("grid copy U4 nt g16384", 2 * B, [&] { copy_kernel<4, true><<<16384, 256>>>(a, r, n4); });
            time("tiled copy R16W8 ticket x1", 2 * (double)ntc * 8192 * 16, [&] {
                hipMemsetAsync(ticket, 0, 4);
                tiled_kernel<16, 8, 1, true><<<cus, 512>>>(a, b, r, ntc, ticket);
            });
            time("grid vadd U4 nt g16384", 3 * B, [&] { vadd_kernel<4, true><<<16384, 256>>>(a, b, r, n4); });
            time("tiled vadd R8W8 ticket x2", 3 * (double)ntv * 4096 * 16, [&] {
                hipMemsetAsync(ticket, 0, 4);
                tiled_kernel<8, 8, 2, true><<<2 * cus, 512>>>(a, b, r, ntv, ticket);
            });
            time("grid axpy(in place) U4 nt g16384", 3 * B, [&] { vadd_kernel<4, true><<<16384, 256>>>(a, b, b, n4); });
            time("tiled axpy(in place) R8W8 ticket x2", 3 * (double)ntv * 4096 * 16, [&] {
                hipMemsetAsync(ticket, 0, 4);
                tiled_kernel<8, 8, 2, true><<<2 * cus, 512>>>(a, b, b, ntv, ticket);
            });
            time("tiled copy R16W8 static x1", 2 * (double)ntc * 8192 * 16,
                 [&] { tiled_kernel<16, 8, 1, false><<<cus, 512>>>(a, b, r, ntc, ticket); });
        }
        return 0;
    }
    if (argc > 2 && argv[2][0] == 's') {  // read-only: grid-stride sum vs ticket-ordered tiles, 5 alternations
        unsigned* ticket;
        CK(hipMalloc(&ticket, 16));
        int cus = 256;
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
        for (int rep = 0; rep < 5; ++rep) {
            printf("-- alternation %d\n", rep);
            time("grid sum U4 g16384", B, [&] { sum_kernel<4><<<16384, 256>>>(a, n4, out); });
            const long long nt16 = n4 / (8 * 64 * 16), nt8 = n4 / (8 * 64 * 8);
            time("ticket sum R16W8 x1", (double)nt16 * 8192 * 16, [&] {
                hipMemsetAsync(ticket, 0, 4);
                tsum_kernel<16, 8><<<cus, 512>>>(a, nt16, ticket, out);
            });
            time("ticket sum R16W8 x2", (double)nt16 * 8192 * 16, [&] {
                hipMemsetAsync(ticket, 0, 4);
                tsum_kernel<16, 8><<<2 * cus, 512>>>(a, nt16, ticket, out);
            });
            time("ticket sum R8W8 x2", (double)nt8 * 4096 * 16, [&] {
                hipMemsetAsync(ticket, 0, 4);
                tsum_kernel<8, 8><<<2 * cus, 512>>>(a, nt8, ticket, out);
            });
            time("ticket sum R8W8 x4", (double)nt8 * 4096 * 16, [&] {
                hipMemsetAsync(ticket, 0, 4);
                tsum_kernel<8, 8><<<4 * cus, 512>>>(a, nt8, ticket, out);
            });
        }
        return 0;
    }
    if (argc > 2 && argv[2][0] == 'o') {  // one-shot + self-resetting ticket vs the memset ticket, 4 alternations
        unsigned* ticket;
        CK(hipMalloc(&ticket, 16));
        CK(hipMemset(ticket, 0, 16));
        int cus = 256;
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
        char nm[96];
#define OS(R, W, NIN)                                                                                         \
    {                                                                                                         \
        const long long tile4 = (long long)W * 64 * R, nt = n4 / tile4;                                      \
        snprintf(nm, sizeof nm, "oneshot %s R%d W%d", NIN == 1 ? "copy" : "vadd", R, W);                     \
        time(nm, (NIN + 1) * (double)nt * tile4 * 16, [&] { oneshot_kernel<R, W, NIN><<<(int)nt, W * 64>>>(a, b, r); }); \
    }
#define SR(R, W, NIN, PERCU)                                                                                  \
    {                                                                                                         \
        const long long tile4 = (long long)W * 64 * R, nt = n4 / tile4;                                      \
        snprintf(nm, sizeof nm, "selfreset %s R%d W%d x%d", NIN == 1 ? "copy" : "vadd", R, W, PERCU);        \
        time(nm, (NIN + 1) * (double)nt * tile4 * 16,                                                        \
             [&] { tiled_selfreset_kernel<R, W, NIN><<<cus * PERCU, W * 64>>>(a, b, r, nt, ticket); });      \
    }
        for (int rep = 0; rep < 4; ++rep) {
            printf("-- alternation %d\n", rep);
            OS(4, 4, 1) OS(8, 4, 1) OS(16, 4, 1) OS(8, 8, 1) OS(16, 8, 1)
            OS(4, 4, 2) OS(8, 4, 2) OS(4, 8, 2) OS(8, 8, 2)
            SR(16, 8, 1, 1) SR(16, 8, 1, 2) SR(8, 8, 2, 1) SR(8, 8, 2, 2) SR(8, 4, 2, 4)
            const long long ntc = n4 / (8 * 64 * 16);
            time("tiled copy R16W8 ticket x1", 2 * (double)ntc * 8192 * 16, [&] {
                hipMemsetAsync(ticket, 0, 4);
                tiled_kernel<16, 8, 1, true><<<cus, 512>>>(a, b, r, ntc, ticket);
            });
            hipMemsetAsync(ticket, 0, 16);
            time("grid copy U4 nt g16384", 2 * B, [&] { copy_kernel<4, true><<<16384, 256>>>(a, r, n4); });
        }
#undef OS
#undef SR
        return 0;
    }
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
