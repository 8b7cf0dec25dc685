// Scan design lab (standalone, not part of the library): measures on one MI355X
//   copy     : f32x4 nontemporal read+write of n floats (the 8 B/element roofline of a single-pass scan)
//   noscan   : the production tile structure (load, in-register wave scans, store) WITHOUT the look-back
//   lib      : the library's pcmx_scan_f32 (linked from libpcmx_hip.so) at rows 4/8/16
// build: hipcc -O3 --offload-arch=gfx950 -Icsrc/include -Icsrc/runtime scripts/scan_lab.hip -o build/scan_lab \
//        -Lparallel_c_programs_amd/lib -lpcmx_hip -Wl,-rpath,$PWD/parallel_c_programs_amd/lib
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <cmath>

#include "pcmx_common.h"
#include "pcmx_hip.h"

extern "C" int pcmx_scan_f32_rows(const float* x, float* out, long long n, int exclusive, const float* init_dev, void* ws,
                                  unsigned* err_flag, int rows, hipStream_t s);
extern "C" int pcmx_scan_f32(const float* x, float* out, long long n, int exclusive, const float* init_dev, void* ws,
                             unsigned* err_flag,
                             hipStream_t s);

using pcmx::f32x4;

__global__ __launch_bounds__(256) void copy_kernel(const f32x4* __restrict__ in, f32x4* __restrict__ out, long long n4) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += stride)
        __builtin_nontemporal_store(__builtin_nontemporal_load(in + i), out + i);
}

// one-shot copy: each block moves a contiguous tile of R f32x4 per lane (like the scan tile), no grid stride
template <int R>
__global__ __launch_bounds__(512) void tile_copy_kernel(const f32x4* __restrict__ in, f32x4* __restrict__ out, long long n4) {
    const long long base = (long long)blockIdx.x * 512 * R + (threadIdx.x / 64) * 64 * R + (threadIdx.x & 63);
    f32x4 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const long long i = base + r * 64;
        if (i < n4) v[r] = __builtin_nontemporal_load(in + i);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const long long i = base + r * 64;
        if (i < n4) __builtin_nontemporal_store(v[r] * 1.0001f, out + i);
    }
}

// block-interleaved tile: row r of the block covers 512 consecutive f32x4 (8 KiB), all waves side by side
template <int R, int T>
__global__ __launch_bounds__(T) void tile_copy_il_kernel(const f32x4* __restrict__ in, f32x4* __restrict__ out, long long n4) {
    const long long base = (long long)blockIdx.x * T * R + threadIdx.x;
    f32x4 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const long long i = base + r * T;
        if (i < n4) v[r] = __builtin_nontemporal_load(in + i);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const long long i = base + r * T;
        if (i < n4) __builtin_nontemporal_store(v[r] * 1.0001f, out + i);
    }
}
// wave-contiguous tile with T threads
template <int R, int T>
__global__ __launch_bounds__(T) void tile_copy_wc_kernel(const f32x4* __restrict__ in, f32x4* __restrict__ out, long long n4) {
    const long long base = (long long)blockIdx.x * T * R + (threadIdx.x / 64) * 64 * R + (threadIdx.x & 63);
    f32x4 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const long long i = base + r * 64;
        if (i < n4) v[r] = __builtin_nontemporal_load(in + i);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const long long i = base + r * 64;
        if (i < n4) __builtin_nontemporal_store(v[r] * 1.0001f, out + i);
    }
}

// ---- lab scan: production structure with switches
//   TICKET: tile id from an atomic ticket (1) or blockIdx.x (0)
//   LB    : 0 = no look-back (prefix = 0, upper bound), 1 = decoupled look-back
//   SLEEP : s_sleep between polls
struct LabWs {
    unsigned ticket, timeout, pad[2];
};
template <int R, int TICKET, int LB, int SLEEP>
__global__ __launch_bounds__(512) void lab_scan(const float* __restrict__ in, float* __restrict__ out, long long n,
                                                LabWs* ws) {
    constexpr int kW = 8;
    unsigned long long* status = reinterpret_cast<unsigned long long*>(ws + 1);
    __shared__ float s_wave_tot[kW];
    __shared__ float s_prefix;
    __shared__ unsigned s_tile;
    constexpr int kWaveItems = R * 256;
    constexpr int kTile = kW * kWaveItems;
    const int lane = pcmx::lane_id();
    const int wave = threadIdx.x / 64;
    long long tile;
    if (TICKET) {
        if (threadIdx.x == 0) s_tile = atomicAdd(&ws->ticket, 1u);
        __syncthreads();
        tile = s_tile;
    } else {
        tile = blockIdx.x;
    }
    const long long base = tile * kTile + (long long)wave * kWaveItems;
    f32x4 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const long long e = base + r * 256 + lane * 4;
        if (e + 3 < n) v[r] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(in + e));
        else v[r] = f32x4{0, 0, 0, 0};
    }
    float carry = 0.f;
    float lane_excl[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        v[r].y += v[r].x;
        v[r].z += v[r].y;
        v[r].w += v[r].z;
        const float incl = pcmx::wave_inclusive_scan(v[r].w);
        float excl = __shfl_up(incl, 1, 64);
        if (lane == 0) excl = 0.f;
        lane_excl[r] = carry + excl;
        carry += __shfl(incl, 63, 64);
    }
    if (lane == 0) s_wave_tot[wave] = carry;
    __syncthreads();
    if (wave == 0) {
        float agg = 0.f;
#pragma unroll
        for (int w = 0; w < kW; ++w) agg += s_wave_tot[w];
        float prefix = 0.f;
        if (LB) {
            if (tile == 0) {
                if (lane == 0) __hip_atomic_store(&status[0], ((2ull << 32) | __float_as_uint(agg)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                if (lane == 0) __hip_atomic_store(&status[tile], ((1ull << 32) | __float_as_uint(agg)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                long long look = tile - 1;
                unsigned spins = 0;
                while (true) {
                    const long long idx = look - lane;
                    unsigned long long sv = idx >= 0 ? __hip_atomic_load(&status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                                     : (2ull << 32);
                    const unsigned flag = (unsigned)(sv >> 32);
                    const float val = __uint_as_float((unsigned)sv);
                    const unsigned long long m_incl = __ballot(flag == 2u);
                    const unsigned long long m_zero = __ballot(flag == 0u);
                    if (m_incl != 0ull) {
                        const int first = __builtin_ctzll(m_incl);
                        const unsigned long long need = (first == 63) ? ~0ull : ((1ull << (first + 1)) - 1ull);
                        if ((m_zero & need) == 0ull) {
                            prefix += pcmx::wave_reduce<float, 0>(lane <= first ? val : 0.f);
                            break;
                        }
                    } else if (m_zero == 0ull) {
                        prefix += pcmx::wave_reduce<float, 0>(val);
                        look -= 64;
                        continue;
                    }
                    if (++spins > (1u << 26)) {
                        if (lane == 0) atomicExch(&ws->timeout, 1u);
                        break;
                    }
                    if (SLEEP) __builtin_amdgcn_s_sleep(SLEEP);
                }
                if (lane == 0) __hip_atomic_store(&status[tile], ((2ull << 32) | __float_as_uint(prefix + agg)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (lane == 0) {
            float wo = 0.f;
            for (int w = 0; w < kW; ++w) {
                float t = s_wave_tot[w];
                s_wave_tot[w] = wo;
                wo += t;
            }
            s_prefix = prefix;
        }
    }
    __syncthreads();
    const float off = s_prefix + s_wave_tot[wave];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const float b = off + lane_excl[r];
        f32x4 o = v[r] + b;
        const long long e = base + r * 256 + lane * 4;
        if (e + 3 < n) __builtin_nontemporal_store(o, reinterpret_cast<f32x4*>(out + e));
    }
}

// ---- persistent, software-pipelined decoupled look-back scan: the loads of the block's NEXT tile are in
// flight while the look-back of the current tile polls its predecessors.
template <int R, int W>
struct PipeTile {
    static constexpr int kWaveItems = R * 256, kTile = W * kWaveItems;
};
template <int R, int W>
__device__ __forceinline__ void pipe_load(const float* __restrict__ in, long long n, long long tile, f32x4 (&v)[R]) {
    const int lane = pcmx::lane_id(), wave = threadIdx.x / 64;
    const long long base = tile * PipeTile<R, W>::kTile + (long long)wave * PipeTile<R, W>::kWaveItems;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const long long e = base + r * 256 + lane * 4;
        if (e + 3 < n) v[r] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(in + e));
        else v[r] = f32x4{0, 0, 0, 0};
    }
}
template <int R, int W, int LPL = 1>
__device__ __forceinline__ void pipe_finish(float* __restrict__ out, long long n, long long tile, f32x4 (&v)[R],
                                            unsigned long long* status, float* s_wave_tot, float* s_prefix,
                                            long long next_tile, const float* __restrict__ in, f32x4 (&vn)[R],
                                            long long ntiles) {
    const int lane = pcmx::lane_id(), wave = threadIdx.x / 64;
    float carry = 0.f;
    float lane_excl[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        v[r].y += v[r].x;
        v[r].z += v[r].y;
        v[r].w += v[r].z;
        const float incl = pcmx::wave_inclusive_scan(v[r].w);
        float excl = __shfl_up(incl, 1, 64);
        if (lane == 0) excl = 0.f;
        lane_excl[r] = carry + excl;
        carry += __shfl(incl, 63, 64);
    }
    if (lane == 0) s_wave_tot[wave] = carry;
    __syncthreads();
    float agg = 0.f;
#pragma unroll
    for (int w = 0; w < W; ++w) agg += s_wave_tot[w];
    if (wave == 0 && lane == 0)
        __hip_atomic_store(&status[tile], ((tile == 0 ? 2ull : 1ull) << 32) | __float_as_uint(agg), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    // next tile's loads go out now: they overlap the look-back below
    if (next_tile < ntiles) pipe_load<R, W>(in, n, next_tile, vn);
    float wexcl = 0.f;
#pragma unroll
    for (int w = 0; w < W; ++w) wexcl += w < wave ? s_wave_tot[w] : 0.f;
    if (wave == 0) {
        float prefix = 0.f;
        if (tile != 0) {
            long long look = tile - 1;
            while (true) {
                // lane l covers statuses look - l*LPL - j, j < LPL (newest first)
                unsigned long long sv[LPL];
#pragma unroll
                for (int j = 0; j < LPL; ++j) {
                    const long long idx = look - (long long)lane * LPL - j;
                    sv[j] = idx >= 0 ? __hip_atomic_load(&status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                     : (2ull << 32);
                }
                // per-lane combine (newest first): stop at the first INCL in this lane's slice
                unsigned lflag = 1u;  // 1 = all AGG, 2 = reached INCL, 0 = not ready
                float lval = 0.f;
#pragma unroll
                for (int j = 0; j < LPL; ++j) {
                    const unsigned f = (unsigned)(sv[j] >> 32);
                    if (lflag == 1u) {
                        if (f == 0u) lflag = 0u;
                        else {
                            lval += __uint_as_float((unsigned)sv[j]);
                            if (f == 2u) lflag = 2u;
                        }
                    }
                }
                const unsigned flag = lflag;
                const float val = lval;
                const unsigned long long m_incl = __ballot(flag == 2u);
                const unsigned long long m_zero = __ballot(flag == 0u);
                if (m_incl != 0ull) {
                    const int first = __builtin_ctzll(m_incl);
                    const unsigned long long need = (first == 63) ? ~0ull : ((1ull << (first + 1)) - 1ull);
                    if ((m_zero & need) == 0ull) {
                        prefix += pcmx::wave_reduce<float, 0>(lane <= first ? val : 0.f);
                        break;
                    }
                } else if (m_zero == 0ull) {
                    prefix += pcmx::wave_reduce<float, 0>(val);
                    look -= 64 * LPL;
                    continue;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (lane == 0)
                __hip_atomic_store(&status[tile], (2ull << 32) | __float_as_uint(prefix + agg), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) *s_prefix = prefix;
    }
    __syncthreads();
    const float off = *s_prefix + wexcl;
    const long long base = tile * PipeTile<R, W>::kTile + (long long)wave * PipeTile<R, W>::kWaveItems;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const float b = off + lane_excl[r];
        const f32x4 o = v[r] + b;
        const long long e = base + r * 256 + lane * 4;
        if (e + 3 < n) __builtin_nontemporal_store(o, reinterpret_cast<f32x4*>(out + e));
    }
}
template <int R, int W, int LPL>
__global__ __launch_bounds__(W * 64) void lab_scan_pipe(const float* __restrict__ in, float* __restrict__ out, long long n,
                                                       LabWs* ws, long long ntiles) {
    unsigned long long* status = reinterpret_cast<unsigned long long*>(ws + 1);
    __shared__ float s_wave_tot[2][W];
    __shared__ float s_prefix[2];
    __shared__ unsigned s_tile[2];
    f32x4 va[R], vb[R];
    if (threadIdx.x == 0) s_tile[0] = atomicAdd(&ws->ticket, 1u);
    __syncthreads();
    long long ta = s_tile[0];
    if (ta >= ntiles) return;
    pipe_load<R, W>(in, n, ta, va);
    while (true) {
        if (threadIdx.x == 0) s_tile[1] = atomicAdd(&ws->ticket, 1u);
        __syncthreads();
        const long long tb = s_tile[1];
        pipe_finish<R, W, LPL>(out, n, ta, va, status, s_wave_tot[0], &s_prefix[0], tb, in, vb, ntiles);
        if (tb >= ntiles) break;
        if (threadIdx.x == 0) s_tile[0] = atomicAdd(&ws->ticket, 1u);
        __syncthreads();
        ta = s_tile[0];
        pipe_finish<R, W, LPL>(out, n, tb, vb, status, s_wave_tot[1], &s_prefix[1], ta, in, va, ntiles);
        if (ta >= ntiles) break;
    }
}

template <class F>
float time_ms(F f, int reps = 10) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    f();
    f();
    hipDeviceSynchronize();
    std::vector<float> t;
    for (int i = 0; i < reps; ++i) {
        hipEventRecord(a);
        f();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main(int argc, char** argv) {
    const long long n = argc > 1 ? (long long)atof(argv[1]) : 1000000000LL;
    float *x, *y;
    void* ws;
    hipMalloc(&x, n * 4);
    hipMalloc(&y, n * 4);
    hipMalloc(&ws, pcmx_scan_workspace_bytes(n) + (n / 512 + 64) * 8);
    pcmx_rand_uniform_f32(x, n, 7, 0.f, 1.f, 0);
    hipDeviceSynchronize();
    const double gb = 8.0 * n / 1e9;
    const long long n4 = n / 4;
    std::vector<float> hx(1 << 20), hy(1 << 20);
    hipMemcpy(hx.data(), x, hx.size() * 4, hipMemcpyDeviceToHost);
    auto check = [&] {
        float tail[4];
        hipMemcpy(hy.data(), y, hy.size() * 4, hipMemcpyDeviceToHost);
        hipMemcpy(tail, y + n - 4, 16, hipMemcpyDeviceToHost);
        double s = 0, worst = 0;
        for (size_t i = 0; i < hx.size(); ++i) {
            s += hx[i];
            worst = std::max(worst, std::abs(hy[i] - s) / s);
        }
        printf("      rel err (first 1M) %.2e, last %.6e (expect ~%.6e)\n", worst, tail[3], 0.5 * n);
    };
    for (int g : {1024}) {
        float ms = time_ms([&] { copy_kernel<<<g, 256>>>((const f32x4*)x, (f32x4*)y, n4); });
        printf("copy grid=%5d        %7.3f ms %7.1f GB/s\n", g, ms, gb / ms * 1e3);
    }
    {
        float ms = time_ms([&] { tile_copy_kernel<8><<<(n4 + 4095) / 4096, 512>>>((const f32x4*)x, (f32x4*)y, n4); });
        printf("tilecopy R=8          %7.3f ms %7.1f GB/s\n", ms, gb / ms * 1e3);
        ms = time_ms([&] { tile_copy_kernel<16><<<(n4 + 8191) / 8192, 512>>>((const f32x4*)x, (f32x4*)y, n4); });
        printf("tilecopy R=16         %7.3f ms %7.1f GB/s\n", ms, gb / ms * 1e3);
        ms = time_ms([&] { tile_copy_kernel<4><<<(n4 + 2047) / 2048, 512>>>((const f32x4*)x, (f32x4*)y, n4); });
        printf("tilecopy R=4          %7.3f ms %7.1f GB/s\n", ms, gb / ms * 1e3);
    }
#define IL(R, T) { float ms = time_ms([&] { tile_copy_il_kernel<R, T><<<(n4 + T * R - 1) / (T * R), T>>>((const f32x4*)x, (f32x4*)y, n4); }); \
        printf("il  R=%2d T=%4d        %7.3f ms %7.1f GB/s\n", R, T, ms, gb / ms * 1e3); }
#define WC(R, T) { float ms = time_ms([&] { tile_copy_wc_kernel<R, T><<<(n4 + T * R - 1) / (T * R), T>>>((const f32x4*)x, (f32x4*)y, n4); }); \
        printf("wc  R=%2d T=%4d        %7.3f ms %7.1f GB/s\n", R, T, ms, gb / ms * 1e3); }
    WC(16, 512) WC(8, 1024) WC(12, 1024) WC(10, 1024)
#define LAB(R, TK, LB, SL) { const long long tiles = (n + R * 2048 - 1) / (R * 2048); \
        float ms = time_ms([&] { hipMemsetAsync(ws, 0, 16 + tiles * 8, 0); lab_scan<R, TK, LB, SL><<<tiles, 512>>>(x, y, n, (LabWs*)ws); }); \
        unsigned to = 0; hipMemcpy(&to, (char*)ws + 4, 4, hipMemcpyDeviceToHost); \
        printf("lab R=%2d ticket=%d lb=%d sleep=%d  %7.3f ms %7.1f GB/s timeout=%u\n", R, TK, LB, SL, ms, gb / ms * 1e3, to); }
#define PIPE(R, W, BPC, LPL) { const long long tiles = (n + R * W * 256 - 1) / (R * W * 256); \
        float ms = time_ms([&] { hipMemsetAsync(ws, 0, 16 + tiles * 8, 0); lab_scan_pipe<R, W, LPL><<<256 * BPC, W * 64>>>(x, y, n, (LabWs*)ws, tiles); }); \
        printf("pipe R=%2d W=%2d bpc=%d lpl=%d    %7.3f ms %7.1f GB/s\n", R, W, BPC, LPL, ms, gb / ms * 1e3); check(); }
    PIPE(16, 8, 1, 1) PIPE(16, 8, 1, 2) PIPE(16, 8, 1, 4) PIPE(8, 16, 1, 1) PIPE(8, 16, 1, 2)
    PIPE(12, 16, 1, 1) PIPE(12, 16, 1, 2) PIPE(10, 16, 1, 2) PIPE(14, 8, 1, 2) PIPE(20, 8, 1, 2) PIPE(6, 16, 1, 2)
    PIPE(8, 8, 2, 2) PIPE(12, 8, 1, 2)
    for (int rows : {4, 8, 16}) {
        float ms = time_ms([&] { pcmx_scan_f32_rows(x, y, n, 0, nullptr, ws, nullptr, rows, 0); });
        printf("lib scan rows=%2d      %7.3f ms %7.1f GB/s\n", rows, ms, gb / ms * 1e3);
    }
    check();
    return 0;
}
