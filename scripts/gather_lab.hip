// Gather-rate lab: how many random 4-B gathers per second can MI355X serve from an L2/MALL/HBM-resident
// table? Each lane issues G independent gathers per round (hash-generated indices, no index loads), R rounds.
// Build: hipcc --offload-arch=gfx950 -O3 scripts/gather_lab.hip -o build/gather_lab
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ __forceinline__ unsigned hash(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

template <int G>
__global__ __launch_bounds__(256) void gather_kernel(const float* __restrict__ t, unsigned mask, int rounds,
                                                     float* __restrict__ out) {
    const unsigned tid = blockIdx.x * 256 + threadIdx.x;
    float acc = 0.f;
    unsigned s = hash(tid * 2654435761U + 1);
    for (int r = 0; r < rounds; ++r) {
        unsigned idx[G];
#pragma unroll
        for (int g = 0; g < G; ++g) { s = hash(s + g); idx[g] = s & mask; }
        float v[G];
#pragma unroll
        for (int g = 0; g < G; ++g) v[g] = t[idx[g]];
#pragma unroll
        for (int g = 0; g < G; ++g) acc += v[g];
    }
    if (acc == 12345.f) out[tid] = acc;
}

// same, but every XCD (block % 8) gathers only from its own 1/8 of the table (XCD-sliced working set)
template <int G>
__global__ __launch_bounds__(256) void gather_xcd_kernel(const float* __restrict__ t, unsigned mask, int rounds,
                                                         float* __restrict__ out) {
    const unsigned tid = blockIdx.x * 256 + threadIdx.x;
    const unsigned base = (blockIdx.x & 7) * (mask + 1);
    float acc = 0.f;
    unsigned s = hash(tid * 2654435761U + 1);
    for (int r = 0; r < rounds; ++r) {
        unsigned idx[G];
#pragma unroll
        for (int g = 0; g < G; ++g) { s = hash(s + g); idx[g] = base + (s & mask); }
        float v[G];
#pragma unroll
        for (int g = 0; g < G; ++g) v[g] = t[idx[g]];
#pragma unroll
        for (int g = 0; g < G; ++g) acc += v[g];
    }
    if (acc == 12345.f) out[tid] = acc;
}

int main() {
    const size_t maxn = 1u << 26;  // 256 MB table
    float *t, *out;
    hipMalloc(&t, maxn * 4);
    hipMemset(t, 0, maxn * 4);
    hipMalloc(&out, 64 << 20);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int blocks = 256 * 8, rounds = 64;
    const double gathers = (double)blocks * 256 * rounds * 16;
    for (int lg = 16; lg <= 26; lg += 1) {
        const unsigned mask = (1u << lg) - 1;
        for (int rep = 0; rep < 2; ++rep) gather_kernel<16><<<blocks, 256>>>(t, mask, rounds, out);
        hipEventRecord(e0);
        for (int rep = 0; rep < 5; ++rep) gather_kernel<16><<<blocks, 256>>>(t, mask, rounds, out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= 5;
        float msx = 0;
        if (lg <= 23) {
            const unsigned m8 = (1u << lg) / 8 - 1;
            for (int rep = 0; rep < 2; ++rep) gather_xcd_kernel<16><<<blocks, 256>>>(t, m8, rounds, out);
            hipEventRecord(e0);
            for (int rep = 0; rep < 5; ++rep) gather_xcd_kernel<16><<<blocks, 256>>>(t, m8, rounds, out);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            hipEventElapsedTime(&msx, e0, e1);
            msx /= 5;
        }
        printf("table %8.2f MB: %7.1f Ggather/s (%.3f ms)   xcd-sliced: %7.1f Ggather/s\n", (4.0 * (1u << lg)) / 1e6,
               gathers / ms / 1e6, ms, msx > 0 ? gathers / msx / 1e6 : 0.0);
    }
    return 0;
}
