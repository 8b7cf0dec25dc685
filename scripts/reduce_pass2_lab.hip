// Reduce pass-2 A/B (round 4, late): the library's pass 1 followed by the former pass 2 (8 scalar partial loads per
// thread per iteration, 8 dependent round trips for 16384 partials) or by the current one (all partials in flight
// as 16-B loads), at 62M (the banded SpMV's 248 MB value stream), 125M (one N = 8 rank of the strong 1e9 reduce) and
// 1e9 floats; pass 1 alone for reference. Same process, same buffers, HIP-event mean of 20 back-to-back calls.
// build: hipcc -O3 --offload-arch=gfx950 -Icsrc/include -Icsrc/runtime scripts/reduce_pass2_lab.hip -o bin_lab/reduce_pass2_lab
#include "../csrc/kernels/reduce.hip"

#include <cstdio>

namespace lab {
// the pass 2 the library used until this lab (kept here for the A/B)
__global__ __launch_bounds__(256) void old_pass2(const float* __restrict__ partials, int np, float* __restrict__ out) {
    __shared__ double lds[4];
    constexpr int kU = 8;
    double acc[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) acc[u] = 0.0;
    for (int i0 = threadIdx.x; i0 < np; i0 += 256 * kU) {
        float v[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) v[u] = i0 + u * 256 < np ? partials[i0 + u * 256] : 0.f;
#pragma unroll
        for (int u = 0; u < kU; ++u) acc[u] += (double)v[u];
    }
#pragma unroll
    for (int u = 1; u < kU; ++u) acc[0] += acc[u];
    const double r = block_reduce<double, 0>(acc[0], lds);
    if (threadIdx.x == 0) out[0] = (float)r;
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
    const long long nmax = 1000000000LL;
    float *x, *out;
    void* ws;
    if (hipMalloc(&x, nmax * 4) || hipMalloc(&out, 64) || hipMalloc(&ws, 1 << 20)) return 1;
    (void)hipMemset(x, 0, nmax * 4);
    for (long long n : {61955590LL, 125000000LL, 1000000000LL}) {
        const int nb = pass1_blocks(n);
        float* part = (float*)ws;
        const float p1 = time_ms([&] { reduce_pass1<float, 0, false><<<nb, kThreads>>>(x, x, n, part); });
        const float po = time_ms([&] {
            reduce_pass1<float, 0, false><<<nb, kThreads>>>(x, x, n, part);
            lab::old_pass2<<<1, 256>>>(part, nb, out);
        });
        const float pn = time_ms([&] { pcmx_reduce_f32(x, n, 0, out, ws, 0); });
        const float o2 = time_ms([&] { lab::old_pass2<<<1, 256>>>(part, nb, out); });
        const float n2 = time_ms([&] { reduce_pass2<float, 0><<<1, kThreads>>>(part, nb, out); });
        printf("n %11lld (%5d partials): pass1 %.4f ms | pass1 + old pass2 %.4f ms (%.0f GB/s) | pass1 + new pass2 %.4f "
               "ms (%.0f GB/s) | old pass2 alone %.2f us, new %.2f us\n",
               n, nb, p1, po, n * 4e-6 / po, pn, n * 4e-6 / pn, o2 * 1e3, n2 * 1e3);
    }
    return 0;
}
