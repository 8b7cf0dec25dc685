// Histogram lab (standalone, not part of the library): timing of the two-pass histeq on one MI355X.
// The library kernels are compiled into this TU (#include of csrc/kernels/histeq.hip).
// Findings of the first ablation round (4096^2, 256 blocks, per-call us): launch 2.5, LDS zeroing 2.2,
// counting 6, 65536 merge atomics onto ONE 1-KiB histogram 9.6 (one memory channel serialises them),
// __threadfence before the ticket 9.2 (agent-scope release = buffer_wbl2, an L2 write-back), tf 1.8
// -> replicated u64 merge slots 4 KiB apart, returning atomics instead of fences.
// build: hipcc -O3 --offload-arch=gfx950 -Icsrc/include -Icsrc/runtime scripts/histeq_lab.hip -o build/histeq_lab
#include "../csrc/kernels/histeq.hip"

#include <cstdio>
#include <vector>

namespace {
__global__ void empty_kernel(int* p) {
    __shared__ unsigned big[32768];
    if (threadIdx.x == 1000) { big[threadIdx.x] = 1; p[0] = big[(threadIdx.x * 7) & 32767]; }
}
}  // namespace

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <class F>
float time_us(F f, int iters = 200) {
    hipEvent_t a, b;
    hipEventCreate(&a), hipEventCreate(&b);
    for (int i = 0; i < 10; ++i) f();
    hipEventRecord(a);
    for (int i = 0; i < iters; ++i) f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms * 1e3f / iters;
}

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    const long long sides[] = {512, 4096, 8192};
    for (long long side : sides) {
        const long long npix = side * side, n16 = npix / 16;
        std::vector<unsigned char> h(npix);
        unsigned x = 12345;
        for (auto& v : h) { x = x * 1664525u + 1013904223u; v = (x >> 24) % 200; }
        unsigned char *img, *out;
        HistWs* ws;
        int* dummy;
        CK(hipMalloc(&img, npix)); CK(hipMalloc(&out, npix)); CK(hipMalloc(&ws, sizeof(HistWs))); CK(hipMalloc(&dummy, 64));
        CK(hipMemcpy(img, h.data(), npix, hipMemcpyHostToDevice));
        CK(hipMemset(ws, 0, sizeof(HistWs)));
        const int g = 256;
        printf("side %lld\n", side);
        printf("  full call (library)      %8.2f us\n", time_us([&] { pcmx_histeq_u8(img, out, npix, ws, 0); }));
        printf("  empty kernel 128KiB LDS  %8.2f us\n", time_us([&] { empty_kernel<<<g, 256>>>(dummy); }));
        auto run = [&](const char* name, auto f) {
            hipMemset(ws, 0, sizeof(HistWs));
            printf("  pass1 %-18s %8.2f us\n", name, time_us(f));
            const hipError_t e = hipDeviceSynchronize();
            if (e != hipSuccess) printf("  error after %s: %s\n", name, hipGetErrorString(e));
        };
        run("8w 2c 256 blocks", [&] { launch_hist<8, 2>(img, npix, ws, 0, 256); });
        run("8w 1c 256 blocks", [&] { launch_hist<8, 1>(img, npix, ws, 0, 256); });
        run("8w 1c 512 blocks", [&] { launch_hist<8, 1>(img, npix, ws, 0, 512); });
        run("8w 1c 1024 blocks", [&] { launch_hist<8, 1>(img, npix, ws, 0, 1024); });
        run("16w 1c 256 blocks", [&] { launch_hist<16, 1>(img, npix, ws, 0, 256); });
        run("16w 2c 256 blocks", [&] { launch_hist<16, 2>(img, npix, ws, 0, 256); });
        run("16w 1c 512 blocks", [&] { launch_hist<16, 1>(img, npix, ws, 0, 512); });
        run("4w 1c 1024 blocks", [&] { launch_hist<4, 1>(img, npix, ws, 0, 1024); });
        for (long long mb : {64LL, 256LL, 512LL, 1024LL, 2048LL}) {
            const long long spread = (n16 + kThreads - 1) / kThreads;
            if (mb > spread) continue;
            printf("  pass2 map %4lld blocks    %8.2f us\n", mb, time_us([&] { map_lut_kernel<<<(int)mb, kThreads>>>(img, out, npix, ws); }));
        }
        CK(hipDeviceSynchronize());
        hipFree(img), hipFree(out), hipFree(ws), hipFree(dummy);
    }
    return 0;
}
