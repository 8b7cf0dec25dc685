// Stencil prefetch-depth lab: the fused v2 kernel with 4 columns per lane (8-B rows, 2 VGPRs per prefetched row)
// on short slabs (one interior rank's rows at N = 8 / 4 of the 16384^2 grid), sweeping the prefetch ring depth kAhead
// against rows per wave. The production rule gives 18-row waves a 3-row ring (sized for the 16-B rows of 8-column
// lanes); a row of 4-column lanes is a quarter of the registers of the full T-level ring, so a deeper ring is cheap.
// Every variant is checked bit for bit against the production launch (pcmx_stencil5xT_bf16).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc/include -Icsrc/runtime scripts/stencil_ahead_lab.hip \
//          -o /tmp/stencil_ahead_lab ; run: /tmp/stencil_ahead_lab [rows]
#include "../csrc/kernels/stencil.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);                       \
            return 1;                                                                              \
        }                                                                                          \
    } while (0)

static int g_rows = 2048;
constexpr int kCols = 16384;

template <int T, int RPW, int AH, int CPL = 4>
void launch(const unsigned short* u, unsigned short* o, int halo, float k) {
    const int rows = g_rows, per = kWaves * RPW;
    const RowSpans sp{0, rows, 0, 0, (rows + per - 1) / per};
    const dim3 grid(strips_for(kCols, CPL, T), sp.nby_a);
    // an interior rank (both neighbours): global row0 = rows of a 16384-row grid
    stencil5xT2_kernel<T, AH, RPW, 1, CPL><<<grid, kWaves * 64>>>(u, o, rows, kCols, kCols, halo, sp, rows, 16384, k);
}

template <int T>
int run(const unsigned short* u, unsigned short* o, unsigned short* ref, size_t elems) {
    const int halo = T;
    const float k = 0.2f;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<unsigned short> a(elems), b(elems);
    CK(hipMemset(ref, 0, elems * 2));
    if (pcmx_stencil5xT_bf16(u, ref, g_rows, kCols, kCols, halo, T, 0, g_rows, g_rows, 16384, k, nullptr)) return 1;
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(a.data(), ref, elems * 2, hipMemcpyDeviceToHost));
    auto one = [&](const char* name, auto fn) -> int {
        CK(hipMemset(o, 0, elems * 2));
        fn();
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(b.data(), o, elems * 2, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t i = (size_t)halo * kCols; i < (size_t)(halo + g_rows) * kCols; ++i) bad += a[i] != b[i];
        for (int i = 0; i < 3; ++i) fn();
        CK(hipEventRecord(e0));
        for (int i = 0; i < 30; ++i) fn();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= 30;
        printf("T=%d rows=%d %-12s %.4f ms %6.0f GLUP/s%s\n", T, g_rows, name, ms,
               (double)g_rows * kCols * T / (ms * 1e-3) / 1e9, bad ? "  MISMATCH" : "");
        fflush(stdout);
        return 0;
    };
    one("production", [&] { pcmx_stencil5xT_bf16(u, o, g_rows, kCols, kCols, halo, T, 0, g_rows, g_rows, 16384, k, nullptr); });
#define V(R, A) one("rpw" #R "_ah" #A, [&] { launch<T, R, A>(u, o, halo, k); });
    V(18, 3) V(18, 6) V(18, 9) V(18, 12) V(18, 15)
    V(24, 6) V(24, 9) V(24, 12) V(24, 15)
    V(32, 6) V(32, 9) V(32, 12) V(32, 15)
    V(48, 9) V(48, 12) V(48, 15)
#undef V
    return 0;
}

int main(int argc, char** argv) {
    if (argc > 1) g_rows = atoi(argv[1]);
    const int hmax = 8;
    const size_t elems = (size_t)(g_rows + 2 * hmax) * kCols;
    std::vector<unsigned short> h(elems);
    unsigned s = 12345;
    for (auto& v : h) {
        s = s * 1664525u + 1013904223u;
        v = (unsigned short)(0x3f00 + ((s >> 16) & 0xff));  // bf16 values in [0.5, 1)
    }
    unsigned short *u, *o, *ref;
    CK(hipMalloc(&u, elems * 2));
    CK(hipMalloc(&o, elems * 2));
    CK(hipMalloc(&ref, elems * 2));
    CK(hipMemcpy(u, h.data(), elems * 2, hipMemcpyHostToDevice));
    if (run<6>(u, o, ref, elems) || run<8>(u, o, ref, elems)) return 1;
    return 0;
}
