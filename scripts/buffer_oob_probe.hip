// Probe (round 6): what a raw buffer_load_dwordx4 returns when its 16 bytes straddle the descriptor's num_records
// (per-dword range check, or the whole access zeroed?). One wave; lane l loads at byte offset 4 * l from a buffer of
// 64 floats (value i + 1 at float i) whose descriptor covers `bytes` bytes. Prints, per lane near the limit, the four
// loaded values. Build: hipcc --offload-arch=gfx950 -O2 scripts/buffer_oob_probe.hip -o bin_lab/buffer_oob_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void probe(const float* src, f32x4* out, int bytes) {
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), 0, bytes, 0x00020000);
    const int lane = threadIdx.x;
    out[lane] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, 4 * lane, 0, 0));
}

int main() {
    float h[128];
    for (int i = 0; i < 128; ++i) h[i] = (float)(i + 1);
    float* d = nullptr;
    f32x4* o = nullptr;
    if (hipMalloc(&d, sizeof(h)) != hipSuccess || hipMalloc(&o, 64 * sizeof(f32x4)) != hipSuccess) return 1;
    if (hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice) != hipSuccess) return 1;
    for (int bytes : {40, 42, 44}) {  // 10 floats, 10.5 floats, 11 floats
        probe<<<1, 64>>>(d, o, bytes);
        f32x4 r[64];
        if (hipMemcpy(r, o, sizeof(r), hipMemcpyDeviceToHost) != hipSuccess) return 1;
        printf("num_records %d bytes:\n", bytes);
        for (int l = 5; l <= 11; ++l) printf("  lane %2d (bytes %2d..%2d): %g %g %g %g\n", l, 4 * l, 4 * l + 15, r[l].x, r[l].y, r[l].z, r[l].w);
    }
    (void)hipFree(d);
    (void)hipFree(o);
    return 0;
}
