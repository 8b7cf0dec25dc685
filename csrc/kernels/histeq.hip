// Histogram equalisation of an 8-bit image on MI355X.
// Reference: 4-histogram-equalization-openmp-pthreads/histogram_serial.c:11-42 (and the OpenMP/pthreads
// variants, histogram_omp.c / histogram_pthreads.c). Output is bit-identical to the serial reference:
// tf[v] = sum_{j<=v} fl(fl(255*h[j]) / npix) accumulated in f32 in increasing j (one lane does the 256
// ordered adds — 256 dependent FMAs are nothing next to the pixel passes), out[i] = (uint8)tf[img[i]].
//
// MI355X design
//  * Small images (the reference's 512x512 = 256 KiB): ONE launch, one 1024-thread workgroup: per-wave
//    privatised LDS histograms (16 x 256 counters, no cross-wave atomic contention), 16-B (uint4) pixel
//    loads, tf in LDS, map pass with 16-B stores. The whole equalisation is a single kernel boundary.
//  * Large images: pass 1 privatises per block in LDS and merges with one global atomic per bin per
//    block; pass 2 re-derives tf in LDS per block (256 ordered adds) and maps with 16-B accesses.
#include "pcmx_common.h"
#include "pcmx_hip.h"

namespace {
constexpr int kBins = 256;

__device__ __forceinline__ void count_word(unsigned w, unsigned* h) {
    atomicAdd(&h[w & 0xff], 1u);
    atomicAdd(&h[(w >> 8) & 0xff], 1u);
    atomicAdd(&h[(w >> 16) & 0xff], 1u);
    atomicAdd(&h[w >> 24], 1u);
}

__device__ __forceinline__ unsigned map_word(unsigned w, const float* tf) {
    return (unsigned)(unsigned char)tf[w & 0xff] | ((unsigned)(unsigned char)tf[(w >> 8) & 0xff] << 8) |
           ((unsigned)(unsigned char)tf[(w >> 16) & 0xff] << 16) | ((unsigned)(unsigned char)tf[w >> 24] << 24);
}

// ordered f32 prefix (exactly the reference's rounding sequence)
__device__ __forceinline__ void build_tf(const unsigned* hist, long long npix, float* tf) {
    float run = 0.f;
    const float n = (float)npix;
    for (int v = 0; v < kBins; ++v) {
        run += (255.0f * (float)hist[v]) / n;
        tf[v] = run;
    }
}

constexpr int kFusedThreads = 1024;
__global__ __launch_bounds__(kFusedThreads) void histeq_fused_kernel(const unsigned char* __restrict__ img,
                                                                    unsigned char* __restrict__ out, long long npix,
                                                                    unsigned* __restrict__ hist_out) {
    constexpr int kWaves = kFusedThreads / 64;
    __shared__ unsigned sh[kWaves][kBins];
    __shared__ unsigned hist[kBins];
    __shared__ float tf[kBins];
    for (int i = threadIdx.x; i < kWaves * kBins; i += kFusedThreads) (&sh[0][0])[i] = 0u;
    __syncthreads();
    unsigned* mine = sh[threadIdx.x / 64];
    const long long n16 = npix >> 4;
    const uint4* v16 = reinterpret_cast<const uint4*>(img);
    for (long long i = threadIdx.x; i < n16; i += kFusedThreads) {
        const uint4 w = v16[i];
        count_word(w.x, mine), count_word(w.y, mine), count_word(w.z, mine), count_word(w.w, mine);
    }
    for (long long i = (n16 << 4) + threadIdx.x; i < npix; i += kFusedThreads) atomicAdd(&mine[img[i]], 1u);
    __syncthreads();
    for (int b = threadIdx.x; b < kBins; b += kFusedThreads) {
        unsigned s = 0;
        for (int w = 0; w < kWaves; ++w) s += sh[w][b];
        hist[b] = s;
        if (hist_out) hist_out[b] = s;
    }
    __syncthreads();
    if (threadIdx.x == 0) build_tf(hist, npix, tf);
    __syncthreads();
    uint4* o16 = reinterpret_cast<uint4*>(out);
    for (long long i = threadIdx.x; i < n16; i += kFusedThreads) {
        const uint4 w = v16[i];
        o16[i] = make_uint4(map_word(w.x, tf), map_word(w.y, tf), map_word(w.z, tf), map_word(w.w, tf));
    }
    for (long long i = (n16 << 4) + threadIdx.x; i < npix; i += kFusedThreads) out[i] = (unsigned char)tf[img[i]];
}

constexpr int kThreads = 256;
__global__ __launch_bounds__(kThreads) void hist_pass_kernel(const unsigned char* __restrict__ img, long long npix,
                                                            unsigned* __restrict__ hist) {
    __shared__ unsigned sh[kThreads / 64][kBins];
    for (int i = threadIdx.x; i < (kThreads / 64) * kBins; i += kThreads) (&sh[0][0])[i] = 0u;
    __syncthreads();
    unsigned* mine = sh[threadIdx.x / 64];
    const long long n16 = npix >> 4;
    const uint4* v16 = reinterpret_cast<const uint4*>(img);
    for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < n16; i += (long long)gridDim.x * kThreads) {
        const uint4 w = v16[i];
        count_word(w.x, mine), count_word(w.y, mine), count_word(w.z, mine), count_word(w.w, mine);
    }
    if (blockIdx.x == 0)
        for (long long i = (n16 << 4) + threadIdx.x; i < npix; i += kThreads) atomicAdd(&mine[img[i]], 1u);
    __syncthreads();
    for (int b = threadIdx.x; b < kBins; b += kThreads) {
        unsigned s = 0;
        for (int w = 0; w < kThreads / 64; ++w) s += sh[w][b];
        if (s) atomicAdd(&hist[b], s);
    }
}

__global__ __launch_bounds__(kThreads) void map_pass_kernel(const unsigned char* __restrict__ img,
                                                           unsigned char* __restrict__ out, long long npix,
                                                           const unsigned* __restrict__ hist) {
    __shared__ unsigned h[kBins];
    __shared__ float tf[kBins];
    for (int b = threadIdx.x; b < kBins; b += kThreads) h[b] = hist[b];
    __syncthreads();
    if (threadIdx.x == 0) build_tf(h, npix, tf);
    __syncthreads();
    const long long n16 = npix >> 4;
    const uint4* v16 = reinterpret_cast<const uint4*>(img);
    uint4* o16 = reinterpret_cast<uint4*>(out);
    for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < n16; i += (long long)gridDim.x * kThreads) {
        const uint4 w = v16[i];
        o16[i] = make_uint4(map_word(w.x, tf), map_word(w.y, tf), map_word(w.z, tf), map_word(w.w, tf));
    }
    if (blockIdx.x == 0)
        for (long long i = (n16 << 4) + threadIdx.x; i < npix; i += kThreads) out[i] = (unsigned char)tf[img[i]];
}
}  // namespace

extern "C" int pcmx_histeq_u8(const unsigned char* img, unsigned char* out, long long npix, unsigned* hist_ws,
                              int force_multiblock, hipStream_t s) {
    if (npix <= 0) return 0;
    if (((uintptr_t)img | (uintptr_t)out) & 15u) return -1;
    if (npix <= (4LL << 20) && !force_multiblock) {
        histeq_fused_kernel<<<1, kFusedThreads, 0, s>>>(img, out, npix, hist_ws);
        return (int)hipGetLastError();
    }
    if (!hist_ws) return -1;
    PCMX_HIP_RET(hipMemsetAsync(hist_ws, 0, kBins * sizeof(unsigned), s));
    long long blocks = ((npix >> 4) + kThreads - 1) / kThreads;
    if (blocks > 2048) blocks = 2048;
    if (blocks < 1) blocks = 1;
    hist_pass_kernel<<<(int)blocks, kThreads, 0, s>>>(img, npix, hist_ws);
    map_pass_kernel<<<(int)blocks, kThreads, 0, s>>>(img, out, npix, hist_ws);
    return (int)hipGetLastError();
}
