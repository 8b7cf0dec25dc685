// Histogram equalisation of an 8-bit image on MI355X.
// Reference: 4-histogram-equalization-openmp-pthreads/histogram_serial.c:11-42 (and the OpenMP/pthreads
// variants, histogram_omp.c / histogram_pthreads.c). Output is bit-identical to the serial reference:
// tf[v] = sum_{j<=v} fl(fl(255*h[j]) / npix) accumulated in f32 in increasing j, out[i] = (uint8)tf[img[i]].
//
// MI355X design — two launches for every image size, no memset, tf derived once:
//  pass 1 (hist_lane_kernel, one 8-wave block per CU): PER-LANE counters in LDS — u16 pairs, bin b of lane l
//    at dword (b/2)*64 + l, half b&1 — so a wave's ds_add_u32 always hits 64 different banks: no bank
//    conflicts and no same-address serialisation however skewed the image is (the reference's dark.bmp
//    piles most pixels into a few bins). Image loads are software-pipelined (the next 8 x 16 B per lane are
//    in flight while the current 8 are counted). Measured (scripts/histeq_lab.hip): the pass is bound by the
//    LDS atomic rate (~14 clk per wave-wide ds_add_u32 per CU) once 8 waves keep it busy; private copies per
//    wave bought nothing, so the 8 waves share ONE 32-KiB copy (less to zero and fold). The block folds the
//    64 lane columns (rotated: conflict-free) and merges into one of 16 u64 histogram replicas 4 KiB apart
//    (65536 merge atomics onto one 1-KiB histogram serialised on one memory channel: 9.6 us). The LAST block
//    (ticket, no fences — see hist_lane_kernel) computes the 256 terms in parallel and the 256 ordered f32
//    adds as a lane-to-lane chain (readlane), writes the u8 LUT and re-zeroes replicas and ticket for the
//    next call (self-cleaning workspace).
//  pass 2 (map_lut_kernel, persistent 512 blocks): the LUT is replicated per LDS bank (entry v of lane l at
//    dword v*64 + l: conflict-free gathers, 2 VALU of addressing per pixel); 16-B loads and stores.
//  Per call on MI355X: 512^2 12.6 us (was 41 us in one fused workgroup), 4096^2 ~20 us (was 74), 8192^2 ~46 us.
#include "pcmx_common.h"
#include "pcmx_hip.h"

namespace {
constexpr int kBins = 256;
constexpr int kThreads = 256;          // map kernel
constexpr int kPairRows = kBins / 2;   // u16-pair counter rows per lane
constexpr int kDepth = 8;              // uint4 per lane per pipeline stage
constexpr int kMaxSlotWords = 4088;    // uint4 per counter slot per launch: 16 * 4088 < 65536 (u16 counters)
constexpr int kHistBlocks = 256;       // one block per CU
constexpr int kHistWaves = 8;         // waves per pass-1 block
constexpr int kHistCopies = 1;        // per-lane counter copies per block (all 8 waves share one: 32 KiB)
constexpr int kMapBlocks = 512;       // persistent map grid
constexpr int kReplicas = 16;          // global histogram replicas (merge atomics spread over channels)
constexpr int kRepStride = 512;        // u64 per replica slot: 4 KiB apart

struct HistWs {  // persistent per (device, stream), zero before the first call, left zero by every call
    unsigned long long rep[kReplicas][kRepStride];  // rep[r][p] = count(bin 2p) | count(bin 2p+1) << 32
    unsigned ticket;
    unsigned pad[63];
    unsigned lut[kBins / 4];  // u8 LUT, 4 entries per word
};

__device__ __forceinline__ void count_word_lane(unsigned w, unsigned* cnt) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const unsigned row = __builtin_amdgcn_ubfe(w, 8 * k + 1, 7);
        const unsigned odd = __builtin_amdgcn_ubfe(w, 8 * k, 1);
        atomicAdd(&cnt[row * 64], 1u + odd * 65535u);  // 1 or 1 << 16; no return value: ds_add_u32
    }
}

__device__ __forceinline__ void count_vec(const uint4& a, unsigned* cnt) {
    count_word_lane(a.x, cnt), count_word_lane(a.y, cnt), count_word_lane(a.z, cnt), count_word_lane(a.w, cnt);
}

// uint4 words [w16_0, w16_1) of the image; the final chunk also counts the npix % 16 tail and finalises.
// Cross-block protocol WITHOUT fences (an agent-scope release is a full L2 write-back on gfx950, measured at
// ~9 us per call): the merge atomics return values, so the s_waitcnt before the block barrier means they are
// performed (device atomics are coherent across XCDs) before thread 0 takes a ticket; the last block reads
// AND re-zeroes the replicas with atomic exchanges, which see every block's performed adds.
// Why this holds although every atomic is memory_order_relaxed (the HIP model alone does not promise it):
//  * Hardware: every atomic here is an agent-scope RMW (atomicAdd / atomicExch, `global_atomic_* sc0`), which
//    gfx950 performs beyond the issuing XCD's L2 (an atomic drops the line from L2; 8-B agent atomics on both
//    sides are one of the valid cross-XCD hand-off forms, MI355X_MICROARCH.md §Workgroup dispatch ... visibility),
//    so there is one coherent order per word. A
//    RETURNING atomic's value comes back only after the RMW was performed there; `sink` is consumed before the
//    barrier, so the compiler must emit s_waitcnt vmcnt(0) for it, i.e. every wave of the block has its merges
//    performed when it reaches the barrier. Thread 0's ticket RMW is issued after the barrier, so it is
//    performed after all of its block's merges. The block that draws the last ticket therefore runs after every
//    block's merges were performed, and its atomicExch reads hit the same coherence point.
//  * Compiler: __syncthreads() is fence(release, workgroup) + llvm.amdgcn.s.barrier + fence(acquire, workgroup);
//    LLVM does not move memory operations (atomics included) across a fence or across the barrier intrinsic (an
//    IntrHasSideEffects, convergent call), and `last` is published through LDS behind the second barrier.
//  * The LUT is written with plain stores and read by the NEXT kernel on the stream: kernel boundaries make it
//    visible (end-of-kernel release, start-of-kernel acquire).
// Test evidence: tests/test_gpu_kernels.py histeq cases (many blocks, repeated calls on one workspace, streams).
template <int WAVES, int COPIES>
__global__ __launch_bounds__(WAVES * 64) void hist_lane_kernel(const unsigned char* __restrict__ img, long long npix,
                                                              long long w16_0, long long w16_1,
                                                              HistWs* __restrict__ ws, int final_chunk) {
    constexpr int T = WAVES * 64;
    static_assert(WAVES % COPIES == 0, "waves share counter copies evenly");
    __shared__ unsigned cnt[COPIES][kPairRows][64];  // 32 KiB per copy (waves w, w + COPIES, ... share one)
    __shared__ unsigned long long part[kPairRows];
    __shared__ float term[kBins];
    __shared__ int last;
    {
        uint4* c4 = reinterpret_cast<uint4*>(&cnt[0][0][0]);
        for (int i = threadIdx.x; i < COPIES * kPairRows * 16; i += T) c4[i] = make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    const int lane = pcmx::lane_id(), wave = threadIdx.x / 64;
    unsigned* mine = &cnt[wave % COPIES][0][lane];
    const uint4* v16 = reinterpret_cast<const uint4*>(img);
    const long long stride = (long long)gridDim.x * T;
    const long long i0 = w16_0 + (long long)blockIdx.x * T + threadIdx.x;
    if (i0 < w16_1) {
        // words i0 + k*stride, k = 0..n-1, in stages of kDepth: stage s+1's loads are issued before stage s
        // is counted. Out-of-range slots load the last word (always valid) and are not counted.
        const int n = (int)((w16_1 - 1 - i0) / stride) + 1;
        auto load = [&](uint4(&r)[kDepth], int k0) {
#pragma unroll
            for (int d = 0; d < kDepth; ++d) {
                const long long idx = i0 + (long long)(k0 + d) * stride;
                r[d] = v16[idx < w16_1 ? idx : w16_1 - 1];
            }
        };
        auto count = [&](const uint4(&r)[kDepth], int k0) {
            if (k0 + kDepth <= n) {
#pragma unroll
                for (int d = 0; d < kDepth; ++d) count_vec(r[d], mine);
            } else {
#pragma unroll
                for (int d = 0; d < kDepth; ++d)
                    if (k0 + d < n) count_vec(r[d], mine);
            }
        };
        uint4 ra[kDepth], rb[kDepth];
        load(ra, 0);
        int k = 0;
        for (;;) {
            if (k + kDepth < n) load(rb, k + kDepth);
            count(ra, k);
            k += kDepth;
            if (k >= n) break;
            if (k + kDepth < n) load(ra, k + kDepth);
            count(rb, k);
            k += kDepth;
            if (k >= n) break;
        }
    }
    if (final_chunk && blockIdx.x == 0)
        for (long long j = ((npix >> 4) << 4) + threadIdx.x; j < npix; j += T) {
            const unsigned v = img[j];
            atomicAdd(&mine[(v >> 1) * 64], 1u + (v & 1u) * 65535u);
        }
    __syncthreads();
    // fold: the T threads split the 128 pair rows x 64 lane columns (rotated columns: 64 lanes -> 64 banks)
    constexpr int kSplit = T / kPairRows;  // column groups per row (1, 2, 4 or 8)
    const int row = threadIdx.x % kPairRows, grp = threadIdx.x / kPairRows;
    unsigned long long sum;
    {
        unsigned lo = 0, hi = 0;
#pragma unroll 4
        for (int c = 0; c < 64 / kSplit; ++c) {
            const int col = (grp * (64 / kSplit) + c + lane) & 63;
#pragma unroll
            for (int w = 0; w < COPIES; ++w) {
                const unsigned v = cnt[w][row][col];
                lo += v & 0xffffu, hi += v >> 16;
            }
        }
        sum = ((unsigned long long)hi << 32) | lo;
    }
    if constexpr (kSplit > 1) {
        for (int g = 1; g < kSplit; ++g) {
            __syncthreads();
            if (grp == g) part[row] = sum;
            __syncthreads();
            if (grp == 0) sum += part[row];
        }
    }
    unsigned long long sink = 0;
    if (grp == 0 && sum) sink = atomicAdd(&ws->rep[blockIdx.x % kReplicas][row], sum);
    if (!final_chunk) return;
    if (sink == ~0ull) ws->pad[0] = 1u;  // never true: consumes the returned value, i.e. waits until performed
    __syncthreads();
    if (threadIdx.x == 0) last = atomicAdd(&ws->ticket, 1u) == gridDim.x - 1;
    __syncthreads();
    if (!last) return;
    if (threadIdx.x < kPairRows) {
        unsigned long long v[kReplicas];
#pragma unroll
        for (int r = 0; r < kReplicas; ++r) v[r] = atomicExch(&ws->rep[r][threadIdx.x], 0ull);
        unsigned long long tot = 0;
#pragma unroll
        for (int r = 0; r < kReplicas; ++r) tot += v[r];
        // the reference's per-bin term, all bins at once
        term[2 * threadIdx.x] = (255.0f * (float)(unsigned)tot) / (float)npix;
        term[2 * threadIdx.x + 1] = (255.0f * (float)(unsigned)(tot >> 32)) / (float)npix;
    }
    __syncthreads();
    if (threadIdx.x < 64) {
        // ordered prefix: lane l owns terms 4l..4l+3; step j extends the running sum through lane j's four
        // terms (the reference's exact add sequence) and broadcasts it with readlane
        const pcmx::f32x4 t = reinterpret_cast<const pcmx::f32x4*>(term)[lane];
        float run = 0.f, r0 = 0.f, r1 = 0.f, r2 = 0.f, r3 = 0.f;
        for (int j = 0; j < 64; ++j) {
            const float a0 = run + t[0], a1 = a0 + t[1], a2 = a1 + t[2], a3 = a2 + t[3];
            if (lane == j) r0 = a0, r1 = a1, r2 = a2, r3 = a3;
            run = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(a3), j));
        }
        ws->lut[lane] = (unsigned)(unsigned char)r0 | ((unsigned)(unsigned char)r1 << 8) |
                        ((unsigned)(unsigned char)r2 << 16) | ((unsigned)(unsigned char)r3 << 24);
        if (lane == 0) atomicExch(&ws->ticket, 0u);
    }
}

__device__ __forceinline__ unsigned map_word_rep(unsigned w, const unsigned* tab) {
    const unsigned t0 = tab[__builtin_amdgcn_ubfe(w, 0, 8) * 64], t1 = tab[__builtin_amdgcn_ubfe(w, 8, 8) * 64];
    const unsigned t2 = tab[__builtin_amdgcn_ubfe(w, 16, 8) * 64], t3 = tab[(w >> 24) * 64];
    return t0 | (t1 << 8) | (t2 << 16) | (t3 << 24);
}

__device__ __forceinline__ uint4 map_vec(const uint4& a, const unsigned* tab) {
    return make_uint4(map_word_rep(a.x, tab), map_word_rep(a.y, tab), map_word_rep(a.z, tab), map_word_rep(a.w, tab));
}

__global__ __launch_bounds__(kThreads) void map_lut_kernel(const unsigned char* __restrict__ img,
                                                          unsigned char* __restrict__ out, long long npix,
                                                          const HistWs* __restrict__ ws) {
    __shared__ uint4 tab4[kBins * 16];  // 64 KiB: entry v replicated in all 64 banks (dword v*64 + lane)
    for (int i = threadIdx.x; i < kBins * 16; i += kThreads) {
        const int v = i >> 4;
        const unsigned e = (ws->lut[v >> 2] >> (8 * (v & 3))) & 0xffu;
        tab4[i] = make_uint4(e, e, e, e);
    }
    __syncthreads();
    const unsigned* tab = reinterpret_cast<const unsigned*>(tab4) + pcmx::lane_id();
    const long long n16 = npix >> 4;
    const uint4* v16 = reinterpret_cast<const uint4*>(img);
    uint4* o16 = reinterpret_cast<uint4*>(out);
    const long long stride = (long long)gridDim.x * kThreads;
    long long i = (long long)blockIdx.x * kThreads + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        const uint4 a = v16[i], b = v16[i + stride], c = v16[i + 2 * stride], d = v16[i + 3 * stride];
        o16[i] = map_vec(a, tab), o16[i + stride] = map_vec(b, tab);
        o16[i + 2 * stride] = map_vec(c, tab), o16[i + 3 * stride] = map_vec(d, tab);
    }
    for (; i < n16; i += stride) o16[i] = map_vec(v16[i], tab);
    if (blockIdx.x == 0)
        for (long long j = (n16 << 4) + threadIdx.x; j < npix; j += kThreads) out[j] = (unsigned char)tab[img[j] * 64];
}
}  // namespace

// pass 1 over the whole image (chunked so a u16 counter slot never sees more than kMaxSlotWords words)
template <int WAVES, int COPIES>
void launch_hist(const unsigned char* img, long long npix, HistWs* w, hipStream_t s, int max_blocks = kHistBlocks) {
    constexpr int T = WAVES * 64;
    const long long n16 = npix >> 4;
    long long blocks = (n16 + T - 1) / T;
    blocks = blocks < 1 ? 1 : (blocks > max_blocks ? max_blocks : blocks);
    const long long chunk = (long long)(kMaxSlotWords / (WAVES / COPIES)) * blocks * T;
    long long w0 = 0;
    do {
        const long long w1 = n16 - w0 > chunk ? w0 + chunk : n16;
        hist_lane_kernel<WAVES, COPIES><<<(int)blocks, T, 0, s>>>(img, npix, w0, w1, w, w1 == n16 ? 1 : 0);
        w0 = w1;
    } while (w0 < n16);
}

// map grid: persistent, 2 blocks per CU (64 KiB LUT each, built once per block); small images spread to
// one word per lane so they still reach every CU
static long long map_blocks(long long n16) {
    const long long spread = (n16 + kThreads - 1) / kThreads;
    return spread < 1 ? 1 : (spread > kMapBlocks ? kMapBlocks : spread);
}

extern "C" long long pcmx_histeq_workspace_bytes(void) { return (long long)sizeof(HistWs); }

extern "C" int pcmx_histeq_u8(const unsigned char* img, unsigned char* out, long long npix, void* ws, hipStream_t s) {
    if (npix <= 0) return 0;
    if (((uintptr_t)img | (uintptr_t)out | (uintptr_t)ws) & 15u || !ws) return -1;
    HistWs* w = static_cast<HistWs*>(ws);
    const long long n16 = npix >> 4;
    launch_hist<kHistWaves, kHistCopies>(img, npix, w, s);
    long long mblocks = map_blocks(n16);
    map_lut_kernel<<<(int)mblocks, kThreads, 0, s>>>(img, out, npix, w);
    return (int)hipGetLastError();
}
