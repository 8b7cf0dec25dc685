// Single-pass prefix scan (inclusive/exclusive, f32) with decoupled look-back — the north-star
// "prefix-scan 1e9 f32" kernel. Reference ancestor: the histogram CDF (ref 4-histogram-equalization-
// openmp-pthreads/histogram_serial.c:29-34) generalised to 1e9 elements.
//
// MI355X design
//  * Tile = 8 waves x 1024 elements (16 per lane = 4 x pcmx::f32x4, each wave instruction a contiguous 1 KiB),
//    so HBM traffic is one read + one write of the array (8 B/element).
//  * Tiles are taken in launch order from an atomic ticket, so every predecessor tile is already running
//    and the look-back cannot deadlock whatever the dispatcher does.
//  * Inter-workgroup hand-off uses 8-byte {flag, value} granules written with ONE agent-scope relaxed
//    atomic store (write-through) and polled with agent-scope relaxed loads: the data IS the flag, so no
//    fence is needed (cdna_hip_programming.md G16 recipe R2). One wave looks back 64 tiles per poll.
//  * Status words and the ticket are zeroed by a hipMemsetAsync on the same stream before every launch
//    (G16 "Re-initialise every call"); spins are bounded and report through a timeout flag.
#include "pcmx_common.h"
#include "pcmx_hip.h"

namespace {
using pcmx::kWave;
constexpr int kWaves = 8;
constexpr int kThreads = kWaves * kWave;
constexpr int kMinRows = 4;                          // smallest tile variant (sizes the workspace)
constexpr int kMinTile = kWaves * kMinRows * 4 * kWave;  // 8192
constexpr unsigned kFlagAgg = 1u, kFlagIncl = 2u;
constexpr unsigned kSpinLimit = 1u << 26;

struct ScanWs {
    unsigned ticket;
    unsigned timeout;
    unsigned pad[2];
    // followed by unsigned long long status[num_tiles]
};

__device__ __forceinline__ unsigned long long pack(unsigned flag, float v) {
    return ((unsigned long long)flag << 32) | (unsigned long long)__float_as_uint(v);
}

// kRows pcmx::f32x4 rows per lane: tile = 8 waves x kRows x 256 elements. Larger tiles amortise the
// look-back round trips (agent-scope polls cross the XCD L2s) over more bytes.
template <int kRows>
__global__ __launch_bounds__(kThreads) void scan_lookback_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                                long long n, int exclusive, const float* init_dev,
                                                                ScanWs* ws) {
    unsigned long long* status = reinterpret_cast<unsigned long long*>(ws + 1);
    __shared__ float s_wave_tot[kWaves];
    __shared__ float s_prefix;
    __shared__ unsigned s_tile;
    constexpr int kWaveItems = kRows * 4 * kWave;
    constexpr int kTile = kWaves * kWaveItems;
    const int lane = pcmx::lane_id();
    const int wave = threadIdx.x / kWave;

    if (threadIdx.x == 0) s_tile = atomicAdd(&ws->ticket, 1u);
    __syncthreads();
    const long long tile = s_tile;
    const long long base = tile * kTile + (long long)wave * kWaveItems;

    // ---- load 4 rows of pcmx::f32x4 (row r covers elements base + r*256 + lane*4 .. +3)
    pcmx::f32x4 v[kRows];
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
        const long long e = base + r * 256 + lane * 4;
        if (e + 3 < n) {
            v[r] = __builtin_nontemporal_load(reinterpret_cast<const pcmx::f32x4*>(in + e));
        } else {
            v[r].x = e < n ? in[e] : 0.f;
            v[r].y = e + 1 < n ? in[e + 1] : 0.f;
            v[r].z = e + 2 < n ? in[e + 2] : 0.f;
            v[r].w = e + 3 < n ? in[e + 3] : 0.f;
        }
    }
    // ---- in-wave scan: per row, lane-local prefix, then a wave scan of the lane totals
    float carry = 0.f;
    float lane_excl[kRows];
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
        v[r].y += v[r].x;
        v[r].z += v[r].y;
        v[r].w += v[r].z;
        const float incl = pcmx::wave_inclusive_scan(v[r].w);
        float excl = __shfl_up(incl, 1, kWave);
        if (lane == 0) excl = 0.f;
        lane_excl[r] = carry + excl;
        carry += __shfl(incl, kWave - 1, kWave);
    }
    if (lane == 0) s_wave_tot[wave] = carry;
    __syncthreads();

    // ---- wave 0: tile aggregate, publish, decoupled look-back
    if (wave == 0) {
        float agg = 0.f;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) agg += s_wave_tot[w];
        float prefix = 0.f;
        if (tile == 0) {
            if (lane == 0) __hip_atomic_store(&status[0], pack(kFlagIncl, agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (lane == 0) __hip_atomic_store(&status[tile], pack(kFlagAgg, agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            long long look = tile - 1;  // newest predecessor still to account for
            unsigned spins = 0;
            while (true) {
                const long long idx = look - lane;
                unsigned long long sv = idx >= 0 ? __hip_atomic_load(&status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                                 : pack(kFlagIncl, 0.f);
                const unsigned flag = (unsigned)(sv >> 32);
                const float val = __uint_as_float((unsigned)sv);
                const unsigned long long m_incl = __ballot(flag == kFlagIncl);
                const unsigned long long m_zero = __ballot(flag == 0u);
                if (m_incl != 0ull) {
                    const int first = __builtin_ctzll(m_incl);
                    const unsigned long long need = (first == 63) ? ~0ull : ((1ull << (first + 1)) - 1ull);
                    if ((m_zero & need) == 0ull) {
                        float contrib = lane <= first ? val : 0.f;
                        prefix += pcmx::wave_reduce<float, 0>(contrib);
                        break;
                    }
                } else if (m_zero == 0ull) {
                    prefix += pcmx::wave_reduce<float, 0>(val);
                    look -= kWave;
                    continue;
                }
                if (++spins > kSpinLimit) {  // bounded spin: report and fall through
                    if (lane == 0) atomicExch(&ws->timeout, 1u);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (lane == 0)
                __hip_atomic_store(&status[tile], pack(kFlagIncl, prefix + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) {
            float init = init_dev ? *init_dev : 0.f;
            float wo = 0.f;
            for (int w = 0; w < kWaves; ++w) {
                float t = s_wave_tot[w];
                s_wave_tot[w] = wo;  // becomes the exclusive wave offset
                wo += t;
            }
            s_prefix = init + prefix;
        }
    }
    __syncthreads();
    const float off = s_prefix + s_wave_tot[wave];

    // ---- write (inclusive or exclusive) results
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
        const float b = off + lane_excl[r];
        pcmx::f32x4 o;
        if (exclusive) {
            const pcmx::f32x4 x = v[r];
            o.x = b;
            o.y = b + x.x;
            o.z = b + x.y;
            o.w = b + x.z;
        } else {
            o.x = b + v[r].x;
            o.y = b + v[r].y;
            o.z = b + v[r].z;
            o.w = b + v[r].w;
        }
        const long long e = base + r * 256 + lane * 4;
        if (e + 3 < n) {
            __builtin_nontemporal_store(o, reinterpret_cast<pcmx::f32x4*>(out + e));
        } else {
            if (e < n) out[e] = o.x;
            if (e + 1 < n) out[e + 1] = o.y;
            if (e + 2 < n) out[e + 2] = o.z;
        }
    }
}

inline long long num_tiles(long long n, int tile) { return (n + tile - 1) / tile; }
int g_scan_rows = 8;
template <int R>
void launch_scan(const float* x, float* out, long long n, int exclusive, const float* init_dev, ScanWs* ws,
                 hipStream_t s) {
    constexpr int tile = kWaves * R * 4 * kWave;
    scan_lookback_kernel<R><<<(unsigned)num_tiles(n, tile), kThreads, 0, s>>>(x, out, n, exclusive, init_dev, ws);
}
}  // namespace

extern "C" int pcmx_scan_set_rows(int rows) {
    if (rows != 4 && rows != 8 && rows != 16) return -1;
    g_scan_rows = rows;
    return 0;
}

extern "C" long long pcmx_scan_workspace_bytes(long long n) {
    return (long long)sizeof(ScanWs) + num_tiles(n, kMinTile) * 8;
}

extern "C" int pcmx_scan_f32(const float* x, float* out, long long n, int exclusive, const float* init_dev, void* workspace,
                             hipStream_t s) {
    if (n <= 0) return 0;
    if ((((uintptr_t)x) & 15u) || (((uintptr_t)out) & 15u) || !workspace) return -1;
    const long long tiles = num_tiles(n, kMinTile);
    if (tiles > 0x7fffffffLL) return -1;
    // only the ticket/timeout header and the status words of the tiles actually launched need zeroing
    const int rows = g_scan_rows;
    const long long used = num_tiles(n, kWaves * rows * 4 * kWave);
    PCMX_HIP_RET(hipMemsetAsync(workspace, 0, sizeof(ScanWs) + (size_t)used * 8, s));
    ScanWs* ws = reinterpret_cast<ScanWs*>(workspace);
    if (rows == 16) launch_scan<16>(x, out, n, exclusive, init_dev, ws, s);
    else if (rows == 4) launch_scan<4>(x, out, n, exclusive, init_dev, ws, s);
    else launch_scan<8>(x, out, n, exclusive, init_dev, ws, s);
    return (int)hipGetLastError();
}
