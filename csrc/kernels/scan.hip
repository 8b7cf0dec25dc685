// Single-pass prefix scan (inclusive/exclusive, f32) with decoupled look-back — the north-star
// "prefix-scan 1e9 f32" kernel. Reference ancestor: the histogram CDF (ref 4-histogram-equalization-
// openmp-pthreads/histogram_serial.c:29-34) generalised to 1e9 elements.
//
// MI355X design (measured in scripts/scan_lab.hip and scripts/scan_tune.py; 1e9 f32 on one MI355X):
//  * HBM traffic is one read + one write of the array (8 B/element); the roofline is a tiled copy
//    (~1.28 ms = 6.2 TB/s for 128-KiB tiles; 64-KiB tiles stream markedly worse on this part).
//  * Tile = 128 KiB: 8 waves x 16 f32x4 rows per lane (or 16 waves x 8 rows), in-register wave scans.
//  * PERSISTENT + SOFTWARE-PIPELINED: one 512-thread block per CU walks tiles in ticket order and keeps
//    the NEXT tile's loads in flight (second register buffer) while a look-back polls predecessors.
//  * PRODUCTION = the PARKED-TILE schedule (scan_parked_kernel, kEarly): tile t is scanned and its aggregate
//    published, its tile-local results are parked in LDS, and it is looked back and written out during the
//    block's NEXT tile, with the first round of polls sent before that tile's scan. Every predecessor then
//    published an iteration ago and the look-back round trip overlaps the scan: 1.47 ms (persistent schedule,
//    look-back right after the scan, scan_persistent_kernel) -> 1.41 ms (parked) -> 1.27 ms = 6.29 TB/s
//    (parked + early polls); the look-back-free structure bound is 1.23 ms.
//  * Tiles come from an atomic ticket, so a tile is only ever owned by a RUNNING block and every predecessor
//    of the oldest unfinished tile has published: the look-back cannot deadlock whatever the dispatcher does.
//  * Hand-off = 8-byte {flag, value} granules written with ONE agent-scope relaxed atomic store and polled
//    with agent-scope relaxed loads (cdna_hip_programming.md G16 recipe R2). Status words and the ticket are
//    zeroed by a hipMemsetAsync on the same stream before every launch. Spins are bounded: a look-back that
//    gives up marks its result invalid in the workspace (ws->timeout) AND in the caller's sticky error word
//    (err_flag, system-scope atomic OR: it may live in host-mapped pinned memory), which pcmx_scan_check /
//    the torch op turn into an error instead of a silently wrong prefix.
#include "pcmx_common.h"
#include "pcmx_hip.h"

namespace {
using pcmx::f32x4;
using pcmx::kWave;
constexpr unsigned kFlagAgg = 1u, kFlagIncl = 2u;
#ifdef PCMX_FAULT_INJECT
// test-only build (libpcmx_faultinj.so): the look-back of tile 1 never sees its predecessor and gives up fast
constexpr unsigned kSpinLimit = 64u;
constexpr long long kFaultTile = 1;
#else
constexpr unsigned kSpinLimit = 1u << 26;
#endif
constexpr int kTileElems = 32768;  // 128 KiB of f32 for every variant

struct ScanWs {
    unsigned ticket;
    unsigned timeout;
    unsigned pad[2];
    // followed by unsigned long long status[num_tiles]
};

__device__ __forceinline__ unsigned long long pack(unsigned flag, float v) {
    return ((unsigned long long)flag << 32) | (unsigned long long)__float_as_uint(v);
}

// W waves x R f32x4 rows per lane; wave w owns the contiguous R*256 elements starting at w*R*256.
template <int R, int W>
struct Tile {
    static constexpr int kWaveItems = R * 4 * kWave, kElems = W * kWaveItems;
    static_assert(kElems == kTileElems, "all variants use 128-KiB tiles");
};

template <int R, int W>
__device__ __forceinline__ void load_tile(const float* __restrict__ in, long long n, long long tile, f32x4 (&v)[R]) {
    const int lane = pcmx::lane_id(), wave = threadIdx.x / kWave;
    const long long base = tile * Tile<R, W>::kElems + (long long)wave * Tile<R, W>::kWaveItems;
    if ((tile + 1) * Tile<R, W>::kElems <= n) {  // block-uniform: full tiles take the branch-free path
#pragma unroll
        for (int r = 0; r < R; ++r)
            v[r] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(in + base + r * 256 + lane * 4));
        return;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const long long e = base + r * 256 + lane * 4;
        if (e + 3 < n) {
            v[r] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(in + e));
        } else {
            v[r].x = e < n ? in[e] : 0.f;
            v[r].y = e + 1 < n ? in[e + 1] : 0.f;
            v[r].z = e + 2 < n ? in[e + 2] : 0.f;
            v[r].w = 0.f;
        }
    }
}

// Branch-free form (round 6 lab): one buffer descriptor per tile whose range ends at n, so the tail of the last tile
// needs no branch. A raw buffer load checks its range per dword: the dwords past the end read as 0 (probed on the
// MI355X, scripts/buffer_oob_probe.hip). Loads carry the nontemporal bit like load_tile's.
template <int R, int W>
__device__ __forceinline__ void load_tile_rs(const float* __restrict__ in, long long n, long long tile, f32x4 (&v)[R]) {
    const int lane = pcmx::lane_id(), wave = threadIdx.x / kWave;
    const long long t0 = tile * Tile<R, W>::kElems;
    const long long rem = n - t0;
    // a tile past the end (the schedule's "next" after the last tile) gets an empty range: every load reads 0 and
    // touches no memory, so the caller issues it without a branch
    const int bytes = (int)((rem <= 0 ? 0 : rem < Tile<R, W>::kElems ? rem : (long long)Tile<R, W>::kElems) * 4);
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(in + t0), 0, bytes, 0x00020000);
    const int off = (wave * Tile<R, W>::kWaveItems + lane * 4) * 4;
#pragma unroll
    for (int r = 0; r < R; ++r)
        v[r] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + r * 1024, 0, 2));
}

// Scans tile `tile` held in v, publishes it, issues the loads of `next` into vn, looks back, stores.
template <int R, int W>
__device__ __forceinline__ void finish_tile(const float* __restrict__ in, float* __restrict__ out, long long n, long long tile,
                                            f32x4 (&v)[R], long long next, f32x4 (&vn)[R], long long ntiles, int exclusive,
                                            float init, ScanWs* ws, unsigned* err_flag, float* s_wave_tot,
                                            float* s_prefix, unsigned* s_next) {
    unsigned long long* status = reinterpret_cast<unsigned long long*>(ws + 1);
    const int lane = pcmx::lane_id(), wave = threadIdx.x / kWave;
    // ---- in-wave scan: per row, lane-local prefix, then a wave scan of the lane totals
    float carry = 0.f;
    float lane_excl[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
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
    float agg = 0.f, wexcl = 0.f;
#pragma unroll
    for (int w = 0; w < W; ++w) {
        const float t = s_wave_tot[w];
        wexcl += w < wave ? t : 0.f;
        agg += t;
    }
    if (threadIdx.x == 0)
        __hip_atomic_store(&status[tile], pack(tile == 0 ? kFlagIncl : kFlagAgg, agg), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    // ---- the next tile's loads go out now and overlap the look-back below
    if (next < ntiles) load_tile<R, W>(in, n, next, vn);
    // ---- the ticket for the tile after `next` is taken HERE, before this tile's stores: vmcnt retires in
    //      order, so an atomic issued after the 16 stores (the previous schedule) made wave 0 - and through the
    //      next barrier the whole block - wait for the stores to complete on every tile. Issued before the
    //      look-back, its return is covered by the poll's wait; published by the barrier below.
    unsigned ticket = 0u;
    if (threadIdx.x == 0) ticket = atomicAdd(&ws->ticket, 1u);

    // ---- wave 0: decoupled look-back over the predecessors' {flag, value} granules
    if (wave == 0) {
        float prefix = 0.f;
        if (tile != 0) {
            long long look = tile - 1;  // newest predecessor still to account for
            unsigned spins = 0;
            while (true) {
                const long long idx = look - lane;
                unsigned long long sv =
                    idx >= 0 ? __hip_atomic_load(&status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                             : pack(kFlagIncl, 0.f);
#ifdef PCMX_FAULT_INJECT
                if (tile == kFaultTile) sv = 0ull;  // fault injection: this tile never sees its predecessors
#endif
                const unsigned flag = (unsigned)(sv >> 32);
                const float val = __uint_as_float((unsigned)sv);
                const unsigned long long m_incl = __ballot(flag == kFlagIncl);
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
                    look -= kWave;
                    continue;
                }
                if (++spins > kSpinLimit) {  // bounded spin: report (workspace + sticky caller word) and fall through
                    if (lane == 0) {
                        atomicExch(&ws->timeout, 1u);
                        if (err_flag) __hip_atomic_fetch_or(err_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (lane == 0)
                __hip_atomic_store(&status[tile], pack(kFlagIncl, prefix + agg), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) *s_prefix = init + prefix;
    }
    if (threadIdx.x == 0) *s_next = ticket;
    __syncthreads();
    const float off = *s_prefix + wexcl;

    // ---- write (inclusive or exclusive) results
    const long long base = tile * Tile<R, W>::kElems + (long long)wave * Tile<R, W>::kWaveItems;
    const bool full = (tile + 1) * Tile<R, W>::kElems <= n;  // block-uniform
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const float b = off + lane_excl[r];
        f32x4 o;
        if (exclusive) {
            o.x = b;
            o.y = b + v[r].x;
            o.z = b + v[r].y;
            o.w = b + v[r].z;
        } else {
            o = v[r] + b;
        }
        const long long e = base + r * 256 + lane * 4;
        if (full || e + 3 < n) {
            __builtin_nontemporal_store(o, reinterpret_cast<f32x4*>(out + e));
        } else {
            if (e < n) out[e] = o.x;
            if (e + 1 < n) out[e + 1] = o.y;
            if (e + 2 < n) out[e + 2] = o.z;
        }
    }
}

template <int R, int W>
__global__ __launch_bounds__(W * kWave) void scan_persistent_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                                    long long n, long long ntiles, int exclusive,
                                                                    const float* init_dev, ScanWs* ws, unsigned* err_flag) {
    // two LDS slots so consecutive tiles never race on the broadcast values
    __shared__ float s_wave_tot[2][W];
    __shared__ float s_prefix[2];
    __shared__ unsigned s_tile[2];
    const float init = init_dev ? *init_dev : 0.f;
    f32x4 va[R], vb[R];
    if (threadIdx.x == 0) {
        s_tile[0] = atomicAdd(&ws->ticket, 1u);
        s_tile[1] = atomicAdd(&ws->ticket, 1u);
    }
    __syncthreads();
    long long ta = s_tile[0], tb = s_tile[1];
    if (ta >= ntiles) return;
    load_tile<R, W>(in, n, ta, va);
    // unrolled by two so both register buffers are statically named (every exit is block-uniform); each
    // finish_tile takes the ticket two tiles ahead and publishes it in s_tile[slot] by its last barrier
    while (true) {
        finish_tile<R, W>(in, out, n, ta, va, tb, vb, ntiles, exclusive, init, ws, err_flag, s_wave_tot[0], &s_prefix[0], &s_tile[0]);
        if (tb >= ntiles) break;
        ta = s_tile[0];
        finish_tile<R, W>(in, out, n, tb, vb, ta, va, ntiles, exclusive, init, ws, err_flag, s_wave_tot[1], &s_prefix[1], &s_tile[1]);
        if (ta >= ntiles) break;
        tb = s_tile[1];
    }
}

// ---- PARKED-TILE schedule (look-back one iteration late).
// The persistent schedule above looks tile t back right after scanning it, while its neighbours t-1, t-2, ...
// are being scanned by other blocks at the same moment: each look-back waits for aggregates that are still
// being produced, and that publication chain cost ~17% (1.23 ms without a look-back vs 1.46 ms, see
// profiles/r1_workloads/scan_lookback_ab.txt). Here a block scans tile t (publishing its aggregate), parks the
// tile-local results in LDS (128 KiB of the 160 KiB) and only looks t back and writes it out during its NEXT
// tile: by then every predecessor published its aggregate an iteration ago, so the look-back is one round of
// polls. The inclusive prefixes now trail by one iteration (~grid tiles), so one wave polls 8 windows of 64
// predecessors with all loads issued at once and combines them newest-first. Each thread parks and later reads
// back only its own f32x4 slots (no barrier guards the park buffer).
constexpr int kParkWindows = 8;

using ParkPoll = unsigned long long[kParkWindows];

// One round of polls: lane l of window k reads the status of tile look - l - 64k (all loads in flight at once).
__device__ __forceinline__ void parked_poll(long long tile, long long look, ScanWs* ws, ParkPoll& sv) {
    unsigned long long* status = reinterpret_cast<unsigned long long*>(ws + 1);
    const int lane = pcmx::lane_id();
#pragma unroll
    for (int k = 0; k < kParkWindows; ++k) {
        const long long idx = look - lane - (long long)k * kWave;
        sv[k] = idx >= 0 ? __hip_atomic_load(&status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                         : pack(kFlagIncl, 0.f);
#ifdef PCMX_FAULT_INJECT
        if (tile == kFaultTile) sv[k] = 0ull;
#endif
    }
    (void)tile;
}

// Exclusive prefix of `tile` from its predecessors' granules; `polled` = sv already holds the first round.
__device__ __forceinline__ float parked_lookback(long long tile, ScanWs* ws, unsigned* err_flag, ParkPoll& sv,
                                                bool polled) {
    const int lane = pcmx::lane_id();
    float acc = 0.f;  // lane-partial sum of the predecessors accounted for so far
    long long look = tile - 1;
    unsigned spins = 0;
    while (true) {
        if (!polled) parked_poll(tile, look, ws, sv);
        polled = false;
        bool done = false, stall = false;
#pragma unroll
        for (int k = 0; k < kParkWindows; ++k) {
            if (done || stall) break;  // wave-uniform
            const unsigned flag = (unsigned)(sv[k] >> 32);
            const float val = __uint_as_float((unsigned)sv[k]);
            const unsigned long long m_incl = __ballot(flag == kFlagIncl);
            const unsigned long long m_zero = __ballot(flag == 0u);
            if (m_incl != 0ull) {
                const int first = __builtin_ctzll(m_incl);
                const unsigned long long need = (first == 63) ? ~0ull : ((1ull << (first + 1)) - 1ull);
                if ((m_zero & need) == 0ull) {
                    acc += lane <= first ? val : 0.f;
                    done = true;
                } else {
                    stall = true;
                }
            } else if (m_zero == 0ull) {
                acc += val;
                look -= kWave;
            } else {
                stall = true;
            }
        }
        if (done) break;
        if (stall) {
            if (++spins > kSpinLimit) {  // bounded spin, reported as in the persistent schedule
                if (lane == 0) {
                    atomicExch(&ws->timeout, 1u);
                    if (err_flag) __hip_atomic_fetch_or(err_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    return pcmx::wave_reduce<float, 0>(acc);
}

// Looks back `prev` (wave 0), publishes its inclusive prefix and writes it out from the park buffer.
template <int R, int W>
__device__ __forceinline__ void parked_flush(float* __restrict__ out, long long n, long long prev, float agg_prev,
                                             float init, ScanWs* ws, unsigned* err_flag, const f32x4* park,
                                             float* s_prefix, unsigned* s_next, unsigned ticket, ParkPoll& sv,
                                             bool polled) {
    unsigned long long* status = reinterpret_cast<unsigned long long*>(ws + 1);
    const int lane = pcmx::lane_id(), wave = threadIdx.x / kWave;
    if (prev >= 0 && wave == 0) {
        const float prefix = prev == 0 ? 0.f : parked_lookback(prev, ws, err_flag, sv, polled);
        if (lane == 0) {
            if (prev != 0)
                __hip_atomic_store(&status[prev], pack(kFlagIncl, prefix + agg_prev), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            *s_prefix = init + prefix;
        }
    }
    if (threadIdx.x == 0) *s_next = ticket;
    __syncthreads();
    if (prev < 0) return;
    const float off = *s_prefix;
    const long long base = prev * Tile<R, W>::kElems + (long long)wave * Tile<R, W>::kWaveItems;
    const bool full = (prev + 1) * Tile<R, W>::kElems <= n;  // block-uniform
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const f32x4 o = park[(wave * R + r) * kWave + lane] + off;
        const long long e = base + r * 256 + lane * 4;
        if (full || e + 3 < n) {
            __builtin_nontemporal_store(o, reinterpret_cast<f32x4*>(out + e));
        } else {
            if (e < n) out[e] = o.x;
            if (e + 1 < n) out[e + 1] = o.y;
            if (e + 2 < n) out[e + 2] = o.z;
        }
    }
}

// One iteration: scan `cur` (in v) and publish its aggregate, issue the loads of `next` into vn, take a ticket,
// flush `prev` from the park buffer, park `cur`. Returns cur's aggregate (thread 0 needs it one iteration later).
// kLoadAt (round 6 lab): where the loads of `next` go out. 0 (production): after cur's scan and publish. 1: at the TOP
// of the iteration (vn is free there: its last tile was parked an iteration ago), before wave 0's early polls. 2:
// right AFTER the early polls, before the scan. vmcnt retires in issue order, so under 1 the look-back's wait for its
// polls also waits for the whole next tile; 2 keeps the polls ahead of the loads.
template <int R, int W, bool kEarly, int kLoadAt = 0, bool kRs = false>
__device__ __forceinline__ float parked_step(const float* __restrict__ in, float* __restrict__ out, long long n,
                                             long long cur, f32x4 (&v)[R], long long next, f32x4 (&vn)[R],
                                             long long prev, float agg_prev, long long ntiles, int exclusive, float init,
                                             ScanWs* ws, unsigned* err_flag, f32x4* park, float* s_wave_tot,
                                             float* s_prefix, unsigned* s_next) {
    unsigned long long* status = reinterpret_cast<unsigned long long*>(ws + 1);
    const int lane = pcmx::lane_id(), wave = threadIdx.x / kWave;
    // kEarly: wave 0 sends prev's first round of polls BEFORE this tile's scan, so their round trip overlaps it
    if constexpr (kLoadAt == 1) {
        if constexpr (kRs)
            load_tile_rs<R, W>(in, n, next, vn);  // branch-free (an empty range past the last tile)
        else if (next < ntiles)
            load_tile<R, W>(in, n, next, vn);
    }
    ParkPoll sv;
    const bool polled = kEarly && wave == 0 && prev > 0;
    if (polled) parked_poll(prev, prev - 1, ws, sv);
    if constexpr (kLoadAt == 2) {
        if constexpr (kRs)
            load_tile_rs<R, W>(in, n, next, vn);  // branch-free (an empty range past the last tile)
        else if (next < ntiles)
            load_tile<R, W>(in, n, next, vn);
    }
    float carry = 0.f;
    float lane_excl[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
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
    float agg = 0.f, wexcl = 0.f;
#pragma unroll
    for (int w = 0; w < W; ++w) {
        const float t = s_wave_tot[w];
        wexcl += w < wave ? t : 0.f;
        agg += t;
    }
    if (threadIdx.x == 0)
        __hip_atomic_store(&status[cur], pack(cur == 0 ? kFlagIncl : kFlagAgg, agg), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    if constexpr (kLoadAt == 0) {
        if constexpr (kRs)
            load_tile_rs<R, W>(in, n, next, vn);  // branch-free (an empty range past the last tile)
        else if (next < ntiles)
            load_tile<R, W>(in, n, next, vn);
    }
    const unsigned ticket = threadIdx.x == 0 ? atomicAdd(&ws->ticket, 1u) : 0u;
    parked_flush<R, W>(out, n, prev, agg_prev, init, ws, err_flag, park, s_prefix, s_next, ticket, sv, polled);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const float b = wexcl + lane_excl[r];
        f32x4 o;
        if (exclusive) {
            o.x = b;
            o.y = b + v[r].x;
            o.z = b + v[r].y;
            o.w = b + v[r].z;
        } else {
            o = v[r] + b;
        }
        park[(wave * R + r) * kWave + lane] = o;
    }
    return agg;
}

template <int R, int W, bool kEarly, int kLoadAt = 0, bool kRs = false>
__global__ __launch_bounds__(W * kWave) void scan_parked_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                                long long n, long long ntiles, int exclusive,
                                                                const float* init_dev, ScanWs* ws, unsigned* err_flag) {
    __shared__ f32x4 park[W * R * kWave];
    __shared__ float s_wave_tot[W];
    __shared__ float s_prefix;
    __shared__ unsigned s_tile[2];
    const float init = init_dev ? *init_dev : 0.f;
    f32x4 va[R], vb[R];
    if (threadIdx.x == 0) {
        s_tile[0] = atomicAdd(&ws->ticket, 1u);
        s_tile[1] = atomicAdd(&ws->ticket, 1u);
    }
    __syncthreads();
    long long ta = s_tile[0], tb = s_tile[1], prev = -1;
    if (ta >= ntiles) return;
    float agg_prev = 0.f;
    if constexpr (kRs)
        load_tile_rs<R, W>(in, n, ta, va);
    else
        load_tile<R, W>(in, n, ta, va);
    // unrolled by two so both register buffers are statically named; every exit is block-uniform and ends with
    // the flush of the last parked tile
    while (true) {
        agg_prev = parked_step<R, W, kEarly, kLoadAt, kRs>(in, out, n, ta, va, tb, vb, prev, agg_prev, ntiles, exclusive, init, ws, err_flag,
                                     park, s_wave_tot, &s_prefix, &s_tile[0]);
        prev = ta;
        ta = s_tile[0];
        if (tb >= ntiles) break;
        agg_prev = parked_step<R, W, kEarly, kLoadAt, kRs>(in, out, n, tb, vb, ta, va, prev, agg_prev, ntiles, exclusive, init, ws, err_flag,
                                     park, s_wave_tot, &s_prefix, &s_tile[0]);
        prev = tb;
        tb = s_tile[0];
        if (ta >= ntiles) break;
    }
    __syncthreads();  // every wave has read s_prefix of the last step before wave 0 rewrites it
    ParkPoll sv;
    parked_flush<R, W>(out, n, prev, agg_prev, init, ws, err_flag, park, &s_prefix, &s_tile[1], 0u, sv, false);
}

inline long long num_tiles(long long n) { return (n + kTileElems - 1) / kTileElems; }

int device_cus() {
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cus[dev] && hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus[dev] = 256;
    return cus[dev] > 0 ? cus[dev] : 256;
}
}  // namespace

extern "C" long long pcmx_scan_workspace_bytes(long long n) { return (long long)sizeof(ScanWs) + num_tiles(n) * 8; }

extern "C" int pcmx_scan_f32_variant(const float* x, float* out, long long n, int exclusive, const float* init_dev,
                                     void* workspace, unsigned* err_flag, int variant, hipStream_t s) {
    if (n <= 0) return 0;
    if (variant < 0 || variant > 8) return PCMX_ERR_ARG;
    if ((((uintptr_t)x) & 15u) || (((uintptr_t)out) & 15u) || !workspace) return PCMX_ERR_ARG;
    const long long tiles = num_tiles(n);
    if (tiles > 0x7fffffffLL) return PCMX_ERR_ARG;
    PCMX_HIP_RET(hipMemsetAsync(workspace, 0, sizeof(ScanWs) + (size_t)tiles * 8, s));
    ScanWs* ws = reinterpret_cast<ScanWs*>(workspace);
    const unsigned grid = (unsigned)(tiles < device_cus() ? tiles : device_cus());  // one resident block per CU
    switch (variant) {
        case 0: scan_persistent_kernel<16, 8><<<grid, 8 * kWave, 0, s>>>(x, out, n, tiles, exclusive, init_dev, ws, err_flag); break;
        case 1: scan_persistent_kernel<8, 16><<<grid, 16 * kWave, 0, s>>>(x, out, n, tiles, exclusive, init_dev, ws, err_flag); break;
        case 2: scan_parked_kernel<16, 8, false><<<grid, 8 * kWave, 0, s>>>(x, out, n, tiles, exclusive, init_dev, ws, err_flag); break;
        case 3: scan_parked_kernel<8, 16, false><<<grid, 16 * kWave, 0, s>>>(x, out, n, tiles, exclusive, init_dev, ws, err_flag); break;
        case 5: scan_parked_kernel<16, 8, true, 1><<<grid, 8 * kWave, 0, s>>>(x, out, n, tiles, exclusive, init_dev, ws, err_flag); break;
        case 6: scan_parked_kernel<16, 8, true, 2><<<grid, 8 * kWave, 0, s>>>(x, out, n, tiles, exclusive, init_dev, ws, err_flag); break;
        case 7: scan_parked_kernel<16, 8, true, 0, true><<<grid, 8 * kWave, 0, s>>>(x, out, n, tiles, exclusive, init_dev, ws, err_flag); break;
        case 8: scan_parked_kernel<16, 8, true, 2, true><<<grid, 8 * kWave, 0, s>>>(x, out, n, tiles, exclusive, init_dev, ws, err_flag); break;
        default: scan_parked_kernel<16, 8, true><<<grid, 8 * kWave, 0, s>>>(x, out, n, tiles, exclusive, init_dev, ws, err_flag); break;
    }
    return (int)hipGetLastError();
}

extern "C" int pcmx_scan_f32_rows(const float* x, float* out, long long n, int exclusive, const float* init_dev,
                                  void* workspace, unsigned* err_flag, int rows, hipStream_t s) {
    if (rows != 8 && rows != 16) return PCMX_ERR_ARG;
    return pcmx_scan_f32_variant(x, out, n, exclusive, init_dev, workspace, err_flag, rows == 16 ? 4 : 1, s);
}

extern "C" int pcmx_scan_f32(const float* x, float* out, long long n, int exclusive, const float* init_dev, void* workspace,
                             unsigned* err_flag, hipStream_t s) {
    return pcmx_scan_f32_variant(x, out, n, exclusive, init_dev, workspace, err_flag, 4, s);
}

extern "C" int pcmx_scan_check(const void* workspace, hipStream_t s) {
    if (!workspace) return PCMX_ERR_ARG;
    unsigned t = 0;
    PCMX_HIP_RET(hipMemcpyAsync(&t, &reinterpret_cast<const ScanWs*>(workspace)->timeout, sizeof(t), hipMemcpyDeviceToHost, s));
    PCMX_HIP_RET(hipStreamSynchronize(s));
    return t ? PCMX_ERR_TIMEOUT : 0;
}
