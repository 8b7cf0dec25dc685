// Sparse matrix-vector products on MI355X (ref 3-serial-optimization/spmv.c: multiply_naive :170-177,
// banded SSE multiply :212-329) — and the north-star 1e8-nnz power-law CSR SpMV.
//
// CSR (any sparsity, power-law safe): CSR-adaptive with nnz-balanced work items. An analysis pass
// (pcmx_spmv_csr_plan, once per matrix) cuts the rows into items of <= kItemNnz nonzeros: runs of short
// rows are packed into one item, a long row is split into several items. One wave per item:
//   * multi-row item: the wave streams the item's values/columns coalesced (16 B per lane), multiplies by
//     the gathered x, parks the products in LDS, then reduces rows with L = 64/rows lanes per row;
//   * long-row piece: straight wave reduction, one float atomic per piece into y (y zeroed first).
// Every wave does about the same number of nonzeros whatever the degree distribution, so the heavy rows
// of a power-law graph do not produce a tail.
//
// Banded (implicit column indices): one wave per row; the 5 bands are contiguous slices of x and of the
// value array, so all loads are unit-stride and no column index is ever read.
#include "pcmx_common.h"
#include "pcmx_hip.h"

namespace {
using pcmx::kWave;
constexpr int kItemNnz = 1024;
constexpr int kWavesPerBlock = 4;

struct Item {
    int row0, row1;        // rows [row0, row1) (row1 == row0 + 1 for a long-row piece)
    long long nz0, nz1;    // nonzeros [nz0, nz1)
};

constexpr int kItemRows = 1024;           // rows per multi-row item (bounds the row-pointer LDS stage)
constexpr int kPerLane = kItemNnz / kWave;  // nonzeros per lane in phase 1

// One wave per item. Phase 1 issues every column/value load of the item up front (kPerLane coalesced
// 256-B wave loads each), then all x gathers, so a lane keeps 2 x kPerLane loads in flight instead of a
// dependent load chain. Products are parked in LDS with the item's row pointers; phase 2 reduces rows
// with L lanes per row out of LDS only.
__global__ __launch_bounds__(kWavesPerBlock * kWave) void spmv_csr_items_kernel(
    const long long* __restrict__ row_ptr, const int* __restrict__ col, const float* __restrict__ val,
    const float* __restrict__ x, float* __restrict__ y, const Item* __restrict__ items, long long n_items) {
    __shared__ float prod[kWavesPerBlock][kItemNnz];
    __shared__ int rps[kWavesPerBlock][kItemRows + 1];
    const int lane = pcmx::lane_id(), w = threadIdx.x / kWave;
    const long long it = (long long)blockIdx.x * kWavesPerBlock + w;
    if (it >= n_items) return;
    const Item item = items[it];
    const long long nz0 = item.nz0;
    const int n = (int)(item.nz1 - nz0);
    const int nrows = item.row1 - item.row0;
    int cj[kPerLane];
    float vj[kPerLane];
#pragma unroll
    for (int j = 0; j < kPerLane; ++j) {
        const int i = j * kWave + lane;
        cj[j] = i < n ? __builtin_nontemporal_load(col + nz0 + i) : 0;
        vj[j] = i < n ? __builtin_nontemporal_load(val + nz0 + i) : 0.f;
    }
    if (nrows == 1) {  // single row (whole short row, or one piece of a long row)
        float acc = 0.f;
#pragma unroll
        for (int j = 0; j < kPerLane; ++j) acc += vj[j] * x[cj[j]];
        acc = pcmx::wave_reduce<float, 0>(acc);
        if (lane == 0) {
            const bool whole = nz0 == row_ptr[item.row0] && item.nz1 == row_ptr[item.row0 + 1];
            if (whole)
                y[item.row0] = acc;
            else
                atomicAdd(&y[item.row0], acc);
        }
        return;
    }
    float* pr = prod[w];
    int* rp = rps[w];
#pragma unroll
    for (int j = 0; j < kPerLane; ++j) pr[j * kWave + lane] = vj[j] * x[cj[j]];
    for (int i = lane; i <= nrows; i += kWave) rp[i] = (int)(row_ptr[item.row0 + i] - nz0);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    // L lanes per row: about avg-row-length / 4 lanes, power of two, at most 64 / (rows per pass)
    const int avg = n / nrows;
    int L = 1;
    while (L < 64 && L * 4 < avg) L <<= 1;
    const int sub = lane & (L - 1), grp = lane / L, ngrp = kWave / L;
    for (int r = grp; r < nrows; r += ngrp) {
        const int b = rp[r], e = rp[r + 1];
        float acc = 0.f;
        for (int i = b + sub; i < e; i += L) acc += pr[i];
        for (int off = L >> 1; off > 0; off >>= 1) acc += __shfl_xor(acc, off, kWave);
        if (sub == 0) y[item.row0 + r] = acc;
    }
}

// one wave per row of the banded matrix
__global__ __launch_bounds__(256) void spmv_banded_kernel(const float* __restrict__ vals,
                                                          const long long* __restrict__ row_off, int n, int a, int b,
                                                          int c, int d, int e, const float* __restrict__ x,
                                                          float* __restrict__ y) {
    const int lane = pcmx::lane_id();
    const int row = blockIdx.x * 4 + threadIdx.x / kWave;
    if (row >= n) return;
    const int ah = a / 2;
    const int r5 = ah, r6 = ah + b, r7 = ah + b + c, r8 = ah + b + c + d, r9 = ah + b + c + d + e;
    int lo[5], hi[5];
    lo[0] = max(0, row - r9), hi[0] = max(0, row - r8);
    lo[1] = max(0, row - r7), hi[1] = max(0, row - r6);
    lo[2] = max(0, row - r5), hi[2] = min(row + r5 + 1, n);
    lo[3] = min(n, row + r6 + 1), hi[3] = min(n, row + r7 + 1);
    lo[4] = min(n, row + r8 + 1), hi[4] = min(n, row + r9 + 1);
    const float* v = vals + row_off[row];
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const int len = hi[k] > lo[k] ? hi[k] - lo[k] : 0;
        for (int j = lane; j < len; j += kWave) acc += v[j] * x[lo[k] + j];
        v += len;
    }
    acc = pcmx::wave_reduce<float, 0>(acc);
    if (lane == 0) y[row] = acc;
}
}  // namespace

// Host-side analysis: row_ptr is a HOST array (n_rows+1, int64). Writes up to max_items items into
// `items_host` (4 x int64 words each: row0, row1, nz0, nz1 packed as in Item) and returns the count, or
// -1 if max_items is too small. pcmx_spmv_csr_plan_count() gives the exact count first.
extern "C" long long pcmx_spmv_csr_plan(const long long* row_ptr, int n_rows, void* items_host, long long max_items) {
    Item* items = reinterpret_cast<Item*>(items_host);
    long long k = 0;
    int r = 0;
    while (r < n_rows) {
        const long long len = row_ptr[r + 1] - row_ptr[r];
        if (len > kItemNnz) {  // long row: split into pieces
            for (long long p = row_ptr[r]; p < row_ptr[r + 1]; p += kItemNnz) {
                if (items && k < max_items) items[k] = Item{r, r + 1, p, p + kItemNnz < row_ptr[r + 1] ? p + kItemNnz : row_ptr[r + 1]};
                ++k;
            }
            ++r;
            continue;
        }
        int r1 = r + 1;
        while (r1 < n_rows && row_ptr[r1 + 1] - row_ptr[r] <= kItemNnz && r1 - r < kItemRows) ++r1;
        if (items && k < max_items) items[k] = Item{r, r1, row_ptr[r], row_ptr[r1]};
        ++k;
        r = r1;
    }
    if (items && k > max_items) return -1;
    return k;
}

extern "C" int pcmx_spmv_csr(const long long* row_ptr, const int* col, const float* val, const float* x, float* y,
                             int n_rows, const void* items, long long n_items, hipStream_t s) {
    if (n_rows <= 0) return 0;
    PCMX_HIP_RET(hipMemsetAsync(y, 0, sizeof(float) * (size_t)n_rows, s));
    if (n_items <= 0) return 0;
    const long long blocks = (n_items + kWavesPerBlock - 1) / kWavesPerBlock;
    if (blocks > 0x7fffffffLL) return -1;
    spmv_csr_items_kernel<<<(unsigned)blocks, kWavesPerBlock * kWave, 0, s>>>(row_ptr, col, val, x, y,
                                                                               reinterpret_cast<const Item*>(items), n_items);
    return (int)hipGetLastError();
}

extern "C" int pcmx_spmv_banded(const float* vals, const long long* row_off, int n, int a, int b, int c, int d, int e,
                                const float* x, float* y, hipStream_t s) {
    if (n <= 0) return 0;
    spmv_banded_kernel<<<(n + 3) / 4, 256, 0, s>>>(vals, row_off, n, a, b, c, d, e, x, y);
    return (int)hipGetLastError();
}
