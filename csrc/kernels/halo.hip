// Halo pack/unpack for 2-D domain decomposition (ref 2-mpi-region-growing/region.c:86-102 derived
// datatypes haloless_col_t/halo_col_t, :250-353 exchange). RCCL has no strided datatypes, so the four
// interior edges of a padded tile are gathered into one contiguous send buffer by ONE launch, exchanged
// with grouped send/recv, and scattered back into the halo ring by one launch.
//
// Padded tile: (H+2) x ld elements, interior rows/cols 1..H / 1..W.
// Send buffer: [top row W | bottom row W | left col H | right col H] (interior edge cells).
// Recv buffer: same order, landing in halo row 0, halo row H+1, halo col 0, halo col W+1.
#include "pcmx_common.h"
#include "pcmx_hip.h"

namespace {
template <class T>
__global__ __launch_bounds__(256) void pack_edges_kernel(const T* __restrict__ tile, int H, int W, int ld,
                                                        T* __restrict__ buf) {
    const int n = 2 * W + 2 * H;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        size_t src;
        if (i < W) src = (size_t)1 * ld + 1 + i;
        else if (i < 2 * W) src = (size_t)H * ld + 1 + (i - W);
        else if (i < 2 * W + H) src = (size_t)(1 + i - 2 * W) * ld + 1;
        else src = (size_t)(1 + i - 2 * W - H) * ld + W;
        buf[i] = tile[src];
    }
}

template <class T>
__global__ __launch_bounds__(256) void unpack_halo_kernel(T* __restrict__ tile, int H, int W, int ld,
                                                         const T* __restrict__ buf, int mask, int* __restrict__ changed) {
    // mask bit 0: top halo valid, 1: bottom, 2: left, 3: right (absent neighbours leave the halo alone).
    // changed (optional): set to 1 when any halo cell takes a new value — the device-resident "halo changed"
    // flag of the distributed fixpoint loops (no host round trip to count halo cells).
    const int n = 2 * W + 2 * H;
    bool diff = false;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        size_t dst;
        int side;
        if (i < W) dst = 1 + i, side = 0;
        else if (i < 2 * W) dst = (size_t)(H + 1) * ld + 1 + (i - W), side = 1;
        else if (i < 2 * W + H) dst = (size_t)(1 + i - 2 * W) * ld, side = 2;
        else dst = (size_t)(1 + i - 2 * W - H) * ld + W + 1, side = 3;
        if (mask & (1 << side)) {
            const T v = buf[i];
            diff |= tile[dst] != v;
            tile[dst] = v;
        }
    }
    if (changed && __any(diff) && pcmx::lane_id() == 0) atomicOr(changed, 1);
}

inline int grid_for(int n) { return max(1, min(1024, (n + 255) / 256)); }
}  // namespace

extern "C" int pcmx_pack_edges(const void* tile, int elem_bytes, int H, int W, int ld, void* buf, hipStream_t s) {
    const int n = 2 * W + 2 * H;
    if (elem_bytes == 1)
        pack_edges_kernel<unsigned char><<<grid_for(n), 256, 0, s>>>((const unsigned char*)tile, H, W, ld, (unsigned char*)buf);
    else if (elem_bytes == 2)
        pack_edges_kernel<unsigned short><<<grid_for(n), 256, 0, s>>>((const unsigned short*)tile, H, W, ld, (unsigned short*)buf);
    else if (elem_bytes == 4)
        pack_edges_kernel<unsigned><<<grid_for(n), 256, 0, s>>>((const unsigned*)tile, H, W, ld, (unsigned*)buf);
    else
        return PCMX_ERR_ARG;
    return (int)hipGetLastError();
}

extern "C" int pcmx_unpack_halo_changed(void* tile, int elem_bytes, int H, int W, int ld, const void* buf, int mask,
                                        int* changed, hipStream_t s) {
    const int n = 2 * W + 2 * H;
    if (elem_bytes == 1)
        unpack_halo_kernel<unsigned char><<<grid_for(n), 256, 0, s>>>((unsigned char*)tile, H, W, ld, (const unsigned char*)buf, mask, changed);
    else if (elem_bytes == 2)
        unpack_halo_kernel<unsigned short><<<grid_for(n), 256, 0, s>>>((unsigned short*)tile, H, W, ld, (const unsigned short*)buf, mask, changed);
    else if (elem_bytes == 4)
        unpack_halo_kernel<unsigned><<<grid_for(n), 256, 0, s>>>((unsigned*)tile, H, W, ld, (const unsigned*)buf, mask, changed);
    else
        return PCMX_ERR_ARG;
    return (int)hipGetLastError();
}

extern "C" int pcmx_unpack_halo(void* tile, int elem_bytes, int H, int W, int ld, const void* buf, int mask, hipStream_t s) {
    return pcmx_unpack_halo_changed(tile, elem_bytes, H, W, ld, buf, mask, nullptr, s);
}
