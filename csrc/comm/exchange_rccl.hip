// Low-host-overhead grouped exchange over a dedicated RCCL communicator (round 6, SpMV ghost exchange and other
// per-step all-to-all-v patterns of parallel/dist.py).
//
// Why: a torch.distributed all_to_all costs ~40 us of HOST time per call (ProcessGroupNCCL work object, events,
// allocator stream records, watchdog), measured with the production N = 8 SpMV rank step on a world-1 RCCL
// communicator: two exchanges per step took the host enqueue from 42 to 126 us per step, above the 116-us device
// step, so the GPU idled between launches (profiles/r6_spmv/). This path issues the same grouped ncclSend / ncclRecv
// per peer straight from C++ on the communicator's own stream, ordered against the caller's stream with two events:
//   exchange(slot): record `ready[slot]` on the compute stream -> the comm stream waits for it -> ncclGroupStart,
//                   one ncclSend / ncclRecv per peer with data (offsets and counts in bytes), ncclGroupEnd ->
//                   record `done[slot]` on the comm stream;
//   wait(slot):     the compute stream waits for `done[slot]` (no host sync).
// A slot is one exchange in flight (the SpMV step keeps one per row chunk). The communicator is separate from
// torch's (its own ncclUniqueId, bootstrapped by the caller over torch.distributed), so its operations never
// interleave with torch's collectives on one communicator; every rank posts the same exchanges in the same order.
// Reference: the MPI exchange of 2-mpi-region-growing/region.c:250-353 (one message per neighbour per step).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdlib>
#include <cstring>
#include <ctime>

#include "pcmx_common.h"
#include "pcmx_errors.h"
#include "pcmx_hip.h"

namespace {
constexpr int kSlots = 8;

struct XComm {
    ncclComm_t comm = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t ready[kSlots] = {}, done[kSlots] = {};
    int world = 0, rank = 0, device = 0;
};

int rc_nccl(ncclResult_t r) { return r == ncclSuccess ? 0 : PCMX_ERR_COMM; }
}  // namespace

extern "C" int pcmx_xcomm_id_bytes() { return (int)sizeof(ncclUniqueId); }

extern "C" int pcmx_xcomm_unique_id(void* out) {
    ncclUniqueId id;
    const int rc = rc_nccl(ncclGetUniqueId(&id));
    if (rc == 0) std::memcpy(out, &id, sizeof(id));
    return rc;
}

extern "C" int pcmx_xcomm_create(const void* id, int world, int rank, int device, void** out) {
    if (!id || !out || world < 1 || rank < 0 || rank >= world) return PCMX_ERR_ARG;
    *out = nullptr;
    PCMX_HIP_RET(hipSetDevice(device));
    XComm* x = new XComm();
    x->world = world, x->rank = rank, x->device = device;
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    int rc = rc_nccl(ncclCommInitRank(&x->comm, world, uid, rank));
    if (rc == 0 && hipStreamCreateWithFlags(&x->stream, hipStreamNonBlocking) != hipSuccess) rc = PCMX_ERR_COMM;
    // PCMX_XCOMM_EVENT_SCOPE (lab knob, read once per communicator): 1 = device-scope release on the "ready" events
    // (compute -> comm), 2 = also on the "done" events (comm -> compute), 0 (default) = the system-scope release of
    // a default event. See profiles/r6_spmv/ for what the wait costs either way.
    const char* sc = getenv("PCMX_XCOMM_EVENT_SCOPE");
    const int scope = sc ? atoi(sc) : 0;
    const unsigned rf = hipEventDisableTiming | (scope >= 1 ? hipEventReleaseToDevice : 0u);
    const unsigned df = hipEventDisableTiming | (scope >= 2 ? hipEventReleaseToDevice : 0u);
    for (int s = 0; rc == 0 && s < kSlots; ++s)
        if (hipEventCreateWithFlags(&x->ready[s], rf) != hipSuccess || hipEventCreateWithFlags(&x->done[s], df) != hipSuccess)
            rc = PCMX_ERR_COMM;
    if (rc != 0) {  // release whatever was created before the failure
        for (int s = 0; s < kSlots; ++s) {
            if (x->ready[s]) (void)hipEventDestroy(x->ready[s]);
            if (x->done[s]) (void)hipEventDestroy(x->done[s]);
        }
        if (x->stream) (void)hipStreamDestroy(x->stream);
        if (x->comm) ncclCommDestroy(x->comm);
        delete x;
        return rc;
    }
    *out = x;
    return 0;
}

// send / recv: device buffers; soff / scnt / roff / rcnt: world entries each, in BYTES. Peers with a zero count move
// nothing; the self entry (q == rank) is a copy through RCCL like any other peer (a world-1 communicator exchanges
// with itself: the lab's stand-in for xGMI).
extern "C" int pcmx_xcomm_exchange(void* handle, int slot, const void* send, const long long* soff,
                                   const long long* scnt, void* recv, const long long* roff, const long long* rcnt,
                                   hipStream_t compute) {
    const char* sb = static_cast<const char*>(send);
    char* rb = static_cast<char*>(recv);
    XComm* x = static_cast<XComm*>(handle);
    if (!x || !x->comm || slot < 0 || slot >= kSlots) return PCMX_ERR_ARG;
    PCMX_HIP_RET(hipEventRecord(x->ready[slot], compute));
    PCMX_HIP_RET(hipStreamWaitEvent(x->stream, x->ready[slot], 0));
    int rc = rc_nccl(ncclGroupStart());
    for (int q = 0; rc == 0 && q < x->world; ++q) {
        if (scnt[q] > 0) rc = rc_nccl(ncclSend(sb + soff[q], (size_t)scnt[q], ncclUint8, q, x->comm, x->stream));
        if (rc == 0 && rcnt[q] > 0) rc = rc_nccl(ncclRecv(rb + roff[q], (size_t)rcnt[q], ncclUint8, q, x->comm, x->stream));
    }
    const int rc_end = rc_nccl(ncclGroupEnd());  // (always closes the group it opened)
    if (rc == 0) rc = rc_end;
    if (rc != 0) return rc;
    PCMX_HIP_RET(hipEventRecord(x->done[slot], x->stream));
    return 0;
}

extern "C" int pcmx_xcomm_wait(void* handle, int slot, hipStream_t compute) {
    XComm* x = static_cast<XComm*>(handle);
    if (!x || slot < 0 || slot >= kSlots) return PCMX_ERR_ARG;
    PCMX_HIP_RET(hipStreamWaitEvent(compute, x->done[slot], 0));
    return 0;
}

// Start-up probe: one float to and from every peer (value 1000 * sender + receiver) through the same grouped path,
// waited for on the host for at most timeout_ms (hipEventQuery polling), then checked. A probe that times out or
// fails ABORTS the communicator (ncclCommAbort ends its pending operations, so nothing is left spinning on the GPU)
// and returns PCMX_ERR_TIMEOUT / PCMX_ERR_COMM: the caller falls back to torch.distributed. Collective.
extern "C" int pcmx_xcomm_probe(void* handle, int timeout_ms) {
    XComm* x = static_cast<XComm*>(handle);
    if (!x || !x->comm) return PCMX_ERR_ARG;
    const int W = x->world;
    float *dev = nullptr;
    if (hipMalloc(&dev, 2 * (size_t)W * sizeof(float)) != hipSuccess) return PCMX_ERR_ALLOC;
    float* host = new float[2 * (size_t)W];
    for (int q = 0; q < W; ++q) host[q] = (float)(1000 * x->rank + q), host[W + q] = -1.f;
    long long* offs = new long long[4 * (size_t)W];
    for (int q = 0; q < W; ++q) offs[q] = 4 * q, offs[W + q] = 4, offs[2 * W + q] = 4 * q, offs[3 * W + q] = 4;
    int rc = hipMemcpy(dev, host, 2 * (size_t)W * sizeof(float), hipMemcpyHostToDevice) == hipSuccess ? 0 : PCMX_ERR_COMM;
    if (rc == 0)
        rc = pcmx_xcomm_exchange(x, kSlots - 1, dev, offs, offs + W, dev + W, offs + 2 * W, offs + 3 * W, x->stream);
    if (rc == 0) {
        const timespec nap{0, 200000};  // 0.2 ms
        for (long waited_us = 0;; waited_us += 200) {
            const hipError_t q = hipEventQuery(x->done[kSlots - 1]);
            if (q == hipSuccess) break;
            if (q != hipErrorNotReady) {
                rc = PCMX_ERR_COMM;
                break;
            }
            ncclResult_t ae = ncclSuccess;
            if (ncclCommGetAsyncError(x->comm, &ae) != ncclSuccess || ae != ncclSuccess) {
                rc = PCMX_ERR_COMM;
                break;
            }
            if (waited_us / 1000 >= timeout_ms) {
                rc = PCMX_ERR_TIMEOUT;
                break;
            }
            nanosleep(&nap, nullptr);
        }
    }
    if (rc == 0 && hipMemcpy(host + W, dev + W, (size_t)W * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
        rc = PCMX_ERR_COMM;
    for (int q = 0; rc == 0 && q < W; ++q)
        if (host[W + q] != (float)(1000 * q + x->rank)) rc = PCMX_ERR_COMM;
    if (rc != 0) {
        ncclCommAbort(x->comm);
        x->comm = nullptr;
    }
    (void)hipStreamSynchronize(x->stream);
    (void)hipFree(dev);
    delete[] host;
    delete[] offs;
    return rc;
}

// Asynchronous RCCL errors of the communicator (a peer that died, a transport failure): 0 when healthy.
extern "C" int pcmx_xcomm_async_error(void* handle) {
    XComm* x = static_cast<XComm*>(handle);
    if (!x || !x->comm) return PCMX_ERR_ARG;
    ncclResult_t e = ncclSuccess;
    const int rc = rc_nccl(ncclCommGetAsyncError(x->comm, &e));
    return rc ? rc : rc_nccl(e);
}

extern "C" int pcmx_xcomm_destroy(void* handle) {
    XComm* x = static_cast<XComm*>(handle);
    if (!x) return 0;
    (void)hipStreamSynchronize(x->stream);
    const int rc = x->comm ? rc_nccl(ncclCommDestroy(x->comm)) : 0;  // (an aborted communicator is gone already)
    for (int s = 0; s < kSlots; ++s) {
        if (x->ready[s]) (void)hipEventDestroy(x->ready[s]);
        if (x->done[s]) (void)hipEventDestroy(x->done[s]);
    }
    (void)hipStreamDestroy(x->stream);
    delete x;
    return rc;
}
