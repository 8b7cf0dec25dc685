// RCCL transport of the native comm layer (pcmx_comm.h) + the device backend of the distributed region
// growing. One process per MI355X; the communicator is bootstrapped over the TCP side-channel (rank 0's
// ncclUniqueId is broadcast), then every collective / point-to-point call is stream-ordered on the
// communicator's HIP stream, and so are the backend's kernels and copies: no host sync is needed between a
// kernel and the send of its output. Grouped send/recv (ncclGroupStart/End) is the deadlock-free halo
// exchange over xGMI point-to-point links.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "pcmx_comm.h"
#include "pcmx_hip.h"

namespace {

struct RcclImpl {
    ncclComm_t comm = nullptr;
    hipStream_t stream = nullptr;
};

int rc_of(ncclResult_t r) { return r == ncclSuccess ? 0 : 1000 + (int)r; }
RcclImpl* impl(pcmx_comm_t* c) { return static_cast<RcclImpl*>(c->impl); }

ncclDataType_t nccl_type(int dt) {
    switch (dt) {
        case PCMX_I32: return ncclInt32;
        case PCMX_F32: return ncclFloat32;
        case PCMX_F64: return ncclFloat64;
        case PCMX_I64: return ncclInt64;
        default: return ncclUint8;
    }
}
ncclRedOp_t nccl_op(int op) { return op == PCMX_MIN ? ncclMin : op == PCMX_MAX ? ncclMax : ncclSum; }

int r_group_start(pcmx_comm_t*) { return rc_of(ncclGroupStart()); }
int r_group_end(pcmx_comm_t*) { return rc_of(ncclGroupEnd()); }
int r_send(pcmx_comm_t* c, const void* b, size_t n, int peer) {
    return rc_of(ncclSend(b, n, ncclUint8, peer, impl(c)->comm, impl(c)->stream));
}
int r_recv(pcmx_comm_t* c, void* b, size_t n, int peer) {
    return rc_of(ncclRecv(b, n, ncclUint8, peer, impl(c)->comm, impl(c)->stream));
}
int r_allreduce(pcmx_comm_t* c, void* b, size_t n, int dt, int op) {
    return rc_of(ncclAllReduce(b, b, n, nccl_type(dt), nccl_op(op), impl(c)->comm, impl(c)->stream));
}
int r_bcast(pcmx_comm_t* c, void* b, size_t n, int root) {
    return rc_of(ncclBroadcast(b, b, n, ncclUint8, root, impl(c)->comm, impl(c)->stream));
}
int r_sync(pcmx_comm_t* c) { return (int)hipStreamSynchronize(impl(c)->stream); }
void r_destroy(pcmx_comm_t* c) {
    RcclImpl* r = impl(c);
    if (r) {
        if (r->stream) hipStreamSynchronize(r->stream);
        if (r->comm) ncclCommDestroy(r->comm);
        if (r->stream) hipStreamDestroy(r->stream);
        delete r;
    }
    if (c->host && c->host != c) pcmx_comm_destroy(c->host);
    free(c);
}

const pcmx_comm_ops_t kRcclOps = {r_group_start, r_group_end, r_send, r_recv, r_allreduce, r_bcast, r_sync, r_destroy};

// ---------------------------------------------------------------- device backend
struct DevCtx {
    hipStream_t s = nullptr;
    void* ws = nullptr;
    long long ws_bytes = 0;
};

void* d_alloc(size_t n, void*) {
    void* p = nullptr;
    return hipMalloc(&p, n ? n : 1) == hipSuccess ? p : nullptr;
}
void d_release(void* p, void*) { hipFree(p); }
int d_memset0(void* p, size_t n, void* ctx) { return (int)hipMemsetAsync(p, 0, n, static_cast<DevCtx*>(ctx)->s); }
int d_h2d(void* d, const void* s, size_t n, void* ctx) {
    hipStream_t st = static_cast<DevCtx*>(ctx)->s;
    int rc = (int)hipMemcpyAsync(d, s, n, hipMemcpyHostToDevice, st);
    return rc ? rc : (int)hipStreamSynchronize(st);  // host source may be a stack temporary
}
int d_d2h(void* d, const void* s, size_t n, void* ctx) {
    hipStream_t st = static_cast<DevCtx*>(ctx)->s;
    int rc = (int)hipMemcpyAsync(d, s, n, hipMemcpyDeviceToHost, st);
    return rc ? rc : (int)hipStreamSynchronize(st);
}
int d_copy2d(void* d, size_t dp, const void* s, size_t sp, size_t w, size_t h, void* ctx) {
    return (int)hipMemcpy2DAsync(d, dp, s, sp, w, h, hipMemcpyDeviceToDevice, static_cast<DevCtx*>(ctx)->s);
}
int d_grow(unsigned char* reg, const unsigned char* img, int h, int w, int thr, void* ctx) {
    DevCtx* c = static_cast<DevCtx*>(ctx);
    const long long need = pcmx_region2d_workspace_bytes(h, w);
    if (need > c->ws_bytes) {
        if (c->ws) hipFree(c->ws);
        if (hipMalloc(&c->ws, need) != hipSuccess) return -1;
        c->ws_bytes = need;
    }
    int launches = 0;
    return pcmx_region2d_grow(img, reg, h, w, w + 2, thr, c->ws, 4, 1 << 20, c->s, &launches);
}
int d_pack(const unsigned char* t, int h, int w, unsigned char* buf, void* ctx) {
    return pcmx_pack_edges(t, 1, h, w, w + 2, buf, static_cast<DevCtx*>(ctx)->s);
}
int d_unpack(unsigned char* t, int h, int w, const unsigned char* buf, int mask, void* ctx) {
    return pcmx_unpack_halo(t, 1, h, w, w + 2, buf, mask, static_cast<DevCtx*>(ctx)->s);
}
int d_sync(void* ctx) { return (int)hipStreamSynchronize(static_cast<DevCtx*>(ctx)->s); }

int env_int(const char* n, int d) {
    const char* v = getenv(n);
    return v && *v ? atoi(v) : d;
}
}  // namespace

extern "C" int pcmx_region_backend_hip(pcmx_region_backend_t* be, void* stream) {
    DevCtx* c = new DevCtx;
    c->s = static_cast<hipStream_t>(stream);
    be->alloc = d_alloc, be->release = d_release, be->memset0 = d_memset0, be->h2d = d_h2d, be->d2h = d_d2h;
    be->copy2d = d_copy2d, be->grow = d_grow, be->pack = d_pack, be->unpack = d_unpack, be->sync = d_sync;
    be->ctx = c;
    return 0;
}

extern "C" int pcmx_comm_init_env_rccl(pcmx_comm_t** out) {
    *out = nullptr;
    pcmx_comm_t* host = nullptr;
    int rc = pcmx_comm_init_env_tcp(&host);
    if (rc) {
        pcmx_comm_destroy(host);
        return rc;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        pcmx_comm_destroy(host);
        return -20;
    }
    const int dev = env_int("LOCAL_RANK", host->rank) % ndev;
    if (hipSetDevice(dev) != hipSuccess) {
        pcmx_comm_destroy(host);
        return -21;
    }
    ncclUniqueId id;
    if (host->rank == 0 && (rc = rc_of(ncclGetUniqueId(&id)))) {
        pcmx_comm_destroy(host);
        return rc;
    }
    if ((rc = host->ops->bcast(host, &id, sizeof id, 0))) {
        pcmx_comm_destroy(host);
        return rc;
    }
    RcclImpl* r = new RcclImpl;
    if (hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking) != hipSuccess ||
        (rc = rc_of(ncclCommInitRank(&r->comm, host->world, id, host->rank)))) {
        if (r->stream) hipStreamDestroy(r->stream);
        delete r;
        pcmx_comm_destroy(host);
        return rc ? rc : -22;
    }
    pcmx_comm_t* c = static_cast<pcmx_comm_t*>(calloc(1, sizeof(pcmx_comm_t)));
    c->rank = host->rank, c->world = host->world, c->local_rank = dev, c->transport = PCMX_TRANSPORT_RCCL;
    c->ops = &kRcclOps, c->impl = r, c->host = host, c->stream = r->stream;
    *out = c;
    return 0;
}
