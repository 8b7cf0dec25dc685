/* Native communication layer: the MPI subset the reference programs use (1-introduction/mpi.c,
 * 2-mpi-region-growing/region.c) rebuilt for one process per MI355X.
 *
 *   transport RCCL : device buffers, ncclSend/ncclRecv/ncclAllReduce/ncclBroadcast over xGMI, grouped
 *                    point-to-point (ncclGroupStart/End) — stream-ordered on the communicator's HIP stream.
 *   transport TCP  : host buffers over loopback/LAN sockets (full mesh, poll-driven group progress) — the
 *                    GPU-less path used by the CPU tests, and the host side-channel/bootstrap of RCCL.
 *   transport TCP_STAGED : device buffers staged through host memory over TCP, so several ranks can share
 *                    one GPU (single-GPU test fixture for the multi-rank device path).
 *
 * Launch contract = torchrun's env: RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR, MASTER_PORT (+ PCMX_PORT to
 * override the bootstrap port). `bin/pcmx_launch -n P prog ...` is the native mpirun equivalent.
 */
#ifndef PCMX_COMM_H
#define PCMX_COMM_H
#include <stddef.h>

#include "pcmx_errors.h" /* every pcmx_comm_* returns 0 or a PCMX_ERR_* code */

#ifdef __cplusplus
extern "C" {
#endif

enum { PCMX_TRANSPORT_TCP = 0, PCMX_TRANSPORT_RCCL = 1, PCMX_TRANSPORT_TCP_STAGED = 2 };
enum { PCMX_I32 = 0, PCMX_F32 = 1, PCMX_F64 = 2, PCMX_I64 = 3, PCMX_U8 = 4 };
enum { PCMX_SUM = 0, PCMX_MIN = 1, PCMX_MAX = 2 };

typedef struct pcmx_comm pcmx_comm_t;

/* transport operations (vtable); buffers live where the transport wants them (host for TCP, device
 * for RCCL). Non-group send/recv are blocking for TCP and stream-ordered for RCCL. */
typedef struct pcmx_comm_ops {
    int (*group_start)(pcmx_comm_t*);
    int (*group_end)(pcmx_comm_t*);
    int (*send)(pcmx_comm_t*, const void* buf, size_t bytes, int peer);
    int (*recv)(pcmx_comm_t*, void* buf, size_t bytes, int peer);
    int (*allreduce)(pcmx_comm_t*, void* buf, size_t count, int dtype, int op);
    int (*bcast)(pcmx_comm_t*, void* buf, size_t bytes, int root);
    int (*sync)(pcmx_comm_t*);
    void (*destroy)(pcmx_comm_t*);
    /* collectives over equal byte blocks (`bytes` per rank; recv/send of the root-side buffers hold world
     * blocks in rank order). RCCL: ncclAllGather / ncclGather / ncclScatter / ncclAllToAll; TCP and staged:
     * one grouped round of point-to-point messages (every peer on its own socket / link at once). */
    int (*allgather)(pcmx_comm_t*, const void* send, void* recv, size_t bytes);
    int (*gather)(pcmx_comm_t*, const void* send, void* recv, size_t bytes, int root);
    int (*scatter)(pcmx_comm_t*, const void* send, void* recv, size_t bytes, int root);
    int (*alltoall)(pcmx_comm_t*, const void* send, void* recv, size_t bytes);
} pcmx_comm_ops_t;

struct pcmx_comm {
    int rank, world, local_rank, transport;
    const pcmx_comm_ops_t* ops;
    void* impl;          /* transport state */
    pcmx_comm_t* host;   /* TCP side-channel (== self for the TCP transport) */
    void* stream;        /* hipStream_t of the RCCL transport, NULL for TCP */
};

/* ---- lifecycle */
int pcmx_comm_init_tcp(int rank, int world, const char* addr, int port, pcmx_comm_t** out);
int pcmx_comm_init_env_tcp(pcmx_comm_t** out);
int pcmx_comm_init_env_rccl(pcmx_comm_t** out); /* in libpcmx_hip: sets the device to LOCAL_RANK % count */
/* in libpcmx_hip: device buffers staged through host memory over TCP — several ranks may share one GPU
 * (single-GPU test fixture for the multi-rank device path; not a performance path) */
int pcmx_comm_init_env_staged(pcmx_comm_t** out);
void pcmx_comm_destroy(pcmx_comm_t* c);
int pcmx_env_port(void);

/* ---- generic API (dispatches through c->ops) */
int pcmx_comm_group_start(pcmx_comm_t* c);
int pcmx_comm_group_end(pcmx_comm_t* c);
int pcmx_comm_send(pcmx_comm_t* c, const void* buf, size_t bytes, int peer);
int pcmx_comm_recv(pcmx_comm_t* c, void* buf, size_t bytes, int peer);
int pcmx_comm_allreduce(pcmx_comm_t* c, void* buf, size_t count, int dtype, int op);
int pcmx_comm_bcast(pcmx_comm_t* c, void* buf, size_t bytes, int root);
int pcmx_comm_sync(pcmx_comm_t* c);
int pcmx_comm_barrier(pcmx_comm_t* c); /* host side-channel barrier (after sync) */
/* MPI_Allgather / Gather / Scatter / Alltoall of `bytes` per rank (recv of allgather/gather/alltoall and send
 * of scatter/alltoall hold world blocks in rank order; the root-only buffers may be NULL elsewhere). In place:
 * allgather with send == recv + rank * bytes, scatter with recv == send + root * bytes on the root. */
int pcmx_comm_allgather(pcmx_comm_t* c, const void* send, void* recv, size_t bytes);
int pcmx_comm_gather(pcmx_comm_t* c, const void* send, void* recv, size_t bytes, int root);
int pcmx_comm_scatter(pcmx_comm_t* c, const void* send, void* recv, size_t bytes, int root);
int pcmx_comm_alltoall(pcmx_comm_t* c, const void* send, void* recv, size_t bytes);

/* point-to-point implementations of the collectives above for transports without native ones; `copy` moves a
 * block between two of the transport's own buffers (memmove for host memory, a device copy for the staged
 * transport) */
typedef int (*pcmx_copy_fn)(pcmx_comm_t* c, void* dst, const void* src, size_t bytes);
int pcmx_p2p_allgather(pcmx_comm_t* c, const void* send, void* recv, size_t bytes, pcmx_copy_fn copy);
int pcmx_p2p_gather(pcmx_comm_t* c, const void* send, void* recv, size_t bytes, int root, pcmx_copy_fn copy);
int pcmx_p2p_scatter(pcmx_comm_t* c, const void* send, void* recv, size_t bytes, int root, pcmx_copy_fn copy);
int pcmx_p2p_alltoall(pcmx_comm_t* c, const void* send, void* recv, size_t bytes, pcmx_copy_fn copy);

/* ---- Cartesian topology (MPI_Dims_create / Cart_create(reorder=0) / Cart_coords / Cart_shift) */
typedef struct {
    int size;
    int dims[2];
} pcmx_cart_t;
void pcmx_dims_create(int nnodes, int dims[2]);
void pcmx_cart_init(pcmx_cart_t* t, int size, const int* dims /* NULL = balanced */);
void pcmx_cart_coords(const pcmx_cart_t* t, int rank, int* row, int* col);
int pcmx_cart_rank(const pcmx_cart_t* t, int row, int col); /* -1 outside */
void pcmx_cart_neighbours(const pcmx_cart_t* t, int rank, int nb[4]); /* north, south, west, east */
void pcmx_cart_tile(const pcmx_cart_t* t, int rank, int height, int width, int out[4]); /* r0 r1 c0 c1 */

/* ---- data-movement backend of the distributed 2-D region growing (host or device memory) */
typedef struct pcmx_region_backend {
    void* (*alloc)(size_t bytes, void* ctx);
    void (*release)(void* p, void* ctx);
    int (*memset0)(void* p, size_t bytes, void* ctx);
    int (*h2d)(void* dst, const void* src, size_t bytes, void* ctx);
    int (*d2h)(void* dst, const void* src, size_t bytes, void* ctx);
    int (*copy2d)(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width, size_t height, void* ctx);
    /* grow a padded (h+2)x(w+2) region tile to its local fixpoint; halo cells are read-only seeds */
    int (*grow)(unsigned char* region_p, const unsigned char* img_p, int h, int w, int threshold, void* ctx);
    int (*pack)(const unsigned char* tile_p, int h, int w, unsigned char* buf, void* ctx);    /* 2w+2h bytes */
    int (*unpack)(unsigned char* tile_p, int h, int w, const unsigned char* buf, int mask, void* ctx);
    /* unpack + set *changed_flag (backend memory) to 1 when any halo cell takes a new value */
    int (*unpack_changed)(unsigned char* tile_p, int h, int w, const unsigned char* buf, int mask, int* changed_flag,
                          void* ctx);
    int (*sync)(void* ctx);
    void* ctx;
    void* stream; /* hipStream_t the backend issues its kernels/copies on (NULL: host backend). When it is the
                   * communicator's stream (RCCL / staged transports), packs and sends are stream-ordered and
                   * the exchange needs no host synchronisation. */
} pcmx_region_backend_t;

#define PCMX_REGION_CHECK_EVERY 2
void pcmx_region_backend_host(pcmx_region_backend_t* be);
int pcmx_region_backend_hip(pcmx_region_backend_t* be, void* stream); /* in libpcmx_hip */

/* Distributed seeded region growing over the Cartesian grid of `c` (ref region.c:582-604).
 * Termination is device-resident: the unpack kernel raises a "halo changed" flag in backend memory, the flag is
 * MAX-all-reduced in place and read by the host once every PCMX_REGION_CHECK_EVERY outer steps.
 * image: H*W bytes on root (host memory; ignored elsewhere); region_out: H*W bytes on root (host).
 * dims: process grid or NULL. stats (optional): [outer_steps, local_grow_calls]. Returns 0 on success. */
int pcmx_region2d_distributed(pcmx_comm_t* c, const pcmx_region_backend_t* be, const unsigned char* image, int H,
                              int W, int threshold, const int* dims, unsigned char* region_out, int* stats);

/* Token chain of ref 1-introduction/mpi.c (prints "Rank %d received %d \n" / "Rank %d sent %d \n");
 * token_buf: 4 bytes in the transport's memory space. Returns the final token value on this rank. */
int pcmx_token_ring(pcmx_comm_t* c, void* token_buf, const pcmx_region_backend_t* be, int verbose);

/* ---- distributed reduce / scan over device vectors split across the ranks (libpcmx_hip; RCCL or staged
 * transport, stream-ordered on c->stream). ws: pcmx_dist_workspace_bytes(n_local, world) bytes of device memory.
 * reduce: *out (device) = op over every rank's x (op = PCMX_OP_SUM / MIN / MAX of pcmx_hip.h).
 * scan: out = inclusive/exclusive prefix of the GLOBAL vector (rank order); err_flag as in pcmx_scan_f32. */
long long pcmx_dist_workspace_bytes(long long n_local, int world);
int pcmx_reduce_distributed(pcmx_comm_t* c, const float* x, long long n_local, int op, float* out, void* ws);
int pcmx_scan_distributed(pcmx_comm_t* c, const float* x, float* out, long long n_local, int exclusive, void* ws,
                          unsigned* err_flag);

/* host flood fill on a padded tile (CPU backend of `grow`) */
void pcmx_region2d_padded_host(unsigned char* region_p, const unsigned char* img_p, int h, int w, int threshold);

#ifdef __cplusplus
}
#endif
#endif
