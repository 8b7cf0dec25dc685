/* TCP transport + generic dispatch + Cartesian topology of the native comm layer (pcmx_comm.h).
 *
 * Bootstrap: rank 0 listens on MASTER_ADDR:port; every other rank opens its own listener, connects to
 * rank 0 and reports (rank, port); rank 0 replies with the whole (ip, port) table; then each rank i >= 1
 * connects to every lower rank j >= 1 and accepts from every higher one -> a full mesh of sockets with
 * TCP_NODELAY. Rank 0's bootstrap sockets are the mesh links to rank 0.
 *
 * Point-to-point semantics: a group (group_start .. group_end) queues sends/receives and completes them
 * together with a poll()-driven progress loop over non-blocking sockets, so any exchange pattern (all ranks
 * sending before receiving, large tiles) completes without relying on socket buffering — the deadlock-free
 * replacement of the reference's parity-ordered blocking MPI_Send/Recv. A lone send/recv
 * is a group of one. Per peer, messages are matched in posting order (byte stream per direction).
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include "pcmx_comm.h"

typedef struct {
    int is_send;
    char* buf;
    size_t bytes, done;
    int peer;
} tcp_op_t;

typedef struct {
    int* fd;  /* fd[peer], -1 for self */
    int in_group;
    tcp_op_t* ops;
    int nops, cap;
} tcp_impl_t;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static int set_opts(int fd) {
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    int big = 4 << 20;
    setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &big, sizeof big);
    setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &big, sizeof big);
    return 0;
}

static int write_all(int fd, const void* p, size_t n) {
    const char* c = (const char*)p;
    while (n) {
        ssize_t k = write(fd, c, n);
        if (k < 0) {
            if (errno == EINTR || errno == EAGAIN) continue;
            return PCMX_ERR_COMM;
        }
        c += k, n -= (size_t)k;
    }
    return 0;
}

static int read_all(int fd, void* p, size_t n) {
    char* c = (char*)p;
    while (n) {
        ssize_t k = read(fd, c, n);
        if (k == 0) return PCMX_ERR_COMM;
        if (k < 0) {
            if (errno == EINTR || errno == EAGAIN) continue;
            return PCMX_ERR_COMM;
        }
        c += k, n -= (size_t)k;
    }
    return 0;
}

static int listen_on(const char* addr, int port, int* bound_port) {
    int fd = socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) return PCMX_ERR_COMM;
    int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    struct sockaddr_in sa;
    memset(&sa, 0, sizeof sa);
    sa.sin_family = AF_INET;
    sa.sin_port = htons((uint16_t)port);
    sa.sin_addr.s_addr = addr ? inet_addr(addr) : htonl(INADDR_ANY);
    if (bind(fd, (struct sockaddr*)&sa, sizeof sa) || listen(fd, 256)) {
        close(fd);
        return PCMX_ERR_COMM;
    }
    socklen_t len = sizeof sa;
    getsockname(fd, (struct sockaddr*)&sa, &len);
    if (bound_port) *bound_port = ntohs(sa.sin_port);
    return fd;
}

static int connect_retry(uint32_t ip_be, int port, double timeout_s) {
    const double t0 = now_s();
    for (;;) {
        int fd = socket(AF_INET, SOCK_STREAM, 0);
        struct sockaddr_in sa;
        memset(&sa, 0, sizeof sa);
        sa.sin_family = AF_INET;
        sa.sin_port = htons((uint16_t)port);
        sa.sin_addr.s_addr = ip_be;
        if (connect(fd, (struct sockaddr*)&sa, sizeof sa) == 0) {
            set_opts(fd);
            return fd;
        }
        close(fd);
        if (now_s() - t0 > timeout_s) return PCMX_ERR_COMM;
        usleep(20000);
    }
}

/* ------------------------------------------------------------------ transport ops */

static int tcp_push(pcmx_comm_t* c, int is_send, void* buf, size_t bytes, int peer) {
    tcp_impl_t* t = (tcp_impl_t*)c->impl;
    if (peer < 0 || peer >= c->world) return PCMX_ERR_ARG;
    if (t->nops == t->cap) {
        const int cap = t->cap ? 2 * t->cap : 16;
        tcp_op_t* ops = (tcp_op_t*)realloc(t->ops, sizeof(tcp_op_t) * (size_t)cap);
        if (!ops) return PCMX_ERR_ALLOC;
        t->ops = ops, t->cap = cap;
    }
    t->ops[t->nops++] = (tcp_op_t){is_send, (char*)buf, bytes, 0, peer};
    return 0;
}

static int tcp_progress(pcmx_comm_t* c) {
    tcp_impl_t* t = (tcp_impl_t*)c->impl;
    const int W = c->world;
    int rc = 0;
    /* self messages: match k-th send to self with k-th recv from self; a size mismatch or an op without a
     * partner is an error (the group is dropped either way, so no stale op survives into the next group) */
    for (int i = 0; i < t->nops && !rc; ++i) {
        tcp_op_t* s = &t->ops[i];
        if (!s->is_send || s->peer != c->rank || s->done == s->bytes + 1) continue;
        int matched = 0;
        for (int j = 0; j < t->nops; ++j) {
            tcp_op_t* r = &t->ops[j];
            if (r->is_send || r->peer != c->rank || r->done == r->bytes + 1) continue;
            if (r->bytes != s->bytes) {
                rc = PCMX_ERR_ARG; /* size mismatch of a send/recv-to-self pair */
                break;
            }
            memcpy(r->buf, s->buf, s->bytes);
            s->done = s->bytes + 1, r->done = r->bytes + 1; /* mark complete */
            matched = 1;
            break;
        }
        if (!matched && !rc) rc = PCMX_ERR_ARG; /* send to self without a recv from self */
    }
    for (int i = 0; i < t->nops && !rc; ++i) /* recv from self without a send to self */
        if (!t->ops[i].is_send && t->ops[i].peer == c->rank && t->ops[i].done != t->ops[i].bytes + 1)
            rc = PCMX_ERR_ARG;
    if (rc) {
        t->nops = 0;
        return rc;
    }
    struct pollfd* pf = (struct pollfd*)calloc((size_t)2 * W, sizeof(struct pollfd));
    if (!pf) {
        t->nops = 0;
        return PCMX_ERR_ALLOC;
    }
    double t_start = now_s(); /* deadline: 60 s without progress */
    const double t_limit = 60.0;
    for (;;) {
        int npf = 0, pending = 0;
        /* head-of-line op per (peer, direction) */
        for (int p = 0; p < W; ++p) {
            if (p == c->rank) continue;
            for (int dir = 0; dir < 2; ++dir) {
                tcp_op_t* head = NULL;
                for (int i = 0; i < t->nops; ++i) {
                    tcp_op_t* o = &t->ops[i];
                    if (o->peer == p && o->is_send == dir && o->done < o->bytes) {
                        head = o;
                        break;
                    }
                    if (o->peer == p && o->is_send == dir && o->bytes == 0) o->done = 1;
                }
                if (!head) continue;
                ++pending;
                pf[npf].fd = t->fd[p];
                pf[npf].events = dir ? POLLOUT : POLLIN;
                pf[npf].revents = 0;
                ++npf;
            }
        }
        if (!pending) break;
        const int left_ms = (int)((t_limit - (now_s() - t_start)) * 1e3);
        int k = left_ms > 0 ? poll(pf, (nfds_t)npf, left_ms) : 0;
        if (k < 0 && errno == EINTR) continue; /* a signal is not a transport failure: retry, same deadline */
        if (k <= 0) {
            rc = k == 0 ? PCMX_ERR_TIMEOUT : PCMX_ERR_COMM; /* no progress for t_limit / poll() failed */
            break;
        }
        t_start = now_s();
        for (int q = 0; q < npf; ++q) {
            if (!pf[q].revents) continue;
            int p = -1;
            for (int r = 0; r < W; ++r)
                if (t->fd[r] == pf[q].fd) p = r;
            const int dir = pf[q].events == POLLOUT;
            for (int i = 0; i < t->nops; ++i) {
                tcp_op_t* o = &t->ops[i];
                if (o->peer != p || o->is_send != dir || o->done >= o->bytes) continue;
                ssize_t n = dir ? send(pf[q].fd, o->buf + o->done, o->bytes - o->done, MSG_DONTWAIT | MSG_NOSIGNAL)
                                : recv(pf[q].fd, o->buf + o->done, o->bytes - o->done, MSG_DONTWAIT);
                if (n > 0) o->done += (size_t)n;
                else if (n == 0 && !dir) rc = PCMX_ERR_COMM; /* peer closed */
                else if (n < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) rc = PCMX_ERR_COMM;
                break;
            }
            if (rc) break;
        }
        if (rc) break;
    }
    free(pf);
    t->nops = 0;
    return rc;
}

static int tcp_group_start(pcmx_comm_t* c) {
    ((tcp_impl_t*)c->impl)->in_group++;
    return 0;
}
static int tcp_group_end(pcmx_comm_t* c) {
    tcp_impl_t* t = (tcp_impl_t*)c->impl;
    if (t->in_group <= 0) return PCMX_ERR_ARG;
    if (--t->in_group == 0) return tcp_progress(c);
    return 0;
}
static int tcp_send(pcmx_comm_t* c, const void* buf, size_t bytes, int peer) {
    int rc = tcp_push(c, 1, (void*)buf, bytes, peer);
    if (rc || ((tcp_impl_t*)c->impl)->in_group) return rc;
    return tcp_progress(c);
}
static int tcp_recv(pcmx_comm_t* c, void* buf, size_t bytes, int peer) {
    int rc = tcp_push(c, 0, buf, bytes, peer);
    if (rc || ((tcp_impl_t*)c->impl)->in_group) return rc;
    return tcp_progress(c);
}

static size_t dsize(int dtype) {
    switch (dtype) {
        case PCMX_I32: case PCMX_F32: return 4;
        case PCMX_F64: case PCMX_I64: return 8;
        default: return 1;
    }
}

#define RED(T)                                                                                  \
    do {                                                                                        \
        T* d = (T*)dst;                                                                         \
        const T* s = (const T*)src;                                                             \
        for (size_t i = 0; i < n; ++i)                                                          \
            d[i] = op == PCMX_SUM ? d[i] + s[i] : op == PCMX_MIN ? (s[i] < d[i] ? s[i] : d[i])  \
                                                              : (s[i] > d[i] ? s[i] : d[i]);    \
    } while (0)

static void reduce_into(void* dst, const void* src, size_t n, int dtype, int op) {
    switch (dtype) {
        case PCMX_I32: RED(int); break;
        case PCMX_F32: RED(float); break;
        case PCMX_F64: RED(double); break;
        case PCMX_I64: RED(long long); break;
        default: RED(unsigned char); break;
    }
}

/* reduce to rank 0 (rank order, deterministic), then broadcast */
static int tcp_allreduce(pcmx_comm_t* c, void* buf, size_t count, int dtype, int op) {
    const size_t bytes = count * dsize(dtype);
    if (c->world == 1) return 0;
    if (c->rank == 0) {
        void* tmp = malloc(bytes ? bytes : 1);
        for (int r = 1; r < c->world; ++r) {
            int rc = tcp_recv(c, tmp, bytes, r);
            if (rc) {
                free(tmp);
                return rc;
            }
            reduce_into(buf, tmp, count, dtype, op);
        }
        free(tmp);
    } else {
        int rc = tcp_send(c, buf, bytes, 0);
        if (rc) return rc;
    }
    return c->ops->bcast(c, buf, bytes, 0);
}

static int tcp_bcast(pcmx_comm_t* c, void* buf, size_t bytes, int root) {
    if (c->world == 1) return 0;
    if (c->rank == root) {
        tcp_group_start(c);
        for (int r = 0; r < c->world; ++r)
            if (r != root) tcp_send(c, buf, bytes, r);
        return tcp_group_end(c);
    }
    return tcp_recv(c, buf, bytes, root);
}

static int tcp_sync(pcmx_comm_t* c) {
    (void)c;
    return 0;
}

static void tcp_destroy(pcmx_comm_t* c) {
    tcp_impl_t* t = (tcp_impl_t*)c->impl;
    if (t) {
        for (int r = 0; r < c->world; ++r)
            if (t->fd[r] >= 0) close(t->fd[r]);
        free(t->fd);
        free(t->ops);
        free(t);
    }
    free(c);
}

/* ------------------------------------------------------------------ collectives over point-to-point */
/* One grouped round: every peer's block moves at once (TCP: all sockets progress together in tcp_progress; staged:
 * one host round trip for the whole group). `copy` handles the rank's own block. */
static char* blk(const void* base, size_t i, size_t bytes) { return (char*)base + i * bytes; }

int pcmx_p2p_allgather(pcmx_comm_t* c, const void* send, void* recv, size_t bytes, pcmx_copy_fn copy) {
    int rc = 0;
    if (send != blk(recv, c->rank, bytes)) rc = copy(c, blk(recv, c->rank, bytes), send, bytes);
    if (rc || c->world == 1) return rc;
    c->ops->group_start(c);
    for (int p = 0; p < c->world && !rc; ++p) {
        if (p == c->rank) continue;
        rc = c->ops->send(c, blk(recv, c->rank, bytes), bytes, p);
        if (!rc) rc = c->ops->recv(c, blk(recv, p, bytes), bytes, p);
    }
    const int rc2 = c->ops->group_end(c);
    return rc ? rc : rc2;
}

int pcmx_p2p_gather(pcmx_comm_t* c, const void* send, void* recv, size_t bytes, int root, pcmx_copy_fn copy) {
    if (root < 0 || root >= c->world) return -1;
    if (c->rank != root) return c->ops->send(c, send, bytes, root);
    int rc = send != blk(recv, root, bytes) ? copy(c, blk(recv, root, bytes), send, bytes) : 0;
    if (rc || c->world == 1) return rc;
    c->ops->group_start(c);
    for (int p = 0; p < c->world && !rc; ++p)
        if (p != root) rc = c->ops->recv(c, blk(recv, p, bytes), bytes, p);
    const int rc2 = c->ops->group_end(c);
    return rc ? rc : rc2;
}

int pcmx_p2p_scatter(pcmx_comm_t* c, const void* send, void* recv, size_t bytes, int root, pcmx_copy_fn copy) {
    if (root < 0 || root >= c->world) return -1;
    if (c->rank != root) return c->ops->recv(c, recv, bytes, root);
    int rc = recv != blk(send, root, bytes) ? copy(c, recv, blk(send, root, bytes), bytes) : 0;
    if (rc || c->world == 1) return rc;
    c->ops->group_start(c);
    for (int p = 0; p < c->world && !rc; ++p)
        if (p != root) rc = c->ops->send(c, blk(send, p, bytes), bytes, p);
    const int rc2 = c->ops->group_end(c);
    return rc ? rc : rc2;
}

int pcmx_p2p_alltoall(pcmx_comm_t* c, const void* send, void* recv, size_t bytes, pcmx_copy_fn copy) {
    if (send == recv) return -1; /* out of place only */
    int rc = copy(c, blk(recv, c->rank, bytes), blk(send, c->rank, bytes), bytes);
    if (rc || c->world == 1) return rc;
    c->ops->group_start(c);
    for (int p = 0; p < c->world && !rc; ++p) {
        if (p == c->rank) continue;
        rc = c->ops->send(c, blk(send, p, bytes), bytes, p);
        if (!rc) rc = c->ops->recv(c, blk(recv, p, bytes), bytes, p);
    }
    const int rc2 = c->ops->group_end(c);
    return rc ? rc : rc2;
}

static int host_copy(pcmx_comm_t* c, void* dst, const void* src, size_t bytes) {
    (void)c;
    memmove(dst, src, bytes);
    return 0;
}
static int tcp_allgather(pcmx_comm_t* c, const void* s, void* r, size_t n) { return pcmx_p2p_allgather(c, s, r, n, host_copy); }
static int tcp_gather(pcmx_comm_t* c, const void* s, void* r, size_t n, int root) {
    return pcmx_p2p_gather(c, s, r, n, root, host_copy);
}
static int tcp_scatter(pcmx_comm_t* c, const void* s, void* r, size_t n, int root) {
    return pcmx_p2p_scatter(c, s, r, n, root, host_copy);
}
static int tcp_alltoall(pcmx_comm_t* c, const void* s, void* r, size_t n) { return pcmx_p2p_alltoall(c, s, r, n, host_copy); }

static const pcmx_comm_ops_t kTcpOps = {tcp_group_start, tcp_group_end, tcp_send,      tcp_recv,
                                        tcp_allreduce,   tcp_bcast,     tcp_sync,      tcp_destroy,
                                        tcp_allgather,   tcp_gather,    tcp_scatter,   tcp_alltoall};

/* ------------------------------------------------------------------ bootstrap */

typedef struct {
    uint32_t ip;
    int32_t port;
} endpoint_t;

int pcmx_comm_init_tcp(int rank, int world, const char* addr, int port, pcmx_comm_t** out) {
    *out = NULL;
    if (world < 1 || rank < 0 || rank >= world) return -1;
    pcmx_comm_t* c = (pcmx_comm_t*)calloc(1, sizeof *c);
    tcp_impl_t* t = (tcp_impl_t*)calloc(1, sizeof *t);
    c->rank = rank, c->world = world, c->local_rank = rank, c->transport = PCMX_TRANSPORT_TCP;
    c->ops = &kTcpOps, c->impl = t, c->host = c;
    t->fd = (int*)malloc(sizeof(int) * (size_t)world);
    for (int i = 0; i < world; ++i) t->fd[i] = -1;
    *out = c;
    if (world == 1) return 0;
    const char* a = addr ? addr : "127.0.0.1";
    struct addrinfo hints, *res = NULL;
    memset(&hints, 0, sizeof hints);
    hints.ai_family = AF_INET;
    if (getaddrinfo(a, NULL, &hints, &res) || !res) return PCMX_ERR_COMM;
    const uint32_t master_ip = ((struct sockaddr_in*)res->ai_addr)->sin_addr.s_addr;
    freeaddrinfo(res);
    endpoint_t* table = (endpoint_t*)calloc((size_t)world, sizeof(endpoint_t));
    int rc = 0;
    if (rank == 0) {
        int lfd = listen_on(NULL, port, NULL);
        if (lfd < 0) return PCMX_ERR_COMM;
        for (int k = 1; k < world; ++k) {
            struct sockaddr_in peer;
            socklen_t len = sizeof peer;
            int fd = accept(lfd, (struct sockaddr*)&peer, &len);
            if (fd < 0) return PCMX_ERR_COMM;
            set_opts(fd);
            int32_t hello[2];
            if (read_all(fd, hello, sizeof hello)) return PCMX_ERR_COMM;
            if (hello[0] <= 0 || hello[0] >= world) return PCMX_ERR_COMM;
            t->fd[hello[0]] = fd;
            table[hello[0]].ip = peer.sin_addr.s_addr;
            table[hello[0]].port = hello[1];
        }
        close(lfd);
        for (int r = 1; r < world; ++r)
            if (write_all(t->fd[r], table, sizeof(endpoint_t) * (size_t)world)) return PCMX_ERR_COMM;
    } else {
        int my_port = 0;
        int lfd = listen_on(NULL, 0, &my_port);
        if (lfd < 0) return PCMX_ERR_COMM;
        int fd0 = connect_retry(master_ip, port, 120.0);
        if (fd0 < 0) return PCMX_ERR_COMM;
        int32_t hello[2] = {rank, my_port};
        if (write_all(fd0, hello, sizeof hello)) return PCMX_ERR_COMM;
        if (read_all(fd0, table, sizeof(endpoint_t) * (size_t)world)) return PCMX_ERR_COMM;
        t->fd[0] = fd0;
        /* connect to lower ranks >= 1, then accept from higher ranks */
        for (int j = 1; j < rank; ++j) {
            int fd = connect_retry(table[j].ip, table[j].port, 120.0);
            if (fd < 0) return PCMX_ERR_COMM;
            int32_t me = rank;
            if (write_all(fd, &me, sizeof me)) return PCMX_ERR_COMM;
            t->fd[j] = fd;
        }
        for (int k = rank + 1; k < world; ++k) {
            int fd = accept(lfd, NULL, NULL);
            if (fd < 0) return PCMX_ERR_COMM;
            set_opts(fd);
            int32_t who;
            if (read_all(fd, &who, sizeof who) || who <= rank || who >= world) return PCMX_ERR_COMM;
            t->fd[who] = fd;
        }
        close(lfd);
    }
    free(table);
    for (int r = 0; r < world; ++r)
        if (r != rank) fcntl(t->fd[r], F_SETFL, fcntl(t->fd[r], F_GETFL) | O_NONBLOCK);
    return rc;
}

static int env_int(const char* name, int dflt) {
    const char* v = getenv(name);
    return v && *v ? atoi(v) : dflt;
}

int pcmx_env_port(void) {
    /* under torchrun, MASTER_PORT is taken by its own store: bootstrap one port above */
    const int p = env_int("PCMX_PORT", 0);
    if (p) return p;
    return env_int("MASTER_PORT", 29500) + (getenv("TORCHELASTIC_RUN_ID") ? 1 : 0);
}

int pcmx_comm_init_env_tcp(pcmx_comm_t** out) {
    const int rank = env_int("RANK", 0), world = env_int("WORLD_SIZE", 1);
    const char* addr = getenv("MASTER_ADDR");
    int rc = pcmx_comm_init_tcp(rank, world, addr ? addr : "127.0.0.1", pcmx_env_port(), out);
    if (*out) (*out)->local_rank = env_int("LOCAL_RANK", rank);
    return rc;
}

/* ------------------------------------------------------------------ generic API */

void pcmx_comm_destroy(pcmx_comm_t* c) {
    if (c) c->ops->destroy(c);
}
int pcmx_comm_group_start(pcmx_comm_t* c) { return pcmx_comm_rc(c->ops->group_start(c)); }
int pcmx_comm_group_end(pcmx_comm_t* c) { return pcmx_comm_rc(c->ops->group_end(c)); }
int pcmx_comm_send(pcmx_comm_t* c, const void* b, size_t n, int p) { return pcmx_comm_rc(c->ops->send(c, b, n, p)); }
int pcmx_comm_recv(pcmx_comm_t* c, void* b, size_t n, int p) { return pcmx_comm_rc(c->ops->recv(c, b, n, p)); }
int pcmx_comm_allreduce(pcmx_comm_t* c, void* b, size_t n, int dt, int op) { return pcmx_comm_rc(c->ops->allreduce(c, b, n, dt, op)); }
int pcmx_comm_bcast(pcmx_comm_t* c, void* b, size_t n, int root) { return pcmx_comm_rc(c->ops->bcast(c, b, n, root)); }
int pcmx_comm_sync(pcmx_comm_t* c) { return pcmx_comm_rc(c->ops->sync(c)); }
int pcmx_comm_allgather(pcmx_comm_t* c, const void* s, void* r, size_t n) { return pcmx_comm_rc(c->ops->allgather(c, s, r, n)); }
int pcmx_comm_gather(pcmx_comm_t* c, const void* s, void* r, size_t n, int root) { return pcmx_comm_rc(c->ops->gather(c, s, r, n, root)); }
int pcmx_comm_scatter(pcmx_comm_t* c, const void* s, void* r, size_t n, int root) {
    return pcmx_comm_rc(c->ops->scatter(c, s, r, n, root));
}
int pcmx_comm_alltoall(pcmx_comm_t* c, const void* s, void* r, size_t n) { return pcmx_comm_rc(c->ops->alltoall(c, s, r, n)); }
int pcmx_comm_barrier(pcmx_comm_t* c) {
    int rc = c->ops->sync(c);
    if (rc) return pcmx_comm_rc(rc);
    int one = 1;
    return pcmx_comm_rc(c->host->ops->allreduce(c->host, &one, 1, PCMX_I32, PCMX_SUM));
}

/* ------------------------------------------------------------------ Cartesian topology */

void pcmx_dims_create(int n, int dims[2]) {
    /* balanced factorisation, non-increasing (MPI_Dims_create): largest prime factors first, each onto
     * the currently smallest dimension */
    int f[64], nf = 0, m = n;
    for (int p = 2; (long long)p * p <= m; ++p)
        while (m % p == 0) f[nf++] = p, m /= p;
    if (m > 1) f[nf++] = m;
    dims[0] = dims[1] = 1;
    for (int i = nf - 1; i >= 0; --i) {
        const int k = dims[0] <= dims[1] ? 0 : 1;
        dims[k] *= f[i];
    }
    if (dims[0] < dims[1]) {
        int t = dims[0];
        dims[0] = dims[1], dims[1] = t;
    }
}

void pcmx_cart_init(pcmx_cart_t* t, int size, const int* dims) {
    t->size = size;
    if (dims) t->dims[0] = dims[0], t->dims[1] = dims[1];
    else pcmx_dims_create(size, t->dims);
}

void pcmx_cart_coords(const pcmx_cart_t* t, int rank, int* row, int* col) {
    *row = rank / t->dims[1];
    *col = rank % t->dims[1];
}

int pcmx_cart_rank(const pcmx_cart_t* t, int row, int col) {
    if (row < 0 || col < 0 || row >= t->dims[0] || col >= t->dims[1]) return -1;
    return row * t->dims[1] + col;
}

void pcmx_cart_neighbours(const pcmx_cart_t* t, int rank, int nb[4]) {
    int r, c;
    pcmx_cart_coords(t, rank, &r, &c);
    nb[0] = pcmx_cart_rank(t, r - 1, c);
    nb[1] = pcmx_cart_rank(t, r + 1, c);
    nb[2] = pcmx_cart_rank(t, r, c - 1);
    nb[3] = pcmx_cart_rank(t, r, c + 1);
}

static void split_block(int n, int parts, int i, int* s, int* e) {
    const int q = n / parts, rem = n % parts;
    *s = i * q + (i < rem ? i : rem);
    *e = *s + q + (i < rem ? 1 : 0);
}

void pcmx_cart_tile(const pcmx_cart_t* t, int rank, int height, int width, int out[4]) {
    int r, c;
    pcmx_cart_coords(t, rank, &r, &c);
    split_block(height, t->dims[0], r, &out[0], &out[1]);
    split_block(width, t->dims[1], c, &out[2], &out[3]);
}
