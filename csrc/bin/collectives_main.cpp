/* bin/collectives [--cpu | --staged] [--bytes N] [--n-local N] [--bench]
 * Self-check (and optional bandwidth run) of the native collectives of pcmx_comm.h — MPI_Allgather / Gather /
 * Scatter / Alltoall (ref 2-mpi-region-growing/region.c:106-143,391-432 use their scatter/gather and all-reduce
 * ancestors) — and of the distributed reduce / prefix scan built on them (north-star NS3). Buffers live in GPU
 * memory moved by RCCL over xGMI (default), in GPU memory staged through host TCP (--staged; ranks may share a
 * GPU) or in host memory over TCP (--cpu; no GPU, no reduce/scan). Every rank checks its buffers byte for byte
 * (reduce/scan on small integers, so the f32 results are exact) and prints one line; rank 0 ends with
 * "collectives ok world=P". --bench (RCCL) adds the all-gather / all-to-all bus bandwidth at 64 MiB per rank.
 * Launch with `pcmx_launch -n P` or torchrun. */
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "pcmx_comm.h"
#include "pcmx_hip.h"

namespace {
int mode = PCMX_TRANSPORT_RCCL;
pcmx_comm_t* comm = nullptr;

unsigned char pat(int a, int b, size_t i, int k) { return (unsigned char)(a * 31 + b * 17 + i * 7 + k * 101); }

void* alloc(size_t n) {
    void* p = nullptr;
    if (mode == PCMX_TRANSPORT_TCP) return malloc(n ? n : 1);
    return hipMalloc(&p, n ? n : 1) == hipSuccess ? p : nullptr;
}
void release(void* p) {
    if (mode == PCMX_TRANSPORT_TCP) free(p);
    else hipFree(p);
}
void put(void* dst, const void* src, size_t n) {
    if (mode == PCMX_TRANSPORT_TCP) memcpy(dst, src, n);
    else hipMemcpy(dst, src, n, hipMemcpyHostToDevice);
}
void get(void* dst, const void* src, size_t n) {
    pcmx_comm_sync(comm);
    if (mode == PCMX_TRANSPORT_TCP) memcpy(dst, src, n);
    else hipMemcpy(dst, src, n, hipMemcpyDeviceToHost);
}

int fail(const char* what, int rc) {
    fprintf(stderr, "rank %d: %s failed (%d)\n", comm->rank, what, rc);
    return 1;
}

// blocks of `bytes` per rank through every collective; returns 0 when all match
int check_collectives(size_t bytes) {
    const int P = comm->world, R = comm->rank;
    std::vector<unsigned char> h(bytes * P), got(bytes * P);
    void* send = alloc(bytes * P);
    void* recv = alloc(bytes * P);
    if (!send || !recv) return fail("alloc", -1);
    int rc, bad = 0;
    // allgather
    for (size_t i = 0; i < bytes; ++i) h[i] = pat(R, 0, i, 0);
    put(send, h.data(), bytes);
    if ((rc = pcmx_comm_allgather(comm, send, recv, bytes))) return fail("allgather", rc);
    get(got.data(), recv, bytes * P);
    for (int p = 0; p < P; ++p)
        for (size_t i = 0; i < bytes; ++i) bad += got[p * bytes + i] != pat(p, 0, i, 0);
    if (bad) return fail("allgather check", bad);
    // allgather in place (send = own block of recv)
    for (size_t i = 0; i < bytes; ++i) h[i] = pat(R, 0, i, 5);
    put(static_cast<char*>(recv) + R * bytes, h.data(), bytes);
    if ((rc = pcmx_comm_allgather(comm, static_cast<char*>(recv) + R * bytes, recv, bytes))) return fail("allgather in place", rc);
    get(got.data(), recv, bytes * P);
    for (int p = 0; p < P; ++p)
        for (size_t i = 0; i < bytes; ++i) bad += got[p * bytes + i] != pat(p, 0, i, 5);
    if (bad) return fail("allgather in-place check", bad);
    // gather to the last rank
    const int groot = P - 1;
    for (size_t i = 0; i < bytes; ++i) h[i] = pat(R, 1, i, 1);
    put(send, h.data(), bytes);
    if ((rc = pcmx_comm_gather(comm, send, R == groot ? recv : nullptr, bytes, groot))) return fail("gather", rc);
    if (R == groot) {
        get(got.data(), recv, bytes * P);
        for (int p = 0; p < P; ++p)
            for (size_t i = 0; i < bytes; ++i) bad += got[p * bytes + i] != pat(p, 1, i, 1);
        if (bad) return fail("gather check", bad);
    }
    // scatter from rank 0
    if (R == 0) {
        for (int p = 0; p < P; ++p)
            for (size_t i = 0; i < bytes; ++i) h[p * bytes + i] = pat(p, 2, i, 2);
        put(send, h.data(), bytes * P);
    }
    if ((rc = pcmx_comm_scatter(comm, R == 0 ? send : nullptr, recv, bytes, 0))) return fail("scatter", rc);
    get(got.data(), recv, bytes);
    for (size_t i = 0; i < bytes; ++i) bad += got[i] != pat(R, 2, i, 2);
    if (bad) return fail("scatter check", bad);
    // all-to-all: block p of rank R's send goes to rank p
    for (int p = 0; p < P; ++p)
        for (size_t i = 0; i < bytes; ++i) h[p * bytes + i] = pat(R, p, i, 3);
    put(send, h.data(), bytes * P);
    if ((rc = pcmx_comm_alltoall(comm, send, recv, bytes))) return fail("alltoall", rc);
    get(got.data(), recv, bytes * P);
    for (int p = 0; p < P; ++p)
        for (size_t i = 0; i < bytes; ++i) bad += got[p * bytes + i] != pat(p, R, i, 3);
    if (bad) return fail("alltoall check", bad);
    release(send);
    release(recv);
    return 0;
}

// global vector of small integers x[g] = (g * 7) % 5 - 2 split raggedly over the ranks
int check_reduce_scan(long long n_base) {
    const int P = comm->world, R = comm->rank;
    std::vector<long long> cnt(P), off(P + 1, 0);
    for (int p = 0; p < P; ++p) cnt[p] = n_base + 37LL * p * (p % 2 ? -1 : 1), off[p + 1] = off[p] + cnt[p];
    const long long n = cnt[R], g0 = off[R];
    std::vector<float> h(n), got(n);
    for (long long i = 0; i < n; ++i) h[i] = (float)(((g0 + i) * 7) % 5 - 2);
    float *x, *y, *red;
    void* ws;
    if (hipMalloc(&x, n * 4) || hipMalloc(&y, n * 4) || hipMalloc(&red, 4) ||
        hipMalloc(&ws, pcmx_dist_workspace_bytes(n, P)))
        return fail("alloc", -1);
    hipMemcpy(x, h.data(), n * 4, hipMemcpyHostToDevice);
    double total = 0, below = 0;
    for (long long g = 0; g < off[P]; ++g) {
        const double v = (double)((g * 7) % 5 - 2);
        total += v;
        if (g < g0) below += v;
    }
    int rc;
    if ((rc = pcmx_reduce_distributed(comm, x, n, PCMX_OP_SUM, red, ws))) return fail("reduce_distributed", rc);
    float r = 0;
    get(&r, red, 4);
    if ((double)r != total) return fail("reduce check", 1);
    if ((rc = pcmx_reduce_distributed(comm, x, n, PCMX_OP_MAX, red, ws))) return fail("reduce_distributed max", rc);
    get(&r, red, 4);
    if (r != 2.f) return fail("reduce max check", 1);
    for (int exclusive = 0; exclusive < 2; ++exclusive) {
        if ((rc = pcmx_scan_distributed(comm, x, y, n, exclusive, ws, nullptr))) return fail("scan_distributed", rc);
        get(got.data(), y, n * 4);
        double acc = below;
        long long bad = 0;
        for (long long i = 0; i < n; ++i) {
            if (!exclusive) acc += h[i];
            bad += (double)got[i] != acc;
            if (exclusive) acc += h[i];
        }
        if (bad) return fail(exclusive ? "exclusive scan check" : "inclusive scan check", (int)bad);
    }
    hipFree(x), hipFree(y), hipFree(red), hipFree(ws);
    return 0;
}

void bench() {
    const size_t bytes = 64u << 20;
    const int P = comm->world;
    void *send = alloc(bytes * P), *recv = alloc(bytes * P);
    for (int k = 0; k < 2; ++k) {
        const bool a2a = k == 1;
        for (int w = 0; w < 2; ++w) a2a ? pcmx_comm_alltoall(comm, send, recv, bytes) : pcmx_comm_allgather(comm, send, recv, bytes);
        pcmx_comm_sync(comm);
        pcmx_comm_barrier(comm);
        const auto t0 = std::chrono::steady_clock::now();
        const int reps = 10;
        for (int i = 0; i < reps; ++i)
            a2a ? pcmx_comm_alltoall(comm, send, recv, bytes) : pcmx_comm_allgather(comm, send, recv, bytes);
        pcmx_comm_sync(comm);
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / reps;
        // bus bandwidth convention of the nccl/rccl tests: (P-1)/P of the gathered size per unit time
        const double busbw = (double)bytes * P * (P - 1) / P / s / 1e9;
        if (comm->rank == 0) printf("%s 64 MiB/rank: %.3f ms  busbw %.1f GB/s\n", a2a ? "alltoall" : "allgather", s * 1e3, busbw);
    }
    release(send);
    release(recv);
}
}  // namespace

int main(int argc, char** argv) {
    size_t bytes = 4099;
    long long n_local = 300001;
    bool do_bench = false;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--cpu")) mode = PCMX_TRANSPORT_TCP;
        else if (!strcmp(argv[i], "--staged")) mode = PCMX_TRANSPORT_TCP_STAGED;
        else if (!strcmp(argv[i], "--bench")) do_bench = true;
        else if (!strcmp(argv[i], "--bytes") && i + 1 < argc) bytes = strtoull(argv[++i], nullptr, 10);
        else if (!strcmp(argv[i], "--n-local") && i + 1 < argc) n_local = strtoll(argv[++i], nullptr, 10);
        else {
            fprintf(stderr, "usage: collectives [--cpu | --staged] [--bytes N] [--n-local N] [--bench]\n");
            return 2;
        }
    }
    int rc = mode == PCMX_TRANSPORT_TCP ? pcmx_comm_init_env_tcp(&comm)
             : mode == PCMX_TRANSPORT_TCP_STAGED ? pcmx_comm_init_env_staged(&comm)
                                                 : pcmx_comm_init_env_rccl(&comm);
    if (rc || !comm) {
        fprintf(stderr, "collectives: communicator init failed (%d)\n", rc);
        return 3;
    }
    int bad = check_collectives(bytes);
    if (!bad && mode != PCMX_TRANSPORT_TCP) bad = check_reduce_scan(n_local);
    printf("rank %d: %s\n", comm->rank, bad ? "FAILED" : mode == PCMX_TRANSPORT_TCP ? "allgather gather scatter alltoall ok"
                                                           : "allgather gather scatter alltoall reduce scan ok");
    fflush(stdout);
    int flag = bad ? 1 : 0;
    pcmx_comm_allreduce(comm->host, &flag, 1, PCMX_I32, PCMX_MAX);  // host side-channel: every rank agrees
    if (!flag && do_bench && mode == PCMX_TRANSPORT_RCCL) bench();
    if (comm->rank == 0 && !flag) printf("collectives ok world=%d\n", comm->world);
    fflush(stdout);
    pcmx_comm_barrier(comm);
    pcmx_comm_destroy(comm);
    return flag ? 1 : 0;
}
