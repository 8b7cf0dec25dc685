/* bin/mpi_ring [--cpu | --staged] — the token chain of 1-introduction/mpi.c:5-44: rank 0
 * sends 0 up the chain, every rank adds one and forwards it, the last rank sends it back down, adding one
 * again; prints "Rank %d received %d " / "Rank %d sent %d " as the reference does. The token lives in GPU
 * memory and moves with ncclSend/ncclRecv over xGMI (default), through host-staged TCP (--staged, ranks may
 * share a GPU) or in host memory over TCP (--cpu). Launch with `pcmx_launch -n P` or torchrun. */
#include <cstdio>
#include <cstring>

#include "pcmx_comm.h"
#include "pcmx_cpu.h"
#include "pcmx_hip.h"

int main(int argc, char** argv) {
    int mode = PCMX_TRANSPORT_RCCL;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--cpu")) mode = PCMX_TRANSPORT_TCP;
        else if (!strcmp(argv[i], "--staged")) mode = PCMX_TRANSPORT_TCP_STAGED;
    }
    pcmx_comm_t* c = nullptr;
    int rc = mode == PCMX_TRANSPORT_TCP ? pcmx_comm_init_env_tcp(&c)
             : mode == PCMX_TRANSPORT_TCP_STAGED ? pcmx_comm_init_env_staged(&c)
                                                 : pcmx_comm_init_env_rccl(&c);
    if (rc || !c) {
        fprintf(stderr, "mpi_ring: communicator init failed (%d)\n", rc);
        return 3;
    }
    pcmx_region_backend_t be;
    if (mode == PCMX_TRANSPORT_TCP) pcmx_region_backend_host(&be);
    else pcmx_region_backend_hip(&be, c->stream);
    void* tok = be.alloc(sizeof(int), be.ctx);
    const int final_value = tok ? pcmx_token_ring(c, tok, &be, 1) : -1;
    if (tok) be.release(tok, be.ctx);
    fflush(stdout);
    pcmx_comm_barrier(c);
    pcmx_comm_destroy(c);
    return final_value < 0 ? 2 : 0;
}
