/* bin/region [--cpu | --staged] [--dims R C] [--threshold T] [--stats] file.bmp
 *
 * The reference's distributed region growing (2-mpi-region-growing/region.c:582-604), one
 * process per MI355X: start it with `pcmx_launch -n P` or torchrun. Rank 0 reads the BMP, the image is
 * scattered as padded tiles over a balanced Cartesian grid, every rank grows its tile to a local fixpoint on
 * the GPU (gfx950 label-propagation kernel), halos go to the 4 neighbours in one grouped exchange and a MIN
 * all-reduce decides termination; rank 0 gathers the region and writes ./out.bmp = image * (region == 0).
 *
 * Transports: default RCCL over xGMI (device buffers, one GPU per rank); --staged = device buffers staged
 * through host memory over TCP, so several ranks may share one GPU (test fixture); --cpu = TCP + host flood
 * fill, no GPU touched. Usage text and exit status (-1) as in the reference (region.c:552-555, B12). */
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "pcmx_comm.h"
#include "pcmx_cpu.h"
#include "pcmx_hip.h"

int main(int argc, char** argv) {
    int mode = PCMX_TRANSPORT_RCCL, thr = 2, dims[2] = {0, 0}, stats_flag = 0;
    const char* file = nullptr;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--cpu")) mode = PCMX_TRANSPORT_TCP;
        else if (!strcmp(argv[i], "--staged")) mode = PCMX_TRANSPORT_TCP_STAGED;
        else if (!strcmp(argv[i], "--stats")) stats_flag = 1;
        else if (!strcmp(argv[i], "--threshold") && i + 1 < argc) thr = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--dims") && i + 2 < argc) dims[0] = atoi(argv[++i]), dims[1] = atoi(argv[++i]);
        else file = argv[i];
    }
    if (!file) {
        printf("Useage: region file");
        fflush(stdout);
        exit(-1);
    }
    pcmx_comm_t* c = nullptr;
    int rc = mode == PCMX_TRANSPORT_TCP ? pcmx_comm_init_env_tcp(&c)
             : mode == PCMX_TRANSPORT_TCP_STAGED ? pcmx_comm_init_env_staged(&c)
                                                 : pcmx_comm_init_env_rccl(&c);
    if (rc || !c) {
        fprintf(stderr, "region: communicator init failed (%d)\n", rc);
        return 3;
    }
    pcmx_region_backend_t be;
    if (mode == PCMX_TRANSPORT_TCP) pcmx_region_backend_host(&be);
    else pcmx_region_backend_hip(&be, c->stream);

    int W = 0, H = 0;
    unsigned char* img = nullptr;
    std::vector<unsigned char> reg;
    if (c->rank == 0) {
        img = pcmx_read_bmp_dims(file, &W, &H);
        if (!img) {
            fprintf(stderr, "region: cannot read %s\n", file);
            H = W = -1;  // still enter the collective so the other ranks learn about the failure
        } else {
            reg.resize((size_t)W * H);
        }
    }
    int stats[2] = {0, 0};
    const double t0 = pcmx_wtime();
    rc = pcmx_region2d_distributed(c, &be, img, H, W, thr, dims[0] ? dims : nullptr, reg.empty() ? nullptr : reg.data(),
                                   stats);
    const double t1 = pcmx_wtime();
    if (!rc && c->rank == 0) {
        long long n = 0;
        for (size_t i = 0; i < reg.size(); ++i) {
            n += reg[i] != 0;
            img[i] = reg[i] ? 0 : img[i];
        }
        write_bmp(img, W, H);
        if (stats_flag)
            fprintf(stderr, "ranks=%d outer_steps=%d local_grows=%d region=%lld time=%.6fs\n", c->world, stats[0],
                    stats[1], n, t1 - t0);
    }
    if (rc) fprintf(stderr, "region: rank %d failed (%d)\n", c->rank, rc);
    pcmx_free(img);
    pcmx_comm_barrier(c);
    pcmx_comm_destroy(c);
    return rc ? 2 : 0;
}
