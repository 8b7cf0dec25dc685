/* Distributed 2-D region growing and the token chain over the native comm layer (pcmx_comm.h).
 *
 * Native counterpart of ref 2-mpi-region-growing/region.c (call stack SURVEY §3.1) and 1-introduction/mpi.c.
 * The algorithm is written once against a data-movement backend (host memory + serial flood fill for the
 * TCP transport; device memory + the gfx950 label-propagation kernel for RCCL, csrc/comm/comm_rccl.hip):
 *
 *   scatter   root cuts every rank's PADDED tile (interior + neighbours' pixels in the halo ring) out of
 *             the zero-padded image and sends one message per rank (ref: one message per row per rank plus
 *             a separate halo pass, region.c:106-246)
 *   grow      local fixpoint on the tile; region cells in the halo ring act as seeds (ref DFS :499-527 +
 *             add_halo_to_stack :355)
 *   exchange  pack 4 edges -> grouped send/recv with N/S/W/E -> unpack (ref exchange :250-353)
 *   finish    device-resident "halo changed" flag raised by the unpack, MAX all-reduce in place, read by the
 *             host every PCMX_REGION_CHECK_EVERY steps (ref finished(): MIN all-reduce of local_finish :435)
 *   gather    one message per rank to root (ref gather_region :391)
 * Any process count and image size (the reference handles square grids only, B8).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pcmx_comm.h"

/* ------------------------------------------------------------------ host backend */

static void* h_alloc(size_t n, void* ctx) {
    (void)ctx;
    return malloc(n ? n : 1);
}
static void h_release(void* p, void* ctx) {
    (void)ctx;
    free(p);
}
static int h_memset0(void* p, size_t n, void* ctx) {
    (void)ctx;
    memset(p, 0, n);
    return 0;
}
static int h_copy(void* d, const void* s, size_t n, void* ctx) {
    (void)ctx;
    memcpy(d, s, n);
    return 0;
}
static int h_copy2d(void* d, size_t dp, const void* s, size_t sp, size_t w, size_t h, void* ctx) {
    (void)ctx;
    for (size_t r = 0; r < h; ++r) memcpy((char*)d + r * dp, (const char*)s + r * sp, w);
    return 0;
}

void pcmx_region2d_padded_host(unsigned char* reg, const unsigned char* img, int h, int w, int thr) {
    const int ld = w + 2;
    const size_t n = (size_t)(h + 2) * ld;
    int* stack = (int*)malloc(sizeof(int) * n);
    size_t top = 0;
    for (size_t i = 0; i < n; ++i)
        if (reg[i]) stack[top++] = (int)i;
    while (top) {
        const int p = stack[--top];
        const int y = p / ld, x = p % ld;
        const int v = img[p];
        const int nbr[4] = {p + ld, p - ld, p + 1, p - 1};
        const int ny[4] = {y + 1, y - 1, y, y}, nx[4] = {x, x, x + 1, x - 1};
        for (int k = 0; k < 4; ++k) {
            if (ny[k] < 1 || ny[k] > h || nx[k] < 1 || nx[k] > w) continue;
            const int q = nbr[k];
            if (reg[q]) continue;
            const int d = (int)img[q] - v;
            if ((d < 0 ? -d : d) < thr) {
                reg[q] = 1;
                stack[top++] = q;
            }
        }
    }
    free(stack);
}

static int h_grow(unsigned char* reg, const unsigned char* img, int h, int w, int thr, void* ctx) {
    (void)ctx;
    pcmx_region2d_padded_host(reg, img, h, w, thr);
    return 0;
}

/* packed edge layout: [top w | bottom w | left h | right h] (same as the gfx950 pack kernel) */
static int h_pack(const unsigned char* t, int h, int w, unsigned char* buf, void* ctx) {
    (void)ctx;
    const int ld = w + 2;
    memcpy(buf, t + ld + 1, (size_t)w);
    memcpy(buf + w, t + (size_t)h * ld + 1, (size_t)w);
    for (int r = 0; r < h; ++r) {
        buf[2 * w + r] = t[(size_t)(r + 1) * ld + 1];
        buf[2 * w + h + r] = t[(size_t)(r + 1) * ld + w];
    }
    return 0;
}

static int h_unpack(unsigned char* t, int h, int w, const unsigned char* buf, int mask, void* ctx) {
    (void)ctx;
    const int ld = w + 2;
    if (mask & 1) memcpy(t + 1, buf, (size_t)w);
    if (mask & 2) memcpy(t + (size_t)(h + 1) * ld + 1, buf + w, (size_t)w);
    for (int r = 0; r < h; ++r) {
        if (mask & 4) t[(size_t)(r + 1) * ld] = buf[2 * w + r];
        if (mask & 8) t[(size_t)(r + 1) * ld + w + 1] = buf[2 * w + h + r];
    }
    return 0;
}

static int h_unpack_changed(unsigned char* t, int h, int w, const unsigned char* buf, int mask, int* changed,
                            void* ctx) {
    const int ld = w + 2;
    int diff = 0;
    if (mask & 1) diff |= memcmp(t + 1, buf, (size_t)w) != 0;
    if (mask & 2) diff |= memcmp(t + (size_t)(h + 1) * ld + 1, buf + w, (size_t)w) != 0;
    for (int r = 0; r < h; ++r) {
        if (mask & 4) diff |= t[(size_t)(r + 1) * ld] != buf[2 * w + r];
        if (mask & 8) diff |= t[(size_t)(r + 1) * ld + w + 1] != buf[2 * w + h + r];
    }
    if (diff) *changed = 1;
    return h_unpack(t, h, w, buf, mask, ctx);
}

static int h_sync(void* ctx) {
    (void)ctx;
    return 0;
}

void pcmx_region_backend_host(pcmx_region_backend_t* be) {
    be->alloc = h_alloc, be->release = h_release, be->memset0 = h_memset0, be->h2d = h_copy, be->d2h = h_copy;
    be->copy2d = h_copy2d, be->grow = h_grow, be->pack = h_pack, be->unpack = h_unpack, be->sync = h_sync;
    be->unpack_changed = h_unpack_changed;
    be->ctx = NULL;
    be->stream = NULL;
}

/* ------------------------------------------------------------------ distributed region growing */

#define TRY(x)                  \
    do {                        \
        int _rc = (x);          \
        if (_rc) {              \
            rc = _rc;           \
            goto done;          \
        }                       \
    } while (0)

int pcmx_region2d_distributed(pcmx_comm_t* c, const pcmx_region_backend_t* be, const unsigned char* image, int H,
                              int W, int threshold, const int* dims, unsigned char* region_out, int* stats) {
    int rc = 0;
    void* ctx = be->ctx;
    const int root = c->rank == 0;
    /* shape is known on root only (ref reads the BMP on rank 0): broadcast over the host side-channel */
    int hw[2] = {H, W};
    if (c->host->ops->bcast(c->host, hw, sizeof hw, 0)) return PCMX_ERR_COMM;
    H = hw[0], W = hw[1];
    pcmx_cart_t topo;
    pcmx_cart_init(&topo, c->world, dims);
    if (topo.dims[0] * topo.dims[1] != c->world) return PCMX_ERR_ARG;
    int tile[4], nb[4];
    pcmx_cart_tile(&topo, c->rank, H, W, tile);
    pcmx_cart_neighbours(&topo, c->rank, nb);
    const int h = tile[1] - tile[0], w = tile[3] - tile[2];
    const size_t tbytes = (size_t)(h + 2) * (w + 2);
    const int nedge = 2 * w + 2 * h;
    /* every rank derives the same answer: equal tiles (1/2/4/8 ranks on a 512^2 image) use the scatter / gather
     * collectives (one ncclScatter / ncclGather), uneven ones one grouped message per rank */
    int equal = 1;
    for (int r = 0; r < c->world; ++r) {
        int t[4];
        pcmx_cart_tile(&topo, r, H, W, t);
        equal &= t[1] - t[0] == h && t[3] - t[2] == w;
    }
    unsigned char *img_p = NULL, *reg_p = NULL, *full_p = NULL, *stage = NULL, *sendb = NULL, *recvb = NULL;
    unsigned char* full_reg = NULL;
    int* flag = NULL;
    int outer = 0;
    img_p = (unsigned char*)be->alloc(tbytes, ctx);
    reg_p = (unsigned char*)be->alloc(tbytes, ctx);
    sendb = (unsigned char*)be->alloc((size_t)nedge, ctx);
    recvb = (unsigned char*)be->alloc((size_t)nedge, ctx);
    flag = (int*)be->alloc(sizeof(int), ctx);
    if (!img_p || !reg_p || !sendb || !recvb || !flag) {
        rc = PCMX_ERR_ALLOC;
        goto done;
    }

    /* ---- scatter padded image tiles (one scatter collective, or one message per rank for uneven tiles) */
    if (root) {
        const size_t pw = (size_t)W + 2;
        unsigned char* padded = (unsigned char*)calloc((size_t)(H + 2) * pw, 1);
        for (int r = 0; r < H; ++r) memcpy(padded + (size_t)(r + 1) * pw + 1, image + (size_t)r * W, (size_t)W);
        full_p = (unsigned char*)be->alloc((size_t)(H + 2) * pw, ctx);
        size_t total = 0;
        for (int r = 0; r < c->world; ++r) {
            int t[4];
            pcmx_cart_tile(&topo, r, H, W, t);
            total += (size_t)(t[1] - t[0] + 2) * (t[3] - t[2] + 2);
        }
        stage = (unsigned char*)be->alloc(total, ctx);
        if (!full_p || !stage) {
            free(padded);
            rc = PCMX_ERR_ALLOC;
            goto done;
        }
        rc = be->h2d(full_p, padded, (size_t)(H + 2) * pw, ctx);
        free(padded);
        if (rc) goto done;
        size_t off = 0;
        if (equal) { /* every padded tile staged in rank order, then ONE scatter collective (ncclScatter) */
            for (int r = 0; r < c->world; ++r) {
                int t[4];
                pcmx_cart_tile(&topo, r, H, W, t);
                TRY(be->copy2d(stage + (size_t)r * tbytes, (size_t)w + 2, full_p + (size_t)t[0] * pw + t[2], pw,
                               (size_t)w + 2, (size_t)h + 2, ctx));
            }
            TRY(be->sync(ctx));
        } else { /* uneven tiles: one grouped message per rank */
            TRY(pcmx_comm_group_start(c));
            for (int r = 0; r < c->world; ++r) {
                int t[4];
                pcmx_cart_tile(&topo, r, H, W, t);
                const size_t th = (size_t)(t[1] - t[0] + 2), tw = (size_t)(t[3] - t[2] + 2);
                unsigned char* dst = r == 0 ? img_p : stage + off;
                TRY(be->copy2d(dst, tw, full_p + (size_t)t[0] * pw + t[2], pw, tw, th, ctx));
                if (r) {
                    TRY(be->sync(ctx));
                    TRY(pcmx_comm_send(c, dst, th * tw, r));
                }
                off += th * tw;
            }
            TRY(pcmx_comm_group_end(c));
        }
    } else if (!equal) {
        TRY(pcmx_comm_recv(c, img_p, tbytes, 0));
    }
    if (equal) TRY(pcmx_comm_scatter(c, root ? stage : NULL, img_p, tbytes, 0));

    /* ---- seeds: the reference's four corner seeds (region.c:450-490) in global coordinates */
    TRY(be->memset0(reg_p, tbytes, ctx));
    {
        const int o = 4;
        const int sx[4] = {o, W - 6, W - 6, o}, sy[4] = {o, o, H - 6, H - 6};
        const unsigned char one = 1;
        for (int k = 0; k < 4; ++k) {
            if (sy[k] >= tile[0] && sy[k] < tile[1] && sx[k] >= tile[2] && sx[k] < tile[3]) {
                const size_t at = (size_t)(sy[k] - tile[0] + 1) * (w + 2) + (sx[k] - tile[2] + 1);
                TRY(be->h2d(reg_p + at, &one, 1, ctx));
            }
        }
    }
    int mask = 0;
    mask |= nb[0] >= 0 ? 1 : 0;
    mask |= nb[1] >= 0 ? 2 : 0;
    mask |= nb[2] >= 0 ? 4 : 0;
    mask |= nb[3] >= 0 ? 8 : 0;
    const int off_e[4] = {0, w, 2 * w, 2 * w + h}, len_e[4] = {w, w, h, h};

    /* ---- bulk-synchronous grow / exchange / terminate. The "halo changed" flag lives in backend (device)
     * memory: the unpack kernel raises it, the MAX all-reduce runs on it in place, and the host reads it once
     * per PCMX_REGION_CHECK_EVERY outer steps (a window with no change on any rank = global fixpoint: a step
     * whose halos did not change cannot grow anything new, so every later step is a no-op too). */
    TRY(be->memset0(flag, sizeof(int), ctx));
    for (;;) {
        TRY(be->grow(reg_p, img_p, h, w, threshold, ctx));
        ++outer;
        if (c->world == 1) break;
        TRY(be->pack(reg_p, h, w, sendb, ctx));
        /* the pack and the sends are stream-ordered when the backend runs on the communicator's stream (device
         * backend + RCCL or staged transport): no host wait per outer step. Only a backend on another stream
         * (or a host backend feeding a device transport) must finish before the transport reads sendb. */
        if (!(be->stream && be->stream == c->stream)) TRY(be->sync(ctx));
        TRY(pcmx_comm_group_start(c));
        for (int k = 0; k < 4; ++k) {
            if (nb[k] < 0) continue;
            TRY(pcmx_comm_send(c, sendb + off_e[k], (size_t)len_e[k], nb[k]));
            TRY(pcmx_comm_recv(c, recvb + off_e[k], (size_t)len_e[k], nb[k]));
        }
        TRY(pcmx_comm_group_end(c));
        TRY(be->unpack_changed(reg_p, h, w, recvb, mask, flag, ctx));
        if (outer % PCMX_REGION_CHECK_EVERY) continue;
        TRY(pcmx_comm_allreduce(c, flag, 1, PCMX_I32, PCMX_MAX));
        int changed = 1;
        TRY(be->d2h(&changed, flag, sizeof changed, ctx));  /* the loop's only host read-back */
        if (!changed) break;
        TRY(be->memset0(flag, sizeof(int), ctx));
    }

    /* ---- gather interiors to root (ONE gather collective for equal tiles, else one message per rank) */
    if (equal) {
        const size_t pw = (size_t)W + 2, n = (size_t)w * h;
        /* contiguous interior, staged through img_p (no longer needed) */
        TRY(be->copy2d(img_p, (size_t)w, reg_p + (w + 2) + 1, (size_t)w + 2, (size_t)w, (size_t)h, ctx));
        TRY(be->sync(ctx));
        TRY(pcmx_comm_gather(c, img_p, root ? stage : NULL, n, 0));
        TRY(pcmx_comm_sync(c));
        if (root) {
            full_reg = (unsigned char*)calloc((size_t)(H + 2) * pw, 1);
            for (int r = 0; r < c->world; ++r) {
                int t[4];
                pcmx_cart_tile(&topo, r, H, W, t);
                TRY(be->copy2d(full_p + (size_t)(t[0] + 1) * pw + t[2] + 1, pw, stage + (size_t)r * n, (size_t)w,
                               (size_t)w, (size_t)h, ctx));
            }
            TRY(be->d2h(full_reg, full_p, (size_t)(H + 2) * pw, ctx));
            for (int r = 0; r < H; ++r)
                memcpy(region_out + (size_t)r * W, full_reg + (size_t)(r + 1) * pw + 1, (size_t)W);
        }
    } else if (root) {
        const size_t pw = (size_t)W + 2;
        full_reg = (unsigned char*)calloc((size_t)(H + 2) * pw, 1);
        /* reuse full_p as the padded device region image */
        TRY(be->copy2d(full_p + (size_t)(tile[0] + 1) * pw + tile[2] + 1, pw, reg_p + (w + 2) + 1, (size_t)w + 2,
                       (size_t)w, (size_t)h, ctx));
        size_t off = 0;
        TRY(pcmx_comm_group_start(c));
        for (int r = 1; r < c->world; ++r) {
            int t[4];
            pcmx_cart_tile(&topo, r, H, W, t);
            const size_t n = (size_t)(t[1] - t[0]) * (t[3] - t[2]);
            TRY(pcmx_comm_recv(c, stage + off, n, r));
            off += n;
        }
        TRY(pcmx_comm_group_end(c));
        TRY(pcmx_comm_sync(c));
        off = 0;
        for (int r = 1; r < c->world; ++r) {
            int t[4];
            pcmx_cart_tile(&topo, r, H, W, t);
            const size_t th = (size_t)(t[1] - t[0]), tw = (size_t)(t[3] - t[2]);
            TRY(be->copy2d(full_p + (size_t)(t[0] + 1) * pw + t[2] + 1, pw, stage + off, tw, tw, th, ctx));
            off += th * tw;
        }
        TRY(be->d2h(full_reg, full_p, (size_t)(H + 2) * pw, ctx));
        for (int r = 0; r < H; ++r) memcpy(region_out + (size_t)r * W, full_reg + (size_t)(r + 1) * pw + 1, (size_t)W);
    } else {
        /* contiguous interior: reuse sendb-sized staging is too small; stage through img_p (no longer needed) */
        TRY(be->copy2d(img_p, (size_t)w, reg_p + (w + 2) + 1, (size_t)w + 2, (size_t)w, (size_t)h, ctx));
        TRY(be->sync(ctx));
        TRY(pcmx_comm_send(c, img_p, (size_t)w * h, 0));
        TRY(pcmx_comm_sync(c));
    }
    if (stats) stats[0] = outer, stats[1] = outer;

done:
    if (img_p) be->release(img_p, ctx);
    if (reg_p) be->release(reg_p, ctx);
    if (full_p) be->release(full_p, ctx);
    if (stage) be->release(stage, ctx);
    if (sendb) be->release(sendb, ctx);
    if (recvb) be->release(recvb, ctx);
    if (flag) be->release(flag, ctx);
    free(full_reg);
    return rc;
}

/* ------------------------------------------------------------------ token chain (ref mpi.c:5-44) */

int pcmx_token_ring(pcmx_comm_t* c, void* tok, const pcmx_region_backend_t* be, int verbose) {
    const int rank = c->rank, size = c->world;
    int msg = 0, rc = 0;
    if (be->h2d(tok, &msg, sizeof msg, be->ctx)) return PCMX_ERR_COMM;
    if (rank != 0) {
        if ((rc = pcmx_comm_recv(c, tok, sizeof msg, rank - 1)) || (rc = pcmx_comm_sync(c))) return rc;
        be->d2h(&msg, tok, sizeof msg, be->ctx);
        if (verbose) printf("Rank %d received %d \n", rank, msg), fflush(stdout);
        msg += 1;
        be->h2d(tok, &msg, sizeof msg, be->ctx);
    }
    if (rank < size - 1) {
        if ((rc = pcmx_comm_send(c, tok, sizeof msg, rank + 1)) || (rc = pcmx_comm_sync(c))) return rc;
        if (verbose) printf("Rank %d sent %d \n", rank, msg), fflush(stdout);
        if ((rc = pcmx_comm_recv(c, tok, sizeof msg, rank + 1)) || (rc = pcmx_comm_sync(c))) return rc;
        be->d2h(&msg, tok, sizeof msg, be->ctx);
        if (verbose) printf("Rank %d received %d \n", rank, msg), fflush(stdout);
        msg += 1;
        be->h2d(tok, &msg, sizeof msg, be->ctx);
    }
    if (rank != 0) {
        if ((rc = pcmx_comm_send(c, tok, sizeof msg, rank - 1)) || (rc = pcmx_comm_sync(c))) return rc;
        if (verbose) printf("Rank %d sent %d \n", rank, msg), fflush(stdout);
    }
    return msg;
}
