"""SpMV rank lab (rounds 4-5): one N = 8 rank's column-split step emulated on one GPU (no exchange): 4 product launches
and per row chunk either the round-4 combine, fix-up and gather pack (three launches) or the round-5 fused combine
(combine + fix-up + send-buffer pack in one launch), interleaved A/B rounds in one process, bit-identity checked; and
the host enqueue time of the production step against its device time. The two exchange calls a real step adds cost
~13-19 us of host time each (scripts/host_overhead_lab.py, profiles/r2_bench/host_overhead_lab.txt).
Run: python scripts/spmv_host_lab.py [world] [reps]
Env: SPMV_LAB_KINDS=paired (comma list of the A/B kinds; "none": no packs), SPMV_LAB_ITEM (0: the production rule), SPMV_LAB_SLICES,
SPMV_LAB_PB=2,4 (resident product blocks per CU of the phase-0 / phase-1 launches),
SPMV_LAB_N1=0 (skip the same-box N = 1 step), SPMV_LAB_FRAC=0.4 (row chunk 0's share), SPMV_LAB_RCCL=1 (the step with both exchanges on a world-1 RCCL
communicator, round 6)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from parallel_c_programs_amd.parallel.dist import Context  # noqa: E402
from parallel_c_programs_amd.parallel.spmv import DistributedSpMV  # noqa: E402


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    dev = torch.device("cuda", 0)
    item = int(os.environ.get("SPMV_LAB_ITEM", "0"))  # 0: the production rule
    slices = int(os.environ.get("SPMV_LAB_SLICES", "16"))
    frac = float(os.environ.get("SPMV_LAB_FRAC", "0.5"))  # row chunk 0's share (round 6: uneven chunks)
    d = DistributedSpMV.powerlaw(Context(rank=0, world=W, device=dev), 10_000_000, 100_000_000, slices=slices, chunks=2,
                                 item_nnz=item, colsplit=True, chunk0_frac=frac)
    print(f"item_nnz {d.parts[0][2].item_nnz}, slices {slices}, phase_blocks {d.parts[0][2].phase_blocks}, "
          f"chunk0_frac {d.chunk0_frac:.3f} (rows {[d.chunk_rows(c) for c in range(2)]})", flush=True)
    xp = torch.rand(d.n_pad, device=dev)
    out = torch.zeros_like(xp)
    Wd, r = d.ctx.world, d.ctx.rank
    # send lists as the real exchange builds them: per chunk, one ascending subset of the chunk's own rows per peer,
    # as many entries in total as this rank receives (a random graph is symmetric on average)
    packs = []
    for c, (a, b, _) in enumerate(d.parts):
        s0, own = d.seg[c * Wd + r], b - a
        k = max(1, d.ghost_len[c] // (Wd - 1))
        packs.append(torch.cat([s0 + torch.sort(torch.randperm(own, device=dev)[:min(k, own)]).values
                                for _ in range(Wd - 1)]))
    packs32 = [p.to(torch.int32) for p in packs]
    bufs = [torch.empty(p.numel(), device=dev) for p in packs]
    from parallel_c_programs_amd.ops.vector import gather_
    print(f"send entries per step {sum(p.numel() for p in packs)}, ghosts received {d.n_ghost}", flush=True)

    # the same send lists inverted per own row for the fused pack (DistributedSpMV.send_csr)
    send_csr = []
    for c, (a, b, _) in enumerate(d.parts):
        lr = packs[c] - d.seg[c * Wd + r]
        order = torch.sort(lr, stable=True).indices
        ptr = torch.zeros(b - a + 1, dtype=torch.int64, device=dev)
        ptr[1:] = torch.bincount(lr, minlength=b - a).cumsum(0)
        send_csr.append((ptr.to(torch.int32), order.to(torch.int32), torch.empty_like(bufs[c])))

    if os.environ.get("SPMV_LAB_PB"):  # resident blocks per CU of the phase-0 / phase-1 product launches (0: 3)
        pb = tuple(int(v) for v in os.environ["SPMV_LAB_PB"].split(","))
        for _, _, part in d.parts:
            part.phase_blocks = pb
        print(f"phase_blocks {pb}", flush=True)

    side = torch.cuda.Stream(dev)

    def step(kind="paired"):
        """kind r4: combine, fix-up and the gather pack as three launches per chunk (round 4); fused_fixup: combine +
        fix-up in one launch, then the gather; fused_pack: combine + fix-up + pack in ONE launch; paired (production):
        fused_pack with both chunks' chunk-0-column products in ONE launch"""
        for c, (a, b, part) in enumerate(d.parts):
            part.fused_combine = kind != "r4"
        if kind == "paired_side":  # paired, with row chunk 0's combine + pack on a side stream beside chunk 1's products
            (_, _, p0), (_, _, p1) = d.parts
            half = p0.n_slices // 16
            p0.products_pair(p1, xp, (0, half), (0, p1.n_slices // 16), mode=p0.phase_blocks[0] << 8)
            main = torch.cuda.current_stream(dev)
            p0.spmv(xp, mode=16 | (p0.phase_blocks[1] << 8), phases=(half, half))
            side.wait_stream(main)
            s0, (a0, b0, _) = d.seg[0 * Wd + r], d.parts[0]
            with torch.cuda.stream(side):
                p0.spmv(xp, out[s0:s0 + (b0 - a0)], mode=32, send=send_csr[0])
            s1, (a1, b1, _) = d.seg[1 * Wd + r], d.parts[1]
            p1.product_phase(xp, 1, 1, out[s1:s1 + (b1 - a1)], send=send_csr[1])
            main.wait_stream(side)
            return
        if kind == "paired":
            (_, _, p0), (_, _, p1) = d.parts
            p0.products_pair(p1, xp, (0, p0.n_slices // 16), (0, p1.n_slices // 16), mode=p0.phase_blocks[0] << 8)
        else:
            for c, (a, b, part) in enumerate(d.parts):
                if b > a:
                    part.product_phase(xp, 0, c)
        for c, (a, b, part) in enumerate(d.parts):
            s0 = d.seg[c * Wd + r]
            if kind in ("fused_pack", "paired"):
                part.product_phase(xp, 1, c, out[s0:s0 + (b - a)], send=send_csr[c])
            else:
                part.product_phase(xp, 1, c, out[s0:s0 + (b - a)])
                if kind:
                    gather_(out, packs32[c], bufs[c])

    def dev_ms(fn):
        for _ in range(5):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / reps

    # bit-identity of the three forms (out rows and send buffers)
    step("r4")
    ref_out, ref_bufs = out.clone(), [bb.clone() for bb in bufs]
    for kind in ("fused_pack", "paired", "paired_side"):
        out.zero_()
        step(kind)
        same = torch.equal(out, ref_out) and all(torch.equal(send_csr[c][2], ref_bufs[c]) for c in range(len(bufs)))
        print(f"{kind}: bit-identical to the round-4 combine, fix-up, gather: {same}", flush=True)
    kinds = os.environ.get("SPMV_LAB_KINDS", "r4,fused_fixup,fused_pack,paired,none").split(",")
    for rnd in range(3):  # interleaved rounds
        for kind in [k if k != "none" else "" for k in kinds]:
            t = dev_ms(lambda: step(kind))
            print(f"round {rnd} N={W} step {kind or 'no packs (r4 combine)'}: device {t:.4f} ms/step", flush=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    host = (t1 - t0) / reps * 1e3
    devt = dev_ms(step)
    print(f"N={W} rank 0 column-split step (production): host enqueue {host:.4f} ms/step, device {devt:.4f} ms/step "
          f"({'launch-bound' if host > devt else 'device-bound'}; + ~0.03 ms of host time for the 2 exchange calls)",
          flush=True)
    if os.environ.get("SPMV_LAB_RCCL") == "1":
        # Round 6: the production step WITH its two exchanges on a world-1 RCCL communicator: each
        # chunk's real send bytes go through an RCCL all_to_all_single to self, posted where _post_chunk posts it (right
        # after that chunk's fused combine + pack) and waited where _step_colsplit waits (chunk 0's at the top of the
        # next step, chunk 1's after the paired phase-0 launch), on RCCL's own stream, concurrently with the products.
        # That prices RCCL's host launch, its kernel's CUs and its HBM / L2 traffic against the L2-bound products; only
        # the xGMI transfer itself is not modelled (the self-exchange is a local copy).
        import torch.distributed as dist
        from parallel_c_programs_amd.parallel.dist import free_port

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        sendb = [sc[2] for sc in send_csr]
        recvb = [torch.empty_like(b) for b in sendb]
        print(f"exchange bytes per chunk: {[4 * b.numel() for b in sendb]}", flush=True)
        pend = [None, None]
        (_, _, q0), (_, _, q1) = d.parts
        from parallel_c_programs_amd.parallel.dist import NativeExchange

        nx = NativeExchange(Context(0, 1, 0, dev, "nccl"))  # the production native path (C++ grouped send/recv)

        side = torch.cuda.Stream(dev)
        evs = [torch.cuda.Event(), torch.cuda.Event()]

        class _Ev:
            def __init__(self, c):
                self.c = c

            def wait(self):
                torch.cuda.current_stream(dev).wait_event(evs[self.c])

        def post(c, native):
            if native == "copy":  # the same event structure, the exchange replaced by torch's copy on a side stream
                side.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(side):
                    recvb[c].copy_(sendb[c])
                    evs[c].record(side)
                return _Ev(c)
            if native:
                n = sendb[c].numel()
                w = nx.post(c, sendb[c], [0], [n], recvb[c], [0], [n])[0]
                return w if native != "nowait" else None
            return dist.all_to_all_single(recvb[c], sendb[c], async_op=True)

        def xstep(comm=True, native=False):
            if pend[0] is not None:
                pend[0].wait()
                pend[0] = None
            q0.products_pair(q1, xp, (0, q0.n_slices // 16), (0, q1.n_slices // 16), mode=q0.phase_blocks[0] << 8)
            if pend[1] is not None:
                pend[1].wait()
                pend[1] = None
            for c, (a, b, part) in enumerate(d.parts):
                s0 = d.seg[c * Wd + r]
                part.fused_combine = True
                part.product_phase(xp, 1, c, out[s0:s0 + (b - a)], send=send_csr[c])
                if comm:
                    pend[c] = post(c, native)

        def flush():
            for k in range(2):
                if pend[k] is not None:
                    pend[k].wait()
                    pend[k] = None

        def xchg_only(native):
            for c in range(2):
                post(c, native).wait()

        for rnd in range(4):
            t_plain = dev_ms(lambda: xstep(False))
            flush()
            t_comm = dev_ms(lambda: xstep(True))
            flush()
            t_nat = dev_ms(lambda: xstep(True, native=True))
            flush()
            t_nw = dev_ms(lambda: xstep(True, native="nowait"))
            flush()
            torch.cuda.synchronize()
            t_cp = dev_ms(lambda: xstep(True, native="copy"))
            flush()
            t_x = dev_ms(lambda: xchg_only(False))
            t_xn = dev_ms(lambda: xchg_only(True))
            print(f"round {rnd} N={W} rank step: no exchange {t_plain:.4f} ms; both RCCL self-exchanges in flight via "
                  f"torch all_to_all_single {t_comm:.4f} ms (+{1e3 * (t_comm - t_plain):.1f} us), via the native "
                  f"exchange {t_nat:.4f} ms (+{1e3 * (t_nat - t_plain):.1f} us); the two exchanges alone, back to back: "
                  f"torch {t_x:.4f} ms, native {t_xn:.4f} ms; native posted but never waited {t_nw:.4f} ms; a side-stream "
                  f"copy with the same waits {t_cp:.4f} ms", flush=True)
        for native in (False, True):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                xstep(True, native)
            t1 = time.perf_counter()
            flush()
            torch.cuda.synchronize()
            print(f"host enqueue with the exchanges ({'native' if native else 'torch all_to_all_single'}): "
                  f"{(t1 - t0) / reps * 1e3:.4f} ms/step", flush=True)
        nx.close()
        dist.destroy_process_group()
    if os.environ.get("SPMV_LAB_N1", "1") == "1":
        # the same-box N = 1 step (the bench's single-GPU section: 1e8 nnz, one sliced product) for the efficiency model
        del d, out, bufs, send_csr, packs, packs32
        torch.cuda.empty_cache()
        d1 = DistributedSpMV.powerlaw(Context(rank=0, world=1, device=dev), 10_000_000, 100_000_000, slices=-1)
        x1 = torch.rand(d1.n_pad, device=dev)
        (_, _, p1), = d1.parts
        y1 = torch.empty(p1.n_rows, device=dev)
        t1 = min(dev_ms(lambda: p1.spmv(x1, y1)) for _ in range(3))
        t8 = devt
        print(f"N=1 step (same box, same process): device {t1:.4f} ms; N={W} production step {t8:.4f} ms -> modelled "
              f"N={W} efficiency t1 / ({W} t{W}) = {100 * t1 / (W * t8):.1f}% (exchange hidden)", flush=True)


if __name__ == "__main__":
    main()
