"""Stencil rank lab: one rank's compute per distributed step of the 16384^2 bf16 grid at N = 2 / 4 / 8
(an interior rank's slab: 8192 / 4096 / 2048 rows, `fuse` halo rows each side), on one GPU without the halo
exchange, for the launch shapes a step can take:

  full      one launch over all rows (no overlap split)
  split3    interior launch + one launch per edge band (round-2 step)
  split2    interior launch + both edge bands in ONE two-span launch
  split2c   split2 with the edge launch on a side stream, concurrent with the interior kernel
  deepM     the deep-halo schedule (StencilSlab halo_mult=M): per M steps an interior launch + one edge launch over
            the two halo-dependent bands, then M - 1 single launches over shrinking extended ranges; time per step

Every variant is checked bit for bit against `full`. Prints ms per step and GLUP/s per GPU; with the 1-GPU
full-grid time this bounds the strong-scaling efficiency of the compute part (docs/ARCHITECTURE.md, stencil).
Run: python scripts/stencil_rank_lab.py [fuse ...]
Env: STENCIL_LAB_WORLDS=8 (subset of 1,2,4,8), STENCIL_LAB_RPW=0,18 (rows per wave forced on the non-edge launches
as an explicit launch shape of each call, ops.stencil.launch_shape; 0 = production rule; one line per value, all in one
process for an A/B); STENCIL_LAB_DEEP=2,3,4 (halo depths m); STENCIL_LAB_ONLY=full (subset of full, split3, split2, split2c); STENCIL_LAB_AHEAD=3 / 6 / 9 (prefetch ring
of the forced shapes); STENCIL_LAB_CPL=4 / 8 (columns per lane of the forced shapes); STENCIL_LAB_PAIRED=0,1 (round 6:
paired waves off / on for the non-edge launches, one line per value); STENCIL_LAB_RCCL=1 (round 6:
each deep-halo variant also runs WITH its exchange: the real halo bytes, 2 x mT rows, through the native exchange on a
world-1 RCCL communicator, posted before the interior launch and waited before the edge launch as StencilSlab.step
does; printed as deepM+x); STENCIL_LAB_DEEP_BUFS=2 (round 6 default: the deep-halo phases ping-pong between two
buffers as StencilSlab does; 0 = one buffer per phase, the rounds 4-6 lab numbers); STENCIL_LAB_EDGE=4:2 (an explicit
cpl:rpw[:ahead] shape for the deep-halo step's edge launch).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from parallel_c_programs_amd import ops  # noqa: E402
from parallel_c_programs_amd.ops.stencil import launch_shape  # noqa: E402

N = 16384


def timed(fn, reps=50):
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


def main():
    fuses = [int(a) for a in sys.argv[1:]] or [4, 6, 8]
    dev = torch.device("cuda", 0)
    nx = None
    if os.environ.get("STENCIL_LAB_RCCL") == "1":
        import torch.distributed as dist

        from parallel_c_programs_amd.parallel.dist import Context, NativeExchange, free_port

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        nx = NativeExchange(Context(0, 1, 0, dev, "nccl"))
    g = torch.Generator(device=dev).manual_seed(1)
    worlds = [int(w) for w in os.environ.get("STENCIL_LAB_WORLDS", "1,2,4,8").split(",")]
    rpws = [int(r) for r in os.environ.get("STENCIL_LAB_RPW", "0").split(",")]
    pairs = [{"": None, "1": True, "0": False}[p] for p in os.environ.get("STENCIL_LAB_PAIRED", "").split(",")]
    # STENCIL_LAB_EDGE=cpl:rpw[:ahead] (round 6): an explicit shape for the deep-halo step's edge launch (the two rank-edge
    # bands, <= 64 rows: production 4 columns per lane x 2-row waves)
    edge_spec = [int(v) for v in os.environ.get("STENCIL_LAB_EDGE", "0:0").split(":")] + [0]
    edge_shape = launch_shape(edge_spec[0], edge_spec[1], edge_spec[2]) if any(edge_spec) else 0
    for T, world, rpw, paired in [(T, w, r, p) for T in fuses for w in worlds for r in rpws for p in pairs]:
        shape = launch_shape(int(os.environ.get("STENCIL_LAB_CPL", "0")), rpw, int(os.environ.get("STENCIL_LAB_AHEAD", "0")),
                             paired)

        def step(*a, shape=shape, **kw):  # the non-edge launches take the forced rows per wave
            return ops.stencil5_fused_step_(*a, shape=shape, **kw)

        if True:
            rows = N // world
            row0 = 0 if world == 1 else rows  # rank 1: both neighbours present (interior rank)
            u = (torch.rand(rows + 2 * T, N, generator=g, device=dev) * 4 - 2).to(torch.bfloat16)
            ref, out = u.clone(), u.clone()

            def full():
                step(u, ref, row0, N, halo=T, steps=T)

            def split3():
                step(u, out, row0, N, halo=T, steps=T, row_range=(T, rows - T))
                step(u, out, row0, N, halo=T, steps=T, row_range=(0, T))
                step(u, out, row0, N, halo=T, steps=T, row_range=(rows - T, rows))

            def split2():
                step(u, out, row0, N, halo=T, steps=T, row_range=(T, rows - T))
                ops.stencil5_fused_spans_(u, out, ((0, T), (rows - T, rows)), row0, N, halo=T, steps=T)

            side = torch.cuda.Stream(dev)

            def split2c():  # the edge launch on a side stream, concurrent with the interior kernel
                main = torch.cuda.current_stream(dev)
                side.wait_stream(main)
                step(u, out, row0, N, halo=T, steps=T, row_range=(T, rows - T))
                with torch.cuda.stream(side):
                    ops.stencil5_fused_spans_(u, out, ((0, T), (rows - T, rows)), row0, N, halo=T, steps=T)
                main.wait_stream(side)

            # deep halo, m = 2, 3, ... (StencilSlab halo_mult=m): a slab with mT halo rows; per m steps an interior
            # launch + ONE two-span edge launch over local rows [-(m-1)T, T) and [rows - T, rows + (m-1)T), then
            # launches over [-e, rows + e) for e = (m-2)T .. 0; checked against the same m steps as single launches
            deeps = {}
            # STENCIL_LAB_DEEP_BUFS (round 6): 2 = the production ping-pong pair (StencilSlab's u / v; at N = 8 the
            # pair, 2 x ~68 MB, can stay in the 256-MB Infinity Cache like the single-launch variants' pair);
            # 0 = one buffer per phase (M + 1, the rounds 4-6 lab numbers: every phase streams from HBM)
            nbufs = int(os.environ.get("STENCIL_LAB_DEEP_BUFS", "2"))
            for M in [int(v) for v in os.environ.get("STENCIL_LAB_DEEP", "2,3,4").split(",")]:
                u4 = (torch.rand(rows + 2 * M * T, N, generator=g, device=dev) * 4 - 2).to(torch.bfloat16)
                nb = nbufs if nbufs >= 2 else M + 1
                b4 = [u4.clone() for _ in range(nb)]
                c4 = [u4.clone() for _ in range(M + 1)]

                rbuf = torch.empty(2 * M * T * N, dtype=torch.bfloat16, device=dev)

                def deep(M=M, b4=b4, comm=False, rbuf=rbuf, nb=nb):
                    e0 = (M - 1) * T
                    works = []
                    if comm:  # both neighbours' halo payload (2 x mT rows) through RCCL, to itself
                        flat = b4[0].view(-1)
                        works = nx.post(4, flat, [M * T * N], [2 * M * T * N], rbuf, [0], [2 * M * T * N])
                    step(b4[0], b4[1], row0, N, halo=M * T, steps=T, row_range=(T, rows - T))
                    for w in works:
                        w.wait()
                    ops.stencil5_fused_spans_(b4[0], b4[1], ((-e0, T), (rows - T, rows + e0)), row0, N,
                                              halo=M * T, steps=T, shape=edge_shape)
                    for ph in range(1, M):
                        e = (M - 1 - ph) * T
                        step(b4[ph % nb], b4[(ph + 1) % nb], row0, N, halo=M * T, steps=T, row_range=(-e, rows + e))

                for ph in range(M):
                    e = (M - 1 - ph) * T
                    step(c4[ph], c4[ph + 1], row0, N, halo=M * T, steps=T, row_range=(-e, rows + e))
                deeps[f"deep{M}"] = (M, deep, b4, c4)
                if nx is not None:
                    deeps[f"deep{M}+x"] = (M, lambda deep=deep: deep(comm=True), b4, c4)
                del u4

            full()
            res = {}
            variants = [("full", full), ("split3", split3), ("split2", split2), ("split2c", split2c)]
            only = os.environ.get("STENCIL_LAB_ONLY")  # e.g. "full,split2": a subset of the single-step shapes
            if only:
                variants = [v for v in variants if v[0] in only.split(",")]
            for name, fn in variants + [(k, v[1]) for k, v in deeps.items()]:
                out.zero_()
                fn()
                torch.cuda.synchronize()
                if name in deeps:
                    M, _, b4, c4 = deeps[name]
                    hh = M * T
                    same = torch.equal(b4[M % len(b4)][hh:-hh], c4[M][hh:-hh])
                    res[name] = (timed(fn) / M, same)
                    continue
                same = name == "full" or torch.equal(out[T:-T], ref[T:-T])
                res[name] = (timed(fn), same)
            line = " ".join(f"{k} {ms:.4f} ms {rows * N * T / ms / 1e6:7.0f} GLUP/s{'' if ok else ' MISMATCH'}"
                            for k, (ms, ok) in res.items())
            tag = (f" rpw={rpw}" if rpw else "") + ("" if paired is None else f" paired={int(paired)}")
            print(f"fuse={T} N={world} rows={rows:5d}{tag}  {line}", flush=True)
            del u, ref, out, deeps
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
