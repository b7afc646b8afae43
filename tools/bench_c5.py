#!/usr/bin/env python3
"""BASELINE config C5 on one GPU: FMG + V-cycles on a 1024^3 4-level
hierarchy (1024/512/256/128), mixed fp32 smoother / fp64 residual, next to
the all-fp64 cycle on the same inputs (SetBinaryBH source of params.txt,
bCoef = 1, Dirichlet-0, harmonic averaging, linear prolongation, nu = 4).

Prints one JSON line: ms per FMG and per V-cycle for both precisions, the
residual max-norm history of each, and the fp32 smoother's per-sweep time
(events around every fine-level sweep).

N-rank mode (round 5; BASELINE C5 as configs[4] states it, "1024^3 4-level
FMG cycle, 8xMI355X"): launched by torchrun with WORLD_SIZE = N > 1, the
domain is split as bench.py splits it (8 ranks: 2 x 2 x 2 boxes of 512^3),
one box per rank, deep halo, the coarsest depth gathered onto rank 0
(bench.agglomerate_default), the peer-mapped transport checked and RCCL as
the fallback (bench.make_comm); times are the max over ranks between
barriers, rank 0 prints the line.  MGIC_BENCH_DEVICE=0 puts every rank on one
GPU (a rehearsal: the ranks then share one GPU's bandwidth).

usage: bench_c5.py [--size 1024] [--levels 4] [--vcycles 6]
       torchrun --nproc-per-node N tools/bench_c5.py [...]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def oracle_check(mg, prm, levels, n=(128, 96, 64)):
    """The same kernels at a small size before the timed run: the mixed
    4-level FMG + one V-cycle of this script's settings (SetBinaryBH source,
    harmonic averaging, linear prolongation, params.txt's BC) on an n[0] x
    n[1] x n[2] box against the float32 restatement oracle/mixed.py, bit for
    bit (tests/test_mixed.py does the same on ragged / multi-box layouts)."""
    import numpy as np
    import oracle
    from oracle.mixed import MixedOracle
    nx, ny, nz = n
    dom = (0, 0, 0, nx - 1, ny - 1, nz - 1)
    dx = prm.L / nx
    grid = mg.Grid(mg.Comm(), dom, [dom], dx)
    fa, fb, frhs, fphi, fres = (mg.LevelData(grid) for _ in range(5))
    bh = prm.bh()
    bh["domain_length"] = prm.L
    mg.set_binary_bh_coefs(fa, frhs, bh)
    fb.set_val(1.0)
    fphi.set_zero()
    op = mg.OperatorParams(alpha=prm.alpha, beta=prm.beta, bc_lo=tuple(prm.bc_lo),
                           bc_hi=tuple(prm.bc_hi), bc_value=prm.bc_value,
                           coefficient_average_type=1, prolong_type=1)
    sp = mg.SolverParams(max_depth=levels - 1, n_pre=4, n_post=4, n_bottom=4, bottom_solver=0)
    mm = mg.MixedMultiGrid(mg.defineOperatorFactory(grid, fa, fb, op), sp)
    a, rhs = fa.download(0), frhs.download(0)
    o = oracle.OracleMG([dom], dom, dx, alpha=prm.alpha, beta=prm.beta, bc_lo=tuple(prm.bc_lo),
                        bc_hi=tuple(prm.bc_hi), bc_value=prm.bc_value, nlevels=levels, avg_type=1,
                        prolong_type=1, bottom_solver=0)
    for f, arr in ((oracle.ACOEF, a), (oracle.BCOEF, np.ones_like(a)), (oracle.RHS, rhs)):
        o.set(0, f, 0, arr)
    o.setup()
    m = MixedOracle(o, prm.alpha, prm.beta, tuple(prm.bc_lo), tuple(prm.bc_hi))
    ok = mm.init_residual(fphi, frhs, fres, 0) == np.abs(m.init_residual(np.zeros((nz, ny, nx)))).max()
    ok &= mm.fmg(fphi, frhs, fres, 0, ncycles=1) == np.abs(m.fmg(1)).max()
    ok &= mm.iteration(fphi, frhs, fres, 0) == np.abs(m.iteration()).max()
    ok &= bool(np.array_equal(fphi.download(0), m.phi))
    return {"size": f"{nx}x{ny}x{nz}", "levels": levels, "bit_identical": bool(ok),
            "against": "oracle/mixed.py (float32 restatement), FMG + 1 V-cycle, phi and norms"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--levels", type=int, default=4)
    ap.add_argument("--vcycles", type=int, default=6)
    ap.add_argument("--kinds", default="mixed,fp64")
    ap.add_argument("--no-oracle-check", action="store_true")
    ap.add_argument("--agglomerate-below", type=int, default=-1, help="-1: bench.py's default")
    ap.add_argument("--deep-halo", type=int, default=-1, help="-1: on for N > 1")
    ap.add_argument("--no-fmg", action="store_true")
    ap.add_argument("--transport", default="auto", choices=("auto", "ipc", "rccl"))
    args = ap.parse_args()
    # torch before the library: torch brings its own HIP runtime, and a
    # process that loads libmgic.so first ends up with two runtimes, which
    # fails at exit ("double free or corruption"); bench.py and the tests do
    # the same
    import torch  # noqa: F401
    import mg_ic_code_amd as mg
    from mg_ic_code_amd.params import read_params_file
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prm = read_params_file(os.path.join(root, "tests", "golden", "params.txt"))
    n = args.size
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dist = None
    sys.path.insert(0, root)
    import bench
    if world > 1:
        import datetime
        import torch.distributed as dist
        dev = int(os.environ.get("MGIC_BENCH_DEVICE", os.environ.get("LOCAL_RANK", "0")))
        torch.cuda.set_device(dev)
        mg.set_device(dev)
        dist.init_process_group("gloo", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=600))
        comm, transport = bench.make_comm(mg, torch, dist, rank, world, args.transport)
    else:
        comm, transport = mg.Comm(), "none"
    from mg_ic_code_amd.decomposition import decompose
    dom, boxes, owners = decompose((n, n, n), world)
    grid = mg.Grid(comm, dom, boxes, prm.L / n, owners=owners)
    fa, fb, frhs, fphi, fres = (mg.LevelData(grid) for _ in range(5))
    bh = prm.bh()
    bh["domain_length"] = prm.L
    mg.set_binary_bh_coefs(fa, frhs, bh)
    fb.set_val(1.0)
    agg = bench.agglomerate_default(world, n, args.levels) if args.agglomerate_below < 0 \
        else args.agglomerate_below
    op = mg.OperatorParams(alpha=prm.alpha, beta=prm.beta, bc_lo=tuple(prm.bc_lo),
                           bc_hi=tuple(prm.bc_hi), bc_value=prm.bc_value,
                           coefficient_average_type=1, prolong_type=1,
                           deep_halo=(1 if world > 1 else 0) if args.deep_halo < 0 else args.deep_halo)
    fac = mg.defineOperatorFactory(grid, fa, fb, op)
    sp = mg.SolverParams(max_depth=args.levels - 1, n_pre=4, n_post=4, n_bottom=4,
                         bottom_solver=0, agglomerate_below=agg)

    def sync():  # every rank's queued work done, then the max over ranks
        comm.synchronize()
        if dist is not None:
            dist.barrier()

    def tmax(x):
        if dist is None:
            return x
        import torch
        v = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(v, op=dist.ReduceOp.MAX)
        return float(v.item())

    where = "1 GPU (BASELINE C5 on one GPU)" if world == 1 else (
        f"{world} ranks, one box each ({'x'.join(str(b[3] - b[0] + 1) for b in boxes[:1])}), "
        f"deep halo, coarsest depth on rank 0 (agglomerate_below {agg}), {transport} transport"
        + (", every rank on one GPU (rehearsal)" if "MGIC_BENCH_DEVICE" in os.environ else ""))
    out = {"config": f"{n}^3 {args.levels}-level FMG + V-cycles, {where}",
           "n_ranks": world, "data": "synthetic (SetBinaryBH source of params.txt on device)",
           "oracle_check": oracle_check(mg, prm, args.levels)
           if rank == 0 and not args.no_oracle_check else None}
    for kind in args.kinds.split(","):
        solver = mg.MixedMultiGrid(fac, sp) if kind == "mixed" else mg.AMRMultiGrid(fac, sp)
        assert solver.num_depths == args.levels, solver.num_depths
        fphi.set_zero()
        hist = [solver.init_residual(fphi, frhs, fres, 0)]
        sync()
        t0 = time.perf_counter()
        hist.append(solver.iteration(fphi, frhs, fres, -1) if args.no_fmg
                    else solver.fmg(fphi, frhs, fres, -1))
        sync()
        t_fmg = tmax(time.perf_counter() - t0)
        hist[-1] = solver.init_residual(fphi, frhs, fres, 0)
        big = max((b[3] - b[0] + 1) * (b[4] - b[1] + 1) * (b[5] - b[2] + 1) for b in boxes)
        mg.prof_smoother(True, big)
        sync()
        t0 = time.perf_counter()
        for _ in range(args.vcycles):
            solver.iteration(fphi, frhs, fres, -1)
        sync()
        t_v = tmax((time.perf_counter() - t0) / args.vcycles)
        launches, passes, ms = mg.prof_smoother_read()
        mg.prof_smoother(False)
        hist.append(solver.init_residual(fphi, frhs, fres, 0))
        out[kind] = {"ms_per_fmg": round(t_fmg * 1e3, 3), "ms_per_vcycle": round(t_v * 1e3, 3),
                     "vcycles_per_s": round(1.0 / t_v, 3),
                     "residual_max_norm": {"initial": hist[0], "after_fmg": hist[1],
                                           f"after_fmg_plus_{args.vcycles}_vcycles": hist[2]},
                     "fine_sweep_ms_events": round(ms / launches, 4) if launches else None}
        del solver
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
