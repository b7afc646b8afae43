#!/usr/bin/env python3
"""V-cycles/s of the 512^3 3-level multigrid V-cycle on MI355X.

BASELINE.json metric: "V-cycles/sec + smoother HBM GB/s vs roofline, 512^3
3-level, 1/2/4/8 GPU".  One step = one AMRMultiGrid iteration on the single
AMR level (the unit the reference's preconditioner runs numMGIterations
times, Main_PoissonSolver.cpp:107-109):
    e = 0; MultiGrid::oneCycle(e, r); phi += e; r = rhs - L(phi)
over depths 512^3 / 256^3 / 128^3 with numMGsmooth = 4 GSRB sweeps pre and
post (params.txt:31) and 4 sweeps at the 128^3 bottom, harmonic coefficient
averaging (params.txt:43), linear prolongation, homogeneous Dirichlet faces.
Inputs: aCoef / rhs from the SetBinaryBH source of params.txt at psi = 1,
bCoef = 1, dpsi = 0 -- generated on device ("synthetic" = no dataset).

N > 1 (torchrun, one rank per GPU): the same 512^3 problem split into N
boxes (z first: 2 -> 512x512x256 slabs, 4 -> 1x2x2, 8 -> 2x2x2), halo
exchange by RCCL over xGMI: strong scaling.  Timing: barrier +
device-synchronize on both sides of exactly K steps, max over ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--size", type=int, default=512, help="cells per side of the fine level")
    ap.add_argument("--levels", type=int, default=3)
    ap.add_argument("--nsmooth", type=int, default=4)
    ap.add_argument("--no-fused", action="store_true", help="per-colour smoother launches")
    ap.add_argument("--boxes-per-rank", default="1,1,1",
                    help="split each rank's share into this many boxes (x,y,z) -- the multi-box "
                         "(exchange) path on one GPU")
    ap.add_argument("--overlap", type=int, default=0,
                    help="halo exchange overlapped with the sweep: 0 off, 1 auto (boxes >= 96^3), "
                         "2 always")
    ap.add_argument("--deep-halo", type=int, default=-1,
                    help="4-deep ghost shells, two sweeps per exchange: 0 off, 1 every level, "
                         "2 levels of boxes <= 128^3; default 1 for N > 1 (RCCL exchanges: "
                         "fewer, larger messages), 0 on one GPU (local copies are cheap)")
    ap.add_argument("--roofline-events", choices=("relax", "launch"), default="relax",
                    help="HIP events for the smoother roofline: one pair per relax call "
                         "(default; time / launches) or one pair per launch")
    ap.add_argument("--no-roofline-events", action="store_true",
                    help="no events in the timed region (roofline fields null)")
    ap.add_argument("--cpu-baseline-iters", type=int, default=10)
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "16")))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_smoother.json"))
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")

    import numpy as np
    import torch

    import mg_ic_code_amd as mg
    from mg_ic_code_amd.decomposition import decompose
    from mg_ic_code_amd.params import read_params_file

    # MGIC_BENCH_DEVICE pins every rank to one device (rehearsing the
    # multi-rank path on a one-GPU machine); default: one GPU per rank
    dev = int(os.environ.get("MGIC_BENCH_DEVICE", local_rank))
    torch.cuda.set_device(dev)
    mg.set_device(dev)

    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        uid = torch.zeros(128, dtype=torch.uint8)
        if rank == 0:
            uid = torch.tensor(list(mg.Comm.unique_id()), dtype=torch.uint8)
        dist.broadcast(uid, 0)
        comm = mg.Comm(rank, world, unique_id=bytes(uid.tolist()))
    else:
        comm = mg.Comm()

    prm = read_params_file(os.path.join(ROOT, "tests", "golden", "params.txt"))
    n = args.size
    dx = prm.L / n
    bh = prm.bh()
    bh["domain_length"] = dx * n
    bpr = tuple(int(v) for v in args.boxes_per_rank.split(","))
    dom, boxes, owners = decompose((n, n, n), world, boxes_per_rank=bpr)
    grid = mg.Grid(comm, dom, boxes, dx, owners=owners)
    fa, fb, frhs, fphi, fres = (mg.LevelData(grid) for _ in range(5))
    mg.set_binary_bh_coefs(fa, frhs, bh)
    fb.set_val(1.0)
    fphi.set_zero()
    op_params = mg.OperatorParams(alpha=prm.alpha, beta=prm.beta, bc_lo=tuple(prm.bc_lo),
                                  bc_hi=tuple(prm.bc_hi), bc_value=prm.bc_value,
                                  coefficient_average_type=1, prolong_type=1, relax_mode=1,
                                  fused_smoother=0 if args.no_fused else 1,
                                  overlap_exchange=args.overlap,
                                  deep_halo=(1 if world > 1 else 0) if args.deep_halo < 0
                                  else args.deep_halo)
    fac = mg.defineOperatorFactory(grid, fa, fb, op_params)
    sp = mg.SolverParams(max_depth=args.levels - 1, n_pre=args.nsmooth, n_post=args.nsmooth,
                         n_bottom=args.nsmooth, bottom_solver=0)
    amg = mg.AMRMultiGrid(fac, sp)
    assert amg.num_depths == args.levels, amg.num_depths
    r0 = amg.init_residual(fphi, frhs, fres, norm_type=0)

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        amg.iteration(fphi, frhs, fres, norm_type=-1)
    comm.synchronize()

    fine_cells = max((b[3] - b[0] + 1) * (b[4] - b[1] + 1) * (b[5] - b[2] + 1) for b in boxes)
    mg.prof_smoother(not args.no_roofline_events, fine_cells,
                     per_relax=args.roofline_events == "relax")
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        amg.iteration(fphi, frhs, fres, norm_type=-1)
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    launches, passes, smooth_ms = mg.prof_smoother_read()
    mg.prof_smoother(False)
    r_final = amg.init_residual(fphi, frhs, fres, norm_type=0)
    if dist is not None:
        import torch.distributed as dist_
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist_.all_reduce(t, op=dist_.ReduceOp.MAX)
        elapsed = float(t.item())

    # dominant kernel: the fine-level smoother; passes_per_launch = 1 (one
    # colour pass), 2 (fused sweep) or 4 (two fused sweeps per launch)
    passes_per_launch = passes / launches if launches else 0.0
    fused = passes_per_launch >= 2
    # SURVEY §8(d)'s per-pass credit (48 B/cell/colour pass: u, rhs, a, b in,
    # u out, every pass): an effective bandwidth, reported beside the roofline
    credit_per_launch = 48.0 * fine_cells * passes_per_launch
    # algorithmic (compulsory) bytes of one launch: u, rhs, a read once (+ b
    # unless it is one value everywhere -- bCoef = 1 here, which the operator
    # detects and does not load) + u written once, however many colour passes
    # it performs: the HBM roofline's numerator, so frac <= 1
    compulsory = 32.0 * fine_cells
    avg_launch_ms = smooth_ms / launches if launches else float("nan")
    achieved = compulsory / (avg_launch_ms * 1e-3) / 1e9 if launches else None
    effective = credit_per_launch / (avg_launch_ms * 1e-3) / 1e9 if launches else None
    traffic = None
    tj = args.traffic_json
    if os.path.exists(tj):
        try:
            with open(tj) as f:
                tinfo = json.load(f)
            key = f"n{n}_w{world}_{ {1: 'pass', 2: 'fused', 4: 'fused2x'}.get(round(passes_per_launch), 'mixed')}"
            if key in tinfo:
                traffic = tinfo[key]["hbm_bytes_per_launch"]
        except Exception:
            traffic = None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.cpu_baseline_iters > 0:
        cpu = cpu_baseline(args, grid, fa, frhs, dom, dx, np)

    if rank == 0:
        vps = args.steps / elapsed
        line = {
            "metric": "V-cycles/sec + smoother HBM GB/s vs roofline, 512^3 3-level, 1/2/4/8 GPU",
            "value": round(vps, 4),
            "unit": "V-cycles/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (SetBinaryBH source of params.txt generated on device; bCoef=1, dpsi=0)",
            "config": {
                "workload": f"{n}^3 {args.levels}-level V-cycle (AMRMultiGrid iteration), "
                            f"GSRB nu={args.nsmooth} pre/post, {args.nsmooth} GSRB sweeps at the bottom, "
                            "harmonic coef averaging, linear prolongation, Dirichlet-0",
                "n": n, "levels": args.levels, "numMGsmooth": args.nsmooth,
                "decomposition": f"{len(boxes)} box(es), {world} rank(s)",
                "halo": ("none (one box)" if len(boxes) == 1 else
                         "4-deep ghost shell per 2 fused sweeps (deep halo)" if op_params.deep_halo
                         else "2-deep ghost shell per fused sweep"),
                "parallelism": f"domain-decomposition x{world} (RCCL halo exchange)" if world > 1
                else "single GPU",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": {4: "two fused red-black GSRB sweeps per launch", 2: "fused red-black GSRB sweep",
                           1: "GSRB colour pass"}.get(round(passes_per_launch), "mixed smoother launches"),
                "colour_passes_per_launch": round(passes_per_launch, 3),
                "achieved": round(achieved, 1) if achieved else None,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                "traffic": traffic,
                "traffic_GBps": round(traffic / (avg_launch_ms * 1e-3) / 1e9, 1) if traffic and launches else None,
                "algorithmic_bytes_per_launch": compulsory,
                "effective_GBps": round(effective, 1) if effective else None,
                "note": "achieved/frac = algorithmic bytes per launch (32 B/cell: u, rhs, aCoef in, "
                        "u out, once per launch whatever its colour passes) / average launch time; "
                        "effective_GBps = SURVEY 8(d)'s 48 B/cell/colour-pass credit over the same "
                        "time (exceeds the peak once a launch fuses passes); traffic = PMC HBM "
                        "bytes per launch (profiles/traffic_smoother.json)",
                "avg_launch_ms": round(avg_launch_ms, 5) if launches else None,
                "timing": ("off" if args.no_roofline_events else
                           "HIP events on the operator stream, one pair per relax call "
                           "(interval / launches)" if args.roofline_events == "relax"
                           else "HIP events on the operator stream, one pair per launch"),
                "launches_timed": launches,
            },
            "cpu_baseline": cpu,
            "residual_max_norm": {"initial": r0, "final": r_final},
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def cpu_baseline(args, grid, fa, frhs, dom, dx, np):
    """The oracle (C restatement, OpenMP) on the same inputs: bounded sample
    of `cpu_baseline_iters` V-cycle iterations of the same workload."""
    import oracle
    n = args.size
    a = fa.download(0)
    rhs = frhs.download(0)
    oracle.set_threads(args.cpu_threads)
    o = oracle.OracleMG([dom], dom, dx, alpha=1.0, beta=-1.0, nlevels=args.levels, avg_type=1,
                        prolong_type=1, bottom_solver=0, n_pre=args.nsmooth, n_post=args.nsmooth,
                        n_bottom=args.nsmooth)
    o.set(0, oracle.ACOEF, 0, a)
    o.set(0, oracle.BCOEF, 0, np.ones_like(a))
    o.set(0, oracle.RHS, 0, rhs)
    del a, rhs
    o.setup()
    o.init_residual(0)
    t0 = time.perf_counter()
    for _ in range(args.cpu_baseline_iters):
        o.iteration(0)
    dt = time.perf_counter() - t0
    return {
        "value": round(args.cpu_baseline_iters / dt, 6),
        "unit": "V-cycles/s",
        "cores": oracle.get_threads(),
        "kind": "port",
        "sample": f"{args.cpu_baseline_iters} V-cycle iteration(s) of the same {n}^3 "
                  f"{args.levels}-level workload (oracle/mgic_oracle.c, OpenMP, -O3), {dt:.1f} s",
    }


if __name__ == "__main__":
    main()
