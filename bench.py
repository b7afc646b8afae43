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
HBM_COPY_GBS = 6290.0  # measured float4 copy rate (MI355X_MICROARCH.md: ≈6.3 TB/s achievable)


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
    ap.add_argument("--deep-halo", type=int, default=-1,
                    help="4-deep ghost shells, two sweeps per exchange: 0 off, 1 every level, "
                         "2 levels of boxes <= 128^3; default 1 for N > 1 (RCCL exchanges: "
                         "fewer, larger messages), 0 on one GPU (local copies are cheap)")
    ap.add_argument("--transport", choices=("auto", "ipc", "rccl"), default="auto",
                    help="N > 1 halo transport: peer-mapped buffers + device flags (ipc), RCCL "
                         "send/recv (rccl), or ipc with an RCCL fallback (auto, default)")
    ap.add_argument("--agglomerate-below", type=int, default=-1,
                    help="gather MG depths whose boxes have a side below this to one box on "
                         "rank 0 (the coarsest levels solved on rank 0); 0 off; default: "
                         "agglomerate_default() (DESIGN.md 6)")
    ap.add_argument("--roofline-events", choices=("relax", "launch"), default="relax",
                    help="HIP events for the smoother roofline: one pair per relax call "
                         "(default; time / launches) or one pair per launch")
    ap.add_argument("--no-roofline-events", action="store_true",
                    help="skip the second, event-instrumented timed region (roofline fields null)")
    ap.add_argument("--no-bottom", action="store_true",
                    help="skip the separately reported BiCGStab-bottom V-cycle timing")
    ap.add_argument("--bottom-vcycles", type=int, default=8,
                    help="V-cycles timed from phi = 0 with the BiCGStab bottom (fixed, so the "
                         "bottom's work does not depend on --steps / --warmup)")
    ap.add_argument("--bottom-replays", type=int, default=10,
                    help="replays of the first V-cycle's bottom solve from e = 0 on its coarse "
                         "residual")
    ap.add_argument("--norm-type", type=int, default=0,
                    help="per-iteration residual norm of AMRMultiGrid's stop test (params.txt:37-38, "
                         "m_normType 0 = max norm; -1 skips it)")
    ap.add_argument("--cpu-baseline-iters", type=int, default=10)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads for the all-cores CPU baseline (0: the CPUs this process may run "
                         "on, capped by the cgroup CPU quota and by OMP_NUM_THREADS when set -- "
                         "the job's CPU share on a shared GPU node); pinned one per CPU")
    ap.add_argument("--cpu-1core-iters", type=int, default=1,
                    help="V-cycle iterations of the 1-thread CPU baseline (0 skips it)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-traffic", action="store_true",
                    help="skip the in-run PMC passes (rocprofv3 FETCH_SIZE / WRITE_SIZE of the "
                         "smoother launches, two child runs of this script)")
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

    # MGIC_BENCH_DEVICE pins every rank to one device (rehearsing the
    # multi-rank path on a one-GPU machine); default: one GPU per rank
    dev = int(os.environ.get("MGIC_BENCH_DEVICE", local_rank))
    torch.cuda.set_device(dev)
    mg.set_device(dev)

    dist = None
    transport = "none"
    if world > 1:
        import datetime
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=300))
        comm, transport = make_comm(mg, torch, dist, rank, world, args.transport)
    else:
        comm = mg.Comm()

    bpr = tuple(int(v) for v in args.boxes_per_rank.split(","))
    case = build_case(mg, comm, world, args.size, args.levels, args.nsmooth, bpr,
                      fused=0 if args.no_fused else 1,
                      deep_halo=(1 if world > 1 else 0) if args.deep_halo < 0 else args.deep_halo,
                      agglomerate_below=agglomerate_default(world, args.size, args.levels)
                      if args.agglomerate_below < 0 else args.agglomerate_below)
    n = args.size
    boxes, grid, fa, frhs, fphi, fres = (case[k] for k in ("boxes", "grid", "fa", "frhs", "fphi",
                                                           "fres"))
    dom, dx, amg, op_params = case["dom"], case["dx"], case["amg"], case["op_params"]
    r0 = amg.init_residual(fphi, frhs, fres, norm_type=0)
    nt = args.norm_type

    def barrier():
        if dist is not None:
            dist.barrier()

    def timed(fn):
        """fn() between barrier + device synchronize on both sides; the max
        over ranks of the wall time"""
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        barrier()
        el = time.perf_counter() - t0
        if dist is not None:
            t = torch.tensor([el], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el, out

    # AMRMultiGrid::solve's loop body K times (amg.iterations: the same phi
    # and norms as K iteration() calls, bit for bit)
    amg.iterations(fphi, frhs, fres, args.warmup, norm_type=nt)
    comm.synchronize()
    # the headline: K AMRMultiGrid iterations -- the V-cycle, r = rhs - L(phi)
    # and (norm_type >= 0) its norm for the stop test, read on the host each
    # iteration before the next iteration's first phi-writing launch is
    # queued (the GPU runs the next V-cycle's earlier part meanwhile) -- with
    # no instrumentation in the timed region
    elapsed, hist = timed(lambda: amg.iterations(fphi, frhs, fres, args.steps, norm_type=nt))

    # the roofline: K more iterations with a HIP event pair around every
    # fine-level smoother relax (or launch) on the operator's stream
    fine_cells = max((b[3] - b[0] + 1) * (b[4] - b[1] + 1) * (b[5] - b[2] + 1) for b in boxes)
    launches = passes = 0
    smooth_ms = 0.0
    elapsed_ev = None
    if not args.no_roofline_events:
        mg.prof_smoother(True, fine_cells, per_relax=args.roofline_events == "relax")
        elapsed_ev, _ = timed(lambda: amg.iterations(fphi, frhs, fres, args.steps, norm_type=nt))
        launches, passes, smooth_ms = mg.prof_smoother_read()
        mg.prof_smoother(False)
    r_final = amg.init_residual(fphi, frhs, fres, norm_type=0)

    # the bottom solve reported separately ("+ bottom (report
    # separately)"): the same V-cycle with the reference's BiCGStab bottom
    # (Main_PoissonSolver.cpp:103-117) at the coarsest depth instead of
    # numMGsmooth GSRB sweeps, from phi = 0 on a second hierarchy
    bottom = None
    if not args.no_bottom:
        bottom = bottom_timing(mg, case, args, timed, nt, elapsed / args.steps)

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
    if rank == 0 and world == 1 and not args.no_traffic and launches:
        traffic = pmc_traffic(args)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.cpu_baseline_iters > 0:
        cpu = cpu_baseline(args, grid, fa, frhs, dom, dx, np)
    hb = traffic.get("hbm_bytes_per_launch") if traffic else None

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
            "timed_region": "K AMRMultiGrid iterations, no instrumentation (the roofline's "
                            "event-timed iterations run after it, separately)",
            "value_with_roofline_events": (round(args.steps / elapsed_ev, 4)
                                           if elapsed_ev else None),
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
                "parallelism": f"domain-decomposition x{world} ({transport} halo exchange)"
                if world > 1 else "single GPU",
                "transport": transport,
                "agglomerate_below": case["agglomerate_below"],
                "bottom_solver": f"{args.nsmooth} GSRB sweeps (the BiCGStab bottom: 'bottom')",
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
                "traffic": hb,
                "traffic_GBps": round(hb / (avg_launch_ms * 1e-3) / 1e9, 1) if hb and launches else None,
                # the guide's measured float4 copy rate: what the memory
                # system delivers in practice, beside the 8 TB/s spec peak
                "copy_rate_GBps": HBM_COPY_GBS,
                "traffic_frac_of_copy_rate": (round(hb / (avg_launch_ms * 1e-3) / 1e9 / HBM_COPY_GBS, 4)
                                              if hb and launches else None),
                "traffic_detail": traffic,
                "algorithmic_bytes_per_launch": compulsory,
                "effective_GBps": round(effective, 1) if effective else None,
                "note": "achieved/frac = algorithmic bytes per launch (32 B/cell: u, rhs, aCoef in, "
                        "u out, once per launch whatever its colour passes) / average launch time; "
                        "effective_GBps = SURVEY 8(d)'s 48 B/cell/colour-pass credit over the same "
                        "time (exceeds the peak once a launch fuses passes); traffic = bytes moved "
                        "between L2 and the memory fabric per fine-level smoother launch (HBM plus "
                        "Infinity-Cache hits, which FETCH_SIZE also counts) from two rocprofv3 --pmc "
                        "passes (FETCH_SIZE x2 gfx950 correction, WRITE_SIZE) run by this bench on the "
                        "same workload; copy_rate_GBps = the measured float4 copy rate of "
                        "MI355X_MICROARCH.md (6.29 TB/s)",
                "avg_launch_ms": round(avg_launch_ms, 5) if launches else None,
                "timing": ("off" if args.no_roofline_events else
                           "HIP events on the operator stream, one pair per relax call "
                           "(interval / launches), in K iterations timed after the headline's"
                           if args.roofline_events == "relax"
                           else "HIP events on the operator stream, one pair per launch, in K "
                                "iterations timed after the headline's"),
                "launches_timed": launches,
            },
            "bottom": bottom,
            "cpu_baseline": cpu,
            "residual_max_norm": {"initial": r0, "final": r_final},
            "norm_type_in_step": nt,
            "residual_norm_history": hist[-3:] if nt >= 0 else None,
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def make_comm(mg, torch, dist, rank, world, transport):
    """The N > 1 communicator: the peer-mapped transport ("ipc": ranks map
    each other's receive buffers, csrc/transport.hpp; works when ranks share
    a device) or RCCL.  "auto" tries ipc, checks it on this job's devices
    (mg_ic_code_amd/commcheck.py: one exchange and one reduction with known
    results), and falls back to RCCL on every rank when any rank could not
    set it up or saw a wrong value (a collective decision)."""
    if transport in ("ipc", "auto"):
        comm, ok, err = None, 1, ""
        try:
            comm = mg.Comm(rank, world, transport="ipc")
            from mg_ic_code_amd.commcheck import check_transport
            if not check_transport(comm, world):
                ok, err = 0, "transport check: wrong halo or reduction values"
        except Exception as e:  # noqa: BLE001 -- decided collectively below
            ok, err = 0, str(e)
        t = torch.tensor([ok], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        if int(t.item()) == 1:
            return comm, "ipc"
        if transport == "ipc":
            raise SystemExit(f"rank {rank}: peer-mapped transport unavailable: {err}")
        del comm
    uid = torch.zeros(128, dtype=torch.uint8)
    if rank == 0:
        uid = torch.tensor(list(mg.Comm.unique_id()), dtype=torch.uint8)
    dist.broadcast(uid, 0)
    return mg.Comm(rank, world, unique_id=bytes(uid.tolist())), "rccl"


def agglomerate_default(world, n, levels):
    """agglomerate_below for an N-rank run: MG depths whose boxes have a side
    below this are gathered onto one box on rank 0 (the coarsest levels
    solved on rank 0, north_star / Main_PoissonSolver.cpp:103-117); 0 on one
    rank.  N > 1: the coarsest depth always (its per-rank boxes, e.g. 64^3 at
    the 8-GPU split's third level, go to one box on rank 0), and every depth
    whose boxes are narrower than 32 cells.  DESIGN.md 6 records the
    measurement: the 8-rank split gathered and distributed run alike
    (profiles/r04a_rank_rehearsal_agg.jsonl)."""
    if world <= 1:
        return 0
    from mg_ic_code_amd.decomposition import decompose
    _, boxes, _ = decompose((n, n, n), world)
    side = min(b[3 + d] - b[d] + 1 for b in boxes for d in range(3)) >> (levels - 1)
    return max(32, side + 1)


def build_case(mg, comm, world, n, levels, nsmooth, boxes_per_rank=(1, 1, 1), fused=1,
               deep_halo=0, agglomerate_below=0, bottom_solver=0):
    """The bench workload (BASELINE config C3 / C4): n^3 split over `world`
    ranks (z first), SetBinaryBH aCoef / rhs of params.txt at psi = 1 on
    device, bCoef = 1, phi = 0, the reference operator settings, and an
    AMRMultiGrid of `levels` depths.  tests/mp_worker.py builds the same."""
    from mg_ic_code_amd.decomposition import decompose
    from mg_ic_code_amd.params import read_params_file
    prm = read_params_file(os.path.join(ROOT, "tests", "golden", "params.txt"))
    dx = prm.L / n
    bh = prm.bh()
    bh["domain_length"] = dx * n
    dom, boxes, owners = decompose((n, n, n), world, boxes_per_rank=tuple(boxes_per_rank))
    grid = mg.Grid(comm, dom, boxes, dx, owners=owners)
    fa, fb, frhs, fphi, fres = (mg.LevelData(grid) for _ in range(5))
    mg.set_binary_bh_coefs(fa, frhs, bh)
    fb.set_val(1.0)
    fphi.set_zero()
    op_params = mg.OperatorParams(alpha=prm.alpha, beta=prm.beta, bc_lo=tuple(prm.bc_lo),
                                  bc_hi=tuple(prm.bc_hi), bc_value=prm.bc_value,
                                  coefficient_average_type=1, prolong_type=1, relax_mode=1,
                                  fused_smoother=fused, deep_halo=deep_halo)
    fac = mg.defineOperatorFactory(grid, fa, fb, op_params)
    sp = mg.SolverParams(max_depth=levels - 1, n_pre=nsmooth, n_post=nsmooth, n_bottom=nsmooth,
                         bottom_solver=bottom_solver, agglomerate_below=agglomerate_below)
    amg = mg.AMRMultiGrid(fac, sp)
    assert amg.num_depths == levels, amg.num_depths
    return dict(dom=dom, boxes=boxes, owners=owners, dx=dx, grid=grid, fa=fa, fb=fb, frhs=frhs,
                fphi=fphi, fres=fres, fac=fac, amg=amg, op_params=op_params,
                agglomerate_below=agglomerate_below)


def bottom_timing(mg, case, args, timed, nt, gsrb_ms):
    """The V-cycle with the reference's bottom solver (bottom_solver = 1,
    Main_PoissonSolver.cpp:103-117: MultilevelLinearOp's BiCGStab at the
    coarsest MG depth, preconditioned by preCond,
    Source/VariableCoeffPoissonOperator.cpp:72-104) on a second hierarchy
    over the same operator factory.  Every timed solve starts from work: the
    K_b = --bottom-vcycles V-cycles are timed from phi = 0 (a fixed count,
    independent of --steps / --warmup, short of the roundoff floor where
    BiCGStab would stop on its absolute tolerance at once), and the solves
    are then replayed from e = 0 on one coarse residual (a fixed amount of
    work per solve).  Reported: ms per V-cycle, the bottom's share, the
    iterations per solve and the coarse residual norms the solves started
    from."""
    amg = mg.AMRMultiGrid(case["fac"], mg.SolverParams(
        max_depth=args.levels - 1, n_pre=args.nsmooth, n_post=args.nsmooth,
        n_bottom=args.nsmooth, bottom_solver=1, agglomerate_below=case["agglomerate_below"]))
    phi, res = mg.LevelData(case["grid"]), mg.LevelData(case["grid"])
    frhs = case["frhs"]
    kb = args.bottom_vcycles

    def fresh():
        phi.set_zero()
        amg.init_residual(phi, frhs, res, norm_type=0)

    # one untimed iteration allocates the solver's temporaries; the first
    # V-cycle's bottom solve (from the largest coarse residual) is then
    # replayed from e = 0: a fixed amount of work per solve
    fresh()
    amg.iterations(phi, frhs, res, 1, norm_type=nt)
    rep_ms, rep_iters, rep_r0, rep_n = amg.bottom_replay(args.bottom_replays)
    fresh()
    el, hist = timed(lambda: amg.iterations(phi, frhs, res, kb, norm_type=nt))
    ms = el / kb * 1e3
    # the same K_b iterations again with HIP events around each solve on the
    # rank that runs it (rank 0 when the coarsest depth is gathered)
    fresh()
    amg.bottom_timer(True)
    amg.iterations(phi, frhs, res, kb, norm_type=nt)
    solve_ms, solves = amg.bottom_ms()
    iters, r0_lo, r0_hi = amg.bottom_iters()
    amg.bottom_timer(False)
    dev = amg.bottom_info()[0]
    out = {"solver": "BiCGStab (imax 80, eps 1e-6, reps 1e-12, restarts 5; preCond = lambda r + "
                     "2 GSRB)",
           "depth": args.levels - 1,
           "vcycles_timed": kb,
           "vcycles_per_s": round(kb / el, 4), "ms_per_vcycle": round(ms, 4),
           "gsrb_bottom_ms_per_vcycle": round(gsrb_ms * 1e3, 4),
           "bottom_delta_ms": round(ms - gsrb_ms * 1e3, 4),
           "bottom_solve_ms_rank0": round(solve_ms / solves, 4) if solves else None,
           "bottom_solves_timed_rank0": solves,
           "iterations_per_solve": round(iters / solves, 3) if solves else None,
           "coarse_residual_norm_range": [r0_lo, r0_hi] if solves else None,
           "on_device": dev,
           "replay": ({"solves": rep_n, "ms_per_solve": round(rep_ms / rep_n, 4),
                       "iterations_per_solve": rep_iters,
                       "ms_per_iteration": round(rep_ms / rep_n / max(1, rep_iters), 5),
                       "coarse_residual_norm": rep_r0} if rep_n else None),
           "residual_norm_history": hist[-3:] if nt >= 0 else None,
           "note": "every timed solve starts from an unconverged coarse residual (the range "
                   "above): K_b V-cycles from phi = 0; the replay re-solves the first V-cycle's "
                   "coarse residual from e = 0; on_device: BiCGStabSolver::solveDevice (scalars "
                   "and stop tests on the GPU, no readback per iteration)"}
    del amg, phi, res
    return out


def host_cpus():
    """(CPUs this process may run on, CPUs of the machine, the cgroup's CPU
    quota in whole CPUs or None when unlimited)."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return avail, os.cpu_count() or avail, quota


def cpu_baseline(args, grid, fa, frhs, dom, dx, np):
    """The oracle (C restatement, OpenMP) on the same inputs: bounded samples
    of the same workload on all the host cores this job may use and on one
    core.  Chombo itself cannot be built here."""
    import oracle
    n = args.size
    a = fa.download(0)
    rhs = frhs.download(0)
    avail, machine, quota = host_cpus()
    threads = args.cpu_threads
    reason = "--cpu-threads"
    if threads <= 0:
        threads, reason = avail, "every CPU this process may run on"
        if quota and quota < threads:
            threads, reason = quota, "the cgroup CPU quota (/sys/fs/cgroup/cpu.max)"
        omp = os.environ.get("OMP_NUM_THREADS")
        if omp and omp.isdigit() and int(omp) < threads:
            threads = int(omp)
            reason = ("OMP_NUM_THREADS, which the GPU pool sets to the job's CPU share (16 host "
                      "CPUs per GPU on a shared node; the machine's other CPUs belong to other "
                      "jobs)")
    try:
        cpus = sorted(os.sched_getaffinity(0))
    except AttributeError:
        cpus = list(range(avail))
    o = oracle.OracleMG([dom], dom, dx, alpha=1.0, beta=-1.0, nlevels=args.levels, avg_type=1,
                        prolong_type=1, bottom_solver=0, n_pre=args.nsmooth, n_post=args.nsmooth,
                        n_bottom=args.nsmooth)
    o.set(0, oracle.ACOEF, 0, a)
    o.set(0, oracle.BCOEF, 0, np.ones_like(a))
    o.set(0, oracle.RHS, 0, rhs)
    del a, rhs
    o.setup()
    o.init_residual(0)

    def timed(nthreads, iters, pin):
        oracle.set_threads(nthreads)
        pinned = 0
        if pin:  # thread t on CPU t of a set spread evenly over this job's CPUs
            step = max(1, len(cpus) // max(1, nthreads))
            pinned = oracle.pin_threads(cpus[::step][:nthreads])
        else:
            oracle.pin_threads(cpus, pin=False)
        t0 = time.perf_counter()
        for _ in range(iters):
            o.iteration(0)
        return time.perf_counter() - t0, oracle.get_threads(), pinned

    # pinned (one thread per CPU, spread over the job's CPU set) and left to
    # the scheduler: on a node shared with other jobs the scheduler can move
    # threads off busy CPUs, so both are timed and the faster one reported
    dtp, used, npin = timed(threads, args.cpu_baseline_iters, True)
    dtu, _, _ = timed(threads, args.cpu_baseline_iters, False)
    vp = round(args.cpu_baseline_iters / dtp, 6)
    vu = round(args.cpu_baseline_iters / dtu, 6)
    dt, pinned = (dtp, npin) if dtp <= dtu else (dtu, 0)
    out = {
        "value": round(args.cpu_baseline_iters / dt, 6),
        "unit": "V-cycles/s",
        "cores": used,
        "kind": "port",
        "sample": f"{args.cpu_baseline_iters} V-cycle iteration(s) of the same {n}^3 "
                  f"{args.levels}-level workload (oracle/mgic_oracle.c, OpenMP, -O3), {dt:.1f} s",
        "cores_reason": reason,
        "pinned_threads": pinned,
        "value_pinned": vp,
        "value_unpinned": vu,
        "host_cpus_available": avail,
        "host_cpus_machine": machine,
        "host_cpu_quota": quota,
    }
    if args.cpu_1core_iters > 0:
        dt1, _, _ = timed(1, args.cpu_1core_iters, True)
        out["one_core"] = {"value": round(args.cpu_1core_iters / dt1, 6), "unit": "V-cycles/s",
                           "cores": 1,
                           "sample": f"{args.cpu_1core_iters} V-cycle iteration(s), 1 thread, "
                                     f"{dt1:.1f} s"}
    oracle.set_threads(threads)
    oracle.pin_threads(cpus, pin=False)  # release the threads to the whole set
    return out


def pmc_traffic(args):
    """HBM bytes per fine-level smoother launch, measured by this bench: two
    child runs of the same workload under rocprofv3 --pmc (FETCH_SIZE, then
    WRITE_SIZE: they do not fit one pass), each under its own time limit.
    MI355X_MICROARCH.md 'HBM': on gfx950 FETCH_SIZE counts half the bytes of
    a wide coalesced read (x2); WRITE_SIZE is exact for 16-B stores; KiB."""
    import csv
    import glob
    import re
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if not prof:
        return None
    work = tempfile.mkdtemp(prefix="mgic_pmc_")
    env = dict(os.environ, TMPDIR="/tmp")
    vals = {}
    kname = None
    try:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(work, ctr)
            # the two-sweep smoother launches
            cmd = ["timeout", "-s", "KILL", "150", prof, "--pmc", ctr, "--kernel-include-regex",
                   "k_gsrb_tb2<double, 64, 22", "-d", d, "-o", "p", "--output-format", "csv", "--",
                   sys.executable, os.path.abspath(__file__), "--steps", "2", "--warmup", "1",
                   "--size", str(args.size), "--levels", str(args.levels), "--nsmooth",
                   str(args.nsmooth), "--no-cpu-baseline", "--no-traffic",
                   "--no-roofline-events", "--no-bottom", "--norm-type", str(args.norm_type)]
            r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, env=env,
                               timeout=200)
            if r.returncode != 0:
                return {"error": f"rocprofv3 --pmc {ctr} pass exited {r.returncode}"}
            rows = []
            for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                rows += list(csv.DictReader(open(f)))
            if not rows:
                return {"error": f"no counter rows for {ctr}"}
            top = max(int(x["Grid_Size"]) for x in rows)  # the fine level's launches
            v = [float(x["Counter_Value"]) for x in rows if int(x["Grid_Size"]) == top]
            m = re.search(r"(k_gsrb_tb2<[^(]*>)", rows[0]["Kernel_Name"])
            kname = m.group(1) if m else rows[0]["Kernel_Name"][:80]
            vals[ctr] = (sum(v) / len(v), len(v))
    except Exception as e:  # the bench line never fails for want of counters
        return {"error": f"{type(e).__name__}: {e}"}
    finally:
        shutil.rmtree(work, ignore_errors=True)
    rd = vals["FETCH_SIZE"][0] * 1024.0 * 2.0
    wr = vals["WRITE_SIZE"][0] * 1024.0
    return {"hbm_bytes_per_launch": rd + wr, "read_bytes_per_launch": rd,
            "write_bytes_per_launch": wr, "launches_sampled": vals["FETCH_SIZE"][1],
            "kernel": kname,
            "method": "this run: rocprofv3 --pmc FETCH_SIZE (x1024 x2, gfx950 half count) and "
                      "WRITE_SIZE (x1024) in separate child passes of the same workload, averaged "
                      "over the fine-level two-sweep launches (plain, ACC and ZIN)"}


if __name__ == "__main__":
    main()
