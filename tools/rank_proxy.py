#!/usr/bin/env python3
"""Per-rank proxy of the N-GPU strong-scaling run on one GPU.

At N = 8 each rank owns one 256^3 box of the 512^3 domain and exchanges its
faces with RCCL.  One GPU cannot run 8 RCCL ranks, so this times one 256^3
box, periodic in every direction (all six faces exchanged, with itself),
with the exchange routed through RCCL self send/recv (the pack -> grouped
ncclSend/ncclRecv -> unpack path the ranks use) or the peer-mapped
transport.  It prints V-cycles/s; xGMI latency is not modelled.

--charge (round 5; the default for the 8-GPU share, a 256^3 box at three
levels) adds what the one-box proxy cannot run, to give the per-rank time of
`bench.py --gpus 8` as it is configured (the coarsest depth gathered onto
rank 0, bench.agglomerate_default):
  * the gathered bottom: the proxy relaxes its own 64^3 coarsest box (four
    sweeps, shell exchanges with itself); the real run gathers the eight
    64^3 boxes into one 128^3 box on rank 0, which relaxes it while the other
    ranks wait, and scatters the correction back.  Charged: - t(4 sweeps on
    the proxy's 64^3 depth) + t(4 sweeps on a 128^3 box, measured here) +
    two exchange latencies (t of one 1-deep exchange of the 64^3 depth,
    measured here);
  * the xGMI byte floor: every exchange's largest per-link
    message at 153 GB/s per link and direction (2 x 2 x 2 split: a rank's
    faces, edges and corner go to 7 different peers, one link each), the
    gather / scatter's 7 x 64^3 (+ faces) into / out of rank 0 included --
    added on top of the measured exchanges (whose self messages already pay
    the latency and a local copy of the same bytes), so an upper bound.
`charged_ms_per_vcycle` is the result.

--parts 2,2,2 --size 512 --periodic 0,0,0 --agglomerate-below 65 (round 5) runs
the whole 8-GPU split on this GPU instead -- the eight 256^3 boxes of
bench.py's decomposition, every box-to-box message through the transport's
put / get kernels, the coarsest depth gathered into one 128^3 box -- and
reports one rank's share of it (split_share below): the exchanged faces,
edges and corners of each box are exactly the real split's, not a periodic
box's six faces.

usage: rank_proxy.py [--size 256] [--transport rccl|ipc] [--deep 1] [--steps 30] [--charge]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--levels", type=int, default=3)
    ap.add_argument("--local", action="store_true", help="local copies instead of RCCL")
    ap.add_argument("--transport", choices=("rccl", "ipc"), default="rccl",
                    help="self messages through RCCL send/recv or the peer-mapped transport")
    ap.add_argument("--deep", type=int, default=0, help="deep halo (two sweeps per exchange)")
    ap.add_argument("--periodic", default="1,1,1", help="periodic directions (exchanged faces)")
    ap.add_argument("--shape", default=None,
                    help="nx,ny,nz of the rank's box (default: a --size cube); e.g. 512,512,256 "
                         "periodic 0,0,1 for one rank of the 2-GPU z-slab split")
    ap.add_argument("--parts", default="1,1,1",
                    help="split the box into this many boxes (all on this rank): the N-GPU "
                         "split's exchanges and gathers on one GPU")
    ap.add_argument("--agglomerate-below", type=int, default=0)
    ap.add_argument("--charge", type=int, default=-1,
                    help="charge the gathered bottom and the xGMI byte floor (1 on, 0 off; "
                         "default on for the 8-GPU share: --size 256, 3 levels, one part)")
    ap.add_argument("--norm-type", type=int, default=-1,
                    help="per-iteration residual norm (bench.py takes 0, the stop test's max "
                         "norm; -1: none, the proxy's default since round 1)")
    args = ap.parse_args()
    import mg_ic_code_amd as mg
    from mg_ic_code_amd.params import read_params_file
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prm = read_params_file(os.path.join(root, "tests", "golden", "params.txt"))
    n = args.size
    if args.local:
        comm = mg.Comm()
    elif args.transport == "ipc":
        comm = mg.Comm(transport="ipc", arena_bytes=64 << 20)
        comm.set_self_messages(True)
    else:
        comm = mg.Comm(0, 1, unique_id=mg.Comm.unique_id(), force_rccl=True)
        comm.set_self_messages(True)
    shp = tuple(int(v) for v in args.shape.split(",")) if args.shape else (n, n, n)
    dom = (0, 0, 0, shp[0] - 1, shp[1] - 1, shp[2] - 1)
    per = tuple(int(v) for v in args.periodic.split(","))
    from mg_ic_code_amd.decomposition import split_domain
    parts = tuple(int(v) for v in args.parts.split(","))
    grid = mg.Grid(comm, dom, split_domain(dom, parts), prm.L / n, periodic=per)
    fa, fb, frhs, fphi, fres = (mg.LevelData(grid) for _ in range(5))
    bh = prm.bh()
    mg.set_binary_bh_coefs(fa, frhs, bh)
    fb.set_val(1.0)
    fphi.set_zero()
    op = mg.OperatorParams(alpha=prm.alpha, beta=prm.beta, coefficient_average_type=1,
                           prolong_type=1, relax_mode=1, fused_smoother=1,
                           deep_halo=args.deep)
    fac = mg.defineOperatorFactory(grid, fa, fb, op)
    amg = mg.AMRMultiGrid(fac, mg.SolverParams(max_depth=args.levels - 1, n_pre=4, n_post=4,
                                               n_bottom=4, bottom_solver=0,
                                               agglomerate_below=args.agglomerate_below))
    amg.init_residual(fphi, frhs, fres, norm_type=0)
    amg.iterations(fphi, frhs, fres, args.warmup, norm_type=args.norm_type)
    comm.synchronize()
    x0 = comm.exchanges
    t0 = time.perf_counter()
    amg.iterations(fphi, frhs, fres, args.steps, norm_type=args.norm_type)
    comm.synchronize()
    dt = time.perf_counter() - t0
    n_x = (comm.exchanges - x0) / args.steps  # exchanges with messages per V-cycle
    r = amg.init_residual(fphi, frhs, fres, norm_type=0)
    out = {"size": n, "shape": shp, "parts": parts,
           "agglomerate_below": args.agglomerate_below, "deep": args.deep, "periodic": per,
           "norm_type": args.norm_type,
           "transport": "local" if args.local else args.transport,
           "vcycles_per_s": round(args.steps / dt, 2),
           "ms_per_vcycle": round(dt / args.steps * 1e3, 4), "final_residual": r}
    charge = args.charge if args.charge >= 0 else int(
        shp == (256, 256, 256) and args.levels == 3 and parts == (1, 1, 1)
        and args.agglomerate_below == 0)
    if charge:
        out.update(charges(mg, comm, amg, prm, args, shp, dt / args.steps * 1e3))
    P = parts[0] * parts[1] * parts[2]
    if P > 1 and args.agglomerate_below > 0 and not any(per):
        out.update(split_share(mg, comm, amg, prm, args, shp, parts, dt / args.steps * 1e3, n_x))
    print(json.dumps(out))


def gathered_bottom_ms(mg, prm, side, reps=50):
    """4 sweeps on one box of `side` cells (the gathered coarsest depth on
    rank 0; bench's coefficients, Dirichlet)"""
    c1 = mg.Comm()
    dom = (0, 0, 0, side[0] - 1, side[1] - 1, side[2] - 1)
    g = mg.Grid(c1, dom, [dom], prm.L / side[0])
    fa, fb, fr, fe = (mg.LevelData(g) for _ in range(4))
    bh = prm.bh()
    bh["domain_length"] = prm.L
    mg.set_binary_bh_coefs(fa, fr, bh)
    fb.set_val(1.0)
    fe.set_zero()
    op = mg.OperatorParams(alpha=prm.alpha, beta=prm.beta, coefficient_average_type=1,
                           prolong_type=1, relax_mode=1, fused_smoother=1)
    op_g = mg.defineOperatorFactory(g, fa, fb, op).AMRnewOp()
    return timed_ms(c1, lambda: op_g.relax(fe, fr, 4), reps)


def xgmi_floor_ms(s0, D, link=153e9):
    """every exchange's largest per-link message (one face of the rank's box
    of side s0 >> level) at `link` B/s, per V-cycle of D + 1 depths (charges()
    below), plus the gather / scatter of 7 coarsest boxes over rank 0's links"""
    floor_s = 0.0
    for lev in range(D):
        s = s0 >> lev
        floor_s += 4 * s * s * 4 * 8 / link + 2 * s * s * 8 / link
    sc = s0 >> D
    floor_s += (sc ** 3 + (sc + 2) ** 3) * 8 / link
    return floor_s * 1e3


def split_share(mg, comm, amg, prm, args, shp, parts, ms, n_x):
    """One rank's share of the N-GPU run from the whole split on this GPU
    (round 5): the N boxes of bench.py's decomposition on one rank, every
    box-to-box message through the transport's put / get kernels (self
    messages), the coarsest depth gathered into one box as bench.py does.
    Each rank's own work is 1/N of what this GPU ran, except
      * the gathered bottom, which rank 0 runs while the others wait;
      * the exchanges' fixed cost: one launch here moves all N boxes'
        messages, where every rank pays its own launch and hand-off, so each
        of the n_x exchanges per V-cycle is charged (1 - 1/N) x t_x more,
        t_x = one 1-deep exchange of the split's coarsest distributed depth
        (small messages: mostly that fixed cost);
    share = (t - t_bottom) / N + t_bottom + n_x (1 - 1/N) t_x, and
    `share_charged_ms` adds the xGMI byte floor (an upper bound: the local
    copies of the same bytes are already in t)."""
    P = parts[0] * parts[1] * parts[2]
    D = args.levels - 1
    side = [s >> D for s in shp]
    t_b = gathered_bottom_ms(mg, prm, side)
    e_d = amg.level_field(D - 1, 0)
    t_x = timed_ms(comm, e_d.exchange, 50)
    lat = n_x * (1.0 - 1.0 / P) * t_x
    share = (ms - t_b) / P + t_b + lat
    floor = xgmi_floor_ms(shp[0] // parts[0], D)
    out = {"split_boxes": P, "gathered_bottom_ms": round(t_b, 4),
           "exchanges_per_vcycle": round(n_x, 2), "exchange_fixed_ms": round(t_x, 4),
           "exchange_latency_charge_ms": round(lat, 4),
           "share_ms_per_vcycle": round(share, 4), "xgmi_floor_ms": round(floor, 4),
           "share_charged_ms_per_vcycle": round(share + floor, 4)}
    # the same charge with t_x as the device sees it (t_x above is the host
    # loop's rate, Python and ctypes included): HIP events around 50
    # exchanges queued behind 16 sweeps of depth 1, so the device runs them
    # back to back
    e1, r1 = amg.level_field(1, 0), amg.level_field(1, 1)
    t_xg = gpu_timed_ms(comm, lambda: amg.op(1).relax(e1, r1, 16), e_d.exchange, 50)
    if t_xg is not None:
        lat_g = n_x * (1.0 - 1.0 / P) * t_xg
        out.update({"exchange_fixed_gpu_ms": round(t_xg, 4),
                    "share_gpu_charge_ms_per_vcycle": round((ms - t_b) / P + t_b + lat_g, 4)})
    # t_x above still moves all N boxes' messages of depth D - 1 (128^3
    # boxes: ~3 MB), whose bytes t / N already holds; the fixed cost alone is
    # the same split's exchange on 16^3 boxes (messages of a few KB)
    from mg_ic_code_amd.decomposition import split_domain
    dom = tuple([0, 0, 0] + [16 * q - 1 for q in parts])
    g0 = mg.Grid(comm, dom, split_domain(dom, parts), 1.0 / (16 * parts[0]), periodic=(0, 0, 0))
    f0 = mg.LevelData(g0)
    f0.set_zero()
    t_x0 = gpu_timed_ms(comm, lambda: amg.op(1).relax(e1, r1, 16), f0.exchange, 50)
    if t_x0 is not None:
        lat0 = n_x * (1.0 - 1.0 / P) * t_x0
        out.update({"exchange_fixed_small_gpu_ms": round(t_x0, 4),
                    "share_small_charge_ms_per_vcycle": round((ms - t_b) / P + t_b + lat0, 4)})
    return out


def timed_ms(comm, fn, reps):
    fn()
    comm.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    comm.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def gpu_timed_ms(comm, blocker, fn, reps):
    """device time per call of fn, from HIP events on the library's stream
    around reps calls queued while `blocker` still runs (None if the host
    did not get ahead of the device, i.e. the events would time the host)"""
    import torch
    fn()
    comm.synchronize()
    s = torch.cuda.ExternalStream(comm.stream)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    blocker()
    a.record(s)
    for _ in range(reps):
        fn()
    b.record(s)
    ahead = not a.query()  # the blocker was still running when the last call was queued
    b.synchronize()
    comm.synchronize()
    return a.elapsed_time(b) / reps if ahead else None


def charges(mg, comm, amg, prm, args, shp, ms):
    """The gathered bottom and the xGMI byte floor of the 8-GPU run (module
    docstring), from measurements in this process."""
    D = args.levels - 1
    reps = 50
    # the proxy's own coarsest depth: 4 sweeps (shell exchanges with itself)
    # and one 1-deep exchange (the latency a gather / scatter pays)
    op_c = amg.op(D)
    e_c, r_c = amg.level_field(D, 0), amg.level_field(D, 1)
    t_own = timed_ms(comm, lambda: op_c.relax(e_c, r_c, 4), reps)
    t_x = timed_ms(comm, e_c.exchange, reps)
    # the gathered box: the 8 ranks' coarsest boxes as one box on rank 0
    # (2 x the side), bench's coefficients coarsened the same way, Dirichlet;
    # the xGMI floor: per exchange the largest per-link message (a face) over
    # 153 GB/s; per level of the 8-GPU split (box side s): e's 4-deep shell
    # before each of the 3 pairs that do not start from zero and r's once
    # (deep halo), plus two 1-deep face exchanges (level 0: phi for the
    # residual, e for the restriction; level 1: e for the restriction and the
    # coarse e for level 0's prolongation); the gather and the scatter move
    # 7 coarsest boxes (+ their faces) over rank 0's 7 links
    t_gath = gathered_bottom_ms(mg, prm, [2 * (s >> D) for s in shp], reps)
    floor_ms = xgmi_floor_ms(shp[0], D)
    charged = ms - t_own + t_gath + 2 * t_x + floor_ms
    return {"bottom_own_ms": round(t_own, 4), "bottom_gathered_ms": round(t_gath, 4),
            "gather_scatter_latency_ms": round(2 * t_x, 4), "xgmi_floor_ms": round(floor_ms, 4),
            "charged_ms_per_vcycle": round(charged, 4)}


if __name__ == "__main__":
    main()
