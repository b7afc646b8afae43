#!/usr/bin/env python3
"""Per-rank proxy of the N-GPU strong-scaling run on one GPU.

At N = 8 each rank owns one 256^3 box of the 512^3 domain and exchanges its
faces with RCCL.  One GPU cannot run 8 RCCL ranks, so this times one 256^3
box, periodic in every direction (all six faces exchanged, with itself),
with the exchange routed through RCCL self send/recv (the pack -> grouped
ncclSend/ncclRecv -> unpack path the ranks use) or the peer-mapped
transport.  It prints V-cycles/s; xGMI latency is not modelled.

usage: rank_proxy.py [--size 256] [--transport rccl|ipc] [--deep 1] [--steps 30]
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
    t0 = time.perf_counter()
    amg.iterations(fphi, frhs, fres, args.steps, norm_type=args.norm_type)
    comm.synchronize()
    dt = time.perf_counter() - t0
    r = amg.init_residual(fphi, frhs, fres, norm_type=0)
    print(json.dumps({"size": n, "shape": shp, "parts": parts,
                      "agglomerate_below": args.agglomerate_below, "deep": args.deep, "periodic": per,
                      "norm_type": args.norm_type,
                      "transport": "local" if args.local else args.transport,
                      "vcycles_per_s": round(args.steps / dt, 2),
                      "ms_per_vcycle": round(dt / args.steps * 1e3, 4), "final_residual": r}))


if __name__ == "__main__":
    main()
