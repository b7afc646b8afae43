#!/usr/bin/env python3
"""Run the reference program's solve (Main_PoissonSolver.cpp main / poissonSolve)
on device: read a params.txt, build the base level, and iterate the
nonlinear loop.  The per-iteration |dpsi| and linear iteration counts are
printed as the reference's pout() does.

usage: python tools/run_poisson.py [params.txt] [--size N] [--boxes-per-rank x,y,z]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("params", nargs="?", default=os.path.join(ROOT, "tests", "golden", "params.txt"))
    ap.add_argument("--size", type=int, default=0, help="override N (cells per side)")
    ap.add_argument("--boxes-per-rank", default="1,1,1")
    ap.add_argument("--max-depth", type=int, default=-1)
    args = ap.parse_args()
    import mg_ic_code_amd as mg
    from mg_ic_code_amd.decomposition import decompose
    from mg_ic_code_amd.nl import poisson_solve
    from mg_ic_code_amd.params import read_params_file
    prm = read_params_file(args.params)
    n = args.size or prm.N[0]
    bpr = tuple(int(v) for v in args.boxes_per_rank.split(","))
    dom, boxes, owners = decompose((n, n, n), 1, boxes_per_rank=bpr)
    grid = mg.Grid(mg.Comm(), dom, boxes, prm.domainLength[0] / n, owners=owners)
    t0 = time.perf_counter()
    res = poisson_solve(grid, prm, max_depth=args.max_depth)
    mg.device_synchronize()
    dt = time.perf_counter() - t0
    for i, (nrm, it) in enumerate(zip(res.dpsi_norms, res.linear_iterations)):
        print(f"Main Loop Iteration {i + 1}: {it} BiCGStab iterations, norm of dpsi {nrm:.6e}")
    print(json.dumps({"n": n, "boxes": len(boxes), "nl_iterations": len(res.dpsi_norms),
                      "converged": res.converged, "seconds": round(dt, 3)}))


if __name__ == "__main__":
    main()
