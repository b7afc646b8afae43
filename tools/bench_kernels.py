#!/usr/bin/env python3
"""Micro-benchmark of the non-smoother V-cycle kernels at n^3 (one box):
residual, restrictResidual, prolongIncrement, applyOp -- ms per call (wall
clock over `reps` back-to-back calls) and the §8(d) bytes/s of each."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    import numpy as np
    import mg_ic_code_amd as mg
    n = args.size
    comm = mg.Comm()
    dom = (0, 0, 0, n - 1, n - 1, n - 1)
    grid = mg.Grid(comm, dom, [dom], 100.0 / n)
    fa, fb, fr, fu, out = (mg.LevelData(grid) for _ in range(5))
    fa.set_val(-1.0)
    fb.set_val(1.0)
    fr.set_val(0.5)
    fu.set_val(0.25)
    fac = mg.defineOperatorFactory(grid, fa, fb, mg.OperatorParams(alpha=1.0, beta=-1.0))
    op = fac.AMRnewOp()
    op1 = fac.MGnewOp(1)
    rc, ec = mg.LevelData(op1.grid), mg.LevelData(op1.grid)
    ec.set_val(0.1)
    cells = n ** 3
    tests = {
        "residual": (lambda: op.residualI(out, fu, fr), 32),
        "restrict": (lambda: op.restrictResidual(rc, fu, fr), 25),
        "prolong": (lambda: op.prolongIncrement(fu, ec), 17),
        "applyOp": (lambda: op.applyOpI(out, fu), 24),
    }
    res = {"size": n, "tag": args.tag}
    for name, (fn, bpc) in tests.items():
        fn()
        comm.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            fn()
        comm.synchronize()
        ms = (time.perf_counter() - t0) / args.reps * 1e3
        res[name] = {"ms": round(ms, 4), "GBps": round(bpc * cells / (ms * 1e-3) / 1e9, 1)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
