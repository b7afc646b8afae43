#!/usr/bin/env python3
"""BASELINE config C5 on one GPU: FMG + V-cycles on a 1024^3 4-level
hierarchy (1024/512/256/128), mixed fp32 smoother / fp64 residual, next to
the all-fp64 cycle on the same inputs (SetBinaryBH source of params.txt,
bCoef = 1, Dirichlet-0, harmonic averaging, linear prolongation, nu = 4).

Prints one JSON line: ms per FMG and per V-cycle for both precisions, the
residual max-norm history of each, and the fp32 smoother's per-sweep time
(events around every fine-level sweep).

usage: bench_c5.py [--size 1024] [--levels 4] [--vcycles 6]
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
    args = ap.parse_args()
    import mg_ic_code_amd as mg
    from mg_ic_code_amd.params import read_params_file
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prm = read_params_file(os.path.join(root, "tests", "golden", "params.txt"))
    n = args.size
    comm = mg.Comm()
    dom = (0, 0, 0, n - 1, n - 1, n - 1)
    grid = mg.Grid(comm, dom, [dom], prm.L / n)
    fa, fb, frhs, fphi, fres = (mg.LevelData(grid) for _ in range(5))
    bh = prm.bh()
    bh["domain_length"] = prm.L
    mg.set_binary_bh_coefs(fa, frhs, bh)
    fb.set_val(1.0)
    op = mg.OperatorParams(alpha=prm.alpha, beta=prm.beta, bc_lo=tuple(prm.bc_lo),
                           bc_hi=tuple(prm.bc_hi), bc_value=prm.bc_value,
                           coefficient_average_type=1, prolong_type=1)
    fac = mg.defineOperatorFactory(grid, fa, fb, op)
    sp = mg.SolverParams(max_depth=args.levels - 1, n_pre=4, n_post=4, n_bottom=4,
                         bottom_solver=0)
    out = {"config": f"{n}^3 {args.levels}-level FMG + V-cycles, 1 GPU (BASELINE C5 on one GPU)",
           "data": "synthetic (SetBinaryBH source of params.txt on device)",
           "oracle_check": oracle_check(mg, prm, args.levels)}
    for kind in ("mixed", "fp64"):
        solver = mg.MixedMultiGrid(fac, sp) if kind == "mixed" else mg.AMRMultiGrid(fac, sp)
        assert solver.num_depths == args.levels, solver.num_depths
        fphi.set_zero()
        hist = [solver.init_residual(fphi, frhs, fres, 0)]
        comm.synchronize()
        t0 = time.perf_counter()
        hist.append(solver.fmg(fphi, frhs, fres, -1))
        comm.synchronize()
        t_fmg = time.perf_counter() - t0
        hist[-1] = solver.init_residual(fphi, frhs, fres, 0)
        mg.prof_smoother(True, n ** 3)
        comm.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.vcycles):
            solver.iteration(fphi, frhs, fres, -1)
        comm.synchronize()
        t_v = (time.perf_counter() - t0) / args.vcycles
        launches, passes, ms = mg.prof_smoother_read()
        mg.prof_smoother(False)
        hist.append(solver.init_residual(fphi, frhs, fres, 0))
        out[kind] = {"ms_per_fmg": round(t_fmg * 1e3, 3), "ms_per_vcycle": round(t_v * 1e3, 3),
                     "vcycles_per_s": round(1.0 / t_v, 3),
                     "residual_max_norm": {"initial": hist[0], "after_fmg": hist[1],
                                           f"after_fmg_plus_{args.vcycles}_vcycles": hist[2]},
                     "fine_sweep_ms_events": round(ms / launches, 4) if launches else None}
        del solver
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
