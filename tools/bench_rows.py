#!/usr/bin/env python3
"""Measurements for SURVEY §8(f) rows 1-3 on one GPU (row 4: bench_output.py).

(f)1 outer BiCGStab + MultilevelLinearOp::preCond: solver.solve(dpsi, rhs) on
     an n^3 level (params.txt coefficients at psi = 1, NL iteration 0): wall
     time, BiCGStab iterations, time per iteration.
(f)2 NL loop: set_a_coef + set_rhs on device (k_binary_bh) at n^3, and
     poisson_solve on an m^3 level (NL iterations to convergence or the cap).
(f)3 AMR V-cycle: a 3-level hierarchy (a^3 base, then a^3-cell patches of the
     2a^3 and 4a^3 domains, properly nested, centred on the punctures), the
     params.txt coefficients on every level; time per AMR iteration.  And the
     NL loop over that hierarchy (poisson_solve with max_level = 2:
     per-level coefficients, multilevel BiCGStab, QuadCFInterp of dpsi,
     Main_PoissonSolver.cpp:129-220).

Prints one JSON line.  usage: bench_rows.py [--n 512] [--m 256] [--amr 128]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--m", type=int, default=256)
    ap.add_argument("--amr", type=int, default=128)
    ap.add_argument("--amr-iters", type=int, default=5)
    ap.add_argument("--nl-iters", type=int, default=3)
    args = ap.parse_args()
    import mg_ic_code_amd as mg
    from mg_ic_code_amd.nl import NLDivergenceError, poisson_solve
    from mg_ic_code_amd.params import read_params_file
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prm = read_params_file(os.path.join(root, "tests", "golden", "params.txt"))
    comm = mg.Comm()
    sync = comm.synchronize
    out = {"data": "synthetic (params.txt BH source on device)"}
    L = prm.domainLength[0]
    op = mg.OperatorParams(alpha=prm.alpha, beta=prm.beta, bc_lo=tuple(prm.bc_lo),
                           bc_hi=tuple(prm.bc_hi), bc_value=prm.bc_value,
                           coefficient_average_type=1, prolong_type=1)

    # ---- (f)1 + the k_binary_bh rate
    n = args.n
    dom = (0, 0, 0, n - 1, n - 1, n - 1)
    grid = mg.Grid(comm, dom, [dom], L / n)
    fa, fb, frhs, fphi = (mg.LevelData(grid) for _ in range(4))
    mg.set_binary_bh_coefs(fa, frhs, prm.bh())
    sync()
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        mg.set_binary_bh_coefs(fa, frhs, prm.bh())
    sync()
    t_bh = (time.perf_counter() - t0) / reps
    out["f2_set_a_coef_set_rhs"] = {"cells": n ** 3, "ms": round(t_bh * 1e3, 3),
                                    "Gcells_per_s": round(n ** 3 / t_bh / 1e9, 2),
                                    "bytes_per_cell": 16,
                                    "note": "FP64 bound: 6 exp + pow per cell"}
    fb.set_val(1.0)
    fac = mg.defineOperatorFactory(grid, fa, fb, op)
    amg = mg.AMRMultiGrid(fac, mg.SolverParams(max_depth=2, n_pre=prm.numMGsmooth,
                                               n_post=prm.numMGsmooth, n_bottom=prm.numMGsmooth,
                                               bottom_solver=0))
    solver = mg.BiCGStabSolver(mg.MultilevelLinearOp(amg, prm.numMGIterations),
                               tolerance=prm.tolerance, max_iterations=prm.max_iterations,
                               norm_type=0)
    fphi.set_zero()
    sync()
    t0 = time.perf_counter()
    its = solver.solve(fphi, frhs)
    sync()
    t_s = time.perf_counter() - t0
    out["f1_bicgstab_solve"] = {
        "config": f"{n}^3, 3-level MG preconditioner (numMGIterations={prm.numMGIterations}, "
                  f"nu={prm.numMGsmooth}), tolerance {prm.tolerance}",
        "iterations": its, "ms_total": round(t_s * 1e3, 2),
        "ms_per_iteration": round(t_s * 1e3 / max(its, 1), 2)}
    del solver, amg, fac, fa, fb, frhs, fphi, grid

    # ---- (f)2 NL loop
    m = args.m
    domm = (0, 0, 0, m - 1, m - 1, m - 1)
    gm = mg.Grid(comm, domm, [domm], L / m)
    sync()
    t0 = time.perf_counter()
    # a truncated loop (--nl-iters) can stop above the divergence threshold
    # (Main_PoissonSolver.cpp:221-225): record the row as such
    status = "converged"
    try:
        res = poisson_solve(gm, prm, max_depth=2, bottom_solver=0, max_NL_iterations=args.nl_iters)
        if not res.converged:
            status = "truncated"
    except NLDivergenceError as e:
        res, status = e.result, "diverged or truncated above the 1e-1 threshold"
    sync()
    t_nl = time.perf_counter() - t0
    out["f2_nl_loop"] = {"config": f"{m}^3 poisson_solve (params.txt)", "status": status,
                         "nl_iterations": len(res.dpsi_norms),
                         "linear_iterations": res.linear_iterations,
                         "dpsi_norms": res.dpsi_norms, "s_total": round(t_nl, 3),
                         "ms_per_nl_iteration": round(t_nl * 1e3 / max(1, len(res.dpsi_norms)), 1)}
    del res, gm

    # ---- (f)3 AMR V-cycle
    a = args.amr
    levels, fields = [], []
    dom, dx = (0, 0, 0, a - 1, a - 1, a - 1), L / a
    for l in range(3):
        if l == 0:
            b = dom
            g = mg.Grid(comm, dom, [b], dx)
        else:
            N = 2 ** l * a
            b = (N // 4, N // 4, N // 4, N - N // 4 - 1, N - N // 4 - 1, N - N // 4 - 1)
            if l == 2:  # a quarter-width patch in the middle of the finest domain
                b = (3 * N // 8, 3 * N // 8, 3 * N // 8, 5 * N // 8 - 1, 5 * N // 8 - 1,
                     5 * N // 8 - 1)
            g = mg.Grid(comm, dom, [b], dx, patches=True)
        fa, fb, fr, fp = (mg.LevelData(g) for _ in range(4))
        mg.set_binary_bh_coefs(fa, fr, prm.bh())
        fb.set_val(1.0)
        fp.set_zero()
        levels.append((g, fa, fb))
        fields.append((fp, fr, b))
        dom = tuple(2 * v if i < 3 else 2 * v + 1 for i, v in enumerate(dom))
        dx /= 2
    amr = mg.AMRSolver(levels, op, mg.SolverParams(max_depth=2, n_pre=prm.numMGsmooth,
                                                   n_post=prm.numMGsmooth,
                                                   n_bottom=prm.numMGsmooth, bottom_solver=0))
    phis = [f[0] for f in fields]
    rhss = [f[1] for f in fields]
    hist = [amr.init_residual(phis, rhss, 0)]
    amr.iteration(phis, rhss, -1)
    sync()
    t0 = time.perf_counter()
    for _ in range(args.amr_iters):
        amr.iteration(phis, rhss, -1)
    sync()
    t_amr = (time.perf_counter() - t0) / args.amr_iters
    hist.append(amr.init_residual(phis, rhss, 0))
    cells = [(f[2][3] - f[2][0] + 1) * (f[2][4] - f[2][1] + 1) * (f[2][5] - f[2][2] + 1)
             for f in fields]
    out["f3_amr_vcycle"] = {
        "config": f"3 AMR levels: {a}^3 base + patches of {cells[1]} and {cells[2]} cells",
        "ms_per_iteration": round(t_amr * 1e3, 3), "cells_per_level": cells,
        "residual_max_norm": {"initial": hist[0], f"after_{args.amr_iters + 1}": hist[1]}}
    del amr, phis, rhss, fields
    grids = [lv[0] for lv in levels]
    del levels
    sync()
    t0 = time.perf_counter()
    status = "converged"
    try:
        res = poisson_solve(grids, prm, max_depth=2, bottom_solver=0,
                            max_NL_iterations=args.nl_iters)
        if not res.converged:
            status = "truncated"
    except NLDivergenceError as e:
        res, status = e.result, "diverged or truncated above the 1e-1 threshold"
    sync()
    t_nl = time.perf_counter() - t0
    out["f3_amr_nl_loop"] = {
        "config": f"poisson_solve over the 3 AMR levels above (max_level = 2, params.txt)",
        "status": status, "nl_iterations": len(res.dpsi_norms),
        "linear_iterations": res.linear_iterations, "dpsi_norms": res.dpsi_norms,
        "s_total": round(t_nl, 3),
        "ms_per_nl_iteration": round(t_nl * 1e3 / max(1, len(res.dpsi_norms)), 1)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
