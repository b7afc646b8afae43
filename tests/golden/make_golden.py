#!/usr/bin/env python3
"""Regenerate the committed fixtures in tests/golden/ from the CPU oracle.

The reference has no tests or vectors and cannot be built here (DESIGN.md
§4), so these fixtures are REGRESSION vectors of the oracle restatement
(SURVEY.md §8(c) "fixtures to commit"), not pins against the reference:

  kernels12.npz   12^3 box (+1 ghost), seed 20261015: inputs u, rhs, a, b;
                  outputs of GSRB pass 0, then pass 1 (one sweep), OP, RES,
                  RESTRICT (6^3), lambda, arithmetic / harmonic averages
                  (ratio 2).  alpha = 1, beta = -1, dx = 100/64 (params.txt).
  vcycle16.npz    16^3, 3 levels, Dirichlet-0, harmonic averaging, linear
                  prolongation, 4 GSRB sweeps at the bottom: inputs a, rhs
                  (b = 1, phi = 0, dx = 1/16 so the Laplacian dominates)
                  and the max-norm residual after init_residual and after
                  each of 4 AMRMultiGrid iterations, plus the final phi.
  binary_bh64.json  params.txt's 64^3 SetBinaryBH aCoef / rhs at 64 sampled
                  cells (float.hex), psi = 1.

usage: python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from oracle import Fab  # noqa: E402

SEED = 20261015
DX = 100.0 / 64
ALPHA, BETA = 1.0, -1.0


def kernels12():
    rng = np.random.default_rng(SEED)
    n = 12
    shp = (n + 2,) * 3
    u = rng.uniform(-1, 1, shp)
    rhs = rng.uniform(-1, 1, shp)
    a = rng.uniform(-2.0, -0.5, shp)
    b = rng.uniform(0.5, 2.0, shp)
    g = (-1, -1, -1)
    lo, hi = (0, 0, 0), (n - 1,) * 3
    lam = np.zeros(shp)
    oracle.lam(Fab(lam, g), Fab(a, g), lo, hi, ALPHA, BETA, DX)
    out = dict(u=u, rhs=rhs, a=a, b=b, lam=lam)
    s = u.copy()
    oracle.gsrb(Fab(s, g), Fab(rhs, g), lo, hi, DX, ALPHA, Fab(a, g), BETA, Fab(b, g), Fab(lam, g), 0)
    out["gsrb_pass0"] = s.copy()
    oracle.gsrb(Fab(s, g), Fab(rhs, g), lo, hi, DX, ALPHA, Fab(a, g), BETA, Fab(b, g), Fab(lam, g), 1)
    out["gsrb_sweep"] = s.copy()
    op = np.zeros(shp)
    oracle.apply_op(Fab(op, g), Fab(u, g), ALPHA, Fab(a, g), BETA, Fab(b, g), lo, hi, DX)
    out["op"] = op
    res = np.zeros(shp)
    oracle.residual(Fab(res, g), Fab(u, g), Fab(rhs, g), ALPHA, Fab(a, g), BETA, Fab(b, g), lo, hi, DX)
    out["res"] = res
    m = n // 2
    rc = np.zeros((m, m, m))
    oracle.restrict_residual(Fab(rc, lo), Fab(u, g), Fab(rhs, g), ALPHA, Fab(a, g), BETA, Fab(b, g),
                             lo, hi, DX)
    out["restrict"] = rc
    inner = np.ascontiguousarray(b[1:-1, 1:-1, 1:-1])
    for name, harm in (("avg_arith", 0), ("avg_harm", 1)):
        c = np.zeros((m, m, m))
        oracle.average(Fab(c, lo), Fab(inner, lo), lo, (m - 1,) * 3, 2, harm)
        out[name] = c
    np.savez(os.path.join(HERE, "kernels12.npz"), **out)


def vcycle16():
    rng = np.random.default_rng(SEED + 1)
    n = 16
    dom = (0, 0, 0, n - 1, n - 1, n - 1)
    a = rng.uniform(-2.0, -0.5, (n, n, n))
    rhs = rng.uniform(-1, 1, (n, n, n))
    o = oracle.OracleMG([dom], dom, 1.0 / n, alpha=ALPHA, beta=BETA, nlevels=3, avg_type=1,
                        prolong_type=1, bottom_solver=0, n_pre=4, n_post=4, n_bottom=4)
    o.set(0, oracle.ACOEF, 0, a)
    o.set(0, oracle.BCOEF, 0, np.ones_like(a))
    o.set(0, oracle.RHS, 0, rhs)
    o.setup()
    hist = [o.init_residual(0)]
    for _ in range(4):
        hist.append(o.iteration(0))
    np.savez(os.path.join(HERE, "vcycle16.npz"), a=a, rhs=rhs, residual_max_norm=np.array(hist),
             phi=o.get(0, oracle.PHI, 0))


def binary_bh64():
    from mg_ic_code_amd.params import read_params_file
    p = read_params_file(os.path.join(HERE, "params.txt"))
    n = p.N[0]
    a, r = oracle.binary_bh(p.bh(), (0, 0, 0), (n - 1,) * 3, p.coarsestDx)
    rng = np.random.default_rng(SEED + 2)
    cells = [tuple(int(v) for v in rng.integers(0, n, 3)) for _ in range(60)]
    cells += [(0, 0, 0), (n - 1, n - 1, n - 1), (n // 2, n // 2, n // 2), (38, 32, 32)]
    data = {"n": n, "dx": p.coarsestDx, "cells_ijk": cells,
            "aCoef": [float(a[k, j, i]).hex() for i, j, k in cells],
            "rhs": [float(r[k, j, i]).hex() for i, j, k in cells]}
    with open(os.path.join(HERE, "binary_bh64.json"), "w") as f:
        json.dump(data, f, indent=0)


if __name__ == "__main__":
    kernels12()
    vcycle16()
    binary_bh64()
    print("fixtures written to", HERE)
