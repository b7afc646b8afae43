"""Worker for test_gpu_parity.py::test_two_sweep_trim_and_round_order_match_oracle:
a fresh interpreter started with MGIC_TB2_TRIM=15 (every two-sweep launch
kind skips the ghost lines of domain faces, at every box size) and
MGIC_TB2_KC=8 or 5 (short z chunks, so a 192 x 132 x 128 box has more than
one dispatch round and takes the round-major tile order with a tail).  Checks
relax() and V-cycle iterations against the oracle bit for bit on ragged
shapes, odd global offsets and every one-rule BC; prints "trim worker OK".
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import mg_ic_code_amd as mg  # noqa: E402
import oracle  # noqa: E402


def relax_case(comm, rng, shape, lo, mode, bcv, nsweeps):
    nx, ny, nz = shape
    dom = (lo[0], lo[1], lo[2], lo[0] + nx - 1, lo[1] + ny - 1, lo[2] + nz - 1)
    dx = 0.7
    a = rng.uniform(-2.0, -0.5, (nz, ny, nx))
    rhs = rng.uniform(-1, 1, (nz, ny, nx))
    u0 = rng.uniform(-1, 1, (nz, ny, nx))
    bc = (mode,) * 3
    grid = mg.Grid(comm, dom, [dom], dx)
    fa, fb, fr, fu = (mg.LevelData(grid) for _ in range(4))
    fa.upload(0, a)
    fb.set_val(1.0)
    fr.upload(0, rhs)
    fu.upload(0, u0)
    prm = mg.OperatorParams(alpha=1.0, beta=-1.0, bc_lo=bc, bc_hi=bc, bc_value=bcv,
                            fused_smoother=2)
    op = mg.defineOperatorFactory(grid, fa, fb, prm).AMRnewOp()
    op.relax(fu, fr, nsweeps)
    got = fu.download(0)
    o = oracle.OracleMG([dom], dom, dx, alpha=1.0, beta=-1.0, bc_lo=bc, bc_hi=bc, bc_value=bcv,
                        nlevels=1)
    o.set(0, oracle.ACOEF, 0, a)
    o.set(0, oracle.BCOEF, 0, np.ones_like(a))
    o.set(0, oracle.RHS, 0, rhs)
    o.set(0, oracle.PHI, 0, u0)
    o.setup()
    o.relax(0, oracle.PHI, oracle.RHS, nsweeps)
    want = o.get(0, oracle.PHI, 0)
    assert np.array_equal(got, want), (shape, lo, mode, bcv, nsweeps)


def vcycle_case(comm, rng, n):
    # ZIN, plain and ACC launches (the V-cycle's pairs) on a 3-level hierarchy
    dom = (0, 0, 0, n - 1, n - 1, n - 1)
    dx = 100.0 / n
    a = rng.uniform(-2.0, -0.5, (n, n, n))
    rhs = rng.uniform(-1, 1, (n, n, n))
    grid = mg.Grid(comm, dom, [dom], dx)
    fa, fb, frhs, fphi, fres = (mg.LevelData(grid) for _ in range(5))
    fa.upload(0, a)
    fb.set_val(1.0)
    frhs.upload(0, rhs)
    fphi.set_zero()
    prm = mg.OperatorParams(alpha=1.0, beta=-1.0, fused_smoother=2)
    fac = mg.defineOperatorFactory(grid, fa, fb, prm)
    amg = mg.AMRMultiGrid(fac, mg.SolverParams(max_depth=2, bottom_solver=0))
    o = oracle.OracleMG([dom], dom, dx, alpha=1.0, beta=-1.0, nlevels=3, bottom_solver=0)
    o.set(0, oracle.ACOEF, 0, a)
    o.set(0, oracle.BCOEF, 0, np.ones_like(a))
    o.set(0, oracle.RHS, 0, rhs)
    o.setup()
    amg.init_residual(fphi, frhs, fres)
    o.init_residual(0)
    got = [amg.iteration(fphi, frhs, fres, 0) for _ in range(2)]
    want = [o.iteration(0) for _ in range(2)]
    assert got == want, (got, want)
    g, w = fphi.download(0), o.get(0, oracle.PHI, 0)
    if not np.array_equal(g, w):
        bad = np.argwhere(g != w)
        print("phi differs at", len(bad), "cells, e.g. (k, j, i)", bad[:8].tolist(),
              "max |diff|", float(np.abs(g - w).max()), flush=True)
    assert np.array_equal(g, w)


def main():
    comm = mg.Comm()
    rng = np.random.default_rng(20261018)
    if os.environ.get("TRIM_WORKER_VCYCLE_ONLY"):
        vcycle_case(comm, rng, int(os.environ["TRIM_WORKER_VCYCLE_ONLY"]))
        print("trim worker OK", flush=True)
        return
    assert os.environ.get("MGIC_TB2_TRIM") == "15" and os.environ.get("MGIC_TB2_KC") in ("8", "5")

    for shape, lo in (((37, 9, 40), (3, -5, 7)), ((130, 47, 45), (-64, 1, 1)),
                      ((65, 23, 17), (1, 0, 2))):
        for mode, bcv in ((0, 0.5), (1, 0.0), (0, 0.0)):
            for nsweeps in (2, 4):
                relax_case(comm, rng, shape, lo, mode, bcv, nsweeps)
    relax_case(comm, rng, (192, 132, 128), (0, 0, 0), 0, 0.0, 2)  # > one dispatch round
    vcycle_case(comm, rng, 48)
    comm.synchronize()
    print("trim worker OK", flush=True)


if __name__ == "__main__":
    main()
