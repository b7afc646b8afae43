"""The nonlinear solve of Main_PoissonSolver.cpp on one AMR level, on device.

`poisson_solve` mirrors `poissonSolve` (Main_PoissonSolver.cpp:51-250) for
max_level = 0:

    psi = 1, dpsi = 0                     set_initial_conditions (SetLevelData.cpp:31-72)
    for NL_iter < max_NL_iterations:      :129-220
        aCoef, rhs from psi               set_a_coef / set_rhs (:155-161)
        bCoef = 1                         set_b_coef
        factory, MG, BiCGStab             defineOperatorFactory, mlOp, solver (:163-178)
        solver.solve(dpsi, rhs)           :184 (dpsi keeps its value between NL iterations)
        psi += dpsi                       set_update_psi0 (:188-207)
        stop if |dpsi| < tolerance or > 1e5   computeNorm (:210-217)

On a periodic domain each NL iteration first sets K from the integrability
condition: K = -sqrt(|sum(integrand) dV| / volume), with the integrand of
set_constant_K_integrand (:133-147).  Every field stays in HBM, and each step
is a libmgic kernel.  With output_dir set, the reference's HDF5 files are
written as it writes them: output_solver_data before every solve (:181) and
output_final_data after the loop (:229), through libmgic_io (output.py).
After the loop the reference stops with MayDay::Error when the final |dpsi|
is above 1e-1 (:221-225), before output_final_data: `poisson_solve` raises
NLDivergenceError at the same point, so a diverged solve writes no
checkpoint.  Not covered: AMR levels (max_level > 0).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import ctypes
import math
import os

from .core import (AMRMultiGrid, BiCGStabSolver, Grid, LevelData, MultilevelLinearOp,
                   OperatorParams, SolverParams, defineOperatorFactory, set_nl_coefs, BH_KEYS)
from ._lib import call
from .output import output_final_data, output_solver_data
from .params import PoissonParameters


# Main_PoissonSolver.cpp:221-225: "a fairly generous threshold"
NL_DIVERGENCE_THRESHOLD = 1e-1


class NLDivergenceError(RuntimeError):
    """MayDay::Error("NL iterations did not converge - may need a better initial
    guess") of Main_PoissonSolver.cpp:223-224.  Carries the loop's result."""

    def __init__(self, result: "NLResult"):
        super().__init__("NL iterations did not converge - may need a better initial guess "
                         f"(final |dpsi| = {result.dpsi_norms[-1]!r})")
        self.result = result


@dataclass
class NLResult:
    psi: LevelData
    dpsi: LevelData
    dpsi_norms: List[float] = field(default_factory=list)
    linear_iterations: List[int] = field(default_factory=list)
    converged: bool = False
    constant_K: List[float] = field(default_factory=list)


def set_nl_integrand(psi: LevelData, out: LevelData, bh: dict) -> None:
    """set_constant_K_integrand (SetLevelData.cpp:131-180) on device."""
    vals = (ctypes.c_double * 13)(*[float(bh[k]) for k in BH_KEYS])
    call("mgic_field_nl_integrand", psi.handle, out.handle, vals)


def poisson_solve(grid: Grid, prm: PoissonParameters, max_depth: int = -1,
                  prolong_type: int = 1, bottom_solver: int = 1,
                  max_NL_iterations: Optional[int] = None,
                  output_dir: Optional[str] = None) -> NLResult:
    periodic = bool(prm.is_periodic)
    if periodic != all(grid.periodic):
        raise ValueError("grid periodicity must match params is_periodic")
    psi, dpsi = LevelData(grid), LevelData(grid)
    a, b, rhs = LevelData(grid), LevelData(grid), LevelData(grid)
    psi.set_val_all(1.0)
    dpsi.set_zero()
    b.set_val(1.0)  # set_b_coef (SetLevelData.cpp:330-340)
    bh = prm.bh(constant_K=0.0)
    avg = prm.coefficient_average_type if prm.coefficient_average_type >= 0 else 0
    op_params = OperatorParams(alpha=prm.alpha, beta=prm.beta, bc_lo=tuple(prm.bc_lo),
                               bc_hi=tuple(prm.bc_hi), bc_value=prm.bc_value,
                               coefficient_average_type=avg, prolong_type=prolong_type,
                               relax_mode=1)
    depth = prm.preCondSolverDepth if prm.preCondSolverDepth >= 0 else max_depth
    res = NLResult(psi=psi, dpsi=dpsi)
    n_nl = prm.max_NL_iterations if max_NL_iterations is None else max_NL_iterations
    dx = grid.dx
    ones = integrand = None
    volume = prm.domainLength[0] * prm.domainLength[1] * prm.domainLength[2]
    for it in range(n_nl):
        if periodic:  # integrability condition for K (:133-147)
            if integrand is None:
                integrand, ones = LevelData(grid), LevelData(grid)
                ones.set_val(1.0)
            bh["constant_K"] = 0.0
            set_nl_integrand(psi, integrand, bh)
            tmp_op = defineOperatorFactory(grid, a, b, op_params).AMRnewOp()
            integral = tmp_op.dotProduct(integrand, ones) * dx ** 3  # computeSum
            bh["constant_K"] = -math.sqrt(abs(integral) / volume)
            res.constant_K.append(bh["constant_K"])
        set_nl_coefs(psi, a, rhs, bh)  # :155-161
        fac = defineOperatorFactory(grid, a, b, op_params)
        # N > 1: depths whose boxes are below 32 cells a side are gathered to
        # one box on rank 0 (the coarsest levels solved on rank 0)
        amg = AMRMultiGrid(fac, SolverParams(max_depth=depth, n_pre=prm.numMGsmooth,
                                             n_post=prm.numMGsmooth, n_bottom=prm.numMGsmooth,
                                             bottom_solver=bottom_solver,
                                             agglomerate_below=32 if grid.comm.size > 1 else 0))
        solver = BiCGStabSolver(MultilevelLinearOp(amg, prm.numMGIterations),
                                tolerance=prm.tolerance, max_iterations=prm.max_iterations,
                                norm_type=0)
        if output_dir is not None:  # :180-181
            output_solver_data([dpsi], [rhs], [psi], bh, it, [2],
                               os.path.join(output_dir, f"vcPoissonOut.3d_{it}.hdf5"))
        res.linear_iterations.append(solver.solve(dpsi, rhs))
        op0 = amg.op(0)
        op0.update_psi(psi, dpsi)
        # computeNorm (L2 over the level, dV = dx^3)
        nrm = op0.norm(dpsi, 2) * dx ** 1.5
        res.dpsi_norms.append(nrm)
        if nrm < prm.tolerance or nrm > 1e5:
            res.converged = nrm < prm.tolerance
            break
    write = None
    if output_dir is not None:  # :227-230
        def write():
            output_final_data([psi], bh, prm.max_level, [2],
                              os.path.join(output_dir, "vcPoissonFinal.3d.hdf5"))
    return finish_nl_loop(res, write)


def finish_nl_loop(res: NLResult, write_final=None) -> NLResult:
    """The end of poissonSolve (Main_PoissonSolver.cpp:218-230): raise when the
    final |dpsi| exceeds 1e-1 (MayDay::Error, :221-225) -- before anything is
    written -- else write the final data (`write_final`, :229) and return.
    The comparison is the reference's `dpsi_norm > 1e-1`, so a NaN norm passes
    it as it does there."""
    if res.dpsi_norms and res.dpsi_norms[-1] > NL_DIVERGENCE_THRESHOLD:
        raise NLDivergenceError(res)
    if write_final is not None:
        write_final()
    return res
