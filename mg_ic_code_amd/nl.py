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
checkpoint.

max_level > 0 (`grid` a list of Grids, coarsest first, finer ones
Grid(patches=True) properly nested; set_grids' tagging/regridding is out of
scope, so the hierarchy is given): every step runs per level as the
reference's loops over ilev do -- coefficients on every level (:154-160),
the outer BiCGStab over MultilevelLinearOp with AMR V-cycles as its
preconditioner (:169-184; AMRSolver), then per level QuadCFInterp of dpsi
from the coarser level before set_update_psi0 (:189-205), and computeNorm /
computeSum over the hierarchy with covered cells masked (:144-145, :208).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import ctypes
import math
import os

from .core import (AMRMultiGrid, AMRSolver, BiCGStabSolver, Grid, LevelData, MultilevelLinearOp,
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
    psi: object   # LevelData, or one per AMR level (max_level > 0)
    dpsi: object
    dpsi_norms: List[float] = field(default_factory=list)
    linear_iterations: List[int] = field(default_factory=list)
    converged: bool = False
    constant_K: List[float] = field(default_factory=list)


def set_nl_integrand(psi: LevelData, out: LevelData, bh: dict) -> None:
    """set_constant_K_integrand (SetLevelData.cpp:131-180) on device."""
    vals = (ctypes.c_double * 13)(*[float(bh[k]) for k in BH_KEYS])
    call("mgic_field_nl_integrand", psi.handle, out.handle, vals)


def poisson_solve(grid, prm: PoissonParameters, max_depth: int = -1,
                  prolong_type: int = 1, bottom_solver: int = 1,
                  max_NL_iterations: Optional[int] = None,
                  output_dir: Optional[str] = None) -> NLResult:
    if isinstance(grid, (list, tuple)):
        if len(grid) > 1:
            return _poisson_solve_amr(list(grid), prm, max_depth, prolong_type, bottom_solver,
                                      max_NL_iterations, output_dir)
        grid = grid[0]
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


def _op_params(prm: PoissonParameters, prolong_type: int) -> OperatorParams:
    avg = prm.coefficient_average_type if prm.coefficient_average_type >= 0 else 0
    return OperatorParams(alpha=prm.alpha, beta=prm.beta, bc_lo=tuple(prm.bc_lo),
                          bc_hi=tuple(prm.bc_hi), bc_value=prm.bc_value,
                          coefficient_average_type=avg, prolong_type=prolong_type, relax_mode=1)


def _poisson_solve_amr(grids: List[Grid], prm: PoissonParameters, max_depth: int,
                       prolong_type: int, bottom_solver: int, max_NL_iterations: Optional[int],
                       output_dir: Optional[str]) -> NLResult:
    """poissonSolve over nlevels = len(grids) AMR levels (Main_PoissonSolver.cpp:51-250)."""
    periodic = bool(prm.is_periodic)
    if periodic != all(grids[0].periodic):
        raise ValueError("grid periodicity must match params is_periodic")
    nlev = len(grids)
    psi = [LevelData(g) for g in grids]
    dpsi = [LevelData(g) for g in grids]
    a = [LevelData(g) for g in grids]
    b = [LevelData(g) for g in grids]
    rhs = [LevelData(g) for g in grids]
    for l in range(nlev):  # set_initial_conditions / set_b_coef per level (:79-99, :157)
        psi[l].set_val_all(1.0)
        dpsi[l].set_zero()
        b[l].set_val(1.0)
    bh = prm.bh(constant_K=0.0)
    op_params = _op_params(prm, prolong_type)
    depth = prm.preCondSolverDepth if prm.preCondSolverDepth >= 0 else max_depth
    sp = SolverParams(max_depth=depth, n_pre=prm.numMGsmooth, n_post=prm.numMGsmooth,
                      n_bottom=prm.numMGsmooth, bottom_solver=bottom_solver,
                      agglomerate_below=32 if grids[0].comm.size > 1 else 0)
    res = NLResult(psi=psi, dpsi=dpsi)
    n_nl = prm.max_NL_iterations if max_NL_iterations is None else max_NL_iterations
    volume = prm.domainLength[0] * prm.domainLength[1] * prm.domainLength[2]
    integrand = geom = None
    refs = [2] * nlev
    for it in range(n_nl):
        if periodic:  # integrability condition for K over the hierarchy (:137-150)
            if integrand is None:
                integrand = [LevelData(g) for g in grids]
                # computeSum only needs the hierarchy's geometry
                geom = AMRSolver(list(zip(grids, a, b)), op_params, sp)
            bh["constant_K"] = 0.0
            for l in range(nlev):
                set_nl_integrand(psi[l], integrand[l], bh)
            integral = geom.computeSum(integrand)
            bh["constant_K"] = -math.sqrt(abs(integral) / volume)
            res.constant_K.append(bh["constant_K"])
        for l in range(nlev):  # :154-160
            set_nl_coefs(psi[l], a[l], rhs[l], bh)
        amr = AMRSolver(list(zip(grids, a, b)), op_params, sp)  # :163-170
        solver = BiCGStabSolver(MultilevelLinearOp(amr, prm.numMGIterations),
                                tolerance=prm.tolerance, max_iterations=prm.max_iterations,
                                norm_type=0)
        if output_dir is not None:  # :180-181
            output_solver_data(dpsi, rhs, psi, bh, it, refs,
                               os.path.join(output_dir, f"vcPoissonOut.3d_{it}.hdf5"))
        res.linear_iterations.append(solver.solve(dpsi, rhs))  # :184
        for l in range(nlev):  # :189-205
            if l > 0:
                amr.cf_interp(l, dpsi[l], dpsi[l - 1])  # QuadCFInterp::coarseFineInterp
            amr.level_op(l).update_psi(psi[l], dpsi[l])
        nrm = amr.computeNorm(dpsi, 2)  # :208-209
        res.dpsi_norms.append(nrm)
        if nrm < prm.tolerance or nrm > 1e5:
            res.converged = nrm < prm.tolerance
            break
    write = None
    if output_dir is not None:  # :227-230
        def write():
            output_final_data(psi, bh, nlev - 1, refs,
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
