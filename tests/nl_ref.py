"""Oracle side of the nonlinear loop (Main_PoissonSolver.cpp:129-220) on one
box, for the NL tests: the same steps as mg_ic_code_amd/nl.py, run through
the C oracle.  Test infrastructure only."""
import numpy as np

import oracle


def oracle_poisson_solve(prm, n, max_depth, n_nl, bottom_solver=1):
    dom = (0, 0, 0, n - 1, n - 1, n - 1)
    dx = prm.domainLength[0] / n
    bh = prm.bh(constant_K=0.0)
    avg = prm.coefficient_average_type if prm.coefficient_average_type >= 0 else 0
    per = (1, 1, 1) if prm.is_periodic else (0, 0, 0)
    volume = prm.domainLength[0] * prm.domainLength[1] * prm.domainLength[2]
    o = oracle.OracleMG([dom], dom, dx, alpha=prm.alpha, beta=prm.beta, periodic=per,
                        bc_lo=prm.bc_lo,
                        bc_hi=prm.bc_hi, bc_value=prm.bc_value, nlevels=max_depth + 1,
                        avg_type=avg, prolong_type=1, bottom_solver=bottom_solver,
                        n_pre=prm.numMGsmooth, n_post=prm.numMGsmooth, n_bottom=prm.numMGsmooth)
    psi = np.ones((n + 2,) * 3)          # set_initial_conditions: psi = 1 incl. ghosts
    o.set(0, oracle.PHI, 0, np.zeros((n,) * 3))
    norms, iters, ks = [], [], []
    for _ in range(n_nl):
        if prm.is_periodic:  # integrability condition for K (Main_PoissonSolver.cpp:133-147)
            bh["constant_K"] = 0.0
            integ = oracle.nl_integrand(bh, (0, 0, 0), (n - 1,) * 3, dx, psi)
            bh["constant_K"] = -np.sqrt(abs(np.sum(integ) * dx ** 3) / volume)
            ks.append(bh["constant_K"])
        a, r = oracle.nl_coefs(bh, (0, 0, 0), (n - 1,) * 3, dx, psi)
        o.set(0, oracle.ACOEF, 0, a)
        o.set(0, oracle.BCOEF, 0, np.ones_like(a))
        o.set(0, oracle.RHS, 0, r)
        o.setup()
        it, _ = o.solve(mg_iters=prm.numMGIterations, imax=prm.max_iterations,
                        eps=prm.tolerance, norm_type=0)
        iters.append(it)
        o.exchange(0, oracle.PHI)          # set_update_psi0
        o.fill_bc(0, oracle.PHI, 0)
        psi += o.get(0, oracle.PHI, 0, full=True)
        dpsi = o.get(0, oracle.PHI, 0)
        nrm = np.sqrt(np.sum(dpsi * dpsi)) * dx ** 1.5
        norms.append(nrm)
        if nrm < prm.tolerance or nrm > 1e5:
            break
    return psi, norms, iters, ks


def oracle_poisson_solve_amr(prm, boxes, n0, max_depth, n_nl, bottom_solver=1):
    """The NL loop over a fixed AMR hierarchy (boxes[0] = the 0..n0-1 domain,
    finer boxes in their level's index space), through oracle/amr.py: per
    level coefficients, the multilevel BiCGStab, QuadCFInterp of dpsi before
    set_update_psi0, computeNorm over the hierarchy (Main_PoissonSolver.cpp:
    129-220 with max_level > 0)."""
    from oracle.amr import AMROracle
    dom0 = (0, 0, 0, n0 - 1, n0 - 1, n0 - 1)
    dx0 = prm.domainLength[0] / n0
    bh = prm.bh(constant_K=0.0)
    avg = prm.coefficient_average_type if prm.coefficient_average_type >= 0 else 0
    nlev = len(boxes)
    shape = [(b[5] - b[2] + 1, b[4] - b[1] + 1, b[3] - b[0] + 1) for b in boxes]
    psi = [np.ones(tuple(s + 2 for s in sh)) for sh in shape]
    dpsi = [np.zeros(tuple(s + 2 for s in sh)) for sh in shape]
    norms, iters = [], []
    o = None
    for _ in range(n_nl):
        levels, rhss = [], []
        for l, b in enumerate(boxes):
            a, r = oracle.nl_coefs(bh, b[:3], b[3:], dx0 / 2 ** l, psi[l])
            levels.append(dict(box=b, a=a, b=np.ones_like(a)))
            rf = np.zeros_like(psi[l])
            rf[1:-1, 1:-1, 1:-1] = r
            rhss.append(rf)
        o = AMROracle(levels, dx0, dom0, alpha=prm.alpha, beta=prm.beta, bc_lo=prm.bc_lo,
                      bc_hi=prm.bc_hi, bc_value=prm.bc_value, n_pre=prm.numMGsmooth,
                      n_post=prm.numMGsmooth,
                      base=dict(nlevels=max_depth + 1, avg_type=avg, prolong_type=1,
                                bottom_solver=bottom_solver, n_pre=prm.numMGsmooth,
                                n_post=prm.numMGsmooth, n_bottom=prm.numMGsmooth))
        it, _ = o.solve(dpsi, rhss, num_mg_iterations=prm.numMGIterations,
                        imax=prm.max_iterations, eps=prm.tolerance, norm_type=0)
        iters.append(it)
        for l in range(nlev):  # QuadCFInterp, then set_update_psi0
            if l > 0:
                cl = o.L[l - 1]
                cl.u_full = dpsi[l - 1]
                o.L[l].cf_interp(dpsi[l], cl, o.cov(l), o.L[l - 1].domain)
            o.L[l].fill_bc(dpsi[l], False)
            psi[l] += dpsi[l]
        nrm = o.norm(o.masked(dpsi), 2)
        norms.append(nrm)
        if nrm < prm.tolerance or nrm > 1e5:
            break
    return psi, norms, iters
