"""AMR levels > 0: coarse-fine interpolation, the
AMRLevelOp multi-level operators and the multi-level AMR V-cycle, GPU against
the numpy restatement oracle/amr.py bit for bit, and multi-box fine levels
against single-box ones.  The CPU test checks the restatement converges.
"""
import numpy as np
import pytest

from oracle.amr import AMROracle

# level 0: 32^3 (one box); level 1: a patch of the 64^3 domain; level 2: a
# patch of the 128^3 domain (even lo, odd hi, properly nested)
DOM0 = (0, 0, 0, 31, 31, 31)
BOXES = [DOM0, (8, 16, 12, 47, 41, 45), (30, 40, 36, 73, 71, 77)]
DX0 = 100.0 / 32
BC = dict(bc_lo=(0, 1, 0), bc_hi=(1, 0, 0), bc_value=0.125)


def _shape(b):
    return (b[5] - b[2] + 1, b[4] - b[1] + 1, b[3] - b[0] + 1)


# patches touching domain faces (level 1: x lo, y hi; level 2: x lo, y hi):
# their boxes mix domain-BC and coarse-fine faces
BOXES_EDGE = [DOM0, (0, 16, 12, 47, 63, 45), (0, 40, 36, 73, 127, 77)]


def _data(rng, nlev, bvar=True, boxes=BOXES):
    out = []
    for l in range(nlev):
        s = _shape(boxes[l])
        out.append(dict(box=boxes[l], a=rng.uniform(-2.0, -0.5, s),
                        b=rng.uniform(0.5, 2.0, s) if bvar else np.ones(s),
                        rhs=rng.uniform(-1, 1, s)))
    return out


def _oracle(levels):
    return AMROracle(levels, DX0, DOM0, alpha=1.0, beta=-1.0, **BC,
                     base=dict(nlevels=3, avg_type=1, prolong_type=1, bottom_solver=0))


def test_amr_oracle_vcycle_converges():
    rng = np.random.default_rng(2)
    lv = _data(rng, 3)
    o = _oracle(lv)
    phis = [o.L[l].full() for l in range(3)]
    res = o.init_residual(phis, [x["rhs"] for x in lv])
    hist = [max(np.abs(r).max() for r in res)]
    for _ in range(4):
        res = o.iteration()
        hist.append(max(np.abs(r).max() for r in res))
    assert hist[-1] < 1e-3 * hist[0]
    assert all(b < a for a, b in zip(hist, hist[1:]))


# ------------------------------------------------------------------ GPU
@pytest.fixture(scope="module")
def comm():
    import mg_ic_code_amd as mg
    return mg.Comm()


def _gpu(comm, lv, split=False):
    import mg_ic_code_amd as mg
    levels, fields = [], []
    dom, dx = DOM0, DX0
    for l, x in enumerate(lv):
        b = x["box"]
        if l == 0:
            grid = mg.Grid(comm, dom, [b], dx)
        else:
            boxes = [b]
            if split:  # two boxes sharing an x face: the exchange replaces their CF ghosts
                m = b[0] + ((b[3] - b[0] + 1) // 4) * 2
                boxes = [(b[0], b[1], b[2], m - 1, b[4], b[5]), (m, b[1], b[2], b[3], b[4], b[5])]
            grid = mg.Grid(comm, dom, boxes, dx, patches=True)
        fa, fb, fr, fphi = (mg.LevelData(grid) for _ in range(4))
        for f, arr in ((fa, x["a"]), (fb, x["b"]), (fr, x["rhs"])):
            for k in range(grid.num_local):
                bx = grid.local_box(k)
                f.upload(k, arr[bx[2] - b[2]:bx[5] - b[2] + 1, bx[1] - b[1]:bx[4] - b[1] + 1,
                                bx[0] - b[0]:bx[3] - b[0] + 1])
        fphi.set_zero()
        levels.append((grid, fa, fb))
        fields.append(dict(grid=grid, rhs=fr, phi=fphi, box=b))
        dom = tuple(2 * v if i < 3 else 2 * v + 1 for i, v in enumerate(dom))
        dx /= 2
    op = mg.OperatorParams(alpha=1.0, beta=-1.0, coefficient_average_type=1, prolong_type=1,
                           **BC)
    amr = mg.AMRSolver(levels, op, mg.SolverParams(max_depth=2, bottom_solver=0))
    return amr, fields


def _get(f, key="phi"):
    g, b = f["grid"], f["box"]
    out = np.zeros(_shape(b))
    for k in range(g.num_local):
        bx = g.local_box(k)
        out[bx[2] - b[2]:bx[5] - b[2] + 1, bx[1] - b[1]:bx[4] - b[1] + 1,
            bx[0] - b[0]:bx[3] - b[0] + 1] = f[key].download(k)
    return out


@pytest.mark.gpu
def test_amr_cf_interp_matches_oracle(comm):
    rng = np.random.default_rng(3)
    lv = _data(rng, 3)
    amr, F = _gpu(comm, lv)
    o = _oracle(lv)
    # random phi on every level; CF ghosts of levels 1, 2 from the coarser level
    us = [rng.uniform(-1, 1, _shape(BOXES[l])) for l in range(3)]
    for l in range(3):
        F[l]["phi"].upload(0, us[l])
    for l in (1, 2):
        for coarse in (True, False):
            F[l]["phi"].upload(0, us[l])
            amr.cf_interp(l, F[l]["phi"], F[l - 1]["phi"] if coarse else None)
            g = F[l]["phi"].download(0, with_ghosts=True)
            u = o.L[l].full(us[l])
            cl = None
            if coarse:
                cl = o.L[l - 1]
                cl.u_full = o.L[l - 1].full(us[l - 1])
            o.L[l].cf_interp(u, cl, o.cov(l), o.L[l - 1].domain)
            for ax in range(3):  # the six ghost faces (edges and corners are not CF cells)
                for side in (0, -1):
                    sl = [slice(1, -1)] * 3
                    sl[ax] = side
                    dom_face = o.L[l].domain_face(2 - ax, 1 if side else 0)
                    if not dom_face:
                        assert np.array_equal(g[tuple(sl)], u[tuple(sl)]), (l, coarse, ax, side)


@pytest.mark.gpu
@pytest.mark.parametrize("bvar", [False, True])
def test_amr_vcycle_matches_oracle_bitwise(comm, bvar):
    rng = np.random.default_rng(4)
    lv = _data(rng, 3, bvar)
    amr, F = _gpu(comm, lv)
    o = _oracle(lv)
    phis = [o.L[l].full() for l in range(3)]
    res = o.init_residual(phis, [x["rhs"] for x in lv])
    g0 = amr.init_residual([f["phi"] for f in F], [f["rhs"] for f in F], 0)
    assert g0 == max(np.abs(r).max() for r in res)
    for _ in range(3):
        g = amr.iteration([f["phi"] for f in F], [f["rhs"] for f in F], 0)
        res = o.iteration()
        assert g == max(np.abs(r).max() for r in res)
    for l in range(3):
        assert np.array_equal(_get(F[l]), o.phis[l][1:-1, 1:-1, 1:-1]), l
    assert g < 5e-2 * g0  # (random bCoef: about 0.34 per iteration for this seed)


@pytest.mark.gpu
def test_amr_vcycle_boundary_patches_bitwise(comm):
    # patches on the domain boundary: the fused sweeps on those levels fold the
    # domain BC and the coarse-fine ghost rule in the same tiles
    rng = np.random.default_rng(6)
    lv = _data(rng, 3, True, BOXES_EDGE)
    amr, F = _gpu(comm, lv)
    o = _oracle(lv)
    phis = [o.L[l].full() for l in range(3)]
    res = o.init_residual(phis, [x["rhs"] for x in lv])
    assert amr.init_residual([f["phi"] for f in F], [f["rhs"] for f in F], 0) == \
        max(np.abs(r).max() for r in res)
    for _ in range(3):
        g = amr.iteration([f["phi"] for f in F], [f["rhs"] for f in F], 0)
        res = o.iteration()
        assert g == max(np.abs(r).max() for r in res)
    for l in range(3):
        assert np.array_equal(_get(F[l]), o.phis[l][1:-1, 1:-1, 1:-1]), l


@pytest.mark.gpu
def test_amr_multibox_fine_level_matches_single_box(comm):
    rng = np.random.default_rng(5)
    lv = _data(rng, 3)
    out = []
    for split in (False, True):
        amr, F = _gpu(comm, lv, split=split)
        h = [amr.init_residual([f["phi"] for f in F], [f["rhs"] for f in F], 0)]
        h += [amr.iteration([f["phi"] for f in F], [f["rhs"] for f in F], 0) for _ in range(2)]
        out.append((h, [_get(f) for f in F]))
    assert out[0][0] == out[1][0]
    for a, b in zip(out[0][1], out[1][1]):
        assert np.array_equal(a, b)


@pytest.mark.gpu
def test_amr_level_operators_match_oracle(comm):
    rng = np.random.default_rng(6)
    lv = _data(rng, 2)
    amr, F = _gpu(comm, lv)
    o = _oracle(lv)
    import mg_ic_code_amd as mg
    g1, g0 = F[1]["grid"], F[0]["grid"]
    u1 = rng.uniform(-1, 1, _shape(BOXES[1]))
    u0 = rng.uniform(-1, 1, _shape(BOXES[0]))
    r1 = rng.uniform(-1, 1, _shape(BOXES[1]))
    fu1, fu0, fr1, fout, frc = (mg.LevelData(g) for g in (g1, g0, g1, g1, g0))
    fu1.upload(0, u1)
    fu0.upload(0, u0)
    fr1.upload(0, r1)
    # AMROperator on level 1 with CF ghosts from level 0 (inhomogeneous phys BC)
    amr.AMROperator(1, fout, fu1, fu0, False)
    U1, U0 = o.L[1].full(u1), o.L[0].full(u0)
    o.fill(1, U1, U0, False)
    lap_o = -o.L[1].residual(U1, np.zeros(_shape(BOXES[1])))  # L(u) = 0 - residual(u, 0)
    assert np.allclose(fout.download(0), lap_o, rtol=1e-13, atol=1e-12)
    # AMRRestrict: covered coarse cells = average(r1 - L(u1)) with homogeneous CF
    fu1.upload(0, u1)
    frc.upload(0, u0)
    amr.AMRRestrict(1, frc, fr1, fu1, None)
    U1 = o.L[1].full(u1)
    rr = o.amr_residual(1, U1, None, r1, True)
    want = u0.copy()
    from oracle.amr import average_down
    o.put_covered(1, want, average_down(rr))
    assert np.array_equal(frc.download(0), want)
    # AMRProlong: piecewise constant
    fu1.upload(0, u1)
    amr.AMRProlong(1, fu1, fu0)
    U1 = o.L[1].full(u1)
    o.prolong_const(1, U1, o.L[0].full(u0))
    assert np.array_equal(fu1.download(0), U1[1:-1, 1:-1, 1:-1])
    # AMRUpdateResidual: r1 - L(u1) with the CF ghosts of u1 from u0
    fu1.upload(0, u1)
    amr.AMRUpdateResidual(1, fr1, fu1, fu0)
    U1 = o.L[1].full(u1)
    assert np.array_equal(fr1.download(0), o.amr_residual(1, U1, o.L[0].full(u0), r1, True))


# ------------------------------------------- MultilevelLinearOp + BiCGStab
def _full_ml(o, arrs):
    return [o.L[l].full(a) for l, a in enumerate(arrs)]


def test_amr_oracle_multilevel_bicgstab_converges():
    # the outer solve over the hierarchy (Main_PoissonSolver.cpp:169-184 with
    # max_level > 0): BiCGStab with AMR V-cycles as the preconditioner
    rng = np.random.default_rng(21)
    lv = _data(rng, 3, bvar=False)
    o = _oracle(lv)
    phis = o.zeros_ml()
    rhss = _full_ml(o, [x["rhs"] for x in lv])
    r0 = o.norm(o.residual_ml([p.copy() for p in phis], rhss), 0)
    it, nrm = o.solve(phis, rhss, num_mg_iterations=2, imax=20, eps=1e-10)
    assert nrm <= 1e-10 * r0 * 10 and it <= 12, (it, nrm, r0)
    # the preconditioner alone reduces the composite residual
    r = o.residual_ml(o.zeros_ml(), rhss)
    e = o.precondition(r, 2)
    r1 = o.residual_ml(e, rhss)
    assert o.norm(r1, 0) < 0.2 * o.norm(r, 0)


def _ml_setup(comm, rng, nlev=3, boxes=BOXES):
    lv = _data(rng, nlev, bvar=False, boxes=boxes)
    amr, F = _gpu(comm, lv)
    o = _oracle(lv)
    return lv, amr, F, o


def _new_fields(F):
    import mg_ic_code_amd as mg
    return [mg.LevelData(f["grid"]) for f in F]


def _up(F, fields, arrs):
    for f, d, a in zip(F, fields, arrs):
        d.upload(0, a[1:-1, 1:-1, 1:-1])


@pytest.mark.gpu
def test_amr_multilevel_apply_op_and_precondition_bitwise(comm):
    rng = np.random.default_rng(22)
    lv, amr, F, o = _ml_setup(comm, rng)
    xs = [o.L[l].full(rng.uniform(-1, 1, _shape(BOXES[l]))) for l in range(3)]
    fx, fl = _new_fields(F), _new_fields(F)
    _up(F, fx, xs)
    amr.applyOp(fl, fx, True)
    want = o.apply_op([x.copy() for x in xs], True)
    for l in range(3):
        assert np.array_equal(fl[l].download(0), want[l][1:-1, 1:-1, 1:-1]), l
    # dot / norms: reductions in another order
    assert amr.dotProduct(fl, fx) == pytest.approx(o.dot(want, xs), rel=1e-12)
    for ord_ in (0, 1, 2):
        assert amr.norm(fl, ord_) == pytest.approx(o.norm(want, ord_), rel=1e-12)
        assert amr.computeNorm(fx, ord_) == pytest.approx(o.norm(o.masked(xs), ord_), rel=1e-12)
    assert amr.computeSum(fx) == pytest.approx(
        sum(o.weight(l) * float(m[1:-1, 1:-1, 1:-1].sum()) for l, m in enumerate(o.masked(xs))),
        rel=1e-11)
    # the preconditioner on a composite residual (covered cells zero)
    r = o.residual_ml(o.zeros_ml(), _full_ml(o, [x["rhs"] for x in lv]))
    fr, fe = _new_fields(F), _new_fields(F)
    _up(F, fr, r)
    amr.precondition(fe, fr, 2)
    e = o.precondition(r, 2)
    for l in range(3):
        assert np.array_equal(fe[l].download(0), e[l][1:-1, 1:-1, 1:-1]), l


@pytest.mark.gpu
@pytest.mark.parametrize("boxes", [BOXES, BOXES_EDGE], ids=["interior", "edge"])
def test_amr_multilevel_bicgstab_solve_matches_oracle(comm, boxes):
    import mg_ic_code_amd as mg
    rng = np.random.default_rng(23)
    lv, amr, F, o = _ml_setup(comm, rng, boxes=boxes)
    solver = mg.BiCGStabSolver(mg.MultilevelLinearOp(amr, 2), tolerance=1e-10,
                               max_iterations=20, norm_type=0)
    it = solver.solve([f["phi"] for f in F], [f["rhs"] for f in F])
    phis = o.zeros_ml()
    it_o, nrm_o = o.solve(phis, _full_ml(o, [x["rhs"] for x in lv]), num_mg_iterations=2,
                          imax=20, eps=1e-10)
    assert it == it_o
    assert solver.final_norm == pytest.approx(nrm_o, rel=1e-6, abs=1e-14)
    for l in range(3):
        got, want = _get(F[l]), phis[l][1:-1, 1:-1, 1:-1]
        assert np.linalg.norm(got - want) <= 1e-10 * np.linalg.norm(want), l


# ------------------------------------------- the NL loop over AMR levels
# params.txt on a 32^3 base with two refined patches around the punctures
NL_BOXES = [(0, 0, 0, 31, 31, 31), (16, 16, 16, 47, 47, 47), (48, 48, 48, 79, 79, 79)]


def test_amr_oracle_nl_loop_converges():
    import os
    from mg_ic_code_amd.params import read_params_file
    from tests.nl_ref import oracle_poisson_solve_amr
    prm = read_params_file(os.path.join(os.path.dirname(__file__), "golden", "params.txt"))
    psi, norms, iters = oracle_poisson_solve_amr(prm, NL_BOXES, 32, max_depth=3, n_nl=4)
    assert norms[-1] < 1e-3 * norms[0], norms
    assert all(b < a for a, b in zip(norms, norms[1:])), norms


@pytest.mark.gpu
def test_amr_nl_loop_matches_oracle(comm):
    # Main_PoissonSolver.cpp:129-220 with max_level = 2 on a fixed hierarchy:
    # per-level coefficients, multilevel BiCGStab, QuadCFInterp of dpsi,
    # set_update_psi0, computeNorm -- GPU against the numpy/C oracle loop
    import os
    import mg_ic_code_amd as mg
    from mg_ic_code_amd.nl import poisson_solve
    from mg_ic_code_amd.params import read_params_file
    from tests.nl_ref import oracle_poisson_solve_amr
    prm = read_params_file(os.path.join(os.path.dirname(__file__), "golden", "params.txt"))
    dx = prm.domainLength[0] / 32
    grids, dom = [], NL_BOXES[0]
    for l, b in enumerate(NL_BOXES):
        grids.append(mg.Grid(comm, dom, [b], dx, patches=l > 0))
        dom = tuple(2 * v if i < 3 else 2 * v + 1 for i, v in enumerate(dom))
        dx /= 2
    res = poisson_solve(grids, prm, max_depth=3, max_NL_iterations=3)
    psi_o, norms_o, iters_o = oracle_poisson_solve_amr(prm, NL_BOXES, 32, max_depth=3, n_nl=3)
    assert res.linear_iterations[:2] == iters_o[:2]
    np.testing.assert_allclose(res.dpsi_norms[:2], norms_o[:2], rtol=1e-6)
    for l in range(3):
        g = res.psi[l].download(0)
        c = psi_o[l][1:-1, 1:-1, 1:-1]
        assert np.linalg.norm(g - c) <= 1e-10 * np.linalg.norm(c), l
