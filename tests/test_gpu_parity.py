"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Integer/byte work would be bit-exact; here every kernel is a fixed
sequence of IEEE fp64 operations compiled with -ffp-contract=off, so the
bar is BIT-EXACT equality with the oracle for the stencils, transfer
operators, coefficient averaging, lambda, BC folding and whole V-cycles
with a relaxation bottom.  Only the Krylov bottom solver (parallel dot
products) is compared with a tolerance: rel-L2 <= 1e-10 (BASELINE.json).
"""
import ctypes
import os

import numpy as np
import pytest

import oracle
from oracle import Fab

pytestmark = pytest.mark.gpu

mg = pytest.importorskip("mg_ic_code_amd")
from mg_ic_code_amd.decomposition import split_domain  # noqa: E402


def dbl(p):
    return p.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def ints(*v):
    return [ctypes.byref(ctypes.c_int(int(x))) for x in v]


def fab_args(arr, lo, ncomp=1):
    nz, ny, nx = arr.shape[-3:]
    hi = (lo[0] + nx - 1, lo[1] + ny - 1, lo[2] + nz - 1)
    return [dbl(arr)] + ints(*lo) + ints(*hi) + ints(ncomp)


@pytest.fixture(scope="module")
def comm():
    return mg.Comm()


def remote_comm(kind, arena_mb=32):
    """A one-rank communicator whose same-rank copies travel the remote path:
    "rccl" -- RCCL self send/recv; "ipc" -- the peer-mapped transport's put /
    get kernels and device flags (csrc/transport.hip) on its own arena."""
    if kind == "rccl":
        c = mg.Comm(0, 1, unique_id=mg.Comm.unique_id(), force_rccl=True)
        assert c.uses_rccl
    else:
        c = mg.Comm(transport="ipc", arena_bytes=arena_mb << 20)
        assert c.transport == "ipc"
    c.set_self_messages(True)
    return c


def make_fields(comm, boxes, dom, dx, periodic=(0, 0, 0), owners=None):
    grid = mg.Grid(comm, dom, boxes, dx, periodic=periodic, owners=owners)
    return grid


def upload_global(field, grid, boxes, arr):
    for n in range(grid.num_local):
        b = grid.local_box(n)
        field.upload(n, arr[b[2]:b[5] + 1, b[1]:b[4] + 1, b[0]:b[3] + 1])


def download_global(field, grid, shape):
    out = np.zeros(shape)
    for n in range(grid.num_local):
        b = grid.local_box(n)
        out[b[2]:b[5] + 1, b[1]:b[4] + 1, b[0]:b[3] + 1] = field.download(n)
    return out


# ----------------------------------------------------------------- ChF drop-ins
@pytest.mark.parametrize("rb", [0, 1])
def test_chf_dropin_gsrb_bitwise(rng, rb):
    # FAB boxes as the reference allocates them: dpsi with 3 ghosts (Main:82),
    # rhs/coefs with none (Main:83-88); region at an odd global offset.
    lo = (5, -3, 2)
    n = (20, 14, 9)
    g3 = tuple(l - 3 for l in lo)
    ncomp = 2
    u = rng.uniform(-1, 1, (ncomp, n[2] + 6, n[1] + 6, n[0] + 6))
    rhs = rng.uniform(-1, 1, (ncomp,) + n[::-1])
    a = rng.uniform(-2, -0.5, (ncomp,) + n[::-1])
    b = rng.uniform(0.5, 2, (ncomp,) + n[::-1])
    lam = rng.uniform(0.1, 0.3, (ncomp,) + n[::-1])
    hi = tuple(lo[d] + n[d] - 1 for d in range(3))
    dx, alpha, beta = 100.0 / 64, 1.0, -1.0
    ug = u.copy()
    mg.lib.gsrbhelmholtzvc3d_(*fab_args(ug, g3, ncomp), *fab_args(rhs, lo, ncomp), *ints(*lo),
                              *ints(*hi), ctypes.byref(ctypes.c_double(dx)),
                              ctypes.byref(ctypes.c_double(alpha)), *fab_args(a, lo, ncomp),
                              ctypes.byref(ctypes.c_double(beta)), *fab_args(b, lo, ncomp),
                              *fab_args(lam, lo, ncomp), ctypes.byref(ctypes.c_int(rb)))
    for c in range(ncomp):
        uo = np.ascontiguousarray(u[c])
        oracle.gsrb(Fab(uo, g3), Fab(np.ascontiguousarray(rhs[c]), lo), lo, hi, dx, alpha,
                    Fab(np.ascontiguousarray(a[c]), lo), beta, Fab(np.ascontiguousarray(b[c]), lo),
                    Fab(np.ascontiguousarray(lam[c]), lo), rb)
        assert np.array_equal(ug[c], uo)


def test_chf_dropin_op_res_restrict_bitwise(rng):
    n = (16, 12, 8)
    lo = (0, 0, 0)  # restrict is called on shifted boxes (.cpp:188-192)
    g1 = (-1, -1, -1)
    u = rng.uniform(-1, 1, (n[2] + 2, n[1] + 2, n[0] + 2))
    rhs, a, b = (rng.uniform(lo_, hi_, n[::-1]) for lo_, hi_ in ((-1, 1), (-2, -0.5), (0.5, 2)))
    hi = tuple(n[d] - 1 for d in range(3))
    dx, alpha, beta = 0.3, 0.7, -1.1
    cd = ctypes.c_double
    out_g = np.zeros(n[::-1])
    mg.lib.vccomputeop3d_(*fab_args(out_g, lo), *fab_args(u, g1), ctypes.byref(cd(alpha)),
                          *fab_args(a, lo), ctypes.byref(cd(beta)), *fab_args(b, lo), *ints(*lo),
                          *ints(*hi), ctypes.byref(cd(dx)))
    out_o = np.zeros(n[::-1])
    oracle.apply_op(Fab(out_o, lo), Fab(u, g1), alpha, Fab(a, lo), beta, Fab(b, lo), lo, hi, dx)
    assert np.array_equal(out_g, out_o)
    mg.lib.vccomputeres3d_(*fab_args(out_g, lo), *fab_args(u, g1), *fab_args(rhs, lo),
                           ctypes.byref(cd(alpha)), *fab_args(a, lo), ctypes.byref(cd(beta)),
                           *fab_args(b, lo), *ints(*lo), *ints(*hi), ctypes.byref(cd(dx)))
    oracle.residual(Fab(out_o, lo), Fab(u, g1), Fab(rhs, lo), alpha, Fab(a, lo), beta, Fab(b, lo),
                    lo, hi, dx)
    assert np.array_equal(out_g, out_o)
    rc_g = np.zeros((n[2] // 2, n[1] // 2, n[0] // 2))
    mg.lib.restrictresvc3d_(*fab_args(rc_g, lo), *fab_args(u, g1), *fab_args(rhs, lo),
                            ctypes.byref(cd(alpha)), *fab_args(a, lo), ctypes.byref(cd(beta)),
                            *fab_args(b, lo), *ints(*lo), *ints(*hi), ctypes.byref(cd(dx)))
    rc_o = np.zeros_like(rc_g)
    oracle.restrict_residual(Fab(rc_o, lo), Fab(u, g1), Fab(rhs, lo), alpha, Fab(a, lo), beta,
                             Fab(b, lo), lo, hi, dx)
    assert np.array_equal(rc_g, rc_o)


# ----------------------------------------------------------------- operator level
def build_pair(comm, rng, n, parts, *, alpha=1.0, beta=-1.0, avg=1, prolong=1, bc_lo=(0, 0, 0),
               bc_hi=(0, 0, 0), bc_value=0.0, periodic=(0, 0, 0), nlevels=3, bottom=0,
               relax_mode=1, agglomerate_below=0, fused=1, bvar=True, deep=0):
    dom = (0, 0, 0, n - 1, n - 1, n - 1)
    dx = 100.0 / n
    boxes = split_domain(dom, parts)
    a = rng.uniform(-2.0, -0.5, (n, n, n))
    b = rng.uniform(0.5, 2.0, (n, n, n)) if bvar else np.ones((n, n, n))
    rhs = rng.uniform(-1, 1, (n, n, n))
    grid = mg.Grid(comm, dom, boxes, dx, periodic=periodic)
    fa, fb, frhs, fphi, fres = (mg.LevelData(grid) for _ in range(5))
    for f, arr in ((fa, a), (fb, b), (frhs, rhs)):
        upload_global(f, grid, boxes, arr)
    fphi.set_zero()
    prm = mg.OperatorParams(alpha=alpha, beta=beta, bc_lo=bc_lo, bc_hi=bc_hi, bc_value=bc_value,
                            coefficient_average_type=avg, prolong_type=prolong,
                            relax_mode=relax_mode, fused_smoother=fused,
                            deep_halo=deep)
    fac = mg.defineOperatorFactory(grid, fa, fb, prm)
    amg = mg.AMRMultiGrid(fac, mg.SolverParams(max_depth=nlevels - 1, bottom_solver=bottom,
                                                agglomerate_below=agglomerate_below))
    o = oracle.OracleMG([dom], dom, dx, alpha=alpha, beta=beta, periodic=periodic, bc_lo=bc_lo,
                        bc_hi=bc_hi, bc_value=bc_value, nlevels=nlevels, avg_type=avg,
                        prolong_type=prolong, relax_mode=relax_mode, bottom_solver=bottom)
    o.set(0, oracle.ACOEF, 0, a)
    o.set(0, oracle.BCOEF, 0, b)
    o.set(0, oracle.RHS, 0, rhs)
    o.setup()
    return dict(grid=grid, boxes=boxes, fa=fa, fb=fb, frhs=frhs, fphi=fphi, fres=fres, fac=fac,
                amg=amg, o=o, n=n, a=a, b=b, rhs=rhs, dx=dx)


@pytest.mark.parametrize("parts", [(1, 1, 1), (2, 2, 2), (1, 2, 3)])
def test_operator_methods_bitwise(comm, rng, parts):
    n = 48 if parts == (1, 2, 3) else 32  # every box coarsenable by 8 (MGnewOp(2))
    S = build_pair(comm, rng, n, parts, bc_lo=(0, 1, 0), bc_hi=(1, 0, 0), bc_value=0.375)
    grid, o = S["grid"], S["o"]
    op = S["fac"].AMRnewOp()
    u = rng.uniform(-1, 1, (n, n, n))
    fu = mg.LevelData(grid)
    upload_global(fu, grid, S["boxes"], u)
    o.set(0, oracle.PHI, 0, u)
    out = mg.LevelData(grid)
    shape = (n, n, n)
    # residualI, inhomogeneous and homogeneous BC
    for hom in (0, 1):
        op.residualI(out, fu, S["frhs"], homogeneous=hom)
        o.residual(0, oracle.RESID, oracle.PHI, oracle.RHS, hom)
        assert np.array_equal(download_global(out, grid, shape), o.get(0, oracle.RESID, 0))
        op.applyOpI(out, fu, homogeneous=hom)
        o.apply_op(0, oracle.TMP, oracle.PHI, hom)
        assert np.array_equal(download_global(out, grid, shape), o.get(0, oracle.TMP, 0))
    # lambda
    lam = op.m_lambda
    assert np.array_equal(download_global(lam, grid, shape), o.get(0, oracle.LAMBDA, 0))
    # levelGSRB x3
    for _ in range(3):
        op.levelGSRB(fu, S["frhs"])
        o.level_gsrb(0, oracle.PHI, oracle.RHS)
    assert np.array_equal(download_global(fu, grid, shape), o.get(0, oracle.PHI, 0))
    # preCond
    op.preCond(out, S["frhs"])
    o.precond(0, oracle.TMP, oracle.RHS)
    assert np.array_equal(download_global(out, grid, shape), o.get(0, oracle.TMP, 0))
    # levelJacobi
    op.levelJacobi(fu, S["frhs"])
    o.level_jacobi(0, oracle.PHI, oracle.RHS)
    assert np.array_equal(download_global(fu, grid, shape), o.get(0, oracle.PHI, 0))
    # restrictResidual into the depth-1 layout, prolongIncrement back
    op1 = S["fac"].MGnewOp(1)
    rc = mg.LevelData(op1.grid)
    op.restrictResidual(rc, fu, S["frhs"])
    o.restrict_residual(0, oracle.PHI, oracle.RHS)
    m = n // 2
    assert np.array_equal(download_global(rc, op1.grid, (m, m, m)), o.get(1, oracle.RESID, 0))
    ec = rng.uniform(-1, 1, (m, m, m))
    fec = mg.LevelData(op1.grid)
    upload_global(fec, op1.grid, None, ec)
    o.set(1, oracle.CORR, 0, ec)
    op.prolongIncrement(fu, fec)
    o.prolong_increment(0, oracle.PHI)
    assert np.array_equal(download_global(fu, grid, shape), o.get(0, oracle.PHI, 0))
    # coefficient coarsening by MGnewOp(2): ratio 4 straight from depth 0
    op2 = S["fac"].MGnewOp(2)
    q = n // 4
    assert np.array_equal(download_global(op2.m_aCoef, op2.grid, (q, q, q)), o.get(2, oracle.ACOEF, 0))
    assert np.array_equal(download_global(op2.m_bCoef, op2.grid, (q, q, q)), o.get(2, oracle.BCOEF, 0))
    # norms / dots agree to rounding (parallel reduction order)
    d_g = op.dotProduct(fu, S["frhs"])
    d_o = o.dot(0, oracle.PHI, oracle.RHS)
    assert abs(d_g - d_o) <= 1e-12 * abs(d_o)
    assert op.norm(fu, 0) == o.norm(0, oracle.PHI, 0)


def test_fill_bc_matches_oracle(comm, rng):
    n = 16
    S = build_pair(comm, rng, n, (1, 1, 1), bc_lo=(0, 1, 0), bc_hi=(1, 0, 2), bc_value=0.25)
    op = S["fac"].AMRnewOp()
    u = rng.uniform(-1, 1, (n, n, n))
    fu = mg.LevelData(S["grid"])
    fu.upload(0, u)
    S["o"].set(0, oracle.PHI, 0, u)
    op.fillBC(fu, homogeneous=False)
    S["o"].fill_bc(0, oracle.PHI, 0)
    g = fu.download(0, with_ghosts=True)
    c = S["o"].get(0, oracle.PHI, 0, full=True)
    for sl in (np.s_[1:-1, 1:-1, 0], np.s_[1:-1, 1:-1, -1], np.s_[1:-1, 0, 1:-1],
               np.s_[1:-1, -1, 1:-1], np.s_[0, 1:-1, 1:-1]):
        assert np.array_equal(g[sl], c[sl])


@pytest.mark.parametrize("parts,prolong,avg", [((1, 1, 1), 1, 1), ((1, 1, 1), 0, 0),
                                               ((2, 2, 2), 1, 1), ((2, 1, 2), 0, 1)])
@pytest.mark.parametrize("fused", [2, 3])  # z-streaming / 3D-block sweep kernel
def test_vcycle_iterations_bitwise(comm, rng, parts, prolong, avg, fused):
    n = 32
    S = build_pair(comm, rng, n, parts, prolong=prolong, avg=avg, nlevels=3, bottom=0,
                   fused=fused)
    amg, o = S["amg"], S["o"]
    assert amg.num_depths == 3
    amg.init_residual(S["fphi"], S["frhs"], S["fres"])
    o.init_residual(0)
    for _ in range(3):
        rg = amg.iteration(S["fphi"], S["frhs"], S["fres"], norm_type=0)
        ro = o.iteration(0)
        assert rg == ro
    assert np.array_equal(download_global(S["fphi"], S["grid"], (n,) * 3), o.get(0, oracle.PHI, 0))


@pytest.mark.parametrize("parts,deep,bottom", [((1, 1, 1), 0, 0), ((1, 1, 1), 0, 1),
                                                ((2, 2, 2), 1, 0), ((2, 2, 2), 1, 1)])
@pytest.mark.parametrize("norm_type", [0, 1, -1])
def test_pipelined_iterations_match_iteration_calls(comm, rng, parts, deep, bottom, norm_type):
    # iterations() takes iteration i's norm on the host while iteration i+1's
    # V-cycle runs up to its phi += e launch (queued only after the read):
    # the same phi, residual and norms as iteration() calls -- with the
    # BiCGStab bottom, whose reductions are published in between, in the
    # deep-halo multi-box layout, and for norms taken outside the residual
    # launch (1) or not at all (-1)
    n = 32
    S = build_pair(comm, rng, n, parts, nlevels=3, bottom=bottom, fused=1, deep=deep)
    amg, grid = S["amg"], S["grid"]
    amg.init_residual(S["fphi"], S["frhs"], S["fres"], norm_type=0)
    want = [amg.iteration(S["fphi"], S["frhs"], S["fres"], norm_type=norm_type)
            for _ in range(3)]
    fphi2, fres2 = mg.LevelData(grid), mg.LevelData(grid)
    fphi2.set_zero()
    amg.init_residual(fphi2, S["frhs"], fres2, norm_type=0)
    got = amg.iterations(fphi2, S["frhs"], fres2, 3, norm_type=norm_type)
    assert got == want
    if norm_type < 0:
        assert got == [-1.0] * 3
    shp = (n,) * 3
    assert np.array_equal(download_global(fphi2, grid, shp), download_global(S["fphi"], grid, shp))
    assert np.array_equal(download_global(fres2, grid, shp), download_global(S["fres"], grid, shp))


@pytest.mark.parametrize("shape", [(76, 44, 52), (256, 132, 64)])
@pytest.mark.parametrize("bvar", [False, True])
def test_lds_staged_residual_restriction_odd_shapes_bitwise(rng, comm, bvar, shape):
    """The LDS-staged residual and restriction (k_residual_zl, k_restrict_zl:
    64 x 4 coarse / 128 x 4 fine tiles, 4- and 32-plane chunks, XCD bands of
    16 tiles) on boxes none of whose sides fills a tile, a row group or a
    chunk: a 2-level V-cycle off the origin with Dirichlet / Neumann faces,
    bit for bit against the oracle, norms included.  (76, 44, 52): fewer
    tiles than one band group (the dispatch order); (256, 132, 64): 132
    residual and 272 restriction tiles, i.e. whole groups of 8 x 16 bands
    plus a tail."""
    # (MGnewOp needs the box coarsenable by 4)
    lo = (8, -12, 16)
    dom = tuple(lo) + tuple(lo[d] + shape[d] - 1 for d in range(3))
    dx = 0.29
    bc_lo, bc_hi, bcv = (0, 1, 0), (1, 0, 0), 0.0
    nz, ny, nx = shape[2], shape[1], shape[0]
    a = rng.uniform(-2.0, -0.5, (nz, ny, nx))
    b = rng.uniform(0.5, 2.0, (nz, ny, nx)) if bvar else np.ones((nz, ny, nx))
    rhs = rng.uniform(-1, 1, (nz, ny, nx))
    grid = mg.Grid(comm, dom, [dom], dx)
    fa, fb, frhs, fphi, fres = (mg.LevelData(grid) for _ in range(5))
    fa.upload(0, a)
    fb.upload(0, b)
    frhs.upload(0, rhs)
    fphi.set_zero()
    prm = mg.OperatorParams(alpha=1.0, beta=-1.0, bc_lo=bc_lo, bc_hi=bc_hi, bc_value=bcv,
                            coefficient_average_type=1, prolong_type=1)
    amg = mg.AMRMultiGrid(mg.defineOperatorFactory(grid, fa, fb, prm),
                          mg.SolverParams(max_depth=1, bottom_solver=0))
    assert amg.num_depths == 2
    o = oracle.OracleMG([dom], dom, dx, alpha=1.0, beta=-1.0, bc_lo=bc_lo, bc_hi=bc_hi,
                        bc_value=bcv, nlevels=2, avg_type=1, prolong_type=1, bottom_solver=0)
    for f, arr in ((oracle.ACOEF, a), (oracle.BCOEF, b), (oracle.RHS, rhs)):
        o.set(0, f, 0, arr)
    o.setup()
    amg.init_residual(fphi, frhs, fres)
    o.init_residual(0)
    for _ in range(3):
        assert amg.iteration(fphi, frhs, fres, 0) == o.iteration(0)
    assert np.array_equal(fphi.download(0), o.get(0, oracle.PHI, 0))


@pytest.mark.parametrize("fused", [2, 3])
@pytest.mark.parametrize("bvar", [False, True])
def test_vcycle_ragged_mixed_bc_bitwise(rng, comm, fused, bvar):
    # non-cubic box at an odd global offset, Dirichlet/Neumann faces with a BC
    # value: covers the sweep+restriction kernel (fused=2: the last
    # pre-smoothing sweep restricts in the same pass) against the oracle
    shape = (48, 40, 56)  # x, y, z
    lo = (-16, 8, 32)
    dom = tuple(lo) + tuple(lo[d] + shape[d] - 1 for d in range(3))
    dx = 0.37
    bc_lo, bc_hi, bcv = (0, 1, 0), (1, 0, 1), 0.25
    nz, ny, nx = shape[2], shape[1], shape[0]
    a = rng.uniform(-2.0, -0.5, (nz, ny, nx))
    b = rng.uniform(0.5, 2.0, (nz, ny, nx)) if bvar else np.ones((nz, ny, nx))
    rhs = rng.uniform(-1, 1, (nz, ny, nx))
    grid = mg.Grid(comm, dom, [dom], dx)
    fa, fb, frhs, fphi, fres = (mg.LevelData(grid) for _ in range(5))
    fa.upload(0, a)
    fb.upload(0, b)
    frhs.upload(0, rhs)
    fphi.set_zero()
    prm = mg.OperatorParams(alpha=1.0, beta=-1.0, bc_lo=bc_lo, bc_hi=bc_hi, bc_value=bcv,
                            coefficient_average_type=1, prolong_type=1, fused_smoother=fused)
    amg = mg.AMRMultiGrid(mg.defineOperatorFactory(grid, fa, fb, prm),
                          mg.SolverParams(max_depth=2, bottom_solver=0))
    o = oracle.OracleMG([dom], dom, dx, alpha=1.0, beta=-1.0, bc_lo=bc_lo, bc_hi=bc_hi,
                        bc_value=bcv, nlevels=3, avg_type=1, prolong_type=1, bottom_solver=0)
    for f, arr in ((oracle.ACOEF, a), (oracle.BCOEF, b), (oracle.RHS, rhs)):
        o.set(0, f, 0, arr)
    o.setup()
    amg.init_residual(fphi, frhs, fres)
    o.init_residual(0)
    for _ in range(3):
        assert amg.iteration(fphi, frhs, fres, 0) == o.iteration(0)
    assert np.array_equal(fphi.download(0), o.get(0, oracle.PHI, 0))


@pytest.mark.parametrize("transport", ["rccl", "ipc"])
@pytest.mark.parametrize("fused", [2, 3])
def test_vcycle_periodic_multibox_rccl_self_messages(rng, fused, transport):
    # the remote path (RCCL pack -> send/recv -> unpack, or the peer-mapped
    # put / get kernels), exercised on one GPU by routing same-rank copies
    # through self messages
    c_local = mg.Comm()
    c_rccl = remote_comm(transport)
    n = 32
    out = []
    for c in (c_local, c_rccl):
        S = build_pair(c, np.random.default_rng(7), n, (2, 2, 2), periodic=(1, 1, 1), alpha=1.0,
                       nlevels=3, bottom=0, fused=fused)
        amg = S["amg"]
        amg.init_residual(S["fphi"], S["frhs"], S["fres"])
        norms = [amg.iteration(S["fphi"], S["frhs"], S["fres"], 0) for _ in range(2)]
        o = S["o"]
        o.init_residual(0)
        onorms = [o.iteration(0) for _ in range(2)]
        assert norms == onorms
        out.append(download_global(S["fphi"], S["grid"], (n,) * 3))
        assert np.array_equal(out[-1], o.get(0, oracle.PHI, 0))
    assert np.array_equal(out[0], out[1])


def test_bicgstab_bottom_within_tolerance(comm, rng):
    n = 32
    S = build_pair(comm, rng, n, (1, 1, 1), nlevels=5, bottom=1)  # 32..2, BiCGStab at 2^3
    amg, o = S["amg"], S["o"]
    amg.init_residual(S["fphi"], S["frhs"], S["fres"])
    o.init_residual(0)
    for _ in range(3):
        amg.iteration(S["fphi"], S["frhs"], S["fres"], 0)
        o.iteration(0)
    g = download_global(S["fphi"], S["grid"], (n,) * 3)
    c = o.get(0, oracle.PHI, 0)
    assert np.linalg.norm(g - c) <= 1e-10 * np.linalg.norm(c)


def test_bicgstab_bottom_pipelined_readbacks_bitwise(comm, rng, monkeypatch):
    """The bottom BiCGStab reads back three times per iteration (the second
    half-step and the next <RT, R> queued behind the norms, op.cpp
    BiCGStabSolver::solve): phi and every residual norm equal the loop with
    five readbacks (MGIC_BICG_PIPE=0) bit for bit."""
    n = 32
    runs = []
    for pipe in ("1", "0"):
        monkeypatch.setenv("MGIC_BICG_PIPE", pipe)
        S = build_pair(comm, np.random.default_rng(7), n, (1, 1, 1), nlevels=3, bottom=1)  # BiCGStab at 8^3
        amg = S["amg"]
        amg.init_residual(S["fphi"], S["frhs"], S["fres"])
        norms = [amg.iteration(S["fphi"], S["frhs"], S["fres"], 0) for _ in range(3)]
        runs.append((norms, download_global(S["fphi"], S["grid"], (n,) * 3)))
    assert runs[0][0] == runs[1][0]
    assert np.array_equal(runs[0][1], runs[1][1])


@pytest.mark.parametrize("n,nlevels", [(32, 3), (64, 3), (64, 2), (128, 2)])
def test_bicgstab_bottom_on_device_bitwise(comm, monkeypatch, n, nlevels):
    """The bottom BiCGStab with its scalars and stop tests on the device
    (op.cpp BiCGStabSolver::solveDevice: fused vector updates + reductions,
    last-block finals, batches without readbacks) equals the host loop --
    pipelined and unpipelined -- bit for bit in phi, every residual norm and
    the iteration count, for batch sizes that stop inside, at the end of and
    long before the end of a batch."""
    runs = []
    for env in ({"MGIC_BICG_DEVICE": "0", "MGIC_BICG_PIPE": "0"},
                {"MGIC_BICG_DEVICE": "0", "MGIC_BICG_PIPE": "1"},
                {"MGIC_BICG_DEVICE": "1", "MGIC_BICG_BATCH": "1"},
                {"MGIC_BICG_DEVICE": "1", "MGIC_BICG_BATCH": "3"},
                {"MGIC_BICG_DEVICE": "1", "MGIC_BICG_BATCH": "16"}):
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        # constant bCoef and fused_smoother 2: preCond is one two-sweep launch
        # (alpha 0 at 128^3: a Poisson bottom of many iterations)
        S = build_pair(comm, np.random.default_rng(7), n, (1, 1, 1), nlevels=nlevels, bottom=1,
                       fused=2, bvar=False, alpha=0.0 if n == 128 else 1.0)
        amg = S["amg"]
        amg.init_residual(S["fphi"], S["frhs"], S["fres"])
        norms, iters = [], []
        for _ in range(3):
            norms.append(amg.iteration(S["fphi"], S["frhs"], S["fres"], 0))
            dev, it, _ = amg.bottom_info()
            assert dev == (env["MGIC_BICG_DEVICE"] == "1")
            iters.append(it)
        runs.append((norms, iters, download_global(S["fphi"], S["grid"], (n,) * 3)))
    for r in runs[1:]:
        assert r[0] == runs[0][0]
        assert r[1] == runs[0][1]
        assert np.array_equal(r[2], runs[0][2])
    # (the 8^3 bottom converges in one iteration, then starts converged)
    assert max(runs[0][1]) >= (8 if n == 128 else 1), runs[0][1]


def test_bicgstab_bottom_replay_is_repeatable(comm):
    """bottom_replay (the bench's fixed-work bottom timing) re-solves the last
    coarse residual from e = 0: the same iterations and the same correction
    every time, equal to the V-cycle's own solve."""
    S = build_pair(comm, np.random.default_rng(3), 128, (1, 1, 1), nlevels=2, bottom=1, fused=2,
                   bvar=False, alpha=0.0)
    amg = S["amg"]
    amg.init_residual(S["fphi"], S["frhs"], S["fres"])
    amg.iteration(S["fphi"], S["frhs"], S["fres"], 0)
    dev, it, r0 = amg.bottom_info()
    assert dev and it >= 2
    e = amg.level_field(1, 0)
    e0 = e.download(0).copy()
    for _ in range(2):
        ms, it2, r02, n = amg.bottom_replay(2)
        assert n == 2 and ms > 0.0 and it2 == it and r02 == r0
        assert np.array_equal(e.download(0), e0)


def test_agglomerated_hierarchy_matches_single_box(comm, rng):
    n = 32
    S = build_pair(comm, rng, n, (2, 2, 2), nlevels=5, bottom=0, agglomerate_below=16)
    amg, o = S["amg"], S["o"]
    assert amg.num_depths == 5
    amg.init_residual(S["fphi"], S["frhs"], S["fres"])
    o.init_residual(0)
    for _ in range(2):
        assert amg.iteration(S["fphi"], S["frhs"], S["fres"], 0) == o.iteration(0)
    assert np.array_equal(download_global(S["fphi"], S["grid"], (n,) * 3), o.get(0, oracle.PHI, 0))


def test_binary_bh_inputs_on_device(comm):
    from mg_ic_code_amd.params import read_params_file
    import os
    p = read_params_file(os.path.join(os.path.dirname(__file__), "golden", "params.txt"))
    n = p.N[0]
    dom = (0, 0, 0, n - 1, n - 1, n - 1)
    grid = mg.Grid(comm, dom, [dom], p.coarsestDx)
    fa, fr = mg.LevelData(grid), mg.LevelData(grid)
    mg.set_binary_bh_coefs(fa, fr, p.bh())
    a_o, r_o = oracle.binary_bh(p.bh(), (0, 0, 0), (n - 1,) * 3, p.coarsestDx)
    np.testing.assert_allclose(fa.download(0), a_o, rtol=1e-13, atol=1e-300)
    np.testing.assert_allclose(fr.download(0), r_o, rtol=1e-13, atol=1e-300)


@pytest.mark.slow
@pytest.mark.parametrize("fused", [2, 3])
def test_large_vcycle_single_vs_multibox_and_oracle(comm, fused):
    # 128^3: GPU single box == GPU 8 boxes == oracle, bit for bit
    n = 128
    res = []
    for parts in ((1, 1, 1), (2, 2, 2)):
        S = build_pair(comm, np.random.default_rng(11), n, parts, nlevels=3, bottom=0, bvar=False,
                       fused=fused)
        amg = S["amg"]
        amg.init_residual(S["fphi"], S["frhs"], S["fres"])
        norms = [amg.iteration(S["fphi"], S["frhs"], S["fres"], 0) for _ in range(2)]
        res.append((norms, download_global(S["fphi"], S["grid"], (n,) * 3), S["o"]))
    assert res[0][0] == res[1][0]
    assert np.array_equal(res[0][1], res[1][1])
    o = res[0][2]
    o.init_residual(0)
    onorms = [o.iteration(0) for _ in range(2)]
    assert onorms == res[0][0]
    assert np.array_equal(o.get(0, oracle.PHI, 0), res[0][1])
    assert onorms[1] < onorms[0]


@pytest.mark.parametrize("bvar", [True, False])
@pytest.mark.parametrize("nsmooth", [1, 3, 4])
@pytest.mark.parametrize("periodic", [(0, 0, 0), (1, 0, 1)])
@pytest.mark.parametrize("parts,n,fused", [((2, 2, 2), 32, 1), ((2, 1, 3), 48, 2), ((3, 2, 1), 48, 3)])
def test_deep_halo_vcycle_bitwise(rng, nsmooth, periodic, parts, n, fused, bvar):
    # 4-deep shells, two sweeps per exchange (grown-box first sweep): the same
    # V-cycle iterates as the 2-deep schedule and the oracle, bit for bit, on
    # local copies, RCCL self messages and the peer-mapped transport, down to
    # 4-cell coarse boxes.  bvar=False (bCoef = 1, detected constant) routes
    # sweep pairs through the two-sweep kernel k_gsrb_tb2 on exchanged faces:
    # odd counts (a pair, then a single sweep after a 2-deep shell), periodic
    # self-exchanged faces, ragged boxes and the zero-input first pair
    for kind in ("local", "rccl", "ipc"):
        c = mg.Comm() if kind == "local" else remote_comm(kind)
        out = []
        for deep in (0, 1):
            S = build_pair(c, np.random.default_rng(9), n, parts, periodic=periodic, alpha=1.0,
                           nlevels=3, bottom=0, fused=fused, deep=deep, bvar=bvar)
            amg = mg.AMRMultiGrid(S["fac"], mg.SolverParams(max_depth=2, n_pre=nsmooth,
                                                            n_post=nsmooth, n_bottom=nsmooth,
                                                            bottom_solver=0))
            amg.init_residual(S["fphi"], S["frhs"], S["fres"])
            norms = [amg.iteration(S["fphi"], S["frhs"], S["fres"], 0) for _ in range(2)]
            out.append((norms, download_global(S["fphi"], S["grid"], (n,) * 3)))
        assert out[0][0] == out[1][0]
        assert np.array_equal(out[0][1], out[1][1])
    if nsmooth == 4:
        o = S["o"]
        o.init_residual(0)
        assert [o.iteration(0) for _ in range(2)] == out[0][0]
        assert np.array_equal(o.get(0, oracle.PHI, 0), out[0][1])


@pytest.mark.parametrize("shape,lo", [((70, 20, 13), (0, 0, 0)), ((37, 9, 40), (3, -5, 7)),
                                      ((128, 64, 33), (-64, 0, 1))])
@pytest.mark.parametrize("nsweeps", [1, 2, 3])
def test_fused_sweep_matches_oracle_and_passes(comm, rng, shape, lo, nsweeps):
    # the fused out-of-place red+black kernel (single box) against the oracle
    # and against the per-colour-pass kernels, bit for bit, on ragged shapes,
    # odd offsets (global colour parity), mixed Dirichlet/Neumann faces
    nx, ny, nz = shape
    dom = (lo[0], lo[1], lo[2], lo[0] + nx - 1, lo[1] + ny - 1, lo[2] + nz - 1)
    dx = 0.7
    a = rng.uniform(-2.0, -0.5, (nz, ny, nx))
    b = rng.uniform(0.5, 2.0, (nz, ny, nx))
    rhs = rng.uniform(-1, 1, (nz, ny, nx))
    u0 = rng.uniform(-1, 1, (nz, ny, nx))
    bc_lo, bc_hi = (0, 1, 0), (1, 0, 1)
    outs = []
    for fused in (2, 3, 1, 0):  # z-streaming, 3D blocks, by size, per-colour passes
        grid = mg.Grid(comm, dom, [dom], dx)
        fa, fb, fr, fu = (mg.LevelData(grid) for _ in range(4))
        fa.upload(0, a)
        fb.upload(0, b)
        fr.upload(0, rhs)
        fu.upload(0, u0)
        prm = mg.OperatorParams(alpha=1.0, beta=-1.0, bc_lo=bc_lo, bc_hi=bc_hi, bc_value=0.5,
                                fused_smoother=fused)
        fac = mg.defineOperatorFactory(grid, fa, fb, prm)
        op = fac.AMRnewOp()
        op.relax(fu, fr, nsweeps)
        outs.append(fu.download(0))
    for x in outs[1:]:
        assert np.array_equal(outs[0], x)
    o = oracle.OracleMG([dom], dom, dx, alpha=1.0, beta=-1.0, bc_lo=bc_lo, bc_hi=bc_hi,
                        bc_value=0.5, nlevels=1)
    o.set(0, oracle.ACOEF, 0, a)
    o.set(0, oracle.BCOEF, 0, b)
    o.set(0, oracle.RHS, 0, rhs)
    o.set(0, oracle.PHI, 0, u0)
    o.setup()
    o.relax(0, oracle.PHI, oracle.RHS, nsweeps)
    assert np.array_equal(outs[0], o.get(0, oracle.PHI, 0))


@pytest.mark.parametrize("shape,lo", [((37, 9, 40), (3, -5, 7)), ((130, 47, 45), (-64, 1, 1))])
@pytest.mark.parametrize("nsweeps", [2, 3])
@pytest.mark.parametrize("coefs", [(1.0, -1.0, 1.0), (0.75, -1.3, 1.7)])
@pytest.mark.parametrize("bc", [(0, 0.5), (1, 0.0), (0, 0.0)])
def test_two_sweep_one_rule_edges_match_oracle(comm, rng, shape, lo, nsweeps, coefs, bc):
    # every x / y domain face with the same ghost rule (the two-sweep
    # kernel's one-rule edge bodies, split into x-face, y-face and corner
    # tiles): inhomogeneous Dirichlet, homogeneous Neumann (ghost + -0) and
    # the reference's Dirichlet-0, against the oracle and the per-colour
    # passes bit for bit (z faces take the same rule)
    mode, bcv = bc
    alpha, beta, bval = coefs
    nx, ny, nz = shape
    dom = (lo[0], lo[1], lo[2], lo[0] + nx - 1, lo[1] + ny - 1, lo[2] + nz - 1)
    dx = 0.7
    a = rng.uniform(-2.0, -0.5, (nz, ny, nx))
    b = np.full((nz, ny, nx), bval)
    rhs = rng.uniform(-1, 1, (nz, ny, nx))
    u0 = rng.uniform(-1, 1, (nz, ny, nx))
    bc_lo = bc_hi = (mode,) * 3
    outs = []
    for fused in (2, 0):
        grid = mg.Grid(comm, dom, [dom], dx)
        fa, fb, fr, fu = (mg.LevelData(grid) for _ in range(4))
        fa.upload(0, a)
        fb.upload(0, b)
        fr.upload(0, rhs)
        fu.upload(0, u0)
        prm = mg.OperatorParams(alpha=alpha, beta=beta, bc_lo=bc_lo, bc_hi=bc_hi, bc_value=bcv,
                                fused_smoother=fused)
        op = mg.defineOperatorFactory(grid, fa, fb, prm).AMRnewOp()
        op.relax(fu, fr, nsweeps)
        outs.append(fu.download(0))
    assert np.array_equal(outs[0], outs[1])
    o = oracle.OracleMG([dom], dom, dx, alpha=alpha, beta=beta, bc_lo=bc_lo, bc_hi=bc_hi,
                        bc_value=bcv, nlevels=1)
    o.set(0, oracle.ACOEF, 0, a)
    o.set(0, oracle.BCOEF, 0, b)
    o.set(0, oracle.RHS, 0, rhs)
    o.set(0, oracle.PHI, 0, u0)
    o.setup()
    o.relax(0, oracle.PHI, oracle.RHS, nsweeps)
    assert np.array_equal(outs[0], o.get(0, oracle.PHI, 0))


@pytest.mark.parametrize("shape,lo", [((70, 20, 13), (0, 0, 0)), ((37, 9, 40), (3, -5, 7)),
                                      ((130, 47, 45), (-64, 1, 1)), ((64, 44, 24), (0, 0, 0))])
@pytest.mark.parametrize("nsweeps", [2, 3, 4, 5])
@pytest.mark.parametrize("coefs", [(1.0, -1.0, 1.0), (0.75, -1.3, 1.7)])
def test_two_sweep_relax_matches_oracle(comm, rng, shape, lo, nsweeps, coefs):
    # the temporally blocked two-sweep kernel (smoother_tb.hip: constant
    # bCoef, fused_smoother=2 forces the streaming path) in relax(): pairs of
    # sweeps plus a single one for odd counts, against the oracle and the
    # per-colour passes bit for bit.  Ragged tiles (64 x 22) in x and y,
    # several z chunks, odd global offsets (colour parity), mixed
    # inhomogeneous Dirichlet / Neumann faces; alpha = 1, beta = -1, b = 1 is
    # the kernel's exact specialisation, the other triple the general path.
    alpha, beta, bval = coefs
    nx, ny, nz = shape
    dom = (lo[0], lo[1], lo[2], lo[0] + nx - 1, lo[1] + ny - 1, lo[2] + nz - 1)
    dx = 0.7
    a = rng.uniform(-2.0, -0.5, (nz, ny, nx))
    b = np.full((nz, ny, nx), bval)
    rhs = rng.uniform(-1, 1, (nz, ny, nx))
    u0 = rng.uniform(-1, 1, (nz, ny, nx))
    bc_lo, bc_hi = (0, 1, 1), (1, 0, 0)
    outs = []
    for fused in (2, 0):
        grid = mg.Grid(comm, dom, [dom], dx)
        fa, fb, fr, fu = (mg.LevelData(grid) for _ in range(4))
        fa.upload(0, a)
        fb.upload(0, b)
        fr.upload(0, rhs)
        fu.upload(0, u0)
        prm = mg.OperatorParams(alpha=alpha, beta=beta, bc_lo=bc_lo, bc_hi=bc_hi, bc_value=0.5,
                                fused_smoother=fused)
        op = mg.defineOperatorFactory(grid, fa, fb, prm).AMRnewOp()
        op.relax(fu, fr, nsweeps)
        outs.append(fu.download(0))
    assert np.array_equal(outs[0], outs[1])
    o = oracle.OracleMG([dom], dom, dx, alpha=alpha, beta=beta, bc_lo=bc_lo, bc_hi=bc_hi,
                        bc_value=0.5, nlevels=1)
    o.set(0, oracle.ACOEF, 0, a)
    o.set(0, oracle.BCOEF, 0, b)
    o.set(0, oracle.RHS, 0, rhs)
    o.set(0, oracle.PHI, 0, u0)
    o.setup()
    o.relax(0, oracle.PHI, oracle.RHS, nsweeps)
    assert np.array_equal(outs[0], o.get(0, oracle.PHI, 0))


@pytest.mark.parametrize("big", [0.0, -1.0e160, -1.0e308])
def test_two_sweep_lambda_range_guard(comm, rng, big):
    # lambda = 1 / (alpha a + 6 beta / dx^2) by the short reciprocal
    # (smoother_tb.hip: rcp_div1) only when the host finds every lambda of the
    # level in [2^-500, 2^500]; a few cells with aCoef -1e160 (lambda ~ 1e-160)
    # or -1e308 (lambda subnormal, where the division's scale / fix-up steps
    # matter) turn the specialised body off.  Bit-identical to the oracle's
    # division either way (alpha = 1, beta = -1, b = 1: the FAST candidate).
    shape = (70, 44, 30)
    nx, ny, nz = shape
    dom = (0, 0, 0, nx - 1, ny - 1, nz - 1)
    dx = 0.7
    a = rng.uniform(-2.0, -0.5, (nz, ny, nx))
    if big:
        a.flat[rng.choice(a.size, 37, replace=False)] = big
    b = np.ones((nz, ny, nx))
    rhs = rng.uniform(-1, 1, (nz, ny, nx))
    u0 = rng.uniform(-1, 1, (nz, ny, nx))
    grid = mg.Grid(comm, dom, [dom], dx)
    fa, fb, fr, fu = (mg.LevelData(grid) for _ in range(4))
    fa.upload(0, a)
    fb.upload(0, b)
    fr.upload(0, rhs)
    fu.upload(0, u0)
    prm = mg.OperatorParams(alpha=1.0, beta=-1.0, fused_smoother=2)
    op = mg.defineOperatorFactory(grid, fa, fb, prm).AMRnewOp()
    op.relax(fu, fr, 4)
    o = oracle.OracleMG([dom], dom, dx, alpha=1.0, beta=-1.0, nlevels=1)
    o.set(0, oracle.ACOEF, 0, a)
    o.set(0, oracle.BCOEF, 0, b)
    o.set(0, oracle.RHS, 0, rhs)
    o.set(0, oracle.PHI, 0, u0)
    o.setup()
    o.relax(0, oracle.PHI, oracle.RHS, 4)
    assert np.array_equal(fu.download(0), o.get(0, oracle.PHI, 0), equal_nan=True)


# ------------------------------------------------- outer solve
@pytest.mark.parametrize("parts", [(1, 1, 1), (2, 1, 2)])
def test_mg_preconditioner_bitwise(comm, rng, parts):
    # MultilevelLinearOp::preCond: e = 0 + numMGIterations AMRMultiGrid
    # iterations (homogeneous BC) -- no reductions, so bit for bit
    n = 32
    S = build_pair(comm, rng, n, parts, nlevels=3, bottom=0, bvar=False)
    e = mg.LevelData(S["grid"])
    mg.MultilevelLinearOp(S["amg"], 2).preCond(e, S["frhs"])
    o = S["o"]
    o.amr_precond(oracle.TMP, oracle.RHS, 2)
    assert np.array_equal(download_global(e, S["grid"], (n,) * 3), o.get(0, oracle.TMP, 0))


@pytest.mark.parametrize("parts", [(1, 1, 1), (2, 2, 2)])
def test_outer_bicgstab_solve_matches_oracle(comm, rng, parts):
    # solver.solve(dpsi, rhs) of Main_PoissonSolver.cpp:174-184 with the
    # params.txt settings; dot products reduce in a different order, so the
    # bar is rel-L2 <= 1e-10 on phi and the same iteration count
    n = 32
    S = build_pair(comm, rng, n, parts, nlevels=3, bottom=0, bvar=False)
    solver = mg.BiCGStabSolver(mg.MultilevelLinearOp(S["amg"], 2), tolerance=1e-10,
                               max_iterations=100, norm_type=0)
    it = solver.solve(S["fphi"], S["frhs"])
    it_o, fin_o = S["o"].solve(mg_iters=2, imax=100, eps=1e-10, norm_type=0)
    assert it == it_o
    g = download_global(S["fphi"], S["grid"], (n,) * 3)
    c = S["o"].get(0, oracle.PHI, 0)
    assert np.linalg.norm(g - c) <= 1e-10 * np.linalg.norm(c)
    assert solver.final_norm <= 1e-9 * np.max(np.abs(S["rhs"]))  # true residual, max norm


# --------------------------------------------- the NL loop
def test_nl_coefs_on_device_match_oracle(comm, rng):
    # set_a_coef / set_rhs at a non-trivial psi (with ghosts), params.txt BH
    import os
    from mg_ic_code_amd.params import read_params_file
    prm = read_params_file(os.path.join(os.path.dirname(__file__), "golden", "params.txt"))
    n = 32
    dom = (0, 0, 0, n - 1, n - 1, n - 1)
    dx = prm.domainLength[0] / n
    grid = mg.Grid(comm, dom, [dom], dx)
    psi, fa, fr = mg.LevelData(grid), mg.LevelData(grid), mg.LevelData(grid)
    pg = 1.0 + 0.01 * rng.uniform(-1, 1, (n + 2,) * 3)
    psi.upload(0, pg, with_ghosts=True)
    mg.set_nl_coefs(psi, fa, fr, prm.bh())
    a_o, r_o = oracle.nl_coefs(prm.bh(), (0, 0, 0), (n - 1,) * 3, dx, pg)
    np.testing.assert_allclose(fa.download(0), a_o, rtol=1e-13, atol=1e-300)
    np.testing.assert_allclose(fr.download(0), r_o, rtol=1e-12, atol=1e-14)


def test_nonlinear_poisson_solve_matches_oracle(comm):
    # Main_PoissonSolver's NL loop: coefficients from psi, MG-preconditioned
    # BiCGStab, psi += dpsi, |dpsi| -- GPU against the oracle loop
    import os
    from mg_ic_code_amd.nl import poisson_solve
    from mg_ic_code_amd.params import read_params_file
    from tests.nl_ref import oracle_poisson_solve
    prm = read_params_file(os.path.join(os.path.dirname(__file__), "golden", "params.txt"))
    n = 32
    dom = (0, 0, 0, n - 1, n - 1, n - 1)
    grid = mg.Grid(comm, dom, [dom], prm.domainLength[0] / n)
    res = poisson_solve(grid, prm, max_depth=3, max_NL_iterations=3)
    psi_o, norms_o, iters_o, _ = oracle_poisson_solve(prm, n, max_depth=3, n_nl=3)
    # the first two NL steps carry the solution; the third dpsi is at the
    # linear solver's roundoff floor, where the two dot-product orders differ
    assert res.linear_iterations[:2] == iters_o[:2]
    np.testing.assert_allclose(res.dpsi_norms[:2], norms_o[:2], rtol=1e-6)
    assert abs(res.dpsi_norms[2] - norms_o[2]) <= 0.1 * norms_o[2]
    g = res.psi.download(0, with_ghosts=True)[1:-1, 1:-1, 1:-1]
    c = psi_o[1:-1, 1:-1, 1:-1]
    assert np.linalg.norm(g - c) <= 1e-10 * np.linalg.norm(c)


def test_periodic_nonlinear_poisson_solve_matches_oracle(comm):
    # periodic domain: K from the integrability condition each NL iteration
    # (Main_PoissonSolver.cpp:133-147), then the same loop as above
    import dataclasses
    import os
    from mg_ic_code_amd.nl import poisson_solve
    from mg_ic_code_amd.params import read_params_file
    from tests.nl_ref import oracle_poisson_solve
    prm = read_params_file(os.path.join(os.path.dirname(__file__), "golden", "params.txt"))
    prm = dataclasses.replace(prm, is_periodic=1)
    n = 32
    dom = (0, 0, 0, n - 1, n - 1, n - 1)
    from mg_ic_code_amd.decomposition import split_domain
    boxes = split_domain(dom, (2, 1, 1))
    grid = mg.Grid(comm, dom, boxes, prm.domainLength[0] / n, periodic=(1, 1, 1))
    # truncated at 3 NL steps |dpsi| is still 0.18 (> 1e-1), where the
    # reference stops with MayDay::Error (Main_PoissonSolver.cpp:221-225); the
    # loop's state travels with the error
    from mg_ic_code_amd.nl import NLDivergenceError
    with pytest.raises(NLDivergenceError) as ei:
        poisson_solve(grid, prm, max_depth=3, max_NL_iterations=3)
    res = ei.value.result
    psi_o, norms_o, iters_o, ks_o = oracle_poisson_solve(prm, n, max_depth=3, n_nl=3)
    # K: a sum over n^3 cells, GPU tree order vs numpy pairwise order
    np.testing.assert_allclose(res.constant_K, ks_o, rtol=1e-11)
    assert res.linear_iterations[:2] == iters_o[:2]
    np.testing.assert_allclose(res.dpsi_norms[:2], norms_o[:2], rtol=1e-6)
    g = np.zeros((n, n, n))
    for i, b in enumerate(boxes):
        g[b[2]:b[5] + 1, b[1]:b[4] + 1, b[0]:b[3] + 1] = res.psi.download(i)
    c = psi_o[1:-1, 1:-1, 1:-1]
    assert np.linalg.norm(g - c) <= 1e-9 * np.linalg.norm(c)


def test_chf_dropin_setleveldata_bitwise(rng):
    # GETLAPLACIANPSIF / GETRHOGRADPHIF (SetLevelDataF_F.H:15-19, :43-47) on
    # host FAB components: FRA1 operands with the box grown by one
    lo = (3, -2, 5)
    n = (17, 12, 9)
    hi = tuple(lo[d] + n[d] - 1 for d in range(3))
    g1 = tuple(l - 1 for l in lo)
    src = rng.uniform(0.5, 1.5, (n[2] + 2, n[1] + 2, n[0] + 2))
    dx = 100.0 / 64
    for name, fn in (("getlaplacianpsif_", oracle.getlaplacianpsif),
                     ("getrhogradphif_", oracle.getrhogradphif)):
        out = np.zeros(n[::-1])
        args = [dbl(out)] + ints(*lo) + ints(*hi) + [dbl(src)] + ints(*g1) + \
            ints(*(h + 1 for h in hi)) + [ctypes.byref(ctypes.c_double(dx))] + ints(*lo) + ints(*hi)
        getattr(mg.lib, name)(*args)
        assert np.array_equal(out, fn(src, lo, hi, dx)), name


_TWO_SWEEPS_CHILD = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
import mg_ic_code_amd as mg, oracle
for shape, lo, bc_lo, bc_hi, bcv in (((48, 40, 56), (-16, 8, 32), (0, 1, 0), (1, 0, 1), 0.25),
                                     ((64, 64, 64), (0, 0, 0), (0, 0, 0), (0, 0, 0), 0.0)):
    rng = np.random.default_rng(17)
    dom = tuple(lo) + tuple(lo[d] + shape[d] - 1 for d in range(3))
    nz, ny, nx = shape[2], shape[1], shape[0]
    a = rng.uniform(-2.0, -0.5, (nz, ny, nx)); rhs = rng.uniform(-1, 1, (nz, ny, nx))
    b = np.ones((nz, ny, nx))
    grid = mg.Grid(mg.Comm(), dom, [dom], 0.37)
    fa, fb, frhs, fphi, fres = (mg.LevelData(grid) for _ in range(5))
    fa.upload(0, a); fb.upload(0, b); frhs.upload(0, rhs); fphi.set_zero()
    prm = mg.OperatorParams(alpha=1.0, beta=-1.0, bc_lo=bc_lo, bc_hi=bc_hi, bc_value=bcv,
                            coefficient_average_type=1, prolong_type=1, fused_smoother=2)
    amg = mg.AMRMultiGrid(mg.defineOperatorFactory(grid, fa, fb, prm),
                          mg.SolverParams(max_depth=2, n_pre=5, n_post=4, n_bottom=4,
                                          bottom_solver=0))
    o = oracle.OracleMG([dom], dom, 0.37, alpha=1.0, beta=-1.0, bc_lo=bc_lo, bc_hi=bc_hi,
                        bc_value=bcv, nlevels=3, avg_type=1, prolong_type=1, bottom_solver=0,
                        n_pre=5, n_post=4, n_bottom=4)
    for f, arr in ((oracle.ACOEF, a), (oracle.BCOEF, b), (oracle.RHS, rhs)):
        o.set(0, f, 0, arr)
    o.setup()
    amg.init_residual(fphi, frhs, fres); o.init_residual(0)
    for _ in range(2):
        assert amg.iteration(fphi, frhs, fres, 0) == o.iteration(0)
    assert np.array_equal(fphi.download(0), o.get(0, oracle.PHI, 0))
print("two-sweep OK")
"""


@pytest.mark.parametrize("spl", ["1", "2"])
def test_two_sweep_kernel_vcycle_bitwise(spl):
    # the two-sweep kernel and its alternative (MGIC_SWEEPS_PER_LAUNCH, read
    # once per process: a child process): 2 = smoother_tb.hip (the default),
    # 1 = one sweep per launch throughout; odd and even sweep counts, ragged
    # mixed-BC box and a cube, against the oracle bit for bit
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MGIC_SWEEPS_PER_LAUNCH=spl)
    r = subprocess.run([sys.executable, "-c", _TWO_SWEEPS_CHILD, root], env=env,
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "two-sweep OK" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("n_post", [1, 2, 3, 4])
@pytest.mark.parametrize("bvar", [False, True])
def test_streaming_vcycle_post_sweeps_bitwise(rng, comm, n_post, bvar):
    # z-streaming kernels at every level, an odd number of post-smoothing
    # sweeps (n_post = 1: the sweep after the prolongation is also the one
    # that adds phi += e), random or constant bCoef; against the oracle bit
    # for bit
    shape = (64, 48, 40)
    lo = (-32, 16, 0)
    dom = tuple(lo) + tuple(lo[d] + shape[d] - 1 for d in range(3))
    bc_lo, bc_hi, bcv = (1, 0, 0), (0, 1, 1), -0.5
    nz, ny, nx = shape[2], shape[1], shape[0]
    a = rng.uniform(-2.0, -0.5, (nz, ny, nx))
    b = rng.uniform(0.5, 2.0, (nz, ny, nx)) if bvar else np.ones((nz, ny, nx))
    rhs = rng.uniform(-1, 1, (nz, ny, nx))
    grid = mg.Grid(comm, dom, [dom], 0.41)
    fa, fb, frhs, fphi, fres = (mg.LevelData(grid) for _ in range(5))
    fa.upload(0, a)
    fb.upload(0, b)
    frhs.upload(0, rhs)
    fphi.set_zero()
    prm = mg.OperatorParams(alpha=1.0, beta=-1.0, bc_lo=bc_lo, bc_hi=bc_hi, bc_value=bcv,
                            coefficient_average_type=1, prolong_type=1, fused_smoother=2)
    amg = mg.AMRMultiGrid(mg.defineOperatorFactory(grid, fa, fb, prm),
                          mg.SolverParams(max_depth=2, n_pre=2, n_post=n_post, n_bottom=3,
                                          bottom_solver=0))
    o = oracle.OracleMG([dom], dom, 0.41, alpha=1.0, beta=-1.0, bc_lo=bc_lo, bc_hi=bc_hi,
                        bc_value=bcv, nlevels=3, avg_type=1, prolong_type=1, bottom_solver=0,
                        n_pre=2, n_post=n_post, n_bottom=3)
    for f, arr in ((oracle.ACOEF, a), (oracle.BCOEF, b), (oracle.RHS, rhs)):
        o.set(0, f, 0, arr)
    o.setup()
    amg.init_residual(fphi, frhs, fres)
    o.init_residual(0)
    for _ in range(3):
        assert amg.iteration(fphi, frhs, fres, 0) == o.iteration(0)
    assert np.array_equal(fphi.download(0), o.get(0, oracle.PHI, 0))


@pytest.mark.gpu
def test_full_size_512_vcycle_bitwise():
    # BASELINE config C3 at its full size: the 512^3 3-level V-cycle of
    # bench.py (SetBinaryBH source on device, harmonic averaging, linear
    # prolongation, nu = 4, 4 bottom sweeps) -- two AMRMultiGrid iterations on
    # the GPU against the C oracle (OpenMP), phi and the residual norms bit
    # for bit.  ~8 GB of host memory, ~20 s.
    import os
    from mg_ic_code_amd.params import read_params_file
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prm = read_params_file(os.path.join(root, "tests", "golden", "params.txt"))
    n = 512
    dx = prm.L / n
    bh = prm.bh()
    bh["domain_length"] = dx * n
    dom = (0, 0, 0, n - 1, n - 1, n - 1)
    grid = mg.Grid(mg.Comm(), dom, [dom], dx)
    fa, fb, frhs, fphi, fres = (mg.LevelData(grid) for _ in range(5))
    mg.set_binary_bh_coefs(fa, frhs, bh)
    fb.set_val(1.0)
    fphi.set_zero()
    op = mg.OperatorParams(alpha=prm.alpha, beta=prm.beta, bc_lo=tuple(prm.bc_lo),
                           bc_hi=tuple(prm.bc_hi), bc_value=prm.bc_value,
                           coefficient_average_type=1, prolong_type=1, relax_mode=1,
                           fused_smoother=1)
    amg = mg.AMRMultiGrid(mg.defineOperatorFactory(grid, fa, fb, op),
                          mg.SolverParams(max_depth=2, n_pre=4, n_post=4, n_bottom=4,
                                          bottom_solver=0))
    r0 = amg.init_residual(fphi, frhs, fres, norm_type=0)
    rg = [amg.iteration(fphi, frhs, fres, norm_type=0) for _ in range(2)]
    oracle.set_threads(min(16, os.cpu_count() or 1))
    o = oracle.OracleMG([dom], dom, dx, alpha=prm.alpha, beta=prm.beta, bc_lo=tuple(prm.bc_lo),
                        bc_hi=tuple(prm.bc_hi), bc_value=prm.bc_value, nlevels=3, avg_type=1,
                        prolong_type=1, bottom_solver=0, n_pre=4, n_post=4, n_bottom=4)
    a = fa.download(0)
    o.set(0, oracle.ACOEF, 0, a)
    o.set(0, oracle.BCOEF, 0, np.ones_like(a))
    del a
    o.set(0, oracle.RHS, 0, frhs.download(0))
    o.setup()
    assert o.init_residual(0) == r0
    assert [o.iteration(0) for _ in range(2)] == rg
    assert np.array_equal(fphi.download(0), o.get(0, oracle.PHI, 0))
    # iterations() (the bench's timed loop): the same phi and norms
    del o
    fphi2, fres2 = mg.LevelData(grid), mg.LevelData(grid)
    fphi2.set_zero()
    assert amg.init_residual(fphi2, frhs, fres2, norm_type=0) == r0
    assert amg.iterations(fphi2, frhs, fres2, 2, norm_type=0) == rg
    assert np.array_equal(fphi2.download(0), fphi.download(0))
    assert np.array_equal(fres2.download(0), fres.download(0))


@pytest.mark.gpu
def test_full_size_256_single_level_gsrb_and_residual_bitwise():
    # BASELINE config C2 at its full size: 256^3 single level, SetBinaryBH
    # source, the GSRB smoother (8 fused sweeps from dpsi = 0) and then the
    # residual rhs - L(dpsi) with the inhomogeneous BC, against the oracle
    # bit for bit (the "GSRB smoother vs CPU residual" of the config)
    import os
    from mg_ic_code_amd.params import read_params_file
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prm = read_params_file(os.path.join(root, "tests", "golden", "params.txt"))
    n = 256
    dx = prm.L / n
    bh = prm.bh()
    bh["domain_length"] = dx * n
    dom = (0, 0, 0, n - 1, n - 1, n - 1)
    grid = mg.Grid(mg.Comm(), dom, [dom], dx)
    fa, fb, frhs, fu, fres = (mg.LevelData(grid) for _ in range(5))
    mg.set_binary_bh_coefs(fa, frhs, bh)
    fb.set_val(1.0)
    fu.set_zero()
    op = mg.defineOperatorFactory(
        grid, fa, fb, mg.OperatorParams(alpha=prm.alpha, beta=prm.beta, bc_lo=tuple(prm.bc_lo),
                                        bc_hi=tuple(prm.bc_hi), bc_value=prm.bc_value,
                                        relax_mode=1, fused_smoother=1)).AMRnewOp()
    op.relax(fu, frhs, 8)
    op.residualI(fres, fu, frhs, homogeneous=False)
    oracle.set_threads(min(16, os.cpu_count() or 1))
    o = oracle.OracleMG([dom], dom, dx, alpha=prm.alpha, beta=prm.beta, bc_lo=tuple(prm.bc_lo),
                        bc_hi=tuple(prm.bc_hi), bc_value=prm.bc_value, nlevels=1)
    a = fa.download(0)
    o.set(0, oracle.ACOEF, 0, a)
    o.set(0, oracle.BCOEF, 0, np.ones_like(a))
    o.set(0, oracle.RHS, 0, frhs.download(0))
    o.set(0, oracle.PHI, 0, np.zeros_like(a))
    o.setup()
    o.relax(0, oracle.PHI, oracle.RHS, 8)
    o.residual(0, oracle.RESID, oracle.PHI, oracle.RHS, 0)
    assert np.array_equal(fu.download(0), o.get(0, oracle.PHI, 0))
    assert np.array_equal(fres.download(0), o.get(0, oracle.RESID, 0))


@pytest.mark.gpu
def test_full_size_512_eight_boxes_rccl_deep_halo_bitwise():
    # BASELINE config C4's code path at its full size on one GPU: 512^3 as the
    # 8-GPU split (2x2x2 boxes of 256^3), every exchange through RCCL
    # self send/recv, the deep halo N > 1 runs with -- against the single-box
    # run (itself bit-identical to the oracle, test_full_size_512_vcycle_
    # bitwise), phi and residual norms bit for bit over two iterations
    import os
    from mg_ic_code_amd.decomposition import decompose
    from mg_ic_code_amd.params import read_params_file
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prm = read_params_file(os.path.join(root, "tests", "golden", "params.txt"))
    n = 512
    dx = prm.L / n
    bh = prm.bh()
    bh["domain_length"] = dx * n
    out = []
    for parts, deep, kind in (((1, 1, 1), 0, "local"), ((2, 2, 2), 1, "rccl"),
                              ((2, 2, 2), 1, "ipc")):
        # one rank owns all 8 boxes: its self message carries every shell
        c = mg.Comm() if kind == "local" else remote_comm(kind, arena_mb=256)
        dom, boxes, owners = decompose((n, n, n), 1, boxes_per_rank=parts)
        grid = mg.Grid(c, dom, boxes, dx, owners=owners)
        fa, fb, frhs, fphi, fres = (mg.LevelData(grid) for _ in range(5))
        mg.set_binary_bh_coefs(fa, frhs, bh)
        fb.set_val(1.0)
        fphi.set_zero()
        op = mg.OperatorParams(alpha=prm.alpha, beta=prm.beta, bc_lo=tuple(prm.bc_lo),
                               bc_hi=tuple(prm.bc_hi), bc_value=prm.bc_value,
                               coefficient_average_type=1, prolong_type=1, relax_mode=1,
                               fused_smoother=1, deep_halo=deep)
        amg = mg.AMRMultiGrid(mg.defineOperatorFactory(grid, fa, fb, op),
                              mg.SolverParams(max_depth=2, n_pre=4, n_post=4, n_bottom=4,
                                              bottom_solver=0))
        norms = [amg.init_residual(fphi, frhs, fres, norm_type=0)]
        norms += [amg.iteration(fphi, frhs, fres, norm_type=0) for _ in range(2)]
        out.append((norms, download_global(fphi, grid, (n,) * 3)))
        del amg, fa, fb, frhs, fphi, fres, grid
    for r in out[1:]:
        assert out[0][0] == r[0]
        assert np.array_equal(out[0][1], r[1])


@pytest.mark.parametrize("kc", ["8", "5"])
def test_two_sweep_trim_and_round_order_match_oracle(kc):
    """The two-sweep launch's ghost-line trim (every launch kind, every box
    size: MGIC_TB2_TRIM=15) and its round-major tile order with a partial
    last round (MGIC_TB2_KC=8 on a 192 x 132 x 128 box) in a fresh process
    (tests/trim_worker.py; the switches are read once per process): relax on
    ragged shapes, odd offsets and every one-rule BC, and V-cycle iterations
    (ZIN / plain / ACC launches), bit-identical to the oracle.  KC=5: the
    short chunks the chooser now picks for small boxes (a 128^3 box takes
    chunks of 7), every chunk boundary inside the 8-slot ring's fill."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MGIC_TB2_TRIM="15", MGIC_TB2_KC=kc, PYTHONUNBUFFERED="1")
    r = subprocess.run([sys.executable, os.path.join(root, "tests", "trim_worker.py")], cwd=root,
                       env=env, capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert "trim worker OK" in r.stdout, out[-3000:]
    assert "double free" not in out and "corruption" not in out, out[-3000:]
