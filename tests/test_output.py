"""the reference's HDF5 output (Source/WriteOutput.H).

CPU: the oracle restatement of set_output_data against hand-evaluated cells,
libmgic_io's exports, and both file layouts written from host arrays, read
back with h5dump (structure, header attributes, boxes, offsets, data).
GPU: the device components (k_output_vars) against the oracle, slab
consistency, device-written files against the oracle and against the
host-written layout, and the NL loop's output files.

Chombo's CH_HDF5 / AMRIO are not in the reference tree: the layout is a
restatement, so parity of the file structure is unpinned; the component
values follow SetLevelData.cpp:343-396 / WriteOutput.H:74-100 (rtol 1e-13:
pow/exp/sqrt differ by an ulp between the GPU and glibc).
"""
import ctypes
import math
import os
import re

import numpy as np
import pytest

import oracle
from mg_ic_code_amd import _lib
from mg_ic_code_amd.output import GRCHOMBO_VARS, SOLVER_VARS, write_host
from tests import h5read

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BH = dict(domain_length=16.0, G_Newton=1.0, phi_amplitude=0.1, phi_wavelength=1.0,
          bh1_bare_mass=0.5, bh2_bare_mass=0.3, bh1_spin=0.1, bh2_spin=-0.2, bh1_offset=2.1,
          bh2_offset=-1.9, bh1_momentum=0.15, bh2_momentum=-0.05, constant_K=-0.3)


def _shape(b):
    return (b[5] - b[2] + 1, b[4] - b[1] + 1, b[3] - b[0] + 1)


def _cell_ref(i, j, k, dx, psi):
    """set_output_data at one cell, evaluated in Python (SetLevelData.cpp:374-393,
    SetBinaryBH.H:15-99, MyPhiFunction.H)."""
    L = BH["domain_length"]
    loc = [(v + 0.5) * dx - L / 2.0 for v in (i, j, k)]
    r1 = math.sqrt((loc[0] - BH["bh1_offset"]) ** 2 + loc[1] ** 2 + loc[2] ** 2)
    r2 = math.sqrt((loc[0] - BH["bh2_offset"]) ** 2 + loc[1] ** 2 + loc[2] ** 2)
    psi_bh = BH["bh1_bare_mass"] / r1 + BH["bh2_bare_mass"] / r2
    chi = (psi + psi_bh) ** -4.0
    phi = BH["phi_amplitude"] * math.exp(-(loc[0] ** 2 + loc[1] ** 2 + loc[2] ** 2)
                                         / BH["phi_wavelength"])
    return chi, phi, chi ** 1.5


def test_oracle_output_vars_known_cells():
    lo, hi, dx = (3, 5, 7), (6, 7, 9), 0.5
    rng = np.random.default_rng(1)
    psi = 1.0 + 0.1 * rng.uniform(-1, 1, _shape(lo + hi))
    o = oracle.output_vars(0, BH, lo, hi, dx, psi)
    assert o.shape == (31,) + _shape(lo + hi)
    const = {1: 1.0, 4: 1.0, 6: 1.0, 18: 1.0, 7: BH["constant_K"]}
    for c in range(31):
        if c in const:
            assert np.all(o[c] == const[c]), GRCHOMBO_VARS[c]
        elif c not in (0, 8, 9, 10, 11, 12, 13, 25):
            assert np.all(o[c] == 0.0), GRCHOMBO_VARS[c]
    for (k, j, i) in ((0, 0, 0), (2, 1, 3), (1, 2, 2)):
        chi, phi, factor = _cell_ref(lo[0] + i, lo[1] + j, lo[2] + k, dx, psi[k, j, i])
        assert o[0, k, j, i] == pytest.approx(chi, rel=1e-14)
        assert o[25, k, j, i] == pytest.approx(phi, rel=1e-14)
    # A_ij = A_ij_0 * chi^1.5, the A_ij_0 of the solver-data components
    s = oracle.output_vars(1, BH, lo, hi, dx, psi, psi * 2, psi * 3)
    assert np.array_equal(s[0], psi * 2) and np.array_equal(s[1], psi * 3)
    assert np.array_equal(s[2], psi)
    fac = o[0] ** 1.5
    for c_out, c_in in zip(range(8, 14), range(3, 9)):
        np.testing.assert_allclose(o[c_out], s[c_in] * fac, rtol=1e-14, atol=0)
    assert np.array_equal(s[9], o[25])
    assert np.any(s[3] != 0) and np.any(s[4] != 0)  # momentum / spin terms present


def test_io_lib_exports_its_header():
    txt = open(os.path.join(ROOT, "include", "mgic_io.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = set(re.findall(r"MGIC_IO_API\s+[\w\s\*]+?\b(mgic_io_\w+)\s*\(", txt))
    assert names == set(_lib.IO_SIGNATURES)
    lib = _lib.io_lib()
    assert all(hasattr(lib, n) for n in names)


def _levels(kind):
    """two levels: 16^3-domain base in two boxes, a refined patch"""
    nc = 31 if kind == 0 else 10
    rng = np.random.default_rng(7 + kind)
    dom0, dom1 = (0, 0, 0, 15, 15, 15), (0, 0, 0, 31, 31, 31)
    b0 = [(0, 0, 0, 7, 15, 15), (8, 0, 0, 15, 15, 15)]
    b1 = [(8, 10, 12, 19, 21, 25)]
    mk = lambda b: rng.uniform(-1, 1, (nc,) + _shape(b))
    return [(dom0, 1.0, [(b, mk(b)) for b in b0]), (dom1, 0.5, [(b, mk(b)) for b in b1])]


def _check_layout(fname, kind, levels, max_level=3, it=5):
    nc = 31 if kind == 0 else 10
    names = GRCHOMBO_VARS if kind == 0 else SOLVER_VARS
    c = h5read.contents(fname)
    for l in range(len(levels)):
        for d in ("boxes", "data:datatype=0", "data:offsets=0", "Processors"):
            assert c[f"/level_{l}/{d}"] == "dataset"
        assert c[f"/level_{l}/data_attributes"] == "group"
    assert c["/Chombo_global"] == "group"
    assert h5read.attr(fname, "/Chombo_global/SpaceDim") == 3
    assert h5read.attr(fname, "/num_components") == nc
    for i in (0, 7, nc - 1):
        assert h5read.attr(fname, f"/component_{i}") == names[i]
    if kind == 0:  # WriteOutput.H:145-173
        assert h5read.attr(fname, "/max_level") == max_level
        assert h5read.attr(fname, "/num_levels") == max_level + 1
        assert h5read.attr(fname, "/iteration") == 0
        assert h5read.attr(fname, "/regrid_interval_1") == 1
        assert h5read.attr(fname, "/steps_since_regrid_0") == 0
    else:
        assert h5read.attr(fname, "/num_levels") == len(levels)
        assert h5read.attr(fname, "/filetype") == "VanillaAMRFileType"
    for l, (dom, dx, bl) in enumerate(levels):
        g = f"/level_{l}"
        assert h5read.attr(fname, g + "/prob_domain") == tuple(dom)
        assert h5read.attr(fname, g + "/dx") == dx
        if kind == 0:  # WriteOutput.H:196-216
            assert h5read.attr(fname, g + "/dt") == 0.25 * dx
            assert h5read.attr(fname, g + "/ref_ratio") == 2
            assert h5read.attr(fname, g + "/tag_buffer_size") == 3
            assert h5read.attr(fname, g + "/is_periodic_2") == 1
            assert h5read.attr(fname, g + "/data_attributes/ghost") == (3, 3, 3)
        else:  # writeLevel: time = iter, dt refined, ref_ratio 1 on the finest
            assert h5read.attr(fname, g + "/time") == float(it)
            assert h5read.attr(fname, g + "/dt") == 1.0 / 2 ** l
            assert h5read.attr(fname, g + "/ref_ratio") == (2 if l < len(levels) - 1 else 1)
            assert h5read.attr(fname, g + "/data_attributes/ghost") == (0, 0, 0)
        assert h5read.attr(fname, g + "/data_attributes/outputGhost") == (0, 0, 0)
        assert h5read.attr(fname, g + "/data_attributes/comps") == nc
        assert h5read.attr(fname, g + "/data_attributes/objectType") == "FArrayBox"
        assert h5read.boxes(fname, l) == [tuple(b) for b, _ in bl]
        off = h5read.dataset(fname, g + "/data:offsets=0", "<i8")
        sizes = [d.size for _, d in bl]
        assert list(off) == list(np.concatenate([[0], np.cumsum(sizes)]))
        data = h5read.dataset(fname, g + "/data:datatype=0", "<f8")
        assert np.array_equal(data, np.concatenate([d.ravel() for _, d in bl]))


@pytest.mark.parametrize("kind", [0, 1])
def test_host_writer_layout(tmp_path, kind):
    levels = _levels(kind)
    f = str(tmp_path / f"out{kind}.hdf5")
    write_host(f, kind, levels, [2, 2], max_level=3, iteration=5)
    _check_layout(f, kind, levels)


def test_host_writer_rejects_bad_arguments(tmp_path):
    with pytest.raises(_lib.MgicError):
        write_host(str(tmp_path / "x.hdf5"), 2, _levels(0), [2, 2])
    with pytest.raises(_lib.MgicError):
        write_host(str(tmp_path / "no_such_dir" / "x.hdf5"), 0, _levels(0), [2, 2])


# ------------------------------------------------------------------ GPU
@pytest.fixture(scope="module")
def comm():
    import mg_ic_code_amd as mg
    return mg.Comm()


def _fields(comm, boxes, dom, dx, rng):
    import mg_ic_code_amd as mg
    grid = mg.Grid(comm, dom, boxes, dx)
    psi, dpsi, rhs = (mg.LevelData(grid) for _ in range(3))
    host = {}
    for k in range(grid.num_local):
        b = grid.local_box(k)
        u = 1.0 + 0.05 * rng.uniform(-1, 1, _shape(b))
        d, r = rng.uniform(-1, 1, _shape(b)), rng.uniform(-1, 1, _shape(b))
        psi.upload(k, u)
        dpsi.upload(k, d)
        rhs.upload(k, r)
        host[k] = (b, u, d, r)
    return grid, psi, dpsi, rhs, host


@pytest.mark.gpu
def test_device_output_vars_match_oracle(comm):
    from mg_ic_code_amd.output import grchombo_vars, solver_vars
    rng = np.random.default_rng(11)
    dom = (0, 0, 0, 39, 31, 23)
    boxes = [(0, 0, 0, 19, 31, 23), (20, 0, 0, 39, 15, 23), (20, 16, 0, 39, 31, 23)]
    grid, psi, dpsi, rhs, host = _fields(comm, boxes, dom, 16.0 / 40, rng)
    for k, (b, u, d, r) in host.items():
        g = grchombo_vars(psi, k, BH)
        o = oracle.output_vars(0, BH, b[:3], b[3:], 16.0 / 40, u)
        exact = [c for c in range(31) if c not in (0, 8, 9, 10, 11, 12, 13, 25)]
        assert np.array_equal(g[exact], o[exact])
        np.testing.assert_allclose(g, o, rtol=1e-13, atol=1e-300)
        s = solver_vars(dpsi, rhs, psi, k, BH)
        so = oracle.output_vars(1, BH, b[:3], b[3:], 16.0 / 40, u, d, r)
        assert np.array_equal(s[:3], so[:3])
        np.testing.assert_allclose(s, so, rtol=1e-13, atol=1e-300)
        # z-slabs reproduce the whole box
        nz = b[5] - b[2] + 1
        parts = [grchombo_vars(psi, k, BH, k0, min(7, nz - k0)) for k0 in range(0, nz, 7)]
        assert np.array_equal(np.concatenate(parts, axis=1), g)


@pytest.mark.gpu
def test_output_final_and_solver_data_files(comm, tmp_path):
    import mg_ic_code_amd as mg
    rng = np.random.default_rng(12)
    dom0 = (0, 0, 0, 15, 15, 15)
    grid0, psi0, dpsi0, rhs0, h0 = _fields(comm, [(0, 0, 0, 7, 15, 15), (8, 0, 0, 15, 15, 15)],
                                           dom0, 1.0, rng)
    # a patch level (no solve needed for output)
    grid1 = mg.Grid(comm, (0, 0, 0, 31, 31, 31), [(8, 10, 12, 19, 21, 25)], 0.5, patches=True)
    psi1, dpsi1, rhs1 = (mg.LevelData(grid1) for _ in range(3))
    b1 = grid1.local_box(0)
    u1 = 1.0 + 0.05 * rng.uniform(-1, 1, _shape(b1))
    d1, r1 = rng.uniform(-1, 1, _shape(b1)), rng.uniform(-1, 1, _shape(b1))
    psi1.upload(0, u1)
    dpsi1.upload(0, d1)
    rhs1.upload(0, r1)
    h1 = {0: (b1, u1, d1, r1)}
    f0 = str(tmp_path / "final.hdf5")
    mg.output_final_data([psi0, psi1], BH, max_level=3, ref_ratio=[2, 2], filename=f0)
    f1 = str(tmp_path / "solver.hdf5")
    mg.output_solver_data([dpsi0, dpsi1], [rhs0, rhs1], [psi0, psi1], BH, 5, [2, 2], f1)
    for kind, f in ((0, f0), (1, f1)):
        levels = []
        for (dom, dx, hh) in (((0, 0, 0, 15, 15, 15), 1.0, h0), ((0, 0, 0, 31, 31, 31), 0.5, h1)):
            bl = []
            for k in sorted(hh):
                b, u, d, r = hh[k]
                bl.append((b, oracle.output_vars(kind, BH, b[:3], b[3:], dx, u, d, r)))
            levels.append((dom, dx, bl))
        # the device-written file has the layout and (to rtol) the oracle's data
        nc = 31 if kind == 0 else 10
        for l, (dom, dx, bl) in enumerate(levels):
            data = h5read.dataset(f, f"/level_{l}/data:datatype=0", "<f8")
            want = np.concatenate([d.ravel() for _, d in bl])
            np.testing.assert_allclose(data, want, rtol=1e-13, atol=1e-300)
            # replace by the file's own values, then the layout check is exact
            pos = 0
            for i, (b, d) in enumerate(bl):
                bl[i] = (b, data[pos:pos + d.size].reshape(d.shape))
                pos += d.size
        _check_layout(f, kind, levels)


@pytest.mark.gpu
def test_nl_loop_writes_reference_files(tmp_path):
    import mg_ic_code_amd as mg
    from mg_ic_code_amd.nl import poisson_solve
    from mg_ic_code_amd.params import read_params_file
    prm = read_params_file(os.path.join(ROOT, "tests", "golden", "params.txt"))
    n = 32
    dom = (0, 0, 0, n - 1, n - 1, n - 1)
    grid = mg.Grid(mg.Comm(), dom, [dom], prm.domainLength[0] / n)
    res = poisson_solve(grid, prm, max_depth=3, max_NL_iterations=2, output_dir=str(tmp_path))
    names = sorted(os.listdir(tmp_path))
    want = [f"vcPoissonOut.3d_{i}.hdf5" for i in range(len(res.dpsi_norms))]
    assert names == sorted(want + ["vcPoissonFinal.3d.hdf5"])
    f = str(tmp_path / "vcPoissonFinal.3d.hdf5")
    data = h5read.dataset(f, "/level_0/data:datatype=0", "<f8").reshape((31, n, n, n))
    bh = prm.bh(constant_K=res.constant_K[-1] if res.constant_K else 0.0)
    o = oracle.output_vars(0, bh, (0, 0, 0), (n - 1,) * 3, prm.domainLength[0] / n,
                           res.psi.download(0))
    np.testing.assert_allclose(data, o, rtol=1e-13, atol=1e-300)
    assert h5read.attr(f, "/max_level") == prm.max_level


@pytest.mark.gpu
def test_nl_loop_divergence_raises_and_writes_no_checkpoint(tmp_path):
    # Main_PoissonSolver.cpp:221-225: MayDay::Error before output_final_data
    # when the final |dpsi| > 1e-1.  Momenta of 50 make |dpsi| ~ 58 after the
    # first NL step (test_nl_host.py pins that on the oracle loop).
    import dataclasses
    import mg_ic_code_amd as mg
    from mg_ic_code_amd.nl import NLDivergenceError, poisson_solve
    from mg_ic_code_amd.params import read_params_file
    prm = read_params_file(os.path.join(ROOT, "tests", "golden", "params.txt"))
    prm = dataclasses.replace(prm, bh1_momentum=50.0, bh2_momentum=-50.0)
    n = 16
    dom = (0, 0, 0, n - 1, n - 1, n - 1)
    grid = mg.Grid(mg.Comm(), dom, [dom], prm.domainLength[0] / n)
    with pytest.raises(NLDivergenceError) as ei:
        poisson_solve(grid, prm, max_depth=2, max_NL_iterations=1, output_dir=str(tmp_path))
    assert ei.value.result.dpsi_norms[-1] > 1e-1
    # the solver-data file before the solve is written (:181), the checkpoint is not
    assert sorted(os.listdir(tmp_path)) == ["vcPoissonOut.3d_0.hdf5"]
