"""CPU tests of the drop-in boundary and host logic (no GPU needed).

* libmgic.so loads and exports every symbol include/*.h declares, and the
  ctypes binding covers exactly that set;
* failures come back as status codes + mgic_last_error (no aborts);
* the params.txt reader reproduces getPoissonParameters;
* the box decomposition tiles the domain.
"""
import ctypes
import os
import re

import numpy as np
import pytest

import mg_ic_code_amd as mg
from mg_ic_code_amd import _lib
from mg_ic_code_amd.decomposition import (chombo_domain_split, decompose, process_grid,
                                          split_domain)
from mg_ic_code_amd.params import read_params_file

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    names = set()
    for h in ("mgic.h", "mgic_chf.h"):
        txt = open(os.path.join(ROOT, "include", h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        names |= set(re.findall(r"MGIC_API\s+[\w\s\*]+?\b(mgic_\w+)\s*\(", txt))
        names |= set(re.findall(r"\bvoid\s+(\w+_)\s*\(", txt))
    return names


def test_every_declared_symbol_is_exported():
    names = declared_symbols()
    assert len(names) >= 70
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in sorted(names) if not hasattr(lib, n)]
    assert not missing, missing
    assert {"gsrbhelmholtzvc3d_", "vccomputeop3d_", "vccomputeres3d_", "restrictresvc3d_"} <= names


def test_binding_covers_header():
    assert declared_symbols() == set(_lib.SIGNATURES)


def test_errors_are_status_codes_not_aborts():
    h = ctypes.c_void_p()
    rc = _lib.lib.mgic_grid_create(None, None, None, 1.0, 1, None, None, ctypes.byref(h))
    assert rc == -1
    assert "null argument" in _lib.last_error()
    with pytest.raises(mg.MgicError):
        _lib.call("mgic_grid_create", None, None, None, 1.0, 1, None, None, ctypes.byref(h))


def test_default_params_match_reference_defaults():
    p = _lib.OpParams()
    _lib.lib.mgic_op_params_default(ctypes.byref(p))
    # VariableCoeffPoissonOperatorFactory::setDefaultValues (Factory.cpp:317-322)
    assert (p.alpha, p.beta, p.coefficient_average_type) == (0.0, -1.0, 0)
    q = _lib.MGParams()
    _lib.lib.mgic_mg_params_default(ctypes.byref(q))
    assert (q.n_pre, q.n_post, q.bottom_solver) == (4, 4, 1)  # numMGsmooth default 4 (Main:111)


def test_params_reader_matches_getPoissonParameters():
    p = read_params_file(os.path.join(ROOT, "tests", "golden", "params.txt"))
    assert (p.alpha, p.beta) == (1.0, -1.0)
    assert p.N == [64, 64, 64] and p.L == 100.0
    assert p.coarsestDx == 100.0 / 64 and p.domainLength == [100.0] * 3
    assert p.coefficient_average_type == 1  # harmonic (params.txt:43)
    assert p.numMGsmooth == 4 and p.numMGIterations == 2
    assert p.tolerance == 1e-10 and p.max_iterations == 100 and p.max_NL_iterations == 6
    assert p.bc_lo == [0, 0, 0] and p.bc_hi == [0, 0, 0] and p.bc_value == 0.0
    assert p.bh1_offset == 10.0 and p.bh2_momentum == -0.05
    assert p.max_grid_size == 16 and p.block_factor == 8


def test_process_grid_and_decomposition():
    assert process_grid(1) == (1, 1, 1)
    assert process_grid(2) == (1, 1, 2)
    assert process_grid(4) == (1, 2, 2)
    assert process_grid(8) == (2, 2, 2)
    for nr in (1, 2, 4, 8):
        dom, boxes, owners = decompose((512, 512, 512), nr)
        assert len(boxes) == nr and sorted(owners) == list(range(nr))
        cells = sum((b[3] - b[0] + 1) * (b[4] - b[1] + 1) * (b[5] - b[2] + 1) for b in boxes)
        assert cells == 512 ** 3
    dom, boxes, owners = decompose((64, 64, 64), 2, boxes_per_rank=(2, 2, 2))
    assert len(boxes) == 16 and owners.count(0) == 8 and owners.count(1) == 8


def test_chombo_domain_split_params_layout():
    # params.txt: 64^3, max_grid_size 16, block_factor 8 -> 64 boxes of 16^3
    boxes = chombo_domain_split((0, 0, 0, 63, 63, 63), 16, 8)
    assert len(boxes) == 64
    assert all(b[3] - b[0] + 1 == 16 for b in boxes)


def test_split_domain_tiles():
    boxes = split_domain((0, 0, 0, 31, 47, 15), (2, 3, 1))
    occ = np.zeros((16, 48, 32), dtype=int)
    for b in boxes:
        occ[b[2]:b[5] + 1, b[1]:b[4] + 1, b[0]:b[3] + 1] += 1
    assert np.all(occ == 1)
