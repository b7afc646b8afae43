"""CPU oracle for parity tests -- TEST INFRASTRUCTURE ONLY.

A ctypes binding of oracle/liboracle.so (plain C restatement of the
reference path, see mgic_oracle.h).  Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg import this package, and only as the
checker.  Parity status: "parity unpinned" (see mgic_oracle.h header and
DESIGN.md).

Arrays are numpy float64 of shape (nz, ny, nx) (i fastest in memory) over
an explicit box; `Fab(arr, lo)` ties an array to its box's low corner.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_double, c_int
from typing import Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


if not os.path.exists(LIB):
    build()
_lib = ctypes.CDLL(LIB)


class _Fab(ctypes.Structure):
    _fields_ = [("p", POINTER(c_double)), ("lo", c_int * 3), ("hi", c_int * 3)]


class MGParams(ctypes.Structure):
    _fields_ = [
        ("nbox", c_int), ("boxes", POINTER(c_int)), ("domain", c_int * 6),
        ("periodic", c_int * 3), ("bc_lo", c_int * 3), ("bc_hi", c_int * 3),
        ("bc_value", c_double), ("dx", c_double), ("alpha", c_double), ("beta", c_double),
        ("nlevels", c_int), ("max_coarse", c_int), ("avg_type", c_int),
        ("prolong_type", c_int), ("relax_mode", c_int), ("n_pre", c_int), ("n_post", c_int),
        ("n_bottom", c_int), ("bottom_solver", c_int), ("bicg_imax", c_int),
        ("bicg_eps", c_double), ("bicg_reps", c_double), ("bicg_small", c_double),
        ("bicg_restarts", c_int), ("bicg_norm_type", c_int),
    ]


class BHParams(ctypes.Structure):
    _fields_ = [(k, c_double) for k in (
        "L", "G_Newton", "phi_amplitude", "phi_wavelength", "bh1_bare_mass", "bh2_bare_mass",
        "bh1_spin", "bh2_spin", "bh1_offset", "bh2_offset", "bh1_momentum", "bh2_momentum",
        "constant_K")]


PF = POINTER(_Fab)
PI = POINTER(c_int)
_sig = {
    "orc_gsrbhelmholtzvc3d": [PF, PF, PI, PI, c_double, c_double, PF, c_double, PF, PF, c_int],
    "orc_vccomputeop3d": [PF, PF, c_double, PF, c_double, PF, PI, PI, c_double],
    "orc_vccomputeres3d": [PF, PF, PF, c_double, PF, c_double, PF, PI, PI, c_double],
    "orc_restrictresvc3d": [PF, PF, PF, c_double, PF, c_double, PF, PI, PI, c_double],
    "orc_lambda": [PF, PF, PI, PI, c_double, c_double, c_double],
    "orc_average": [PF, PF, PI, PI, c_int, c_int],
    "orc_prolong": [PF, PF, PI, PI, PI, PI, PI, PI, c_int],
    "orc_mg_create": [POINTER(MGParams)],
    "orc_mg_destroy": [ctypes.c_void_p],
    "orc_mg_nlevels": [ctypes.c_void_p],
    "orc_mg_box": [ctypes.c_void_p, c_int, c_int, PI],
    "orc_mg_dx": [ctypes.c_void_p, c_int],
    "orc_mg_set": [ctypes.c_void_p, c_int, c_int, c_int, POINTER(c_double)],
    "orc_mg_get": [ctypes.c_void_p, c_int, c_int, c_int, POINTER(c_double)],
    "orc_mg_set_full": [ctypes.c_void_p, c_int, c_int, c_int, POINTER(c_double)],
    "orc_mg_get_full": [ctypes.c_void_p, c_int, c_int, c_int, POINTER(c_double)],
    "orc_mg_setup": [ctypes.c_void_p],
    "orc_mg_exchange": [ctypes.c_void_p, c_int, c_int],
    "orc_mg_fill_bc": [ctypes.c_void_p, c_int, c_int, c_int],
    "orc_mg_level_gsrb": [ctypes.c_void_p, c_int, c_int, c_int],
    "orc_mg_level_jacobi": [ctypes.c_void_p, c_int, c_int, c_int],
    "orc_mg_relax": [ctypes.c_void_p, c_int, c_int, c_int, c_int],
    "orc_mg_residual": [ctypes.c_void_p, c_int, c_int, c_int, c_int, c_int],
    "orc_mg_apply_op": [ctypes.c_void_p, c_int, c_int, c_int, c_int],
    "orc_mg_restrict_residual": [ctypes.c_void_p, c_int, c_int, c_int],
    "orc_mg_prolong_increment": [ctypes.c_void_p, c_int, c_int],
    "orc_mg_precond": [ctypes.c_void_p, c_int, c_int, c_int],
    "orc_mg_one_cycle": [ctypes.c_void_p, c_int],
    "orc_mg_iteration": [ctypes.c_void_p, c_int],
    "orc_mg_fmg": [ctypes.c_void_p, c_int, c_int],
    "orc_mg_init_residual": [ctypes.c_void_p, c_int],
    "orc_mg_bicgstab": [ctypes.c_void_p, c_int, c_int, c_int, c_int],
    "orc_mg_amr_precond": [ctypes.c_void_p, c_int, c_int, c_int],
    "orc_mg_solve": [ctypes.c_void_p, c_int, c_int, c_double, c_int, POINTER(c_double)],
    "orc_mg_norm": [ctypes.c_void_p, c_int, c_int, c_int],
    "orc_mg_dot": [ctypes.c_void_p, c_int, c_int, c_int],
    "orc_mg_last_bicg_iters": [ctypes.c_void_p],
    "orc_binary_bh_coefs": [POINTER(BHParams), PI, PI, c_double, POINTER(c_double), POINTER(c_double)],
    "orc_nl_coefs": [POINTER(BHParams), PI, PI, c_double, POINTER(c_double), POINTER(c_double),
                     POINTER(c_double)],
    "orc_nl_integrand": [POINTER(BHParams), PI, PI, c_double, POINTER(c_double),
                         POINTER(c_double)],
    "orc_getlaplacianpsif": [POINTER(c_double), POINTER(c_double), PI, PI, c_double, c_int],
    "orc_output_vars": [c_int, POINTER(BHParams), PI, PI, c_double, POINTER(c_double),
                        POINTER(c_double), POINTER(c_double), POINTER(c_double)],
    "orc_set_threads": [c_int],
    "orc_get_threads": [],
    "orc_pin_threads": [PI, c_int, c_int],
}
_res = {"orc_mg_create": ctypes.c_void_p, "orc_mg_dx": c_double, "orc_mg_iteration": c_double, "orc_mg_fmg": c_double,
        "orc_mg_init_residual": c_double, "orc_mg_norm": c_double, "orc_mg_dot": c_double}
for _n, _a in _sig.items():
    _f = getattr(_lib, _n)
    _f.argtypes = _a
    _f.restype = _res.get(_n, c_int if _n in ("orc_mg_nlevels", "orc_mg_bicgstab",
                                               "orc_mg_last_bicg_iters", "orc_get_threads",
                                               "orc_pin_threads")
                          else None)
_lib.orc_mg_solve.restype = c_int

# field ids (mgic_oracle.h)
PHI, RHS, ACOEF, BCOEF, LAMBDA, RESID, CORR, TMP = range(8)


def _i3(v: Sequence[int]):
    return (c_int * 3)(*[int(x) for x in v])


def _dp(a: np.ndarray):
    return a.ctypes.data_as(POINTER(c_double))


class Fab:
    """numpy array (nz, ny, nx) over the box whose low corner is `lo`."""

    def __init__(self, arr: np.ndarray, lo: Sequence[int]):
        assert arr.dtype == np.float64 and arr.flags.c_contiguous and arr.ndim == 3
        self.arr = arr
        self.lo = tuple(int(x) for x in lo)
        nz, ny, nx = arr.shape
        self.hi = (self.lo[0] + nx - 1, self.lo[1] + ny - 1, self.lo[2] + nz - 1)
        self._c = _Fab(_dp(arr), _i3(self.lo), _i3(self.hi))

    @property
    def c(self):
        return ctypes.byref(self._c)


def gsrb(u: Fab, rhs: Fab, rlo, rhi, dx, alpha, a: Fab, beta, b: Fab, lam: Fab, red_black: int):
    _lib.orc_gsrbhelmholtzvc3d(u.c, rhs.c, _i3(rlo), _i3(rhi), dx, alpha, a.c, beta, b.c, lam.c,
                               int(red_black))


def apply_op(lof: Fab, u: Fab, alpha, a: Fab, beta, b: Fab, rlo, rhi, dx):
    _lib.orc_vccomputeop3d(lof.c, u.c, alpha, a.c, beta, b.c, _i3(rlo), _i3(rhi), dx)


def residual(res: Fab, u: Fab, rhs: Fab, alpha, a: Fab, beta, b: Fab, rlo, rhi, dx):
    _lib.orc_vccomputeres3d(res.c, u.c, rhs.c, alpha, a.c, beta, b.c, _i3(rlo), _i3(rhi), dx)


def restrict_residual(res: Fab, u: Fab, rhs: Fab, alpha, a: Fab, beta, b: Fab, rlo, rhi, dx):
    _lib.orc_restrictresvc3d(res.c, u.c, rhs.c, alpha, a.c, beta, b.c, _i3(rlo), _i3(rhi), dx)


def lam(out: Fab, a: Fab, rlo, rhi, alpha, beta, dx):
    _lib.orc_lambda(out.c, a.c, _i3(rlo), _i3(rhi), alpha, beta, dx)


def average(coarse: Fab, fine: Fab, crlo, crhi, ratio: int, harmonic: int):
    _lib.orc_average(coarse.c, fine.c, _i3(crlo), _i3(crhi), int(ratio), int(harmonic))


def prolong(fine: Fab, coarse: Fab, frlo, frhi, cvlo, cvhi, avail_lo, avail_hi, ptype: int):
    _lib.orc_prolong(fine.c, coarse.c, _i3(frlo), _i3(frhi), _i3(cvlo), _i3(cvhi), _i3(avail_lo),
                     _i3(avail_hi), int(ptype))


def _bh_params(bh: dict) -> BHParams:
    return BHParams(L=bh["domain_length"], G_Newton=bh["G_Newton"],
                    phi_amplitude=bh["phi_amplitude"], phi_wavelength=bh["phi_wavelength"],
                    bh1_bare_mass=bh["bh1_bare_mass"], bh2_bare_mass=bh["bh2_bare_mass"],
                    bh1_spin=bh["bh1_spin"], bh2_spin=bh["bh2_spin"], bh1_offset=bh["bh1_offset"],
                    bh2_offset=bh["bh2_offset"], bh1_momentum=bh["bh1_momentum"],
                    bh2_momentum=bh["bh2_momentum"], constant_K=bh["constant_K"])


def binary_bh(bh: dict, lo, hi, dx):
    """aCoef, rhs at psi = 1 over [lo, hi] (arrays (nz, ny, nx))."""
    return nl_coefs(bh, lo, hi, dx, None)


def nl_coefs(bh: dict, lo, hi, dx, psi=None):
    """set_a_coef / set_rhs at psi given over [lo-1, hi+1] (None: psi = 1)."""
    p = _bh_params(bh)
    shape = (hi[2] - lo[2] + 1, hi[1] - lo[1] + 1, hi[0] - lo[0] + 1)
    a = np.empty(shape)
    r = np.empty(shape)
    if psi is None:
        _lib.orc_binary_bh_coefs(ctypes.byref(p), _i3(lo), _i3(hi), dx, _dp(a), _dp(r))
    else:
        g = np.ascontiguousarray(psi, dtype=np.float64)
        assert g.shape == tuple(n + 2 for n in shape)
        _lib.orc_nl_coefs(ctypes.byref(p), _i3(lo), _i3(hi), dx, _dp(g), _dp(a), _dp(r))
    return a, r


def nl_integrand(bh: dict, lo, hi, dx, psi):
    """set_constant_K_integrand at psi over [lo-1, hi+1]."""
    p = _bh_params(bh)
    g = np.ascontiguousarray(psi, dtype=np.float64)
    out = np.empty((hi[2] - lo[2] + 1, hi[1] - lo[1] + 1, hi[0] - lo[0] + 1))
    assert g.shape == tuple(n + 2 for n in out.shape)
    _lib.orc_nl_integrand(ctypes.byref(p), _i3(lo), _i3(hi), dx, _dp(g), _dp(out))
    return out


def output_vars(kind: int, bh: dict, lo, hi, dx, psi, dpsi=None, rhs=None):
    """WriteOutput.H's components over [lo, hi]: kind 0 the 31 GRChombo
    variables of set_output_data, kind 1 output_solver_data's 10; arrays
    (nz, ny, nx), result (ncomp, nz, ny, nx)."""
    p = _bh_params(bh)
    shape = (hi[2] - lo[2] + 1, hi[1] - lo[1] + 1, hi[0] - lo[0] + 1)
    f = lambda a: np.ascontiguousarray(a if a is not None else np.zeros(shape), dtype=np.float64)
    u, d, r = f(psi), f(dpsi), f(rhs)
    assert u.shape == d.shape == r.shape == shape
    out = np.empty((31 if kind == 0 else 10,) + shape)
    _lib.orc_output_vars(int(kind), ctypes.byref(p), _i3(lo), _i3(hi), float(dx), _dp(u), _dp(d),
                         _dp(r), _dp(out))
    return out


def getlaplacianpsif(psi_g, lo, hi, dx):
    """GETLAPLACIANPSIF over [lo, hi]; psi_g over the box grown by one."""
    return _fd(psi_g, lo, hi, dx, 1)


def getrhogradphif(phi_g, lo, hi, dx):
    """GETRHOGRADPHIF over [lo, hi]; phi_g over the box grown by one."""
    return _fd(phi_g, lo, hi, dx, 0)


def _fd(g, lo, hi, dx, lap):
    g = np.ascontiguousarray(g, dtype=np.float64)
    out = np.empty((hi[2] - lo[2] + 1, hi[1] - lo[1] + 1, hi[0] - lo[0] + 1))
    assert g.shape == tuple(n + 2 for n in out.shape)
    _lib.orc_getlaplacianpsif(_dp(out), _dp(g), _i3(lo), _i3(hi), float(dx), int(lap))
    return out


def set_threads(n: int) -> None:
    _lib.orc_set_threads(int(n))


def get_threads() -> int:
    return _lib.orc_get_threads()


def pin_threads(cpus, pin: bool = True) -> int:
    """Pin OpenMP thread t to cpus[t] (pin) or release every thread to the
    set `cpus` (the process's own CPUs); returns the threads set."""
    arr = (c_int * max(1, len(cpus)))(*cpus)
    return _lib.orc_pin_threads(arr, len(cpus), int(bool(pin)))


class OracleMG:
    """Multi-box level hierarchy + MultiGrid/AMRMultiGrid/BiCGStab restated."""

    def __init__(self, boxes, domain, dx, alpha=1.0, beta=-1.0, periodic=(0, 0, 0),
                 bc_lo=(0, 0, 0), bc_hi=(0, 0, 0), bc_value=0.0, nlevels=-1, avg_type=0,
                 prolong_type=1, relax_mode=1, n_pre=4, n_post=4, n_bottom=4, bottom_solver=1,
                 bicg_imax=80, bicg_eps=1e-6, bicg_reps=1e-12, bicg_small=1e-30,
                 bicg_restarts=5, bicg_norm_type=2, max_coarse=2):
        flat = [int(v) for b in boxes for v in b]
        self._boxes = (c_int * len(flat))(*flat)
        p = MGParams()
        p.nbox = len(boxes)
        p.boxes = ctypes.cast(self._boxes, PI)
        p.domain[:] = [int(v) for v in domain]
        p.periodic[:] = list(periodic)
        p.bc_lo[:] = list(bc_lo)
        p.bc_hi[:] = list(bc_hi)
        p.bc_value = bc_value
        p.dx, p.alpha, p.beta = dx, alpha, beta
        p.nlevels, p.max_coarse, p.avg_type = nlevels, max_coarse, avg_type
        p.prolong_type, p.relax_mode = prolong_type, relax_mode
        p.n_pre, p.n_post, p.n_bottom, p.bottom_solver = n_pre, n_post, n_bottom, bottom_solver
        p.bicg_imax, p.bicg_eps, p.bicg_reps, p.bicg_small = bicg_imax, bicg_eps, bicg_reps, bicg_small
        p.bicg_restarts, p.bicg_norm_type = bicg_restarts, bicg_norm_type
        self._p = p
        h = _lib.orc_mg_create(ctypes.byref(p))
        if not h:
            raise ValueError("orc_mg_create failed (boxes not coarsenable?)")
        self._h = ctypes.c_void_p(h)
        self.nbox = len(boxes)
        self.nlevels = _lib.orc_mg_nlevels(self._h)

    def box(self, level: int, b: int):
        lohi = (c_int * 6)()
        _lib.orc_mg_box(self._h, level, b, lohi)
        return tuple(lohi)

    def dx(self, level: int) -> float:
        return _lib.orc_mg_dx(self._h, level)

    def shape(self, level: int, b: int, ghost: int = 0):
        x = self.box(level, b)
        return (x[5] - x[2] + 1 + 2 * ghost, x[4] - x[1] + 1 + 2 * ghost, x[3] - x[0] + 1 + 2 * ghost)

    def set(self, level, field, b, arr, full=False):
        a = np.ascontiguousarray(arr, dtype=np.float64)
        assert a.shape == self.shape(level, b, 1 if full else 0)
        (_lib.orc_mg_set_full if full else _lib.orc_mg_set)(self._h, level, field, b, _dp(a))

    def get(self, level, field, b, full=False):
        out = np.empty(self.shape(level, b, 1 if full else 0))
        (_lib.orc_mg_get_full if full else _lib.orc_mg_get)(self._h, level, field, b, _dp(out))
        return out

    def setup(self):
        _lib.orc_mg_setup(self._h)

    def exchange(self, level, field):
        _lib.orc_mg_exchange(self._h, level, field)

    def fill_bc(self, level, field, homogeneous=1):
        _lib.orc_mg_fill_bc(self._h, level, field, int(homogeneous))

    def level_gsrb(self, level, fu, frhs):
        _lib.orc_mg_level_gsrb(self._h, level, fu, frhs)

    def level_jacobi(self, level, fu, frhs):
        _lib.orc_mg_level_jacobi(self._h, level, fu, frhs)

    def relax(self, level, fu, frhs, n):
        _lib.orc_mg_relax(self._h, level, fu, frhs, int(n))

    def residual(self, level, fr, fu, frhs, homogeneous=0):
        _lib.orc_mg_residual(self._h, level, fr, fu, frhs, int(homogeneous))

    def apply_op(self, level, flu, fu, homogeneous=0):
        _lib.orc_mg_apply_op(self._h, level, flu, fu, int(homogeneous))

    def restrict_residual(self, level, fu, frhs):
        _lib.orc_mg_restrict_residual(self._h, level, fu, frhs)

    def prolong_increment(self, level, fu):
        _lib.orc_mg_prolong_increment(self._h, level, fu)

    def precond(self, level, fe, fr):
        _lib.orc_mg_precond(self._h, level, fe, fr)

    def one_cycle(self, level=0):
        _lib.orc_mg_one_cycle(self._h, level)

    def iteration(self, norm_type=0) -> float:
        return _lib.orc_mg_iteration(self._h, int(norm_type))

    def fmg(self, ncycles=1, norm_type=0) -> float:
        return _lib.orc_mg_fmg(self._h, int(ncycles), int(norm_type))

    def init_residual(self, norm_type=0) -> float:
        return _lib.orc_mg_init_residual(self._h, int(norm_type))

    def bicgstab(self, level, fe, fr, homogeneous=1) -> int:
        return _lib.orc_mg_bicgstab(self._h, level, fe, fr, int(homogeneous))

    def amr_precond(self, fe, fr, iters):
        _lib.orc_mg_amr_precond(self._h, fe, fr, int(iters))

    def solve(self, mg_iters=1, imax=10, eps=1e-7, norm_type=0):
        """Outer MG-preconditioned BiCGStab on level-0 PHI/RHS: (iterations, final norm)."""
        out = c_double()
        it = _lib.orc_mg_solve(self._h, int(mg_iters), int(imax), float(eps), int(norm_type),
                               ctypes.byref(out))
        return it, out.value

    def norm(self, level, field, norm_type=2) -> float:
        return _lib.orc_mg_norm(self._h, level, field, int(norm_type))

    def dot(self, level, fx, fy) -> float:
        return _lib.orc_mg_dot(self._h, level, fx, fy)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            _lib.orc_mg_destroy(h)
            self._h = None
