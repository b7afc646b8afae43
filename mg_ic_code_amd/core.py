"""Python host layer over libmgic: the reference's operator-plugin API.

Names and argument meaning follow the reference so a Chombo user finds the
same surface:

* :class:`VariableCoeffPoissonOperatorFactory` --
  Source/VariableCoeffPoissonOperatorFactory.H:34-117 (``define``,
  ``MGnewOp``, ``AMRnewOp``, ``refToFiner``, ``m_coefficient_average_type``);
  :func:`defineOperatorFactory` -- Factory.cpp:29-49.
* :class:`VariableCoeffPoissonOperator` --
  Source/VariableCoeffPoissonOperator.H:25-170 (``residualI``, ``preCond``,
  ``applyOpI``, ``applyOpNoBoundary``, ``restrictResidual``,
  ``setAlphaAndBeta``, ``setCoefs``, ``resetLambda``, ``levelGSRB``,
  ``levelJacobi``, ...) plus the inherited [Chombo] AMRPoissonOp/LinearOp
  methods the solvers call (``relax``, ``prolongIncrement``, ``incr``,
  ``dotProduct``, ``norm``, ...).
* :class:`AMRMultiGrid` / :func:`bicgstab` -- the [Chombo] drivers
  (MultiGrid::oneCycle, AMRMultiGrid::solve, BiCGStabSolver::solve).

Errors raise :class:`MgicError` (the reference aborts via MayDay).
Everything runs on the GPU through libmgic.so; nothing here computes.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import MGParams, MgicError, OpParams, call, lib

__all__ = [
    "Comm",
    "Grid",
    "LevelData",
    "OperatorParams",
    "SolverParams",
    "VariableCoeffPoissonOperatorFactory",
    "VariableCoeffPoissonOperator",
    "AMRMultiGrid",
    "MultilevelLinearOp",
    "BiCGStabSolver",
    "defineOperatorFactory",
    "bicgstab",
    "set_binary_bh_coefs",
    "set_nl_coefs",
    "prof_smoother",
    "prof_smoother_read",
    "MgicError",
]

Box6 = Tuple[int, int, int, int, int, int]


def _ints(vals: Iterable[int]):
    v = list(vals)
    return (ctypes.c_int * len(v))(*v)


def set_device(dev: int) -> None:
    _lib.check_single_hip_runtime()
    call("mgic_set_device", int(dev))


def device_synchronize() -> None:
    call("mgic_device_synchronize")


# mgic_allgather_fn: int (*)(const void *in, size_t nbytes, void *out, void *user)
_ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                 ctypes.c_void_p)


def gloo_allgather(group=None):
    """A host allgather over an initialised torch.distributed process group
    (the control plane of the peer-mapped transport's one-time setup)."""
    import torch
    import torch.distributed as dist

    def fn(data: bytes) -> List[bytes]:
        t = torch.frombuffer(bytearray(data), dtype=torch.uint8)
        out = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
        dist.all_gather(out, t, group=group)
        return [bytes(o.numpy().tobytes()) for o in out]

    return fn


class Comm:
    """One rank of the job (MPI process in the reference) and the HIP stream
    all work is queued on.  transport:
      "rccl" -- an RCCL communicator (when size > 1 or forced; needs
                `unique_id`, one rank per device);
      "ipc"  -- the peer-mapped transport (csrc/transport.hpp): every rank
                maps the others' receive buffers and signal pages; ranks may
                share a device.  `allgather(bytes) -> [bytes per rank]` is
                the host collective for the one-time setup (default: gloo
                over torch.distributed)."""

    def __init__(self, rank: int = 0, size: int = 1, unique_id: Optional[bytes] = None,
                 force_rccl: bool = False, transport: str = "rccl",
                 allgather=None, arena_bytes: int = 0):
        _lib.check_single_hip_runtime()
        h = ctypes.c_void_p()
        self.rank, self.size = rank, size
        if transport == "ipc":
            if allgather is None and size > 1:
                allgather = gloo_allgather()

            def _cb(inp, nbytes, out, _user):
                try:
                    parts = allgather(ctypes.string_at(inp, nbytes))
                    if len(parts) != size or any(len(x) != nbytes for x in parts):
                        return 1
                    ctypes.memmove(out, b"".join(parts), nbytes * size)
                    return 0
                except Exception:  # noqa: BLE001 -- reported as a status code
                    return 1

            cb = _ALLGATHER_FN(_cb)
            call("mgic_comm_create_ipc", int(rank), int(size), ctypes.cast(cb, ctypes.c_void_p),
                 None, int(arena_bytes), ctypes.byref(h))
            self._h = h
            return
        if transport != "rccl":
            raise ValueError(f"unknown transport {transport!r}")
        uid = None
        if unique_id is not None:
            assert len(unique_id) == 128
            uid = ctypes.c_char_p(bytes(unique_id))
        call("mgic_comm_create", int(rank), int(size), uid, int(bool(force_rccl)), ctypes.byref(h))
        self._h = h

    @property
    def transport(self) -> str:
        t = ctypes.c_int()
        call("mgic_comm_transport", self._h, ctypes.byref(t))
        return {0: "none", 1: "rccl", 2: "ipc"}[t.value]

    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(128)
        call("mgic_comm_unique_id", buf)
        return buf.raw

    @property
    def handle(self):
        return self._h

    def set_stream(self, stream_ptr: int) -> None:
        call("mgic_comm_set_stream", self._h, ctypes.c_void_p(stream_ptr))

    @property
    def stream(self) -> int:
        p = ctypes.c_void_p()
        call("mgic_comm_get_stream", self._h, ctypes.byref(p))
        return p.value or 0

    def set_self_messages(self, on: bool) -> None:
        call("mgic_comm_set_self_messages", self._h, int(bool(on)))

    @property
    def exchanges(self) -> int:
        """Exchanges with messages issued on this communicator so far (a
        measurement counter)."""
        n = ctypes.c_ulonglong()
        call("mgic_comm_exchanges", self._h, ctypes.byref(n))
        return n.value

    @property
    def uses_rccl(self) -> bool:
        u = ctypes.c_int()
        call("mgic_comm_rank", self._h, None, None, ctypes.byref(u))
        return bool(u.value)

    def synchronize(self) -> None:
        call("mgic_comm_synchronize", self._h)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib.mgic_comm_destroy(h)
            self._h = None


class Grid:
    """DisjointBoxLayout + ProblemDomain + dx of one level."""

    def __init__(self, comm: Comm, domain: Box6, boxes: Sequence[Box6], dx: float,
                 periodic: Sequence[int] = (0, 0, 0), owners: Optional[Sequence[int]] = None,
                 _handle=None, patches: bool = False):
        """patches: an AMR level > 0 (disjoint boxes inside the domain, not
        tiling it)"""
        self.comm = comm
        self.domain = tuple(int(v) for v in domain)
        self.boxes = [tuple(int(v) for v in b) for b in boxes]
        self.dx = float(dx)
        self.periodic = tuple(int(p) for p in periodic)
        self.owners = list(owners) if owners is not None else [0] * len(self.boxes)
        if _handle is not None:
            self._h = _handle
        else:
            h = ctypes.c_void_p()
            flat = [v for b in self.boxes for v in b]
            call("mgic_grid_create_patches" if patches else "mgic_grid_create", comm.handle,
                 _ints(self.domain), _ints(self.periodic), ctypes.c_double(self.dx),
                 len(self.boxes), _ints(flat), _ints(self.owners), ctypes.byref(h))
            self._h = h

    @property
    def handle(self):
        return self._h

    @property
    def num_local(self) -> int:
        n = ctypes.c_int()
        call("mgic_grid_num_local", self._h, ctypes.byref(n))
        return n.value

    def local_box(self, n: int) -> Box6:
        lohi = (ctypes.c_int * 6)()
        gi = ctypes.c_int()
        call("mgic_grid_local_box", self._h, int(n), lohi, ctypes.byref(gi))
        return tuple(lohi)

    def coarsen(self, ratio: int) -> "Grid":
        h = ctypes.c_void_p()
        call("mgic_grid_coarsen", self._h, int(ratio), ctypes.byref(h))
        dom = coarsen_box(self.domain, ratio)
        return Grid(self.comm, dom, [coarsen_box(b, ratio) for b in self.boxes],
                    self.dx * ratio, self.periodic, self.owners, _handle=h)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib.mgic_grid_destroy(h)
            self._h = None


def coarsen_box(b: Box6, r: int) -> Box6:
    return tuple(int(np.floor_divide(v, r)) for v in b)


def box_shape(b: Box6, ghost: int = 0) -> Tuple[int, int, int]:
    """numpy shape (nz, ny, nx) of a box (i fastest in memory)."""
    return (b[5] - b[2] + 1 + 2 * ghost, b[4] - b[1] + 1 + 2 * ghost, b[3] - b[0] + 1 + 2 * ghost)


class LevelData:
    """LevelData<FArrayBox>: one fp64 component, one ghost layer, on device."""

    def __init__(self, grid: Grid, _handle=None, _owner=None):
        self.grid = grid
        self._owner = _owner  # keeps a borrowed handle's parent alive
        if _handle is not None:
            self._h = _handle
        else:
            h = ctypes.c_void_p()
            call("mgic_field_create", grid.handle, ctypes.byref(h))
            self._h = h

    @property
    def handle(self):
        return self._h

    def upload(self, n: int, arr: np.ndarray, with_ghosts: bool = False) -> None:
        b = self.grid.local_box(n)
        a = np.ascontiguousarray(arr, dtype=np.float64)
        if a.shape != box_shape(b, 1 if with_ghosts else 0):
            raise ValueError(f"shape {a.shape} != {box_shape(b, 1 if with_ghosts else 0)}")
        call("mgic_field_upload", self._h, int(n), a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
             int(with_ghosts))

    def download(self, n: int = 0, with_ghosts: bool = False) -> np.ndarray:
        b = self.grid.local_box(n)
        out = np.empty(box_shape(b, 1 if with_ghosts else 0), dtype=np.float64)
        call("mgic_field_download", self._h, int(n),
             out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), int(with_ghosts))
        return out

    def device_ptr(self, n: int = 0) -> Tuple[int, Tuple[int, int, int]]:
        p = ctypes.c_void_p()
        s = (ctypes.c_long * 3)()
        call("mgic_field_device_ptr", self._h, int(n), ctypes.byref(p), s)
        return p.value, tuple(s)

    def set_val(self, v: float) -> None:
        call("mgic_field_set_val", self._h, ctypes.c_double(v))

    def set_zero(self) -> None:
        call("mgic_field_set_zero", self._h)

    def set_val_all(self, v: float) -> None:
        """Every cell of the allocation, ghosts included."""
        call("mgic_field_set_val_all", self._h, ctypes.c_double(v))

    def exchange(self) -> None:
        call("mgic_field_exchange", self._h)

    def copy_to(self, dst: "LevelData", with_faces: bool = False) -> None:
        call("mgic_field_copy_to", self._h, dst.handle, int(bool(with_faces)))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib.mgic_field_destroy(h)
            self._h = None


@dataclass
class OperatorParams:
    """Operator constants / BC flags (params.txt: alpha, beta, bc_lo, bc_hi,
    bc_value, coefficient_average_type) plus [Chombo] statics."""

    alpha: float = 0.0
    beta: float = -1.0
    bc_lo: Tuple[int, int, int] = (0, 0, 0)
    bc_hi: Tuple[int, int, int] = (0, 0, 0)
    bc_value: float = 0.0
    coefficient_average_type: int = 0  # 0 arithmetic, 1 harmonic
    prolong_type: int = 1               # 0 piecewise constant, 1 linear
    relax_mode: int = 1                 # 1 GSRB, 4 Jacobi
    fused_smoother: int = 1             # 0 per-colour passes, 1 by size, 2 z-streaming, 3 3D blocks
    deep_halo: int = 0                  # 4-deep ghost shells, two sweeps per exchange: 0 off,
    #                                     1 every level, 2 levels of boxes <= 128^3

    def to_c(self) -> OpParams:
        p = OpParams()
        p.alpha, p.beta = self.alpha, self.beta
        p.bc_lo[:] = list(self.bc_lo)
        p.bc_hi[:] = list(self.bc_hi)
        p.bc_value = self.bc_value
        p.coefficient_average_type = self.coefficient_average_type
        p.prolong_type = self.prolong_type
        p.relax_mode = self.relax_mode
        p.fused_smoother = self.fused_smoother
        p.deep_halo = self.deep_halo
        return p


@dataclass
class SolverParams:
    """MultiGrid / bottom BiCGStab knobs (numMGsmooth, preCondSolverDepth,
    Chombo BiCGStabSolver defaults)."""

    max_depth: int = -1
    n_pre: int = 4
    n_post: int = 4
    n_bottom: int = 4
    bottom_solver: int = 1  # 0 relax, 1 BiCGStab
    cycles: int = 1
    agglomerate_below: int = 0
    bicg_imax: int = 80
    bicg_eps: float = 1.0e-6
    bicg_reps: float = 1.0e-12
    bicg_small: float = 1.0e-30
    bicg_restarts: int = 5
    bicg_norm_type: int = 2

    def to_c(self) -> MGParams:
        p = MGParams()
        for f in MGParams._fields_:
            setattr(p, f[0], getattr(self, f[0]))
        return p


class VariableCoeffPoissonOperator:
    """Handle on a device-side VariableCoeffPoissonOperator."""

    def __init__(self, handle, grid: Grid, owner=None, owned: bool = True):
        self._h = handle
        self.grid = grid
        self._owner = owner
        self._owned = owned

    @property
    def handle(self):
        return self._h

    def _coef(self, which: int) -> LevelData:
        h = ctypes.c_void_p()
        call("mgic_op_coef", self._h, which, ctypes.byref(h))
        return LevelData(self.grid, _handle=h, _owner=self)

    @property
    def m_aCoef(self) -> LevelData:
        return self._coef(0)

    @property
    def m_bCoef(self) -> LevelData:
        return self._coef(1)

    @property
    def m_lambda(self) -> LevelData:
        return self._coef(2)

    def create(self) -> LevelData:
        return LevelData(self.grid)

    # --- VariableCoeffPoissonOperator.H overrides
    def residualI(self, lhs: LevelData, dpsi: LevelData, rhs: LevelData, homogeneous=False):
        call("mgic_op_residual", self._h, lhs.handle, dpsi.handle, rhs.handle, int(bool(homogeneous)))

    residual = residualI

    def preCond(self, correction: LevelData, residual: LevelData):
        call("mgic_op_precond", self._h, correction.handle, residual.handle)

    def applyOpI(self, lhs: LevelData, dpsi: LevelData, homogeneous=False):
        call("mgic_op_apply_op", self._h, lhs.handle, dpsi.handle, int(bool(homogeneous)))

    applyOp = applyOpI

    def applyOpNoBoundary(self, lhs: LevelData, dpsi: LevelData):
        call("mgic_op_apply_op_no_boundary", self._h, lhs.handle, dpsi.handle)

    def restrictResidual(self, resCoarse: LevelData, dpsiFine: LevelData, rhsFine: LevelData):
        call("mgic_op_restrict_residual", self._h, resCoarse.handle, dpsiFine.handle, rhsFine.handle)

    def prolongIncrement(self, phiThisLevel: LevelData, correctCoarse: LevelData):
        call("mgic_op_prolong_increment", self._h, phiThisLevel.handle, correctCoarse.handle)

    def setAlphaAndBeta(self, alpha: float, beta: float):
        call("mgic_op_set_alpha_beta", self._h, ctypes.c_double(alpha), ctypes.c_double(beta))

    def setCoefs(self, aCoef: LevelData, bCoef: LevelData, alpha: float, beta: float):
        call("mgic_op_set_coefs", self._h, aCoef.handle, bCoef.handle, ctypes.c_double(alpha),
             ctypes.c_double(beta))

    def resetLambda(self):
        call("mgic_op_reset_lambda", self._h)

    def computeLambda(self):
        call("mgic_op_reset_lambda", self._h)

    def setTime(self, t: float):
        call("mgic_op_set_time", self._h, ctypes.c_double(t))

    def relax(self, e: LevelData, r: LevelData, iterations: int):
        call("mgic_op_relax", self._h, e.handle, r.handle, int(iterations))

    def levelGSRB(self, dpsi: LevelData, rhs: LevelData):
        call("mgic_op_level_gsrb", self._h, dpsi.handle, rhs.handle)

    def levelJacobi(self, dpsi: LevelData, rhs: LevelData):
        call("mgic_op_level_jacobi", self._h, dpsi.handle, rhs.handle)

    def fillBC(self, u: LevelData, homogeneous: bool = True):
        call("mgic_op_fill_bc", self._h, u.handle, int(bool(homogeneous)))

    def update_psi(self, psi: LevelData, dpsi: LevelData):
        """set_update_psi0 (SetLevelData.cpp:236-256): psi += dpsi incl. ghost layer 1."""
        call("mgic_op_update_psi", self._h, psi.handle, dpsi.handle)

    # --- LinearOp vector interface
    def setToZero(self, x: LevelData):
        call("mgic_op_set_to_zero", self._h, x.handle)

    def assignLocal(self, lhs: LevelData, rhs: LevelData):
        call("mgic_op_assign", self._h, lhs.handle, rhs.handle)

    assign = assignLocal

    def incr(self, lhs: LevelData, x: LevelData, scale: float):
        call("mgic_op_incr", self._h, lhs.handle, x.handle, ctypes.c_double(scale))

    def axby(self, lhs: LevelData, x: LevelData, y: LevelData, a: float, b: float):
        call("mgic_op_axby", self._h, lhs.handle, x.handle, y.handle, ctypes.c_double(a),
             ctypes.c_double(b))

    def scale(self, lhs: LevelData, s: float):
        call("mgic_op_scale", self._h, lhs.handle, ctypes.c_double(s))

    def dotProduct(self, x: LevelData, y: LevelData) -> float:
        out = ctypes.c_double()
        call("mgic_op_dot", self._h, x.handle, y.handle, ctypes.byref(out))
        return out.value

    def norm(self, x: LevelData, ord: int = 2) -> float:
        out = ctypes.c_double()
        call("mgic_op_norm", self._h, x.handle, int(ord), ctypes.byref(out))
        return out.value

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib.mgic_op_destroy(h)  # borrowed handles only drop the wrapper
            self._h = None


class VariableCoeffPoissonOperatorFactory:
    """Handle on a device-side VariableCoeffPoissonOperatorFactory."""

    def __init__(self):
        self._h = None
        self.grid: Optional[Grid] = None
        self.params: Optional[OperatorParams] = None
        self._keep: List[LevelData] = []

    def define(self, grid: Grid, params: OperatorParams, aCoef: LevelData, bCoef: LevelData):
        h = ctypes.c_void_p()
        p = params.to_c()
        call("mgic_factory_define", grid.handle, ctypes.byref(p), aCoef.handle, bCoef.handle,
             ctypes.byref(h))
        self._h, self.grid, self.params = h, grid, params
        self._keep = [aCoef, bCoef]
        return self

    @property
    def handle(self):
        return self._h

    @property
    def m_coefficient_average_type(self) -> int:
        return self.params.coefficient_average_type

    def MGnewOp(self, depth: int, homoOnly: bool = True) -> Optional[VariableCoeffPoissonOperator]:
        h = ctypes.c_void_p()
        rc = call("mgic_factory_mg_new_op", self._h, int(depth), ctypes.byref(h))
        if rc == 1:
            return None
        return VariableCoeffPoissonOperator(h, self.grid.coarsen(1 << depth) if depth else self.grid,
                                            owner=self)

    def AMRnewOp(self) -> VariableCoeffPoissonOperator:
        h = ctypes.c_void_p()
        call("mgic_factory_amr_new_op", self._h, ctypes.byref(h))
        return VariableCoeffPoissonOperator(h, self.grid, owner=self)

    def refToFiner(self) -> int:
        r = ctypes.c_int()
        call("mgic_factory_ref_to_finer", self._h, ctypes.byref(r))
        return r.value

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib.mgic_factory_destroy(h)
            self._h = None


def defineOperatorFactory(grid: Grid, aCoef: LevelData, bCoef: LevelData,
                          params: OperatorParams) -> VariableCoeffPoissonOperatorFactory:
    """defineOperatorFactory (VariableCoeffPoissonOperatorFactory.cpp:29-49)."""
    return VariableCoeffPoissonOperatorFactory().define(grid, params, aCoef, bCoef)


def bicgstab(op: VariableCoeffPoissonOperator, phi: LevelData, rhs: LevelData,
             homogeneous: bool = True, params: Optional[SolverParams] = None) -> int:
    """BiCGStabSolver<LevelData>::solve with `op` (returns iterations)."""
    p = (params or SolverParams()).to_c()
    it = ctypes.c_int()
    call("mgic_op_bicgstab", op.handle, phi.handle, rhs.handle, int(bool(homogeneous)),
         ctypes.byref(p), ctypes.byref(it))
    return it.value


class AMRMultiGrid:
    """AMRMultiGrid on one AMR level with its MultiGrid hierarchy."""

    def __init__(self, factory: VariableCoeffPoissonOperatorFactory,
                 params: Optional[SolverParams] = None):
        self.factory = factory
        self.params = params or SolverParams()
        h = ctypes.c_void_p()
        p = self.params.to_c()
        call("mgic_mg_create", factory.handle, ctypes.byref(p), ctypes.byref(h))
        self._h = h
        n = ctypes.c_int()
        call("mgic_mg_num_depths", h, ctypes.byref(n))
        self.num_depths = n.value

    @property
    def handle(self):
        return self._h

    def op(self, depth: int) -> VariableCoeffPoissonOperator:
        h = ctypes.c_void_p()
        call("mgic_mg_op", self._h, int(depth), ctypes.byref(h))
        g = ctypes.c_void_p()
        call("mgic_op_grid", h, ctypes.byref(g))
        grid = Grid(self.factory.grid.comm, (0,) * 6, [], 1.0, _handle=g)
        return VariableCoeffPoissonOperator(h, grid, owner=self, owned=False)

    def level_field(self, depth: int, which: int) -> LevelData:
        h = ctypes.c_void_p()
        call("mgic_mg_level_field", self._h, int(depth), int(which), ctypes.byref(h))
        g = ctypes.c_void_p()
        op = self.op(depth)
        return LevelData(op.grid, _handle=h, _owner=self)

    def oneCycle(self, e: LevelData, r: LevelData) -> None:
        call("mgic_mg_one_cycle", self._h, e.handle, r.handle)

    def iteration(self, phi: LevelData, rhs: LevelData, resid: LevelData, norm_type: int = 0,
                  homogeneous: bool = False) -> float:
        out = ctypes.c_double()
        call("mgic_mg_iteration", self._h, phi.handle, rhs.handle, resid.handle, int(norm_type),
             int(bool(homogeneous)), ctypes.byref(out))
        return out.value

    def iterations(self, phi: LevelData, rhs: LevelData, resid: LevelData, count: int,
                   norm_type: int = 0, homogeneous: bool = False) -> List[float]:
        """`count` iteration() calls (same phi, resid and norms, bit for bit);
        iteration i's norm is read while iteration i+1's V-cycle runs up to
        its first phi-writing launch (mgic_mg_iterations)."""
        out = (ctypes.c_double * max(1, count))()
        call("mgic_mg_iterations", self._h, phi.handle, rhs.handle, resid.handle, int(count),
             int(norm_type), int(bool(homogeneous)), out)
        return [out[i] for i in range(count)]

    def init_residual(self, phi: LevelData, rhs: LevelData, resid: LevelData, norm_type: int = 0,
                      homogeneous: bool = False) -> float:
        out = ctypes.c_double()
        call("mgic_mg_init_residual", self._h, phi.handle, rhs.handle, resid.handle,
             int(norm_type), int(bool(homogeneous)), ctypes.byref(out))
        return out.value

    def bottom_timer(self, on: bool = True) -> None:
        """Time every BiCGStab bottom solve this rank runs (HIP events)."""
        call("mgic_mg_bottom_timer", self._h, int(bool(on)))

    def bottom_ms(self) -> Tuple[float, int]:
        """(total ms, solves) of the bottom solves timed since bottom_timer(True)."""
        ms, n = ctypes.c_double(), ctypes.c_int()
        call("mgic_mg_bottom_ms", self._h, ctypes.byref(ms), ctypes.byref(n))
        return ms.value, n.value

    def bottom_iters(self) -> Tuple[int, float, float]:
        """(BiCGStab iterations summed over the timed solves, smallest and
        largest norm of the coarse residual they started from)."""
        it, lo, hi = ctypes.c_longlong(), ctypes.c_double(), ctypes.c_double()
        call("mgic_mg_bottom_iters", self._h, ctypes.byref(it), ctypes.byref(lo), ctypes.byref(hi))
        return it.value, lo.value, hi.value

    def bottom_info(self) -> Tuple[bool, int, float]:
        """The last BiCGStab bottom solve: (ran on the device, iterations,
        norm of the residual it started from)."""
        dv, it, r0 = ctypes.c_int(), ctypes.c_int(), ctypes.c_double()
        call("mgic_mg_bottom_info", self._h, ctypes.byref(dv), ctypes.byref(it), ctypes.byref(r0))
        return bool(dv.value), it.value, r0.value

    def bottom_replay(self, n: int) -> Tuple[float, int, float, int]:
        """The last bottom solve again, n times from e = 0 on the same coarse
        residual: (total ms, iterations per solve, residual norm, solves run;
        0 solves on a rank that does not run the coarsest depth)."""
        ms, it, r0, k = ctypes.c_double(), ctypes.c_int(), ctypes.c_double(), ctypes.c_int()
        call("mgic_mg_bottom_replay", self._h, int(n), ctypes.byref(ms), ctypes.byref(it),
             ctypes.byref(r0), ctypes.byref(k))
        return ms.value, it.value, r0.value, k.value

    def fmg(self, phi: LevelData, rhs: LevelData, resid: LevelData, norm_type: int = 0,
            homogeneous: bool = False, ncycles: int = 1) -> float:
        """Full multigrid on the current resid (from init_residual/iteration):
        phi += FMG correction; resid = rhs - L(phi); returns its norm."""
        out = ctypes.c_double()
        call("mgic_mg_fmg", self._h, phi.handle, rhs.handle, resid.handle, int(norm_type),
             int(bool(homogeneous)), int(ncycles), ctypes.byref(out))
        return out.value

    def solve(self, phi: LevelData, rhs: LevelData, resid: LevelData, max_iter: int = 20,
              eps: float = 1e-10, norm_type: int = 0) -> List[float]:
        """AMRMultiGrid::solve: iterate until norm(resid) <= eps*norm(resid0)."""
        hist = [self.init_residual(phi, rhs, resid, norm_type)]
        for _ in range(max_iter):
            if hist[-1] <= eps * hist[0] or hist[-1] == 0.0:
                break
            hist.append(self.iteration(phi, rhs, resid, norm_type))
        return hist

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib.mgic_mg_destroy(h)
            self._h = None


class MixedMultiGrid:
    """Mixed-precision V-cycle (BASELINE config C5): the correction equation
    cycled in fp32 (GSRB / restrictResidual / prolongIncrement in float,
    coefficients rounded from the fp64 hierarchy), the fine residual
    rhs - L(phi) in fp64 rounded once, phi += e in fp64.  Bottom: relax."""

    def __init__(self, factory: VariableCoeffPoissonOperatorFactory,
                 params: Optional[SolverParams] = None):
        self.factory = factory
        self.params = params or SolverParams(bottom_solver=0)
        h = ctypes.c_void_p()
        p = self.params.to_c()
        call("mgic_mixed_create", factory.handle, ctypes.byref(p), ctypes.byref(h))
        self._h = h
        n = ctypes.c_int()
        call("mgic_mixed_num_depths", h, ctypes.byref(n))
        self.num_depths = n.value

    def _run(self, name, phi, rhs, resid, norm_type, *extra):
        out = ctypes.c_double()
        call(name, self._h, phi.handle, rhs.handle, resid.handle if resid is not None else None,
             int(norm_type), *extra, ctypes.byref(out))
        return out.value

    def init_residual(self, phi: LevelData, rhs: LevelData, resid: Optional[LevelData] = None,
                      norm_type: int = 0) -> float:
        return self._run("mgic_mixed_init_residual", phi, rhs, resid, norm_type)

    def iteration(self, phi: LevelData, rhs: LevelData, resid: Optional[LevelData] = None,
                  norm_type: int = 0) -> float:
        return self._run("mgic_mixed_iteration", phi, rhs, resid, norm_type)

    def fmg(self, phi: LevelData, rhs: LevelData, resid: Optional[LevelData] = None,
            norm_type: int = 0, ncycles: int = 1) -> float:
        return self._run("mgic_mixed_fmg", phi, rhs, resid, norm_type, int(ncycles))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib.mgic_mixed_destroy(h)
            self._h = None


class AMRSolver:
    """AMR levels > 0: levels = [(grid, aCoef, bCoef), ...]
    from the coarsest; each finer grid is Grid(..., patches=True) on the
    coarser domain refined by 2, properly nested.  The [Chombo] AMRPoissonOp
    multi-level operators (QuadCFInterp, AMROperator/AMRResidual with reflux a
    no-op, AMRRestrict, AMRProlong, AMRUpdateResidual) and AMRMultiGrid's
    multi-level V-cycle; level 0 is solved by its own MultiGrid (params)."""

    def __init__(self, levels, op_params: OperatorParams, params: Optional[SolverParams] = None):
        self.levels = list(levels)
        n = len(self.levels)
        grids = (ctypes.c_void_p * n)(*[g.handle.value for g, _, _ in self.levels])
        acs = (ctypes.c_void_p * n)(*[a.handle.value for _, a, _ in self.levels])
        bcs = (ctypes.c_void_p * n)(*[b.handle.value for _, _, b in self.levels])
        op = op_params.to_c()
        self.params = params or SolverParams()
        mp = self.params.to_c()
        h = ctypes.c_void_p()
        call("mgic_amr_create", n, grids, acs, bcs, ctypes.byref(op), ctypes.byref(mp),
             ctypes.byref(h))
        self._h = h
        self.num_levels = n

    @property
    def handle(self):
        return self._h

    @staticmethod
    def _f(x):
        return x.handle if x is not None else None

    def cf_interp(self, level: int, u: LevelData, coarse: Optional[LevelData] = None) -> None:
        call("mgic_amr_cf_interp", self._h, int(level), u.handle, self._f(coarse))

    def average_down(self, level: int, coarse: LevelData, fine: LevelData) -> None:
        call("mgic_amr_average_down", self._h, int(level), coarse.handle, fine.handle)

    def AMROperator(self, level, lphi, phi, phi_coarse=None, homogeneous=False) -> None:
        call("mgic_amr_operator", self._h, int(level), lphi.handle, phi.handle,
             self._f(phi_coarse), int(bool(homogeneous)))

    def AMRResidual(self, level, r, phi, phi_coarse, rhs, homogeneous=False) -> None:
        call("mgic_amr_residual", self._h, int(level), r.handle, phi.handle,
             self._f(phi_coarse), rhs.handle, int(bool(homogeneous)))

    def AMRRestrict(self, level, res_coarse, res, corr, corr_coarse=None) -> None:
        call("mgic_amr_restrict", self._h, int(level), res_coarse.handle, res.handle,
             corr.handle, self._f(corr_coarse))

    def AMRProlong(self, level, corr, corr_coarse) -> None:
        call("mgic_amr_prolong", self._h, int(level), corr.handle, corr_coarse.handle)

    def AMRUpdateResidual(self, level, res, corr, corr_coarse=None) -> None:
        call("mgic_amr_update_residual", self._h, int(level), res.handle, corr.handle,
             self._f(corr_coarse))

    def _fields(self, fs):
        assert len(fs) == self.num_levels
        return (ctypes.c_void_p * self.num_levels)(*[f.handle.value for f in fs])

    def init_residual(self, phis, rhss, norm_type: int = 0) -> float:
        out = ctypes.c_double()
        call("mgic_amr_init_residual", self._h, self._fields(phis), self._fields(rhss),
             int(norm_type), ctypes.byref(out))
        return out.value

    def iteration(self, phis, rhss, norm_type: int = 0) -> float:
        out = ctypes.c_double()
        call("mgic_amr_iteration", self._h, self._fields(phis), self._fields(rhss),
             int(norm_type), ctypes.byref(out))
        return out.value

    def residual_field(self, level: int) -> LevelData:
        h = ctypes.c_void_p()
        call("mgic_amr_residual_field", self._h, int(level), ctypes.byref(h))
        return LevelData(self.levels[level][0], _handle=h, _owner=self)

    def level_op(self, level: int) -> VariableCoeffPoissonOperator:
        """the operator of AMR level `level` (level 0: its MultiGrid's depth 0)"""
        h = ctypes.c_void_p()
        call("mgic_amr_level_op", self._h, int(level), ctypes.byref(h))
        return VariableCoeffPoissonOperator(h, self.levels[level][0], owner=self, owned=False)

    # MultilevelLinearOp over the hierarchy (one LevelData per level)
    def applyOp(self, lhs, x, homogeneous: bool = True) -> None:
        call("mgic_amr_apply_op", self._h, self._fields(lhs), self._fields(x),
             int(bool(homogeneous)))

    def dotProduct(self, x, y) -> float:
        out = ctypes.c_double()
        call("mgic_amr_dot", self._h, self._fields(x), self._fields(y), ctypes.byref(out))
        return out.value

    def norm(self, x, ord: int = 0) -> float:
        out = ctypes.c_double()
        call("mgic_amr_norm", self._h, self._fields(x), int(ord), ctypes.byref(out))
        return out.value

    def computeNorm(self, x, ord: int = 2) -> float:
        """computeNorm (Main_PoissonSolver.cpp:208-209): covered cells masked,
        levels weighted by dx^3"""
        out = ctypes.c_double()
        call("mgic_amr_composite_norm", self._h, self._fields(x), int(ord), ctypes.byref(out))
        return out.value

    def computeSum(self, x) -> float:
        """computeSum (Main_PoissonSolver.cpp:144-145): covered cells masked,
        levels weighted by dx^3"""
        out = ctypes.c_double()
        call("mgic_amr_composite_sum", self._h, self._fields(x), ctypes.byref(out))
        return out.value

    def precondition(self, e, r, iters: int = 1) -> None:
        call("mgic_amr_precondition", self._h, self._fields(e), self._fields(r), int(iters))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib.mgic_amr_destroy(h)
            self._h = None


class MultilevelLinearOp:
    """MultilevelLinearOp<FArrayBox> (Main_PoissonSolver.cpp:103-117,169-170): the
    operator plus the MG preconditioner of `num_mg_iterations` AMRMultiGrid iterations
    (pre = post = bottom = the SolverParams smoothing counts).  Over an AMRMultiGrid
    (one AMR level: vectors are LevelData) or an AMRSolver (max_level > 0: vectors
    are one LevelData per level, AMR V-cycles as the preconditioner)."""

    def __init__(self, amg, num_mg_iterations: int = 1):
        self.amg = amg
        self.num_mg_iterations = int(num_mg_iterations)
        self.multilevel = isinstance(amg, AMRSolver)

    def preCond(self, e, r) -> None:
        if self.multilevel:
            self.amg.precondition(e, r, self.num_mg_iterations)
        else:
            call("mgic_mg_precondition", self.amg.handle, e.handle, r.handle,
                 self.num_mg_iterations)


class BiCGStabSolver:
    """BiCGStabSolver<Vector<LevelData*>> over a MultilevelLinearOp
    (Main_PoissonSolver.cpp:104,172-184): m_normType, m_eps = tolerance,
    m_imax = max_iterations, inhomogeneous BC."""

    def __init__(self, mlop: MultilevelLinearOp, tolerance: float = 1.0e-7,
                 max_iterations: int = 10, norm_type: int = 0):
        self.mlop = mlop
        self.m_eps = tolerance
        self.m_imax = max_iterations
        self.m_normType = norm_type
        self.iterations = 0
        self.final_norm = None

    def solve(self, phi, rhs) -> int:
        p = _lib.SolveParams()
        lib.mgic_solve_params_default(ctypes.byref(p))
        p.num_mg_iterations = self.mlop.num_mg_iterations
        p.max_iterations = int(self.m_imax)
        p.tolerance = float(self.m_eps)
        p.norm_type = int(self.m_normType)
        it = ctypes.c_int()
        nrm = ctypes.c_double()
        if self.mlop.multilevel:  # phi, rhs: one LevelData per AMR level
            a = self.mlop.amg
            call("mgic_amr_solve", a.handle, a._fields(phi), a._fields(rhs), ctypes.byref(p),
                 ctypes.byref(it), ctypes.byref(nrm))
        else:
            call("mgic_mg_solve", self.mlop.amg.handle, phi.handle, rhs.handle, ctypes.byref(p),
                 ctypes.byref(it), ctypes.byref(nrm))
        self.iterations, self.final_norm = it.value, nrm.value
        return it.value


BH_KEYS = ("domain_length", "G_Newton", "phi_amplitude", "phi_wavelength", "bh1_bare_mass",
           "bh2_bare_mass", "bh1_spin", "bh2_spin", "bh1_offset", "bh2_offset", "bh1_momentum",
           "bh2_momentum", "constant_K")


def set_nl_coefs(psi: Optional[LevelData], acoef: LevelData, rhs: LevelData, bh: dict) -> None:
    """set_a_coef + set_rhs (SetLevelData.cpp:73-127, :281-325) at conformal factor psi
    (None: psi = 1) on device."""
    vals = (ctypes.c_double * 13)(*[float(bh[k]) for k in BH_KEYS])
    call("mgic_field_nl_coefs", psi.handle if psi is not None else None, acoef.handle, rhs.handle,
         vals)


def set_binary_bh_coefs(acoef: LevelData, rhs: LevelData, bh: dict) -> None:
    """set_a_coef + set_rhs at psi = 1 (SetLevelData.cpp:73-127, :281-325) on device."""
    vals = (ctypes.c_double * 13)(*[float(bh[k]) for k in BH_KEYS])
    call("mgic_field_binary_bh", acoef.handle, rhs.handle, vals)


def prof_smoother(enable: bool, min_cells: int = 0, per_relax: bool = False) -> None:
    """HIP events around the fine-level smoother launches: one pair per launch,
    or (per_relax) one pair per run of consecutive launches in a relax call
    (fewer event records in the timed stream; time / launches = the average)."""
    call("mgic_prof_smoother", (2 if per_relax else 1) if enable else 0, int(min_cells))


def prof_smoother_read() -> Tuple[int, int, float]:
    """(launches, colour passes, total ms) since prof_smoother(True)."""
    n = ctypes.c_int()
    np_ = ctypes.c_long()
    t = ctypes.c_double()
    call("mgic_prof_smoother_read", ctypes.byref(n), ctypes.byref(np_), ctypes.byref(t))
    return n.value, np_.value, t.value
