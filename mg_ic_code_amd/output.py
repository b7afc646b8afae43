"""HDF5 output in the reference's layouts, through
libmgic_io.so (include/mgic_io.h).

    output_final_data   WriteOutput.H:127-227 (the GRChombo checkpoint,
                        set_output_data's 31 variables, SetLevelData.cpp:343-396)
    output_solver_data  WriteOutput.H:52-123 (the per-NL-iteration file:
                        dpsi, rhs and the 8 multigrid_vars)

The per-box components are computed on the GPU (k_output_vars) and streamed
into the file in z-slabs; there is no host fallback.  The multigrid_vars
A_ij_0 and phi_0 are not stored fields here: set_initial_conditions sets them
analytically and nothing changes them, so the kernels evaluate them in place.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import numpy as np

from ._lib import call, io_call
from .core import BH_KEYS, LevelData

GRCHOMBO_VARS = (  # GRChomboUserVariables.hpp:58-75
    "chi", "h11", "h12", "h13", "h22", "h23", "h33", "K", "A11", "A12", "A13", "A22", "A23",
    "A33", "Theta", "Gamma1", "Gamma2", "Gamma3", "lapse", "shift1", "shift2", "shift3", "B1",
    "B2", "B3", "phi", "Pi", "Ham", "Mom1", "Mom2", "Mom3")
SOLVER_VARS = ("dpsi", "rhs", "psi", "A11_0", "A12_0", "A13_0", "A22_0", "A23_0", "A33_0",
               "phi_0")  # WriteOutput.H:74-80 + MultigridUserVariables.hpp:29-33


def _bh(bh: dict):
    return (ctypes.c_double * 13)(*[float(bh[k]) for k in BH_KEYS])


def _handles(fields: Sequence[LevelData]):
    return (ctypes.c_void_p * len(fields))(*[f.handle for f in fields])


def _enc(filename: Optional[str]):
    return filename.encode() if filename is not None else None


def output_final_data(psi: Sequence[LevelData], bh: dict, max_level: int = 0,
                      ref_ratio: Optional[Sequence[int]] = None,
                      filename: Optional[str] = None) -> None:
    """output_final_data (WriteOutput.H:127-227); constant_K = bh['constant_K'].
    filename None: "vcPoissonFinal.3d.hdf5" in the working directory."""
    n = len(psi)
    rr = list(ref_ratio) if ref_ratio is not None else [2] * n
    io_call("mgic_io_write_final_data", _enc(filename), n, _handles(psi), _bh(bh), int(max_level),
            (ctypes.c_int * n)(*rr))


def output_solver_data(dpsi: Sequence[LevelData], rhs: Sequence[LevelData],
                       psi: Sequence[LevelData], bh: dict, iteration: int,
                       ref_ratio: Optional[Sequence[int]] = None,
                       filename: Optional[str] = None) -> None:
    """output_solver_data (WriteOutput.H:52-123) for NL iteration `iteration`.
    filename None: "vcPoissonOut.3d_<iteration>.hdf5"."""
    n = len(psi)
    rr = list(ref_ratio) if ref_ratio is not None else [2] * n
    io_call("mgic_io_write_solver_data", _enc(filename), n, _handles(dpsi), _handles(rhs),
            _handles(psi), _bh(bh), (ctypes.c_int * n)(*rr), int(iteration))


def grchombo_vars(psi: LevelData, n: int, bh: dict, k0: int = 0, nk: Optional[int] = None,
                  out_device_ptr: Optional[int] = None) -> Optional[np.ndarray]:
    """set_output_data for local box n, planes [k0, k0+nk): (31, nk, ny, nx) on
    the host, or written to device memory at out_device_ptr (returns None)."""
    return _vars(0, psi, None, None, n, bh, k0, nk, out_device_ptr)


def solver_vars(dpsi: LevelData, rhs: LevelData, psi: LevelData, n: int, bh: dict, k0: int = 0,
                nk: Optional[int] = None, out_device_ptr: Optional[int] = None):
    """output_solver_data's 10 components for local box n: (10, nk, ny, nx)."""
    return _vars(1, psi, dpsi, rhs, n, bh, k0, nk, out_device_ptr)


def _vars(kind, psi, dpsi, rhs, n, bh, k0, nk, dev):
    lo, hi = psi.grid.local_box(n)[:3], psi.grid.local_box(n)[3:]
    nx, ny, nz = (hi[d] - lo[d] + 1 for d in range(3))
    nk = nz - k0 if nk is None else nk
    nc = 31 if kind == 0 else 10
    if dev is not None:
        ptr, out = ctypes.c_void_p(dev), None
    else:
        out = np.empty((nc, nk, ny, nx))
        ptr = out.ctypes.data_as(ctypes.c_void_p)
    if kind == 0:
        call("mgic_field_grchombo_vars", psi.handle, n, k0, nk, _bh(bh), ptr, int(dev is not None))
    else:
        call("mgic_field_solver_vars", dpsi.handle, rhs.handle, psi.handle, n, k0, nk, _bh(bh), ptr,
             int(dev is not None))
    return out


def write_host(filename: str, kind: int, levels, ref_ratio: Sequence[int], max_level: int = 0,
               iteration: int = 0) -> None:
    """Either layout from host arrays.  levels: [(domain lohi6, dx, [(box lohi6,
    data (ncomp, nz, ny, nx)), ...]), ...] in layout order."""
    nbox, boxes, domains, dxs, chunks = [], [], [], [], []
    nc = 31 if kind == 0 else 10
    for dom, dx, bl in levels:
        nbox.append(len(bl))
        domains += list(dom)
        dxs.append(float(dx))
        for b, data in bl:
            boxes += list(b)
            shape = (nc, b[5] - b[2] + 1, b[4] - b[1] + 1, b[3] - b[0] + 1)
            a = np.ascontiguousarray(data, dtype=np.float64)
            if kind in (0, 1) and a.shape != shape:
                raise ValueError(f"box {b}: data shape {a.shape} != {shape}")
            chunks.append(a.ravel())
    data = np.concatenate(chunks) if chunks else np.zeros(1)
    nl = len(levels)
    io_call("mgic_io_write_host", filename.encode(), int(kind), nl, (ctypes.c_int * nl)(*nbox),
            (ctypes.c_int * max(1, len(boxes)))(*boxes), (ctypes.c_int * (6 * nl))(*domains),
            (ctypes.c_double * nl)(*dxs), (ctypes.c_int * nl)(*list(ref_ratio)),
            data.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), int(max_level), int(iteration))
