"""ctypes binding of libmgic.so (the C ABI declared in include/mgic.h).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc,
gfx950).  There is no fallback: if the shared object is missing or fails to
load, importing this module raises, so nothing can silently run on a CPU
path.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_int, c_long, c_size_t, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
# MGIC_LIB_PATH: another build of the library (A/B measurements only)
LIB_PATH = os.environ.get("MGIC_LIB_PATH") or os.path.join(_HERE, "libmgic.so")


class MgicError(RuntimeError):
    """A libmgic call returned a negative status."""

    def __init__(self, func: str, code: int, msg: str):
        super().__init__(f"{func} failed ({code}): {msg}")
        self.code = code


class OpParams(ctypes.Structure):
    """mgic_op_params (include/mgic.h)."""

    _fields_ = [
        ("alpha", c_double),
        ("beta", c_double),
        ("bc_lo", c_int * 3),
        ("bc_hi", c_int * 3),
        ("bc_value", c_double),
        ("coefficient_average_type", c_int),
        ("prolong_type", c_int),
        ("relax_mode", c_int),
        ("fused_smoother", c_int),
        ("deep_halo", c_int),
    ]


class SolveParams(ctypes.Structure):
    """mgic_solve_params (include/mgic.h)."""

    _fields_ = [
        ("num_mg_iterations", c_int),
        ("max_iterations", c_int),
        ("tolerance", c_double),
        ("norm_type", c_int),
    ]


class MGParams(ctypes.Structure):
    """mgic_mg_params (include/mgic.h)."""

    _fields_ = [
        ("max_depth", c_int),
        ("n_pre", c_int),
        ("n_post", c_int),
        ("n_bottom", c_int),
        ("bottom_solver", c_int),
        ("cycles", c_int),
        ("agglomerate_below", c_int),
        ("bicg_imax", c_int),
        ("bicg_eps", c_double),
        ("bicg_reps", c_double),
        ("bicg_small", c_double),
        ("bicg_restarts", c_int),
        ("bicg_norm_type", c_int),
    ]


H = c_void_p  # every opaque handle
PI = POINTER(c_int)
PD = POINTER(c_double)
PH = POINTER(c_void_p)
PLL = POINTER(ctypes.c_longlong)

# name -> argtypes (all return int status unless listed in _RESTYPE)
SIGNATURES = {
    "mgic_version": [],
    "mgic_abi_version": [],
    "mgic_last_error": [],
    "mgic_set_device": [c_int],
    "mgic_get_device_count": [PI],
    "mgic_device_synchronize": [],
    "mgic_op_params_default": [POINTER(OpParams)],
    "mgic_mg_params_default": [POINTER(MGParams)],
    "mgic_comm_unique_id": [ctypes.c_char_p],
    "mgic_comm_create": [c_int, c_int, ctypes.c_char_p, c_int, PH],
    "mgic_comm_create_ipc": [c_int, c_int, c_void_p, c_void_p, ctypes.c_size_t, PH],
    "mgic_comm_transport": [H, PI],
    "mgic_comm_destroy": [H],
    "mgic_comm_set_stream": [H, c_void_p],
    "mgic_comm_get_stream": [H, PH],
    "mgic_comm_set_self_messages": [H, c_int],
    "mgic_comm_exchanges": [H, ctypes.POINTER(ctypes.c_ulonglong)],
    "mgic_comm_synchronize": [H],
    "mgic_comm_rank": [H, PI, PI, PI],
    "mgic_grid_create": [H, PI, PI, c_double, c_int, PI, PI, PH],
    "mgic_grid_destroy": [H],
    "mgic_grid_num_local": [H, PI],
    "mgic_grid_local_box": [H, c_int, PI, PI],
    "mgic_grid_coarsen": [H, c_int, PH],
    "mgic_field_nl_coefs": [H, H, H, PD],
    "mgic_field_nl_integrand": [H, H, PD],
    "mgic_field_set_val_all": [H, c_double],
    "mgic_op_update_psi": [H, H, H],
    "mgic_plan_create": [c_int, c_int, PI, PI, c_int, PI, PI, c_int, PI, PI, c_int, c_int, PH],
    "mgic_plan_create_shell": [c_int, c_int, PI, PI, c_int, PI, PI, c_int, PH],
    "mgic_plan_check_transport": [H, c_int],
    "mgic_plan_ipc_blocks": [H, PI, PLL],
    "mgic_plan_ipc_blocks_per": [H, ctypes.c_longlong, PI, PLL],
    "mgic_plan_destroy": [H],
    "mgic_plan_sizes": [H, PI, PI, PI, PI],
    "mgic_plan_items": [H, c_int, PLL],
    "mgic_plan_peers": [H, PI, PLL, PLL, PLL, PLL],
    "mgic_plan_geom": [H, c_int, c_int, PLL],
    "mgic_field_create": [H, PH],
    "mgic_field_destroy": [H],
    "mgic_field_device_ptr": [H, c_int, PH, POINTER(c_long)],
    "mgic_field_upload": [H, c_int, PD, c_int],
    "mgic_field_download": [H, c_int, PD, c_int],
    "mgic_field_set_val": [H, c_double],
    "mgic_field_set_zero": [H],
    "mgic_field_exchange": [H],
    "mgic_field_copy_to": [H, H, c_int],
    "mgic_field_binary_bh": [H, H, PD],
    "mgic_factory_define": [H, POINTER(OpParams), H, H, PH],
    "mgic_factory_destroy": [H],
    "mgic_factory_mg_new_op": [H, c_int, PH],
    "mgic_factory_amr_new_op": [H, PH],
    "mgic_factory_ref_to_finer": [H, PI],
    "mgic_op_destroy": [H],
    "mgic_op_grid": [H, PH],
    "mgic_op_coef": [H, c_int, PH],
    "mgic_op_residual": [H, H, H, H, c_int],
    "mgic_op_apply_op": [H, H, H, c_int],
    "mgic_op_apply_op_no_boundary": [H, H, H],
    "mgic_op_precond": [H, H, H],
    "mgic_op_relax": [H, H, H, c_int],
    "mgic_op_level_gsrb": [H, H, H],
    "mgic_op_level_jacobi": [H, H, H],
    "mgic_op_restrict_residual": [H, H, H, H],
    "mgic_op_prolong_increment": [H, H, H],
    "mgic_op_set_alpha_beta": [H, c_double, c_double],
    "mgic_op_set_coefs": [H, H, H, c_double, c_double],
    "mgic_op_reset_lambda": [H],
    "mgic_op_set_time": [H, c_double],
    "mgic_op_fill_bc": [H, H, c_int],
    "mgic_op_set_to_zero": [H, H],
    "mgic_op_assign": [H, H, H],
    "mgic_op_incr": [H, H, H, c_double],
    "mgic_op_axby": [H, H, H, H, c_double, c_double],
    "mgic_op_scale": [H, H, c_double],
    "mgic_op_dot": [H, H, H, PD],
    "mgic_op_norm": [H, H, c_int, PD],
    "mgic_op_bicgstab": [H, H, H, c_int, POINTER(MGParams), PI],
    "mgic_mg_create": [H, POINTER(MGParams), PH],
    "mgic_mg_destroy": [H],
    "mgic_mg_num_depths": [H, PI],
    "mgic_mg_op": [H, c_int, PH],
    "mgic_mg_level_field": [H, c_int, c_int, PH],
    "mgic_mg_one_cycle": [H, H, H],
    "mgic_mg_iteration": [H, H, H, H, c_int, c_int, PD],
    "mgic_mg_iterations": [H, H, H, H, c_int, c_int, c_int, PD],
    "mgic_mg_init_residual": [H, H, H, H, c_int, c_int, PD],
    "mgic_mg_precondition": [H, H, H, c_int],
    "mgic_mg_bottom_timer": [H, c_int],
    "mgic_mg_bottom_ms": [H, PD, PI],
    "mgic_mg_bottom_iters": [H, PLL, PD, PD],
    "mgic_mg_bottom_replay": [H, c_int, PD, PI, PD, PI],
    "mgic_mg_bottom_info": [H, PI, PI, PD],
    "mgic_mg_fmg": [H, H, H, H, c_int, c_int, c_int, PD],
    "mgic_grid_create_patches": [H, PI, PI, c_double, c_int, PI, PI, PH],
    "mgic_amr_create": [c_int, POINTER(H), POINTER(H), POINTER(H), POINTER(OpParams),
                        POINTER(MGParams), PH],
    "mgic_amr_destroy": [H],
    "mgic_amr_num_levels": [H, PI],
    "mgic_amr_level_op": [H, c_int, PH],
    "mgic_amr_cf_interp": [H, c_int, H, H],
    "mgic_amr_average_down": [H, c_int, H, H],
    "mgic_amr_operator": [H, c_int, H, H, H, c_int],
    "mgic_amr_residual": [H, c_int, H, H, H, H, c_int],
    "mgic_amr_restrict": [H, c_int, H, H, H, H],
    "mgic_amr_prolong": [H, c_int, H, H],
    "mgic_amr_update_residual": [H, c_int, H, H, H],
    "mgic_amr_init_residual": [H, POINTER(H), POINTER(H), c_int, PD],
    "mgic_amr_iteration": [H, POINTER(H), POINTER(H), c_int, PD],
    "mgic_amr_residual_field": [H, c_int, PH],
    "mgic_amr_apply_op": [H, POINTER(H), POINTER(H), c_int],
    "mgic_amr_dot": [H, POINTER(H), POINTER(H), PD],
    "mgic_amr_norm": [H, POINTER(H), c_int, PD],
    "mgic_amr_composite_norm": [H, POINTER(H), c_int, PD],
    "mgic_amr_composite_sum": [H, POINTER(H), PD],
    "mgic_amr_precondition": [H, POINTER(H), POINTER(H), c_int],
    "mgic_mixed_create": [H, POINTER(MGParams), PH],
    "mgic_mixed_destroy": [H],
    "mgic_mixed_num_depths": [H, PI],
    "mgic_mixed_init_residual": [H, H, H, H, c_int, PD],
    "mgic_mixed_iteration": [H, H, H, H, c_int, PD],
    "mgic_mixed_fmg": [H, H, H, H, c_int, c_int, PD],
    "mgic_solve_params_default": [POINTER(SolveParams)],
    "mgic_mg_solve": [H, H, H, POINTER(SolveParams), PI, PD],
    "mgic_amr_solve": [H, POINTER(H), POINTER(H), POINTER(SolveParams), PI, PD],
    "mgic_field_grchombo_vars": [H, c_int, c_int, c_int, PD, c_void_p, c_int],
    "mgic_field_solver_vars": [H, H, H, c_int, c_int, c_int, PD, c_void_p, c_int],
    "mgic_field_layout": [H, PI, PI, PD, PI, PI, PI],
    "mgic_field_box": [H, c_int, PI, PI, PI],
    "mgic_field_barrier": [H],
    "mgic_host_alloc": [c_size_t, PH],
    "mgic_host_free": [c_void_p],
    "mgic_prof_smoother": [c_int, c_long],
    "mgic_prof_smoother_read": [PI, POINTER(c_long), PD],
    # ChomboFortran drop-ins (include/mgic_chf.h); argtypes left open
    "gsrbhelmholtzvc3d_": None,
    "vccomputeop3d_": None,
    "vccomputeres3d_": None,
    "restrictresvc3d_": None,
    "getlaplacianpsif_": None,
    "getrhogradphif_": None,
}

_RESTYPE = {
    "mgic_version": c_char_p,
    "mgic_last_error": c_char_p,
    "mgic_op_params_default": None,
    "mgic_mg_params_default": None,
    "mgic_solve_params_default": None,
    "gsrbhelmholtzvc3d_": None,
    "vccomputeop3d_": None,
    "vccomputeres3d_": None,
    "restrictresvc3d_": None,
    "getlaplacianpsif_": None,
    "getrhogradphif_": None,
}


def hip_runtime_images() -> list:
    """The distinct HIP runtime files (libamdhip64*) mapped into this process,
    from /proc/self/maps ([] where that file does not exist)."""
    paths = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                parts = line.split(None, 5)
                if len(parts) == 6:
                    p = parts[5].strip()
                    if os.path.basename(p).startswith("libamdhip64"):
                        paths.add(os.path.realpath(p))
    except OSError:
        return []
    return sorted(paths)


def check_single_hip_runtime() -> None:
    """Fail loudly when this process maps more than one HIP runtime: torch
    bundles its own libamdhip64 under another path, and a process that loads
    libmgic.so (which binds /opt/rocm's by soname) before torch holds both --
    they corrupt each other's heap at exit ("double free or corruption",
    status -6).  Checked at load, and again wherever a Comm or a device is
    set up (torch may be imported after this package)."""
    imgs = hip_runtime_images()
    if len(imgs) > 1:
        raise RuntimeError(
            "two HIP runtimes in one process (" + ", ".join(imgs) + "): import torch before "
            "mg_ic_code_amd (the default preload does this unless MGIC_NO_TORCH_PRELOAD is set)")


def _preload_torch() -> None:
    """Import torch (when installed) before the library, so that libmgic.so
    binds to torch's HIP runtime by soname instead of loading a second one
    (check_single_hip_runtime).  MGIC_NO_TORCH_PRELOAD=1 skips it (a process
    that never imports torch); a torch that is present but broken is not this
    library's failure: any exception is swallowed, and the runtime check
    still guards the process."""
    if os.environ.get("MGIC_NO_TORCH_PRELOAD", "0") not in ("", "0"):
        return
    try:
        import torch  # noqa: F401
    except Exception:  # noqa: BLE001 -- see the docstring
        pass


def _load() -> ctypes.CDLL:
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
        )
    _preload_torch()
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    check_single_hip_runtime()
    for name, argtypes in SIGNATURES.items():
        fn = getattr(lib, name)  # AttributeError = missing export: fail loudly
        if argtypes is not None:
            fn.argtypes = argtypes
        fn.restype = _RESTYPE.get(name, c_int)
    return lib


lib = _load()


# ---- libmgic_io.so (include/mgic_io.h): the HDF5 writers, loaded on first
# use (it links libhdf5); missing or unloadable = an ImportError, no fallback
IO_LIB_PATH = os.path.join(_HERE, "libmgic_io.so")
IO_SIGNATURES = {
    "mgic_io_last_error": [],
    "mgic_io_write_final_data": [c_char_p, c_int, PH, PD, c_int, PI],
    "mgic_io_write_solver_data": [c_char_p, c_int, PH, PH, PH, PD, PI, c_int],
    "mgic_io_write_host": [c_char_p, c_int, c_int, PI, PI, PI, PD, PI, PD, c_int, c_int],
}
_io = None


def io_lib() -> ctypes.CDLL:
    global _io
    if _io is None:
        if not os.path.exists(IO_LIB_PATH):
            raise ImportError(f"{IO_LIB_PATH} not found: build it with __graft_entry__.build()")
        L = ctypes.CDLL(IO_LIB_PATH)
        for name, argtypes in IO_SIGNATURES.items():
            fn = getattr(L, name)
            fn.argtypes = argtypes
            fn.restype = c_char_p if name == "mgic_io_last_error" else c_int
        _io = L
    return _io


def io_call(name: str, *args) -> int:
    L = io_lib()
    st = getattr(L, name)(*args)
    if st < 0:
        msg = L.mgic_io_last_error()
        raise MgicError(name, st, msg.decode() if msg else "")
    return st


def last_error() -> str:
    msg = lib.mgic_last_error()
    return msg.decode() if msg else ""


def check(func: str, status: int) -> int:
    """Raise MgicError on a negative status; pass through 0 / 1."""
    if status < 0:
        raise MgicError(func, status, last_error())
    return status


def call(name: str, *args) -> int:
    return check(name, getattr(lib, name)(*args))
