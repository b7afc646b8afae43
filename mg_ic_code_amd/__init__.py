"""mg_ic_code_amd -- MI355X-native multigrid V-cycle for the
VariableCoeffPoissonOperator hot path of eugenealim/MG_IC_code.

The compute lives in libmgic.so (hand-written HIP kernels for gfx950 behind
the C ABI in include/mgic.h); this package is the host-side mirror of the
reference's operator / factory / solver interface (see core.py).
"""
from .core import (  # noqa: F401
    AMRMultiGrid,
    AMRSolver,
    BiCGStabSolver,
    Comm,
    Grid,
    LevelData,
    MgicError,
    MixedMultiGrid,
    MultilevelLinearOp,
    OperatorParams,
    SolverParams,
    VariableCoeffPoissonOperator,
    VariableCoeffPoissonOperatorFactory,
    bicgstab,
    defineOperatorFactory,
    device_synchronize,
    prof_smoother,
    prof_smoother_read,
    set_binary_bh_coefs,
    set_nl_coefs,
    set_device,
)
from ._lib import IO_LIB_PATH, LIB_PATH, lib  # noqa: F401
from .output import output_final_data, output_solver_data  # noqa: F401

__version__ = "0.1.0"
