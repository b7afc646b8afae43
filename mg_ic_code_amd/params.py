"""params.txt reader: the ParmParse keys the reference reads for this path.

Mirrors getPoissonParameters (Source/PoissonParameters.cpp:26-131) and the
solver knobs of Main_PoissonSolver.cpp:107-126, with the same defaults and
the same derived values (coarsestDx = L / N[0], domainLength = coarsestDx *
N, refRatio forced to 2, one periodicity flag for all directions).
"""
from __future__ import annotations

import shlex
from dataclasses import dataclass, field
from typing import Dict, List, Optional


def parse_parmparse(text: str) -> Dict[str, List[str]]:
    """Parse ``key = v1 v2 ...`` lines; '#' starts a comment (ParmParse)."""
    out: Dict[str, List[str]] = {}
    for raw in text.splitlines():
        line = raw.split("#", 1)[0].strip()
        if not line or "=" not in line:
            continue
        key, val = line.split("=", 1)
        out[key.strip()] = shlex.split(val.strip())
    return out


@dataclass
class PoissonParameters:
    alpha: float = 1.0
    beta: float = -1.0
    N: List[int] = field(default_factory=lambda: [64, 64, 64])
    L: float = 100.0
    max_level: int = 0
    coarsestDx: float = 100.0 / 64
    domainLength: List[float] = field(default_factory=lambda: [100.0] * 3)
    is_periodic: int = 0
    bc_lo: List[int] = field(default_factory=lambda: [0, 0, 0])
    bc_hi: List[int] = field(default_factory=lambda: [0, 0, 0])
    bc_value: float = 0.0
    coefficient_average_type: int = -1  # -1: factory default (arithmetic)
    numMGsmooth: int = 4
    numMGIterations: int = 1
    preCondSolverDepth: int = -1
    tolerance: float = 1.0e-7
    max_iterations: int = 10
    max_NL_iterations: int = 4
    max_grid_size: int = 16
    block_factor: int = 8
    verbosity: int = 3
    G_Newton: float = 1.0
    phi_amplitude: float = 0.0
    phi_wavelength: float = 1.0
    bh1_bare_mass: float = 0.0
    bh2_bare_mass: float = 0.0
    bh1_spin: float = 0.0
    bh2_spin: float = 0.0
    bh1_offset: float = 0.0
    bh2_offset: float = 0.0
    bh1_momentum: float = 0.0
    bh2_momentum: float = 0.0

    def bh(self, constant_K: float = 0.0) -> dict:
        """Inputs of set_a_coef / set_rhs (domain length of direction 0)."""
        return dict(domain_length=self.domainLength[0], G_Newton=self.G_Newton,
                    phi_amplitude=self.phi_amplitude, phi_wavelength=self.phi_wavelength,
                    bh1_bare_mass=self.bh1_bare_mass, bh2_bare_mass=self.bh2_bare_mass,
                    bh1_spin=self.bh1_spin, bh2_spin=self.bh2_spin, bh1_offset=self.bh1_offset,
                    bh2_offset=self.bh2_offset, bh1_momentum=self.bh1_momentum,
                    bh2_momentum=self.bh2_momentum, constant_K=constant_K)


def read_params(text: str, overrides: Optional[Dict[str, str]] = None) -> PoissonParameters:
    kv = parse_parmparse(text)
    for k, v in (overrides or {}).items():  # CLI overrides (Main_PoissonSolver.cpp:272)
        kv[k] = shlex.split(str(v))
    p = PoissonParameters()

    def get(key, conv, required=True):
        if key not in kv:
            if required:
                raise KeyError(f"ParmParse::get: key '{key}' not found")
            return None
        return conv(kv[key][0])

    p.alpha = get("alpha", float)
    p.beta = get("beta", float)
    for k in ("G_Newton", "phi_amplitude", "phi_wavelength", "bh1_bare_mass", "bh2_bare_mass",
              "bh1_spin", "bh2_spin", "bh1_offset", "bh2_offset", "bh1_momentum",
              "bh2_momentum"):
        setattr(p, k, get(k, float))
    v = get("verbosity", int, required=False)
    if v is not None:
        p.verbosity = v
    p.max_level = get("max_level", int)
    p.N = [int(x) for x in kv["N"][:3]]
    p.L = get("L", float)
    p.coarsestDx = p.L / p.N[0]                               # PoissonParameters.cpp:82
    p.domainLength = [p.coarsestDx * n for n in p.N]          # :83-85
    p.max_grid_size = get("max_grid_size", int)
    p.block_factor = get("block_factor", int)
    if "coefficient_average_type" in kv:                      # :97-108
        s = kv["coefficient_average_type"][0]
        if s == "arithmetic":
            p.coefficient_average_type = 0
        elif s == "harmonic":
            p.coefficient_average_type = 1
        else:
            raise ValueError("bad coefficient_average_type in input")
    p.is_periodic = get("is_periodic", int)                   # :119-128
    if "bc_lo" in kv:
        p.bc_lo = [int(x) for x in kv["bc_lo"][:3]]
    if "bc_hi" in kv:
        p.bc_hi = [int(x) for x in kv["bc_hi"][:3]]
    bv = get("bc_value", float, required=False)
    if bv is not None:
        p.bc_value = bv
    # solver knobs, Main_PoissonSolver.cpp:107-126 (query with defaults)
    for k, conv in (("numMGIterations", int), ("numMGsmooth", int), ("preCondSolverDepth", int),
                    ("tolerance", float), ("max_iterations", int), ("max_NL_iterations", int)):
        val = get(k, conv, required=False)
        if val is not None:
            setattr(p, k, val)
    return p


def read_params_file(path: str, overrides: Optional[Dict[str, str]] = None) -> PoissonParameters:
    with open(path) as f:
        return read_params(f.read(), overrides)
