"""Debug helper: V-cycle iterations of the fp64 or mixed fp32 path on one box
against the oracle (bitwise), for a given shape / smoother kind.  Env vars of
the library (MGIC_*) select kernel variants; run one process per variant."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mg_ic_code_amd as mg  # noqa: E402
from oracle.mixed import MixedOracle  # noqa: E402
from tests.test_mixed import _gpu, _oracle, _phi, _problem  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--prec", type=int, default=32)
ap.add_argument("--shape", default="264,72,40")
ap.add_argument("--fused", type=int, default=2)
ap.add_argument("--levels", type=int, default=3)
ap.add_argument("--iters", type=int, default=2)
ap.add_argument("--bvar", action="store_true")
args = ap.parse_args()
shape = tuple(int(v) for v in args.shape.split(","))
rng = np.random.default_rng(11)
lo = (0, -8, 8)
dom = tuple(lo) + tuple(lo[d] + shape[d] - 1 for d in range(3))
dx = 0.21
bc_lo, bc_hi, bcv = (0, 0, 1), (1, 0, 0), 0.5
a, b, rhs = _problem(rng, shape, args.bvar)
S = _gpu(mg.Comm(), dom, [dom], dx, a, b, rhs, args.levels, args.fused, bc_lo, bc_hi, bcv)
o = _oracle(dom, dx, a, b, rhs, args.levels, bc_lo, bc_hi, bcv)
tag = f"prec={args.prec} shape={shape} fused={args.fused} env=" + " ".join(
    f"{k}={v}" for k, v in os.environ.items() if k.startswith("MGIC_"))
if args.prec == 32:
    mm = mg.MixedMultiGrid(S["fac"], S["sp"])
    m = MixedOracle(o, 1.0, -1.0, bc_lo, bc_hi)
    g = [mm.init_residual(S["fphi"], S["frhs"], S["fres"], 0)]
    c = [np.abs(m.init_residual(np.zeros(shape[::-1]))).max()]
    for _ in range(args.iters):
        g.append(mm.iteration(S["fphi"], S["frhs"], S["fres"], 0))
        c.append(np.abs(m.iteration()).max())
    ref = m.phi
else:
    amg = mg.AMRMultiGrid(S["fac"], S["sp"])
    g = [amg.init_residual(S["fphi"], S["frhs"], S["fres"], norm_type=0)]
    o.init_residual(0)
    c = [g[0]]
    for _ in range(args.iters):
        g.append(amg.iteration(S["fphi"], S["frhs"], S["fres"], norm_type=0))
        c.append(o.iteration(0))
    import oracle
    ref = o.get(0, oracle.PHI, 0)
phi = _phi(S)
ok = np.array_equal(phi, ref)
d = np.abs(phi - ref)
idx = np.unravel_index(np.argmax(d), d.shape)
bad = np.argwhere(d > 0)
print(f"{tag}: bitwise={ok} norms gpu={g} cpu={c} maxdiff={d.max():.3e} at (z,y,x)={idx} "
      f"nbad={len(bad)} xs={sorted(set(bad[:, 2].tolist()))[:20]} ys={sorted(set(bad[:, 1].tolist()))[:20]} "
      f"zs={sorted(set(bad[:, 0].tolist()))[:20]}", flush=True)
