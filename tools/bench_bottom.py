#!/usr/bin/env python3
"""The BiCGStab bottom solve on its own: bench.py's 512^3 3-level hierarchy
with bottom_solver = 1, one V-cycle from phi = 0 to fill the 128^3 coarse
residual, then --replays solves of it from e = 0 (a fixed amount of work per
solve; Main_PoissonSolver.cpp:103-117, preCond at
Source/VariableCoeffPoissonOperator.cpp:72-104).  Prints one JSON line:
ms per solve, iterations per solve, ms per iteration.  Under rocprofv3 the
trace's tail is the replayed solves alone.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--levels", type=int, default=3)
    ap.add_argument("--nsmooth", type=int, default=4)
    ap.add_argument("--replays", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3, help="replay rounds (each reported)")
    ap.add_argument("--vcycles", type=int, default=1, help="V-cycles from phi = 0 before replaying")
    a = ap.parse_args()
    import torch

    import bench
    import mg_ic_code_amd as mg
    torch.cuda.set_device(0)
    mg.set_device(0)
    comm = mg.Comm()
    case = bench.build_case(mg, comm, 1, a.size, a.levels, a.nsmooth, bottom_solver=1)
    amg, phi, res, rhs = case["amg"], case["fphi"], case["fres"], case["frhs"]
    amg.init_residual(phi, rhs, res, norm_type=0)
    amg.iterations(phi, rhs, res, a.vcycles, norm_type=0)
    rounds = []
    for _ in range(a.rounds):
        ms, it, r0, n = amg.bottom_replay(a.replays)
        rounds.append({"ms_per_solve": round(ms / n, 4), "iterations": it,
                       "us_per_iteration": round(ms / n / max(1, it) * 1e3, 2)})
    env = {k: v for k, v in os.environ.items() if k.startswith("MGIC_")}
    print(json.dumps({"size": a.size, "levels": a.levels, "replays": a.replays,
                      "coarse_residual_norm": r0, "rounds": rounds, "env": env}), flush=True)


if __name__ == "__main__":
    main()
