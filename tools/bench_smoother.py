#!/usr/bin/env python3
"""Micro-benchmark of the fine-level smoother: time `relax(nsweeps)` on one
n^3 box (SetBinaryBH inputs) and print one JSON line with per-sweep time,
effective GB/s (48 B/cell/pass credited) and a checksum of the result.
Kernel selection: --kind, MGIC_SWEEPS_PER_LAUNCH (1 or 2), MGIC_FUSED_VARIANT /
MGIC_FUSED2X_VARIANT / MGIC_BLOCK_VARIANT (tile shapes)."""
import argparse
import hashlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--sweeps", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--no-fused", action="store_true")
    ap.add_argument("--tag", default=None)
    ap.add_argument("--kind", type=int, default=1,
                    help="fused_smoother: 1 by size, 2 z-streaming, 3 3D blocks")
    args = ap.parse_args()
    import mg_ic_code_amd as mg
    from mg_ic_code_amd.params import read_params_file
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prm = read_params_file(os.path.join(root, "tests", "golden", "params.txt"))
    n = args.n
    comm = mg.Comm()
    dom = (0, 0, 0, n - 1, n - 1, n - 1)
    grid = mg.Grid(comm, dom, [dom], prm.L / n)
    fa, fb, fr, fu = (mg.LevelData(grid) for _ in range(4))
    bh = prm.bh()
    mg.set_binary_bh_coefs(fa, fr, bh)
    fb.set_val(1.0)
    fu.set_zero()
    op = mg.defineOperatorFactory(grid, fa, fb, mg.OperatorParams(
        alpha=1.0, beta=-1.0, coefficient_average_type=1,
        fused_smoother=0 if args.no_fused else args.kind)).AMRnewOp()
    op.relax(fu, fr, 2)  # warm-up
    comm.synchronize()
    mg.prof_smoother(True, n ** 3)
    t0 = time.perf_counter()
    for _ in range(args.reps):
        op.relax(fu, fr, args.sweeps)
    comm.synchronize()
    wall = time.perf_counter() - t0
    launches, passes, ms = mg.prof_smoother_read()
    mg.prof_smoother(False)
    sweeps = args.reps * args.sweeps
    per_sweep = wall / sweeps * 1e3
    h = hashlib.sha1(fu.download(0).tobytes()).hexdigest()[:16]
    print(json.dumps({"variant": "passes" if args.no_fused else (args.tag or "default"),
                      "n": n, "ms_per_sweep_wall": round(per_sweep, 4),
                      "ms_per_launch_events": round(ms / max(launches, 1), 4),
                      "launches": launches, "passes": passes,
                      "ms_per_sweep_events": round(ms / max(passes, 1) * 2, 4),
                      "eff_GBps": round(96.0 * n ** 3 / (per_sweep * 1e-3) / 1e9, 1),
                      "checksum": h}), flush=True)


if __name__ == "__main__":
    main()
