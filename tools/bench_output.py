#!/usr/bin/env python3
"""SURVEY §8(f) row 4 measurement: the output kernels and the HDF5 write.

* k_output_vars<0> (set_output_data, 31 components) and <1> (output_solver_data,
  10) on a 512^3 box into device memory, z-slabs of 64 planes (4.2 GB per
  slab for the 31 components): time per launch from events on the library's
  stream (the launches are synchronous to it; wall clock around R repeats
  after a device sync), and algorithmic bytes 256 / 104 B per cell (psi in +
  31 doubles out; dpsi, rhs, psi in + 10 out).
* the whole output_final_data of a 256^3 level to a file under /tmp
  (4.2 GB): wall time, split into device+PCIe and HDF5.

Prints one JSON line.  usage: bench_output.py [--n 512] [--file-n 256] [--reps 5]
"""
import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--file-n", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--slab", type=int, default=64)
    args = ap.parse_args()
    import numpy as np
    import torch

    import mg_ic_code_amd as mg
    from mg_ic_code_amd.output import grchombo_vars, solver_vars
    from mg_ic_code_amd.params import read_params_file
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prm = read_params_file(os.path.join(root, "tests", "golden", "params.txt"))
    bh = prm.bh(constant_K=-0.1)
    comm = mg.Comm()
    out = {"config": f"output kernels on a {args.n}^3 box (slabs of {args.slab} planes); "
                     f"output_final_data of a {args.file_n}^3 level to /tmp",
           "data": "synthetic (psi = 1 + small noise, params.txt BH)"}
    n = args.n
    dom = (0, 0, 0, n - 1, n - 1, n - 1)
    grid = mg.Grid(comm, dom, [dom], prm.domainLength[0] / n)
    psi, dpsi, rhs = mg.LevelData(grid), mg.LevelData(grid), mg.LevelData(grid)
    psi.set_val(1.0)
    dpsi.set_val(0.01)
    rhs.set_val(0.02)
    buf = torch.empty(31 * args.slab * n * n, dtype=torch.float64, device="cuda")
    for kind, nc, bpc in ((0, 31, 256), (1, 10, 104)):
        def launch_all():
            for k0 in range(0, n, args.slab):
                nk = min(args.slab, n - k0)
                if kind == 0:
                    grchombo_vars(psi, 0, bh, k0, nk, out_device_ptr=buf.data_ptr())
                else:
                    solver_vars(dpsi, rhs, psi, 0, bh, k0, nk, out_device_ptr=buf.data_ptr())
        launch_all()
        comm.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            launch_all()
        comm.synchronize()
        dt = (time.perf_counter() - t0) / args.reps
        cells = n ** 3
        out[f"k_output_vars<{kind}>"] = {
            "components": nc, "ms_per_box": round(dt * 1e3, 3),
            "algorithmic_bytes_per_cell": bpc,
            "achieved_GBps": round(bpc * cells / dt / 1e9, 1),
            "frac_of_8TBps": round(bpc * cells / dt / 8e12, 3)}
    del buf
    torch.cuda.empty_cache()
    # the whole write
    m = args.file_n
    domf = (0, 0, 0, m - 1, m - 1, m - 1)
    gf = mg.Grid(comm, domf, [domf], prm.domainLength[0] / m)
    pf = mg.LevelData(gf)
    pf.set_val(1.0)
    with tempfile.TemporaryDirectory(dir="/tmp") as d:
        f = os.path.join(d, "vcPoissonFinal.3d.hdf5")
        t0 = time.perf_counter()
        host = grchombo_vars(pf, 0, bh)  # device kernel + D2H of the whole box
        t_dev = time.perf_counter() - t0
        del host
        t0 = time.perf_counter()
        mg.output_final_data([pf], bh, 0, [2], f)
        t_all = time.perf_counter() - t0
        size = os.path.getsize(f)
    out["output_final_data"] = {"cells": m ** 3, "file_bytes": size, "s_total": round(t_all, 3),
                                "file_GBps": round(size / t_all / 1e9, 3),
                                "s_kernel_plus_d2h_whole_box": round(t_dev, 3)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
