#!/usr/bin/env python3
"""One rank of a multi-process run of the bench workload (bench.build_case)
on a GPU, for tests/test_multiprocess.py: BASELINE config C4's real form --
separate processes, one box per rank, halo exchange through the
peer-mapped transport (csrc/transport.hpp) -- on however many devices the
box has (all ranks may share device 0).

    mp_worker.py --rank R --world W --port P --n N --out DIR [--device D]
                 [--mode vcycle|mixed]
mode vcycle (config C4): init_residual + `iters` AMRMultiGrid iterations of
the fp64 V-cycle, deep halo (--bottom-solver 1: the reference's BiCGStab
bottom, on rank 0 when the coarsest depth is gathered).  mode mixed (config
C5): init_residual, one FMG cycle and `iters` V-cycle iterations of the mixed
fp32 smoother / fp64 residual MultiGrid (fp32 messages), deep halo; both
modes gather the depths --agglomerate-below names onto rank 0.
Writes DIR/rank<R>.npz: this rank's phi boxes, the residual max norms, the
transport used.  gloo (127.0.0.1) is the control
plane; nothing touches the GPU before the process group exists.
"""
import argparse
import datetime
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--levels", type=int, default=3)
    ap.add_argument("--iters", type=int, default=2)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--agglomerate-below", type=int, default=0)
    ap.add_argument("--bottom-solver", type=int, default=0)
    ap.add_argument("--mode", choices=("vcycle", "mixed"), default="vcycle")
    ap.add_argument("--fmg", type=int, default=0,
                    help="vcycle mode: one fp64 FMG cycle (MultiGrid::fmg) before the iterations")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    import bench
    import mg_ic_code_amd as mg
    from mg_ic_code_amd._lib import check_single_hip_runtime

    check_single_hip_runtime()  # one libamdhip64 image (the exit abort of two)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{a.port}", rank=a.rank,
                            world_size=a.world, timeout=datetime.timedelta(seconds=120))
    mg.set_device(a.device)
    comm = mg.Comm(a.rank, a.world, transport="ipc")
    from mg_ic_code_amd.commcheck import check_transport
    checked = check_transport(comm, a.world)  # bench.py's transport check
    mixed = a.mode == "mixed"
    case = bench.build_case(mg, comm, a.world, a.n, a.levels, 4, deep_halo=1,
                            agglomerate_below=a.agglomerate_below, bottom_solver=a.bottom_solver)
    amg, fphi, frhs, fres, grid = (case[k] for k in ("amg", "fphi", "frhs", "fres", "grid"))
    if mixed:
        amg = mg.MixedMultiGrid(case["fac"], mg.SolverParams(
            max_depth=a.levels - 1, n_pre=4, n_post=4, n_bottom=4, bottom_solver=0,
            agglomerate_below=a.agglomerate_below))
        norms = [amg.init_residual(fphi, frhs, fres, 0), amg.fmg(fphi, frhs, fres, 0)]
        norms += [amg.iteration(fphi, frhs, fres, 0) for _ in range(a.iters)]
    else:
        norms = [amg.init_residual(fphi, frhs, fres, norm_type=0)]
        if a.fmg:
            norms.append(amg.fmg(fphi, frhs, fres, norm_type=0))
        norms += [amg.iteration(fphi, frhs, fres, norm_type=0) for _ in range(a.iters)]
    comm.synchronize()
    out = {"norms": np.array(norms), "transport": np.array(comm.transport),
           "checked": np.array(checked)}
    for i in range(grid.num_local):
        out[f"box{i}"] = np.array(grid.local_box(i))
        out[f"phi{i}"] = fphi.download(i)
    np.savez(os.path.join(a.out, f"rank{a.rank}.npz"), **out)
    dist.barrier()
    del amg, case
    dist.destroy_process_group()
    print(json.dumps({"rank": a.rank, "norms": norms}), flush=True)
    del torch


if __name__ == "__main__":
    main()
