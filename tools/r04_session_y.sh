#!/bin/bash
# round-4 GPU session y: BASELINE config C5 (tools/bench_c5.py: 1024^3
# 4-level FMG + V-cycles, mixed fp32 / fp64, one GPU) with the one-rule,
# direction-split edge tiles against the library before them (gpurun_ab/prev,
# c9334f1), two interleaved rounds, and the share proxy A/B (the 256^3 rank
# box with Dirichlet-free periodic faces has no edge tiles; a 2x2x2-split rank
# box of the real run has three domain faces: --periodic 0,0,0 --parts 1,1,1
# on 256^3 shows the edge path).  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/c5_ab.log
for r in 1 2; do
  for v in prev new; do
    if [ $v = prev ]; then L=gpurun_ab/prev/libmgic.so; else L=""; fi
    echo -n "$v " >> gpurun_out/c5_ab.log
    MGIC_LIB_PATH=$L timeout -k 10 300 python tools/bench_c5.py >> gpurun_out/c5_ab.log 2> gpurun_out/c5_err.log || { echo "bench_c5 $v failed"; tail gpurun_out/c5_err.log; exit 1; }
  done
done
python3 - <<'PY'
import json
for line in open("gpurun_out/c5_ab.log"):
    v, j = line.split(" ", 1)
    d = json.loads(j)
    print(v, d["oracle_check"]["bit_identical"], "mixed", d["mixed"]["ms_per_fmg"], d["mixed"]["ms_per_vcycle"], d["mixed"]["fine_sweep_ms_events"], "fp64", d["fp64"]["ms_per_fmg"], d["fp64"]["ms_per_vcycle"], d["fp64"]["fine_sweep_ms_events"])
PY
echo "session done"
