#!/bin/bash
# round-4 GPU session sc: machine scheduler strategies for the sweep kernels
# (gpurun_ab/<name> from tools/ab_build.sh with -Xarch_device -mllvm=-amdgpu-sched-strategy=
# max-ilp (ilp), max-memory-clause (mc), iterative-minreg (mr)): parity subset on each, then the
# interleaved A/B against the in-tree library
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ilp mc mr; do
  MGIC_LIB_PATH=gpurun_ab/$v/libmgic.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -rf -k "two_sweep or vcycle or fused" --timeout 200 --timeout-method thread > gpurun_out/pytest_$v.log 2>&1; rc=$?
  echo "$v: $(tail -1 gpurun_out/pytest_$v.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/pytest_$v.log; exit $rc; }
done
: > gpurun_out/ab.jsonl
VARIANTS="base ilp mc mr" ROUNDS=3 bash tools/ab_run.sh || exit 1
echo "session done"
