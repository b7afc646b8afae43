#!/bin/bash
# round-4 GPU session sdy: the steady-step loop (SDY) for the plain fp64 two-sweep launch
# (gpurun_ab/sdy: SDY = true, which spills 7 VGPRs in the plain kernel; the SQ counters put the
# plain step at ~138 SALU per wave, most of them the range tests and plane clamps SDY compiles out)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in sdy; do
  MGIC_LIB_PATH=gpurun_ab/$v/libmgic.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -rf -k "two_sweep or vcycle or fused" --timeout 200 --timeout-method thread > gpurun_out/pytest_$v.log 2>&1; rc=$?
  echo "$v: $(tail -1 gpurun_out/pytest_$v.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/pytest_$v.log; exit $rc; }
done
: > gpurun_out/ab.jsonl
VARIANTS="head sdy" ROUNDS=4 bash tools/ab_run.sh || exit 1
echo "session done"
