#!/bin/bash
# round-5 GPU session i: the device-loop BiCGStab (tests, then the bench's
# 'bottom' at 1 rank and in the 8-rank one-GPU rehearsal), then the C5
# teardown bisect.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_multiprocess.py -q -x -rf \
  -k "bicgstab" --timeout 300 --timeout-method thread > gpurun_out/pytest_bicg.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_bicg.log; [ $rc -ne 0 ] && { tail -60 gpurun_out/pytest_bicg.log; exit $rc; }
STEPS_TO_RUN="bench bench8" BSTEPS=20 bash tools/gpu_session.sh > gpurun_out/sess_i.log 2>&1 || { tail -20 gpurun_out/sess_i.log; exit 1; }
for f in bench bench8; do
  python3 -c "import json; d=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['bottom'])"
done
bash tools/r05_c5_teardown.sh
echo "session i done"
