#!/bin/bash
# round-4 GPU session um: interior tiles (EM 0) of the two-sweep kernel write
# every lane's value unmasked.  GPU suite on the in-tree library, then an
# interleaved A/B against the previous sweep kernels (gpurun_ab/head, from
# tools/ab_build_rev.sh HEAD head)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
: > gpurun_out/ab.jsonl
VARIANTS="head base" ROUNDS=5 bash tools/ab_run.sh > /dev/null || exit 1
python3 - <<'PY'
import json
r = {}
for l in open('gpurun_out/ab.jsonl'):
    d = json.loads(l)
    k = 'bench' if 'vcycles' in d else 'smoother'
    r.setdefault((d['variant'], k), []).append(d.get('vcycles') or d.get('ms_per_launch_events'))
for k, v in sorted(r.items()):
    print(k, [round(x, 4) for x in v], 'mean', round(sum(v) / len(v), 4))
PY
echo "session done"
