#!/bin/bash
# round-5 last GPU check at HEAD: the GPU suite, smoke and the default bench
# line.  Measurement only; each step bounded.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/last
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 400 --timeout-method thread > gpurun_out/last/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/last/pytest_gpu.log; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; tail -40 gpurun_out/last/pytest_gpu.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/last/smoke.log 2>&1 || { cat gpurun_out/last/smoke.log; exit 1; }
cat gpurun_out/last/smoke.log
timeout -k 10 900 python bench.py > gpurun_out/last/bench.log 2>&1 || { tail gpurun_out/last/bench.log; exit 1; }
tail -n 1 gpurun_out/last/bench.log > gpurun_out/last/bench_line.json
python3 -c "import json; d=json.load(open('gpurun_out/last/bench_line.json')); print(d['value'], d['steps'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['cpu_baseline']['value'])"
echo "session done"
