#!/bin/bash
# round-5 GPU checkpoint at HEAD: the driver's round-end sequence (GPU suite,
# smoke, default bench line) plus the evidence for profiles/: a rocprofv3
# kernel trace of the bench and the SQ counter passes of the two-sweep launch
# (tools/r04_session_pmc_sq.sh).  Measurement only; each step bounded.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 900 python bench.py > gpurun_out/bench.log 2>&1 || { tail gpurun_out/bench.log; exit 1; }
tail -n 1 gpurun_out/bench.log > gpurun_out/bench_line.json
python3 -c "import json; d=json.load(open('gpurun_out/bench_line.json')); print(d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['roofline']['traffic'], d['cpu_baseline']['value'], d['bottom'])"
TAG=r05f BSTEPS=10 bash tools/trace_bench.sh > /dev/null || exit 1
grep -E "k_gsrb_tb2" gpurun_out/trace_r05f.txt | head -8
bash tools/r04_session_pmc_sq.sh > gpurun_out/pmcsq.log 2>&1 || { tail gpurun_out/pmcsq.log; exit 1; }
tail -30 gpurun_out/pmcsq.log
echo "session done"
