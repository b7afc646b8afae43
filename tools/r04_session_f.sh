#!/bin/bash
# round-4 GPU session f: the whole GPU suite, smoke and bench at HEAD (the
# driver's round-end sequence), then a rocprofv3 trace of the 8-GPU share
# proxy (what one rank's V-cycle is made of)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 900 python bench.py --steps 20 --warmup 2 > gpurun_out/bench.log 2>&1 || { tail gpurun_out/bench.log; exit 1; }
tail -n 1 gpurun_out/bench.log > gpurun_out/bench_line.json
python3 -c "import json; d=json.load(open('gpurun_out/bench_line.json')); print(d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['cpu_baseline']['value'], d['bottom']['ms_per_vcycle'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/ptrace" -o p --output-format csv -- python3 "$R/tools/rank_proxy.py" --transport ipc --deep 1 --steps 20 > gpurun_out/ptrace.log 2>&1 || { tail gpurun_out/ptrace.log; exit 1; }
f=$(find gpurun_out/ptrace -name "*kernel_trace.csv" | head -n 1)
python3 tools/trace_summary.py "$f" > gpurun_out/ptrace.txt 2>&1
rm -rf gpurun_out/ptrace
head -40 gpurun_out/ptrace.txt
echo "session done"
