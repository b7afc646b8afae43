#!/bin/bash
# round-4 GPU session m: HEAD (per-block exchange flags, cap 2 per CU) -- the
# GPU suite, smoke, the 8-GPU share proxy (three runs) with its kernel trace,
# and the 1-GPU bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -rf --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
: > gpurun_out/proxy_ab.txt
CONFIGS="new:0:0" ROUNDS=3 bash tools/proxy_ab.sh || exit 1
python3 tools/proxy_ab_summary.py gpurun_out/proxy_ab.txt
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/xt" -o p --output-format csv -- python3 "$R/tools/rank_proxy.py" --transport ipc --deep 1 --steps 20 > gpurun_out/xt.log 2>&1 || { tail gpurun_out/xt.log; exit 1; }
f=$(find gpurun_out/xt -name "*kernel_trace.csv" | head -n 1)
python3 tools/trace_summary.py "$f" > gpurun_out/ptrace_m.txt
rm -rf gpurun_out/xt
timeout -k 10 900 python bench.py --steps 20 --warmup 2 > gpurun_out/bench.log 2>&1 || { tail gpurun_out/bench.log; exit 1; }
tail -n 1 gpurun_out/bench.log > gpurun_out/bench_line.json
python3 -c "import json; d=json.load(open('gpurun_out/bench_line.json')); print(d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['cpu_baseline']['value'], d['bottom']['ms_per_vcycle'])"
echo "session done"
