#!/bin/bash
# round-4 GPU session s (checkpoint at HEAD, the driver's round-end sequence
# plus evidence): the GPU suite, smoke, the default bench line, a rocprofv3
# kernel trace of the bench, and the 8-GPU share proxy without and with the
# per-iteration norm (three runs each) with its kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 900 python bench.py > gpurun_out/bench.log 2>&1 || { tail gpurun_out/bench.log; exit 1; }
tail -n 1 gpurun_out/bench.log > gpurun_out/bench_line.json
python3 -c "import json; d=json.load(open('gpurun_out/bench_line.json')); print(d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['roofline']['traffic'], d['cpu_baseline']['value'], d['bottom']['ms_per_vcycle'])"
TAG=r04s BSTEPS=5 bash tools/trace_bench.sh > /dev/null || exit 1
: > gpurun_out/proxy_ab.txt
for r in 1 2 3; do
  for nt in -1 0; do
    echo -n "norm_type $nt " >> gpurun_out/proxy_ab.txt
    timeout -k 10 180 python3 tools/rank_proxy.py --transport ipc --deep 1 --steps 30 --norm-type $nt >> gpurun_out/proxy_ab.txt 2> gpurun_out/proxy_err.log || { tail gpurun_out/proxy_err.log; exit 1; }
  done
done
python3 tools/proxy_ab_summary.py gpurun_out/proxy_ab.txt
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/xt" -o p --output-format csv -- python3 "$R/tools/rank_proxy.py" --transport ipc --deep 1 --steps 20 > gpurun_out/xt.log 2>&1 || { tail gpurun_out/xt.log; exit 1; }
f=$(find gpurun_out/xt -name "*kernel_trace.csv" | head -n 1)
python3 tools/trace_summary.py "$f" > gpurun_out/ptrace_s.txt
rm -rf gpurun_out/xt
echo "session done"
