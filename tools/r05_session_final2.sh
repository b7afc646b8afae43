#!/bin/bash
# round-5 GPU checkpoint 2 at HEAD: the GPU suite, smoke, the default bench
# line (PMC traffic and the CPU baseline), a rocprofv3 kernel trace of the
# bench, the 8-GPU share proxies (the periodic 256^3 box charged, and the
# whole 2x2x2 split on this GPU), and the 1/2/4/8-rank rehearsal with the
# driver's settings.  Measurement only; each step bounded.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/f2
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 400 --timeout-method thread > gpurun_out/f2/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/f2/pytest_gpu.log; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; tail -40 gpurun_out/f2/pytest_gpu.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f2/smoke.log 2>&1 || { cat gpurun_out/f2/smoke.log; exit 1; }
cat gpurun_out/f2/smoke.log
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > gpurun_out/f2/bench.log 2>&1 || { tail gpurun_out/f2/bench.log; exit 1; }
tail -n 1 gpurun_out/f2/bench.log > gpurun_out/f2/bench_line.json
python3 -c "import json; d=json.load(open('gpurun_out/f2/bench_line.json')); print(d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['roofline']['traffic'], d['cpu_baseline']['value'], d['bottom'])"
TAG=${FTAG:-r05k} BSTEPS=10 bash tools/trace_bench.sh > /dev/null || exit 1
grep -E "k_gsrb_tb2" gpurun_out/trace_${FTAG:-r05k}.txt | head -8
: > gpurun_out/f2/proxy.txt
for r in 1 2 3; do
  timeout -k 10 200 python3 tools/rank_proxy.py --transport ipc --deep 1 --steps 30 --charge 1 >> gpurun_out/f2/proxy.txt 2> gpurun_out/f2/proxy_err.log || { tail gpurun_out/f2/proxy_err.log; exit 1; }
  timeout -k 10 200 python3 tools/rank_proxy.py --size 512 --parts 2,2,2 --periodic 0,0,0 --agglomerate-below 65 --deep 1 --transport ipc --steps 20 >> gpurun_out/f2/proxy.txt 2>> gpurun_out/f2/proxy_err.log || { tail gpurun_out/f2/proxy_err.log; exit 1; }
done
cat gpurun_out/f2/proxy.txt
SKIP_PROXY=1 bash tools/r05_session_ranks.sh || exit 1
echo "session done"
