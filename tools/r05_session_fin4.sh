#!/bin/bash
# round-5 GPU session fin4: HEAD (restriction in 4-plane chunks and XCD
# bands): the GPU suite and smoke, the V-cycle against the previous
# restriction defaults (MGIC_RESTRICT_ZL=2 MGIC_RESTRICT_XCD=0) in three
# interleaved rounds, the default bench line and a kernel trace.
# Measurement only; each step bounded.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/f4
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 400 --timeout-method thread > gpurun_out/f4/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/f4/pytest_gpu.log; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; tail -40 gpurun_out/f4/pytest_gpu.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f4/smoke.log 2>&1 || { cat gpurun_out/f4/smoke.log; exit 1; }
cat gpurun_out/f4/smoke.log
o=gpurun_out/f4/ab.txt; : > $o
for r in 1 2 3; do
  for v in "2 0" "4 16"; do
    set -- $v
    MGIC_RESTRICT_ZL=$1 MGIC_RESTRICT_XCD=$2 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-bottom > gpurun_out/f4/b.tmp 2> gpurun_out/f4/err.log || { tail gpurun_out/f4/err.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/f4/b.tmp').read().strip().splitlines()[-1]); print('zl$1x$2', d['value'])" >> $o
  done
done
cat $o
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > gpurun_out/f4/bench.log 2>&1 || { tail gpurun_out/f4/bench.log; exit 1; }
tail -n 1 gpurun_out/f4/bench.log > gpurun_out/f4/bench_line.json
python3 -c "import json; d=json.load(open('gpurun_out/f4/bench_line.json')); print(d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['roofline']['traffic'], d['cpu_baseline']['value'])"
TAG=r05ai BSTEPS=10 bash tools/trace_bench.sh > /dev/null || exit 1
grep -E "k_restrict_zl|k_residual_zl|k_gsrb_tb2" gpurun_out/trace_r05ai.txt | head -8
echo "session done"
