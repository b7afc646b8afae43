#!/bin/bash
# round-5 GPU session hb: the default bench line at HEAD, interleaved with
# the residual in the dispatch order (MGIC_RESIDUAL_XCD=0), two rounds.
# Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/hb
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/hb/bench$r.log 2>&1 || { tail gpurun_out/hb/bench$r.log; exit 1; }
  tail -n 1 gpurun_out/hb/bench$r.log > gpurun_out/hb/bench$r.json
  python3 -c "import json; d=json.load(open('gpurun_out/hb/bench$r.json')); print('head', d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
  MGIC_RESIDUAL_XCD=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-bottom > gpurun_out/hb/b0.tmp 2> gpurun_out/hb/err.log || { tail gpurun_out/hb/err.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/hb/b0.tmp').read().strip().splitlines()[-1]); print('xcd0', d['value'])"
done
echo "session done"
