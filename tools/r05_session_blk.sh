#!/bin/bash
# round-5 GPU session blk: the 128^3 level on the one-shot block kernel
# (MGIC_BLOCK_MAX_CELLS=2300000, grown 132^3 boxes included) against the
# two-sweep kernel (default 100^3): the whole-split 8-GPU proxy and the 1-GPU
# bench, interleaved.  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/blk
export TMPDIR=/tmp
out=gpurun_out/blk/ab.jsonl; : > $out
for r in 1 2 3; do
  for b in 1000000 2300000; do
    MGIC_BLOCK_MAX_CELLS=$b timeout -k 10 200 python3 tools/rank_proxy.py --size 512 --parts 2,2,2 --periodic 0,0,0 --agglomerate-below 65 --deep 1 --transport ipc --steps 20 > gpurun_out/blk/p.tmp 2> gpurun_out/blk/err.log || { tail gpurun_out/blk/err.log; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/blk/p.tmp')); print(json.dumps({'block_max': $b, 'proxy_ms': d['ms_per_vcycle'], 'share_ms': d['share_ms_per_vcycle'], 'residual': d['final_residual']}))" >> $out
    MGIC_BLOCK_MAX_CELLS=$b timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-bottom > gpurun_out/blk/b.tmp 2> gpurun_out/blk/err.log || { tail gpurun_out/blk/err.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/blk/b.tmp').read().strip().splitlines()[-1]); print(json.dumps({'block_max': $b, 'vcycles': d['value']}))" >> $out
  done
done
cat $out
echo "session done"
