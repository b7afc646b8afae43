#!/bin/bash
# round-5: the exit-time heap error of the multi-rank C5 bench (every rank
# aborts with "double free or corruption" after printing its line): 2 ranks,
# 128^3, 3 levels, fp64, one setting changed per run.  Diagnostics only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
port=29620
i=0
for extra in "" "--agglomerate-below 0" "--deep-halo 0" "--no-fmg" "--agglomerate-below 0 --deep-halo 0 --no-fmg"; do
  port=$((port + 1)); i=$((i + 1))
  MGIC_BENCH_DEVICE=0 timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $port tools/bench_c5.py --size 128 --levels 3 --vcycles 2 \
    --kinds fp64 --no-oracle-check $extra > gpurun_out/c5td_$i.log 2>&1
  rc=$?
  echo "[$extra] rc=$rc $(grep -c 'double free' gpurun_out/c5td_$i.log) double-free lines"
done
echo "session done"
