#!/bin/bash
# round-5 GPU session a: where the two-sweep launch issues its global loads
# (TB2_SPREAD 0 = all before the first barrier, the in-tree library; 1 / 2 / 3
# spread over the colour phases, built into gpurun_ab/s1..s3) -- three
# interleaved rounds of bench_smoother (512^3 / 256^3) and bench.py.
# Measurement only; the checksums must agree bit for bit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r05a_spread_ab.txt; : > $out
for r in 1 2 3; do
  for v in base s1 s2 s3; do
    L=""; [ $v != base ] && L=gpurun_ab/$v/libmgic.so
    MGIC_LIB_PATH=$L timeout -k 10 120 python tools/bench_smoother.py --n 512 --sweeps 8 --tag $v >> $out || exit 1
    MGIC_LIB_PATH=$L timeout -k 10 120 python tools/bench_smoother.py --n 256 --sweeps 8 --tag $v >> $out || exit 1
    MGIC_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic --no-bottom > gpurun_out/ab_bench.tmp 2> gpurun_out/ab_err.log || { tail gpurun_out/ab_err.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_bench.tmp').read().strip().splitlines()[-1]); print(json.dumps({'variant':'$v','vcycles':d['value'],'ms':d['ms_per_step'],'launch_ms':d['roofline']['avg_launch_ms'],'frac':d['roofline']['frac']}))" >> $out
  done
done
cat $out
echo "session done"
