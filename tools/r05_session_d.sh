#!/bin/bash
# round-5 GPU session d: the in-tree library now issues the two-sweep loads
# spread over the step (TB2_SPREAD 1, the default; gpurun_ab/s0 = all loads
# before the first barrier, round 4's placement); against it: loads one step
# ahead (pf1), the steady step for the plain launch (sdy), both (pf1sdy) --
# the two-sweep parity tests on each variant, three interleaved A/B rounds,
# then C5 (fp32 two-sweep launches) in-tree vs s0.  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="pf1 sdy pf1sdy"
for v in $V; do
  MGIC_LIB_PATH=gpurun_ab/$v/libmgic.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x \
    -k "two_sweep or full_size_512_vcycle or full_size_256 or deep_halo_vcycle or streaming_vcycle or vcycle_iterations" \
    --timeout 200 --timeout-method thread > gpurun_out/pytest_$v.log 2>&1; rc=$?
  echo "$v: $(tail -1 gpurun_out/pytest_$v.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/pytest_$v.log; exit $rc; }
done
out=gpurun_out/r05d_ab.txt; : > $out
for r in 1 2 3; do
  for v in base s0 $V; do
    L=""; [ $v != base ] && L=gpurun_ab/$v/libmgic.so
    MGIC_LIB_PATH=$L timeout -k 10 120 python tools/bench_smoother.py --n 512 --sweeps 8 --tag $v >> $out || exit 1
    MGIC_LIB_PATH=$L timeout -k 10 120 python tools/bench_smoother.py --n 256 --sweeps 8 --tag $v >> $out || exit 1
    MGIC_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic --no-bottom > gpurun_out/ab_bench.tmp 2> gpurun_out/ab_err.log || { tail gpurun_out/ab_err.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_bench.tmp').read().strip().splitlines()[-1]); print(json.dumps({'variant':'$v','vcycles':d['value'],'ms':d['ms_per_step'],'launch_ms':d['roofline']['avg_launch_ms'],'frac':d['roofline']['frac']}))" >> $out
  done
done
cat $out
for r in 1 2; do
  for v in base s0; do
    L=""; [ $v != base ] && L=gpurun_ab/$v/libmgic.so
    echo -n "$v " >> gpurun_out/r05d_c5.txt
    MGIC_LIB_PATH=$L timeout -k 10 300 python tools/bench_c5.py --vcycles 4 >> gpurun_out/r05d_c5.txt 2> gpurun_out/c5_err.log || { tail gpurun_out/c5_err.log; exit 1; }
  done
done
cat gpurun_out/r05d_c5.txt
echo "session done"
