#!/bin/bash
# round-5 GPU session b: delayed stores on top of the spread loads
# (gpurun_ab/s1 = TB2_SPREAD 1; s1d1 / s1d2 / s1d3 / s2d2 = + TB2_DSTORE):
# the two-sweep parity tests on each variant, then three interleaved rounds
# of bench_smoother (512^3 / 256^3) and bench.py against the in-tree library.
# Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${VARIANTS:-s1d1 s1d2 s1d3 s2d2}"
for v in $V; do
  MGIC_LIB_PATH=gpurun_ab/$v/libmgic.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x \
    -k "two_sweep or full_size_512_vcycle or full_size_256 or deep_halo_vcycle or streaming_vcycle or vcycle_iterations" \
    --timeout 200 --timeout-method thread > gpurun_out/pytest_$v.log 2>&1; rc=$?
  echo "$v: $(tail -1 gpurun_out/pytest_$v.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/pytest_$v.log; exit $rc; }
done
out=gpurun_out/r05b_dstore_ab.txt; : > $out
for r in 1 2 3; do
  for v in base s1 $V; do
    L=""; [ $v != base ] && L=gpurun_ab/$v/libmgic.so
    MGIC_LIB_PATH=$L timeout -k 10 120 python tools/bench_smoother.py --n 512 --sweeps 8 --tag $v >> $out || exit 1
    MGIC_LIB_PATH=$L timeout -k 10 120 python tools/bench_smoother.py --n 256 --sweeps 8 --tag $v >> $out || exit 1
    MGIC_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic --no-bottom > gpurun_out/ab_bench.tmp 2> gpurun_out/ab_err.log || { tail gpurun_out/ab_err.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_bench.tmp').read().strip().splitlines()[-1]); print(json.dumps({'variant':'$v','vcycles':d['value'],'ms':d['ms_per_step'],'launch_ms':d['roofline']['avg_launch_ms'],'frac':d['roofline']['frac']}))" >> $out
  done
done
cat $out
echo "session done"
