#!/bin/bash
# round-4 GPU session st: store offsets precomputed per parity (branch st-offsets, gpurun_ab/st) vs main; the slot-interleaved ring with byte-offset LDS
# addressing (branch lds-bytes, built into gpurun_ab/lds) -- the GPU suite on
# that library, then three interleaved rounds of bench_smoother (512^3 /
# 256^3) and bench.py against the in-tree library (main).  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
MGIC_LIB_PATH=gpurun_ab/st/libmgic.so timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -rf --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
out=gpurun_out/st_ab.txt; : > $out
for r in 1 2 3; do
  for v in main st; do
    L=""; [ $v = st ] && L=gpurun_ab/st/libmgic.so
    MGIC_LIB_PATH=$L timeout -k 10 120 python tools/bench_smoother.py --n 512 --sweeps 8 --tag $v >> $out || exit 1
    MGIC_LIB_PATH=$L timeout -k 10 120 python tools/bench_smoother.py --n 256 --sweeps 8 --tag $v >> $out || exit 1
    MGIC_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic --no-bottom > gpurun_out/ab_bench.tmp 2> gpurun_out/ab_err.log || { tail gpurun_out/ab_err.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_bench.tmp').read().strip().splitlines()[-1]); print(json.dumps({'variant':'$v','vcycles':d['value'],'ms':d['ms_per_step'],'launch_ms':d['roofline']['avg_launch_ms'],'frac':d['roofline']['frac']}))" >> $out
  done
done
cat $out
echo "session done"
