#!/bin/bash
# round-4 GPU session z: the two-sweep ring slot-interleaved with byte-offset LDS addressing (lane offsets + constants in the ds offset field; no scratch) vs prev (element indexing)
# domain face (UBC: one ghost per update, four selects) vs prev (one ghost
# per face) -- the GPU suite, then three interleaved rounds of
# bench_smoother (512^3 two-sweep launches) and bench.py, and a kernel trace
# of the new library's bench.  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -rf --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
out=gpurun_out/lds_ab.txt; : > $out
for r in 1 2 3; do
  for v in prev new; do
    L=""; [ $v = prev ] && L=gpurun_ab/prev/libmgic.so
    MGIC_LIB_PATH=$L timeout -k 10 120 python tools/bench_smoother.py --n 512 --sweeps 8 --tag $v >> $out || exit 1
    MGIC_LIB_PATH=$L timeout -k 10 120 python tools/bench_smoother.py --n 256 --sweeps 8 --tag $v >> $out || exit 1
    MGIC_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic --no-bottom > gpurun_out/ab_bench.tmp 2> gpurun_out/ab_err.log || { tail gpurun_out/ab_err.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_bench.tmp').read().strip().splitlines()[-1]); print(json.dumps({'variant':'$v','vcycles':d['value'],'ms':d['ms_per_step'],'launch_ms':d['roofline']['avg_launch_ms'],'frac':d['roofline']['frac']}))" >> $out
  done
done
cat $out
TAG=lds BSTEPS=5 bash tools/trace_bench.sh > /dev/null || exit 1
grep "avg=" gpurun_out/trace_lds.txt | head -12
bash tools/r04_session_t.sh > /dev/null || exit 1
grep -E "==|k_gsrb_tb2" gpurun_out/edge_cost.txt | head -20
echo "session done"
