#!/bin/bash
# round-4 GPU session e: fp32 short reciprocal -- the fp32 / mixed parity
# tests, then bench_c5 (1024^3 4-level, mixed and fp64) A/B against the
# previous library (gpurun_ab/prev: fp32 lambda by division), interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_mixed.py tests/test_gpu_parity.py -m gpu -x -q -k "mixed or fp32 or lambda_range or two_sweep" --timeout 300 --timeout-method thread > gpurun_out/mixed_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/mixed_tests.log; exit 1; }
tail -2 gpurun_out/mixed_tests.log
for r in 1 2; do
  for v in prev new; do
    if [ $v = prev ]; then L=gpurun_ab/prev/libmgic.so; else L=""; fi
    echo -n "$v " >> gpurun_out/c5_ab.log
    MGIC_LIB_PATH=$L timeout -k 10 300 python tools/bench_c5.py >> gpurun_out/c5_ab.log 2> gpurun_out/c5_err.log || { echo "bench_c5 $v failed"; tail gpurun_out/c5_err.log; exit 1; }
  done
done
cat gpurun_out/c5_ab.log
echo "session done"
