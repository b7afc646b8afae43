#!/bin/bash
# round-4 GPU session c: FETCH_SIZE calibration for the two-sweep kernel's
# access shapes (tools/fetch_calib.hip), the counter list, and the rocprofv3
# kernel trace of bench.py at HEAD
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/calib
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "lambda_range or two_sweep_relax" --timeout 200 --timeout-method thread > gpurun_out/lam_tests.log 2>&1 || { echo "lambda tests failed"; tail -30 gpurun_out/lam_tests.log; exit 1; }
tail -2 gpurun_out/lam_tests.log
timeout -k 10 60 tools/fetch_calib > gpurun_out/calib/plain.log 2>&1 || { echo "calib failed"; exit 1; }
cat gpurun_out/calib/plain.log
timeout -s KILL 60 rocprofv3 -L > gpurun_out/calib/counters.txt 2>&1 || echo "counter list rc=$?"
grep -i "TCC_EA0_RD\|TCC_EA_RD\|TCC_BUBBLE\|TCC_REQ\|TCC_READ\|MALL\|TCC_EA0_RDREQ" gpurun_out/calib/counters.txt | head -40
for C in "FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_REQ_sum TCC_READ_sum"; do
  n=$(echo $C | tr ' ' '_')
  timeout -s KILL 60 rocprofv3 --pmc $C -d "$R/gpurun_out/calib/$n" -o c --output-format csv -- "$R/tools/fetch_calib" > gpurun_out/calib/$n.log 2>&1 || echo "pmc $C rc=$?"
  f=$(find gpurun_out/calib/$n -name "*counter_collection.csv" | head -n 1)
  [ -n "$f" ] && python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    print('$n', r['Kernel_Name'][:14], r['Counter_Name'], r['Counter_Value'])
"
done
TAG=r04c BSTEPS=5 bash tools/trace_bench.sh || exit $?
echo "session done"
