#!/bin/bash
# round-4 GPU session h: one counter update per workgroup and peer in the
# exchange launch (waits passed once per launch) -- the GPU suite, then the
# 8-GPU share proxy A/B against the previous library (gpurun_ab/prev: one
# counter update and one wait per block) over block sizes, interleaved, and a
# kernel trace of the new default.  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
out=gpurun_out/exch_ab.txt
: > $out
CONFIGS=${CONFIGS:-"prev:4096 new:4096 new:8192 new:2048 new:16384"}
for r in 1 2; do
  for c in $CONFIGS; do
    v=${c%%:*}; be=${c##*:}
    L=""; [ $v = prev ] && L=gpurun_ab/prev/libmgic.so
    echo -n "$v block $be " >> $out
    MGIC_LIB_PATH=$L MGIC_IPC_BLOCK_ELEMS=$be timeout -k 10 180 python3 tools/rank_proxy.py --transport ipc --deep 1 --steps 30 >> $out 2> gpurun_out/xp_err.log || { tail gpurun_out/xp_err.log; exit 1; }
  done
done
for be in 4096 8192; do
  MGIC_IPC_BLOCK_ELEMS=$be timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/xt" -o p --output-format csv -- python3 "$R/tools/rank_proxy.py" --transport ipc --deep 1 --steps 20 > gpurun_out/xt.log 2>&1 || { tail gpurun_out/xt.log; exit 1; }
  f=$(find gpurun_out/xt -name "*kernel_trace.csv" | head -n 1)
  echo "== new block $be" >> $out
  python3 tools/trace_summary.py "$f" | grep "avg=" | grep k_exchange >> $out
  [ $be = 4096 ] && python3 tools/trace_summary.py "$f" > gpurun_out/ptrace_new.txt
  rm -rf gpurun_out/xt
done
cat $out
echo "session done"
