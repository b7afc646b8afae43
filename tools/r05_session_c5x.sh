#!/bin/bash
# round-5 GPU session c5x: C5 (tools/bench_c5.py, 1024^3 mixed and fp64 on
# one GPU) at HEAD, and the mixed cycle with the residual-to-fp32 in the
# dispatch order (MGIC_RESIDUAL_XCD=0) against the XCD bands, two
# interleaved rounds.  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/c5x
export TMPDIR=/tmp
timeout -k 10 600 python tools/bench_c5.py --vcycles 4 > gpurun_out/c5x/c5.log 2>&1 || { tail gpurun_out/c5x/c5.log; exit 1; }
tail -n 1 gpurun_out/c5x/c5.log
for r in 1 2; do
  for v in 0 16; do
    MGIC_RESIDUAL_XCD=$v timeout -k 10 400 python tools/bench_c5.py --vcycles 4 --kinds mixed > gpurun_out/c5x/m$v.log 2>&1 || { tail gpurun_out/c5x/m$v.log; exit 1; }
    echo "xcd=$v $(tail -n 1 gpurun_out/c5x/m$v.log)"
  done
done
echo "session done"
