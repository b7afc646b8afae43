#!/bin/bash
# round-4 GPU session rz: the z-streaming restriction (k_restrict over chunks
# of MGIC_RESTRICT_KC coarse planes): GPU suite, then an interleaved A/B of
# the chunk length (kc 1 = one coarse plane per workgroup, the former
# layout) and kernel traces at kc 1 and the default
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
: > gpurun_out/ab_env.jsonl
VARIANTS="kc1:MGIC_RESTRICT_KC=1 base kc4:MGIC_RESTRICT_KC=4 kc16:MGIC_RESTRICT_KC=16" ROUNDS=3 bash tools/ab_env.sh || exit 1
MGIC_RESTRICT_KC=1 TAG=rz1 BSTEPS=5 bash tools/trace_bench.sh > /dev/null || exit 1
TAG=rz8 BSTEPS=5 bash tools/trace_bench.sh > /dev/null || exit 1
grep -E "k_restrict|k_prolong|k_residual" gpurun_out/trace_rz1.txt gpurun_out/trace_rz8.txt
echo "session done"
