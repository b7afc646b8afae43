#!/bin/bash
# round-5 GPU session bicg: the BiCGStab bottom with three readbacks per
# iteration (queued second half-step and next <RT, R>) and the preconditioner's
# copy and scale in one launch, against the library before it (gpurun_ab/base0):
# the BiCGStab / preconditioner / solve tests, the multi-process bottom test,
# then three interleaved rounds of bench.py's bottom block (driver settings).
# Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bicg
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -k "bicgstab or precond or solve or nonlinear or nl_loop or amr or bottom" \
  --timeout 300 --timeout-method thread > gpurun_out/bicg/tests.log 2>&1; rc=$?
tail -1 gpurun_out/bicg/tests.log; [ $rc -ne 0 ] && { tail -30 gpurun_out/bicg/tests.log; exit $rc; }
out=gpurun_out/bicg/ab.jsonl; : > $out
for r in 1 2 3; do
  for v in new base0; do
    L=""; [ $v != new ] && L=gpurun_ab/$v/libmgic.so
    MGIC_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > gpurun_out/bicg/b.tmp 2> gpurun_out/bicg/err.log || { tail gpurun_out/bicg/err.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/bicg/b.tmp').read().strip().splitlines()[-1]); b=d['bottom']; print(json.dumps({'variant':'$v','vcycles':d['value'],'bicg_ms_per_vcycle':b['ms_per_vcycle'],'bottom_delta_ms':b['bottom_delta_ms'],'bottom_solve_ms_rank0':b['bottom_solve_ms_rank0'],'hist':b['residual_norm_history']}))" >> $out
  done
done
cat $out
echo "session done"
