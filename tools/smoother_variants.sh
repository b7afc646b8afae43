#!/bin/bash
# Time smoother configurations: each entry of $VARIANTS is a comma-separated
# list of VAR=value settings, e.g.
#   VARIANTS="MGIC_SWEEPS_PER_LAUNCH=1 MGIC_SWEEPS_PER_LAUNCH=2,MGIC_FUSED2X_VARIANT=1"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
N=${N:-512}
SWEEPS=${SWEEPS:-8}
timeout -k 10 300 python tools/bench_smoother.py --n $N --sweeps $SWEEPS --no-fused || exit $?
for v in ${VARIANTS:-MGIC_SWEEPS_PER_LAUNCH=1 MGIC_SWEEPS_PER_LAUNCH=2}; do
  env ${v//,/ } timeout -k 10 300 python tools/bench_smoother.py --n $N --sweeps $SWEEPS --tag "$v" || exit $?
done
