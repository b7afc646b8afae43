#!/bin/bash
# Time fused-sweep variants: VARIANTS="v[:zs] ..." (zs -> MGIC_FUSED_ZS)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
N=${N:-512}
timeout -k 10 300 python tools/bench_smoother.py --n $N --no-fused || exit $?
for vz in ${VARIANTS:-0 1 2 3 4}; do
  v=${vz%%:*}; zs=0; [[ $vz == *:* ]] && zs=${vz##*:}
  MGIC_FUSED_VARIANT=$v MGIC_FUSED_ZS=$zs timeout -k 10 300 python tools/bench_smoother.py --n $N --tag "$vz" || exit $?
done
