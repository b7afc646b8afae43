#!/bin/bash
# A/B of the fused residual (bench.py lines): the in-tree library with the
# fused launch (bench.py --fused-residual 1) and without it (0), plus the
# measurement builds named in $VARIANTS (gpurun_ab/<name>/libmgic.so),
# ROUNDS times interleaved.  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-2}
out=gpurun_out/ab_fused.jsonl
one() {  # name, then env assignments
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic $FR \
    > gpurun_out/ab_fused.tmp || return $?
  python3 -c "import json; d=json.loads(open('gpurun_out/ab_fused.tmp').read().strip().splitlines()[-1]); print(json.dumps({'variant':'$name','vcycles':d['value'],'ms':d['ms_per_step'],'launch_ms':d['roofline']['avg_launch_ms'],'fused':d['config'].get('residual_fused')}))" >> $out
}
for r in $(seq $ROUNDS); do
  FR="--fused-residual 1"; one fused MGIC_LIB_PATH=mg_ic_code_amd/libmgic.so || exit $?
  FR="--fused-residual 0"; one unfused MGIC_LIB_PATH=mg_ic_code_amd/libmgic.so || exit $?
  for v in ${VARIANTS:-}; do
    FR="--fused-residual 1"; one "$v" MGIC_LIB_PATH=gpurun_ab/$v/libmgic.so || exit $?
  done
done
cat $out
