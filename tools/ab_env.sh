#!/bin/bash
# A/B of environment settings on the in-tree library (bench.py lines), e.g.
#   VARIANTS="base kc96:MGIC_TB2_KC=96 kc192:MGIC_TB2_KC=192" ROUNDS=2 bash tools/ab_env.sh
# (name:VAR=VAL[,VAR=VAL...]; "base" = no change), ROUNDS interleaved.
# Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-2}
out=gpurun_out/ab_env.jsonl
for r in $(seq $ROUNDS); do
  for spec in ${VARIANTS}; do
    name=${spec%%:*}; envs=""
    [ "$spec" != "$name" ] && envs=${spec#*:} && envs=${envs//,/ }
    env $envs timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic \
      ${BENCH_ARGS:-} > gpurun_out/ab_env.tmp || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_env.tmp').read().strip().splitlines()[-1]); print(json.dumps({'variant':'$name','vcycles':d['value'],'ms':d['ms_per_step'],'launch_ms':d['roofline']['avg_launch_ms']}))" >> $out
  done
done
cat $out
