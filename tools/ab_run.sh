#!/bin/bash
# Runs tools/bench_smoother.py and bench.py for each A/B build named in
# $VARIANTS (gpurun_ab/<name>/libmgic.so; "base" = the in-tree library),
# ROUNDS times interleaved.  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
N=${N:-512}
ROUNDS=${ROUNDS:-2}
out=gpurun_out/ab.jsonl
timeout -k 10 120 python tools/bench_smoother.py --n $N --sweeps 8 --no-fused >> $out || exit $?
for r in $(seq $ROUNDS); do
  for v in ${VARIANTS}; do
    lib=gpurun_ab/$v/libmgic.so; [ "$v" = base ] && lib=mg_ic_code_amd/libmgic.so
    MGIC_LIB_PATH=$lib timeout -k 10 120 python tools/bench_smoother.py --n $N --sweeps 8 --tag "$v" >> $out || exit $?
    if [ -z "${NO_BENCH:-}" ]; then
      MGIC_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic > gpurun_out/ab_bench.tmp || exit $?
      python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_bench.tmp').read().strip().splitlines()[-1]); print(json.dumps({'variant':'$v','vcycles':d['value'],'ms':d['ms_per_step'],'launch_ms':d['roofline']['avg_launch_ms']}))" >> $out
    fi
  done
done
cat $out
