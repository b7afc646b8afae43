#!/bin/bash
# bench.py V-cycles/s under each setting in $SETTINGS (space-separated;
# each a comma-separated VAR=value list), one line per run.  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in ${SETTINGS}; do
  env ${v//,/ } timeout -k 10 150 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline > gpurun_out/sweep.tmp || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/sweep.tmp').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
done
