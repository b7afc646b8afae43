#!/bin/bash
# round-5 GPU session c5r: the mixed cycle's fp32 restriction in 4-plane
# chunks and XCD bands (MGIC_RESTRICT_F_ZL / MGIC_RESTRICT_F_XCD) against
# its defaults (2 / 0), C5 1024^3 mixed, two interleaved rounds.
# Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/c5r
export TMPDIR=/tmp
for r in 1 2; do
  for v in "2 0" "4 16" "2 16"; do
    set -- $v
    MGIC_RESTRICT_F_ZL=$1 MGIC_RESTRICT_F_XCD=$2 timeout -k 10 400 python tools/bench_c5.py --vcycles 4 --kinds mixed > gpurun_out/c5r/m.log 2>&1 || { tail gpurun_out/c5r/m.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/c5r/m.log').read().strip().splitlines()[-1]); m=d['mixed']; print('zl$1x$2', m['ms_per_vcycle'], m['ms_per_fmg'], d['oracle_check']['bit_identical'])"
  done
done
echo "session done"
