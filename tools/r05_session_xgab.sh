#!/bin/bash
# round-5 GPU session xgab: the whole-split share proxy with the previous
# restriction defaults (MGIC_RESTRICT_ZL=2 MGIC_RESTRICT_XCD=0) against HEAD
# (4-plane chunks, bands of 16), two interleaved rounds.  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/xgab
o=gpurun_out/xgab/proxy.txt; : > $o
for r in 1 2; do
  for v in "2 0" "4 16"; do
    set -- $v
    MGIC_RESTRICT_ZL=$1 MGIC_RESTRICT_XCD=$2 timeout -k 10 200 python3 tools/rank_proxy.py --size 512 --parts 2,2,2 --periodic 0,0,0 --agglomerate-below 65 --deep 1 --transport ipc --steps 20 > gpurun_out/xgab/p.tmp 2>> gpurun_out/xgab/err.log || { tail gpurun_out/xgab/err.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/xgab/p.tmp').read().strip().splitlines()[-1]); print('zl$1x$2', d['ms_per_vcycle'], d['share_small_charge_ms_per_vcycle'], d['share_ms_per_vcycle'])" >> $o
  done
done
cat $o
echo "session done"
