#!/bin/bash
# round-5 GPU session fzl: the mixed cycle's fp64 -> fp32 residual on
# LDS-staged u planes (MGIC_RESIDUAL_F_ZL = chunk) against k_residual_z2:
# the fp32 / mixed tests, then two interleaved rounds of tools/bench_c5.py
# (mixed, 1024^3).  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fzl
export TMPDIR=/tmp
MGIC_RESIDUAL_F_ZL=16 timeout -k 10 600 python -u -m pytest tests/test_mixed.py tests/test_multiprocess.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/fzl/tests.log 2>&1; rc=$?
tail -1 gpurun_out/fzl/tests.log; [ $rc -ne 0 ] && { tail -30 gpurun_out/fzl/tests.log; exit $rc; }
out=gpurun_out/fzl/ab.txt; : > $out
for r in 1 2; do
  for v in 0 16 32; do
    MGIC_RESIDUAL_F_ZL=$v timeout -k 10 400 python tools/bench_c5.py --kinds mixed --vcycles 4 > gpurun_out/fzl/c5.tmp 2> gpurun_out/fzl/err.log || { tail gpurun_out/fzl/err.log; exit 1; }
    echo "fzl=$v $(tail -n 1 gpurun_out/fzl/c5.tmp)" >> $out
  done
done
python3 - $out <<'PY'
import json, sys
for l in open(sys.argv[1]):
    v, j = l.split(" ", 1); d = json.loads(j); m = d["mixed"]
    print(v, "fmg", m["ms_per_fmg"], "vcycle", m["ms_per_vcycle"], "oracle", d.get("oracle_check", {}).get("bit_identical"), "res", m["residual_max_norm"]["after_fmg_plus_4_vcycles"])
PY
echo "session done"
