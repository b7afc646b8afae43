#!/bin/bash
# round-5 GPU session frz: the fp32 restriction on LDS-staged fine planes
# (k_restrict_zl<float>, MGIC_RESTRICT_F_ZL = chunk) against k_restrict<float>
# (0): fp64 restriction parity subset (the templated kernel), the fp32 / mixed
# tests, two interleaved rounds of tools/bench_c5.py (mixed, 1024^3).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/frz
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "restrict or vcycle_iterations or full_size_512_vcycle or multibox" --timeout 200 --timeout-method thread > gpurun_out/frz/p64.log 2>&1; rc=$?
echo "fp64: $(tail -1 gpurun_out/frz/p64.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/frz/p64.log; exit $rc; }
MGIC_RESTRICT_F_ZL=2 timeout -k 10 600 python -u -m pytest tests/test_mixed.py tests/test_multiprocess.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/frz/tests.log 2>&1; rc=$?
echo "fp32: $(tail -1 gpurun_out/frz/tests.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/frz/tests.log; exit $rc; }
out=gpurun_out/frz/ab.txt; : > $out
for r in 1 2; do
  for v in 0 2 4; do
    MGIC_RESTRICT_F_ZL=$v timeout -k 10 400 python tools/bench_c5.py --kinds mixed --vcycles 4 > gpurun_out/frz/c5.tmp 2> gpurun_out/frz/err.log || { tail gpurun_out/frz/err.log; exit 1; }
    echo "frz=$v $(tail -n 1 gpurun_out/frz/c5.tmp)" >> $out
  done
done
python3 - $out <<'PY'
import json, sys
for l in open(sys.argv[1]):
    v, j = l.split(" ", 1); d = json.loads(j); m = d["mixed"]
    print(v, "fmg", m["ms_per_fmg"], "vcycle", m["ms_per_vcycle"], "oracle", d.get("oracle_check", {}).get("bit_identical"), "res", m["residual_max_norm"]["after_fmg_plus_4_vcycles"])
PY
echo "session done"
