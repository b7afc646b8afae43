#!/bin/bash
# round-5 GPU session rzl: the residual with LDS-staged u planes
# (MGIC_RESIDUAL_ZL=1, z chunk MGIC_RESIDUAL_KC) against k_residual_z2:
# parity subset (fp64 and mixed), three interleaved rounds of bench_kernels
# 512^3 / 256^3 and the V-cycle.  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rzl
export TMPDIR=/tmp
MGIC_RESIDUAL_ZL=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_mixed.py -q -x \
  -k "residual or operator_methods or vcycle or multibox or agglomerat or periodic or mixed or fmg" --timeout 200 --timeout-method thread > gpurun_out/rzl/pytest.log 2>&1; rc=$?
echo "zl: $(tail -1 gpurun_out/rzl/pytest.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/rzl/pytest.log; exit $rc; }
o=gpurun_out/rzl/ab.txt; : > $o
for r in 1 2 3; do
  for v in "0 16" "1 16" "1 8" "1 32"; do
    set -- $v
    MGIC_RESIDUAL_ZL=$1 MGIC_RESIDUAL_KC=$2 timeout -k 10 120 python tools/bench_kernels.py --size 512 --reps 30 --tag zl$1kc$2 >> $o || exit 1
    MGIC_RESIDUAL_ZL=$1 MGIC_RESIDUAL_KC=$2 timeout -k 10 120 python tools/bench_kernels.py --size 256 --reps 50 --tag zl$1kc$2 >> $o || exit 1
    MGIC_RESIDUAL_ZL=$1 MGIC_RESIDUAL_KC=$2 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-bottom > gpurun_out/rzl/b.tmp 2> gpurun_out/rzl/err.log || { tail gpurun_out/rzl/err.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/rzl/b.tmp').read().strip().splitlines()[-1]); print(json.dumps({'tag':'zl$1kc$2','vcycles':d['value']}))" >> $o
  done
done
python3 - $o <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    j = json.loads(l)
    if "residual" in j: d[(j["tag"], str(j["size"]))].append(j["residual"]["ms"])
    else: d[(j["tag"], "vcycles")].append(j["vcycles"])
for k in sorted(d): print(k, d[k])
PY
echo "session done"
