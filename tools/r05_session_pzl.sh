#!/bin/bash
# round-5 GPU session pzl: the linear prolongation with LDS-staged coarse
# planes (MGIC_PROLONG_ZL = z chunk in coarse planes) against k_prolong (0):
# parity subset, three interleaved rounds of bench_kernels 512^3 / 256^3 and
# the V-cycle.  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pzl
export TMPDIR=/tmp
V="${PZLS:-4 8 16}"
for v in $V; do
  MGIC_PROLONG_ZL=$v timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -x \
    -k "prolong or operator_methods or vcycle or multibox or agglomerat or periodic or ragged" --timeout 200 --timeout-method thread > gpurun_out/pzl/pytest_$v.log 2>&1; rc=$?
  echo "pzl=$v: $(tail -1 gpurun_out/pzl/pytest_$v.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/pzl/pytest_$v.log; exit $rc; }
done
o=gpurun_out/pzl/ab.txt; : > $o
for r in 1 2 3; do
  for v in 0 $V; do
    MGIC_PROLONG_ZL=$v timeout -k 10 120 python tools/bench_kernels.py --size 512 --reps 30 --tag pzl=$v >> $o || exit 1
    MGIC_PROLONG_ZL=$v timeout -k 10 120 python tools/bench_kernels.py --size 256 --reps 50 --tag pzl=$v >> $o || exit 1
    MGIC_PROLONG_ZL=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-bottom > gpurun_out/pzl/b.tmp 2> gpurun_out/pzl/err.log || { tail gpurun_out/pzl/err.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/pzl/b.tmp').read().strip().splitlines()[-1]); print(json.dumps({'tag':'pzl=$v','vcycles':d['value']}))" >> $o
  done
done
python3 - $o <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    j = json.loads(l)
    if "prolong" in j: d[(j["tag"], str(j["size"]))].append(j["prolong"]["ms"])
    else: d[(j["tag"], "vcycles")].append(j["vcycles"])
for k in sorted(d): print(k, d[k])
PY
echo "session done"
