#!/bin/bash
# round-5 GPU session zl: the restriction streaming in z with the fine u
# planes staged in LDS (MGIC_RESTRICT_ZL = z chunk in coarse planes) against
# k_restrict (0): parity subset per chunk, three interleaved rounds of
# bench_kernels 512^3 / 256^3 and the V-cycle.  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/zl
export TMPDIR=/tmp
V="${ZLS:-8 16 32}"
for v in $V; do
  MGIC_RESTRICT_ZL=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x \
    -k "restrict or operator_methods or vcycle_iterations or full_size_512_vcycle or multibox or agglomerat or periodic" --timeout 200 --timeout-method thread > gpurun_out/zl/pytest_$v.log 2>&1; rc=$?
  echo "zl=$v: $(tail -1 gpurun_out/zl/pytest_$v.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/zl/pytest_$v.log; exit $rc; }
done
o=gpurun_out/zl/ab.txt; : > $o
for r in 1 2 3; do
  for v in 0 $V; do
    MGIC_RESTRICT_ZL=$v timeout -k 10 120 python tools/bench_kernels.py --size 512 --reps 30 --tag zl=$v >> $o || exit 1
    MGIC_RESTRICT_ZL=$v timeout -k 10 120 python tools/bench_kernels.py --size 256 --reps 50 --tag zl=$v >> $o || exit 1
    MGIC_RESTRICT_ZL=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-bottom > gpurun_out/zl/b.tmp 2> gpurun_out/zl/err.log || { tail gpurun_out/zl/err.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/zl/b.tmp').read().strip().splitlines()[-1]); print(json.dumps({'tag':'zl=$v','vcycles':d['value']}))" >> $o
  done
done
python3 - $o <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    j = json.loads(l)
    if "restrict" in j: d[(j["tag"], str(j["size"]))].append(j["restrict"]["ms"])
    else: d[(j["tag"], "vcycles")].append(j["vcycles"])
for k in sorted(d): print(k, d[k])
PY
echo "session done"
