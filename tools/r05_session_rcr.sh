#!/bin/bash
# round-5 GPU session rcr: k_restrict_zl with 8 coarse rows per workgroup
# (MGIC_RESTRICT_CR=8: 512 threads, 76 KB LDS, 16 waves per CU) against 4
# (256 threads, 42 KB, 12 waves), chunks 2 and 4: parity subset, three
# interleaved rounds of bench_kernels 512^3 / 256^3 and the V-cycle.
# Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rcr
export TMPDIR=/tmp
MGIC_RESTRICT_CR=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x \
  -k "restrict or lds_staged or operator_methods or vcycle_iterations or full_size_512_vcycle or multibox or agglomerat or periodic" --timeout 200 --timeout-method thread > gpurun_out/rcr/pytest.log 2>&1; rc=$?
echo "cr=8: $(tail -1 gpurun_out/rcr/pytest.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/rcr/pytest.log; exit $rc; }
o=gpurun_out/rcr/ab.txt; : > $o
for r in 1 2 3; do
  for v in "4 2" "8 2" "8 4"; do
    set -- $v
    MGIC_RESTRICT_CR=$1 MGIC_RESTRICT_ZL=$2 timeout -k 10 120 python tools/bench_kernels.py --size 512 --reps 30 --tag cr$1kc$2 >> $o || exit 1
    MGIC_RESTRICT_CR=$1 MGIC_RESTRICT_ZL=$2 timeout -k 10 120 python tools/bench_kernels.py --size 256 --reps 50 --tag cr$1kc$2 >> $o || exit 1
    MGIC_RESTRICT_CR=$1 MGIC_RESTRICT_ZL=$2 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-bottom > gpurun_out/rcr/b.tmp 2> gpurun_out/rcr/err.log || { tail gpurun_out/rcr/err.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/rcr/b.tmp').read().strip().splitlines()[-1]); print(json.dumps({'tag':'cr$1kc$2','vcycles':d['value']}))" >> $o
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
