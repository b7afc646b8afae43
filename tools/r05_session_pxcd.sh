#!/bin/bash
# round-5 GPU session pxcd: the linear prolongation in XCD bands
# (MGIC_PROLONG_XCD = band) against the dispatch order: parity subset,
# FETCH_SIZE per 512^3 launch, three interleaved rounds of bench_kernels
# 512^3 / 256^3 and the V-cycle.  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pxcd
export TMPDIR=/tmp
R=$(pwd)
MGIC_PROLONG_XCD=16 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x \
  -k "prolong or operator_methods or vcycle_iterations or full_size_512_vcycle or multibox or agglomerat or periodic" --timeout 200 --timeout-method thread > gpurun_out/pxcd/pytest.log 2>&1; rc=$?
echo "band 16: $(tail -1 gpurun_out/pxcd/pytest.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/pxcd/pytest.log; exit $rc; }
for v in 0 16 64; do
  MGIC_PROLONG_XCD=$v timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_prolong -d "$R/gpurun_out/pxcd/f$v" -o p --output-format csv -- python3 "$R/tools/bench_kernels.py" --size 512 --reps 5 > gpurun_out/pxcd/f.log 2>&1 || { tail gpurun_out/pxcd/f.log; exit 1; }
  echo "fetch band=$v: $(PMC_KERNELS='k_prolong' python3 tools/pmc_sq_summary.py gpurun_out/pxcd/f$v | grep FETCH_SIZE | head -1)"
done
o=gpurun_out/pxcd/ab.txt; : > $o
for r in 1 2 3; do
  for v in 0 16 64; do
    MGIC_PROLONG_XCD=$v timeout -k 10 120 python tools/bench_kernels.py --size 512 --reps 30 --tag "p$v" >> $o || exit 1
    MGIC_PROLONG_XCD=$v timeout -k 10 120 python tools/bench_kernels.py --size 256 --reps 50 --tag "p$v" >> $o || exit 1
    MGIC_PROLONG_XCD=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-bottom > gpurun_out/pxcd/b.tmp 2> gpurun_out/pxcd/err.log || { tail gpurun_out/pxcd/err.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/pxcd/b.tmp').read().strip().splitlines()[-1]); print(json.dumps({'tag':'p$v','vcycles':d['value']}))" >> $o
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
find gpurun_out/pxcd -name "*.csv" -size +20M -delete
echo "session done"
