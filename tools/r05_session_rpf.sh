#!/bin/bash
# round-5 GPU session rpf: k_residual_zl with rhs / aCoef one plane ahead
# (MGIC_RESIDUAL_PF=1) against the default:
# parity subset (fp64 and mixed), three interleaved rounds of bench_kernels
# 512^3 / 256^3 and the V-cycle.  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rpf
export TMPDIR=/tmp
MGIC_RESIDUAL_PF=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_mixed.py -q -x \
  -k "residual or operator_methods or vcycle or multibox or agglomerat or periodic or mixed or fmg" --timeout 200 --timeout-method thread > gpurun_out/rpf/pytest.log 2>&1; rc=$?
echo "pf: $(tail -1 gpurun_out/rpf/pytest.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/rpf/pytest.log; exit $rc; }
o=gpurun_out/rpf/ab.txt; : > $o
for r in 1 2 3; do
  for v in "0" "1"; do
    set -- $v
    MGIC_RESIDUAL_PF=$1 timeout -k 10 120 python tools/bench_kernels.py --size 512 --reps 30 --tag pf$1 >> $o || exit 1
    MGIC_RESIDUAL_PF=$1 timeout -k 10 120 python tools/bench_kernels.py --size 256 --reps 50 --tag pf$1 >> $o || exit 1
    MGIC_RESIDUAL_PF=$1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-bottom > gpurun_out/rpf/b.tmp 2> gpurun_out/rpf/err.log || { tail gpurun_out/rpf/err.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/rpf/b.tmp').read().strip().splitlines()[-1]); print(json.dumps({'tag':'pf$1','vcycles':d['value']}))" >> $o
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
