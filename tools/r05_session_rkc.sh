#!/bin/bash
# round-5 GPU session rkc: the banded residual's z chunk (MGIC_RESIDUAL_KC)
# and band (MGIC_RESIDUAL_XCD): parity subset, three interleaved rounds of
# bench_kernels 512^3 / 256^3 and the V-cycle per "chunk band" pair.
# Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rkc
export TMPDIR=/tmp
for v in "16 16" "64 16"; do
  set -- $v
  MGIC_RESIDUAL_KC=$1 MGIC_RESIDUAL_XCD=$2 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_mixed.py -q -x \
    -k "residual or restrict or lds_staged or operator_methods or vcycle or multibox or agglomerat or periodic or mixed or fmg" --timeout 200 --timeout-method thread > gpurun_out/rkc/pytest.log 2>&1; rc=$?
  echo "xcd $1 $2: $(tail -1 gpurun_out/rkc/pytest.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/rkc/pytest.log; exit $rc; }
done
o=gpurun_out/rkc/ab.txt; : > $o
for r in 1 2 3; do
  for v in "32 16" "16 16" "64 16" "32 32"; do
    set -- $v
    export MGIC_RESIDUAL_KC=$1 MGIC_RESIDUAL_XCD=$2
    timeout -k 10 120 python tools/bench_kernels.py --size 512 --reps 30 --tag "kc$1b$2" >> $o || exit 1
    timeout -k 10 120 python tools/bench_kernels.py --size 256 --reps 50 --tag "kc$1b$2" >> $o || exit 1
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-bottom > gpurun_out/rkc/b.tmp 2> gpurun_out/rkc/err.log || { tail gpurun_out/rkc/err.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/rkc/b.tmp').read().strip().splitlines()[-1]); print(json.dumps({'tag':'kc$1b$2','vcycles':d['value']}))" >> $o
  done
done
unset MGIC_RESIDUAL_KC MGIC_RESIDUAL_XCD
python3 - $o <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    j = json.loads(l)
    if "restrict" in j:
        d[(j["tag"], str(j["size"]), "restrict")].append(j["restrict"]["ms"])
        d[(j["tag"], str(j["size"]), "residual")].append(j["residual"]["ms"])
    else: d[(j["tag"], "vcycles")].append(j["vcycles"])
for k in sorted(d): print(k, d[k])
PY
echo "session done"
