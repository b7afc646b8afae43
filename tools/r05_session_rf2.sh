#!/bin/bash
# round-5 GPU session rf2: the fp32 restriction and prolongation with two coarse cells per
# thread (16-B fine-row accesses; MGIC_RESTRICT_F2=1 MGIC_PROLONG_F2=1, the defaults) against one
# (=0): the fp32 / mixed tests, then two interleaved rounds of
# tools/bench_c5.py (mixed, 1024^3).  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rf2
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_mixed.py tests/test_multiprocess.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/rf2/tests.log 2>&1; rc=$?
tail -1 gpurun_out/rf2/tests.log; [ $rc -ne 0 ] && { tail -30 gpurun_out/rf2/tests.log; exit $rc; }
out=gpurun_out/rf2/ab.txt; : > $out
for r in 1 2; do
  for v in 1 0; do
    MGIC_RESTRICT_F2=$v MGIC_PROLONG_F2=$v timeout -k 10 400 python tools/bench_c5.py --kinds mixed --vcycles 4 > gpurun_out/rf2/c5.tmp 2> gpurun_out/rf2/err.log || { tail gpurun_out/rf2/err.log; exit 1; }
    echo "f2=$v $(tail -n 1 gpurun_out/rf2/c5.tmp)" >> $out
  done
done
python3 - $out <<'PY'
import json, sys
for l in open(sys.argv[1]):
    v, j = l.split(" ", 1); d = json.loads(j); m = d["mixed"]
    print(v, "fmg", m["ms_per_fmg"], "vcycle", m["ms_per_vcycle"], "oracle", d.get("oracle_check", {}).get("bit_identical"), "res", m["residual_max_norm"]["after_fmg_plus_4_vcycles"])
PY
# the fp64 restriction with two coarse cells per thread (MGIC_RESTRICT_D2=1,
# a measurement switch): parity subset, three interleaved rounds of
# bench_kernels at 512^3 / 256^3 and the V-cycle
MGIC_RESTRICT_D2=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x \
  -k "restrict or operator_methods or vcycle_iterations or full_size_512_vcycle or multibox or agglomerat" \
  --timeout 200 --timeout-method thread > gpurun_out/rf2/pytest_d2.log 2>&1; rc=$?
echo "d2: $(tail -1 gpurun_out/rf2/pytest_d2.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/rf2/pytest_d2.log; exit $rc; }
o2=gpurun_out/rf2/d2.txt; : > $o2
for r in 1 2 3; do
  for v in 0 1; do
    MGIC_RESTRICT_D2=$v timeout -k 10 120 python tools/bench_kernels.py --size 512 --reps 30 --tag d2=$v >> $o2 || exit 1
    MGIC_RESTRICT_D2=$v timeout -k 10 120 python tools/bench_kernels.py --size 256 --reps 50 --tag d2=$v >> $o2 || exit 1
    MGIC_RESTRICT_D2=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-bottom > gpurun_out/rf2/b.tmp 2> gpurun_out/rf2/err.log || { tail gpurun_out/rf2/err.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/rf2/b.tmp').read().strip().splitlines()[-1]); print(json.dumps({'tag':'d2=$v','vcycles':d['value']}))" >> $o2
  done
done
python3 - $o2 <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    j = json.loads(l)
    if "restrict" in j: d[(j["tag"], j["size"])].append(j["restrict"]["ms"])
    else: d[(j["tag"], "vcycles")].append(j["vcycles"])
for k in sorted(d): print(k, d[k])
PY
echo "session done"
