#!/bin/bash
# round-5 GPU session wpe: k_restrict compiled for 6 / 8 waves per SIMD
# (RESTRICT_WPE, gpurun_ab/wpe6, wpe8: 94 -> <= 80 / 64 VGPRs) against the
# in-tree library (5 waves): parity subset, three interleaved rounds of
# bench_kernels 512^3 / 256^3 and the V-cycle.  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/wpe
export TMPDIR=/tmp
for v in wpe6 wpe8; do
  MGIC_LIB_PATH=gpurun_ab/$v/libmgic.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x \
    -k "restrict or operator_methods or vcycle_iterations or full_size_512_vcycle" --timeout 200 --timeout-method thread > gpurun_out/wpe/pytest_$v.log 2>&1; rc=$?
  echo "$v: $(tail -1 gpurun_out/wpe/pytest_$v.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/wpe/pytest_$v.log; exit $rc; }
done
o=gpurun_out/wpe/ab.txt; : > $o
for r in 1 2 3; do
  for v in base wpe6 wpe8; do
    L=""; [ $v != base ] && L=gpurun_ab/$v/libmgic.so
    MGIC_LIB_PATH=$L timeout -k 10 120 python tools/bench_kernels.py --size 512 --reps 30 --tag $v >> $o || exit 1
    MGIC_LIB_PATH=$L timeout -k 10 120 python tools/bench_kernels.py --size 256 --reps 50 --tag $v >> $o || exit 1
    MGIC_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-bottom > gpurun_out/wpe/b.tmp 2> gpurun_out/wpe/err.log || { tail gpurun_out/wpe/err.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/wpe/b.tmp').read().strip().splitlines()[-1]); print(json.dumps({'tag':'$v','vcycles':d['value']}))" >> $o
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
