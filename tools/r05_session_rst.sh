#!/bin/bash
# round-5 GPU session rst: restriction tiles (MGIC_RESTRICT_TILE = WX RY KC,
# k_restrict_t) against the per-cell grid (0): parity subset per tile, three
# interleaved rounds of tools/bench_kernels.py at 512^3 and 256^3, FETCH_SIZE
# of each tile's 512^3 launch, the V-cycle for the candidates.  Measurement only
# (k_restrict_t and its switch were removed after this A/B: profiles/r05g_restrict_tiles.txt).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rst
export TMPDIR=/tmp
R=$(pwd)
T="${TILES:-0 141 242 424 441 482}"
for t in $T; do
  MGIC_RESTRICT_TILE=$t timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x \
    -k "restrict or operator_methods or vcycle_iterations or full_size_512_vcycle" \
    --timeout 200 --timeout-method thread > gpurun_out/rst/pytest_$t.log 2>&1; rc=$?
  echo "$t: $(tail -1 gpurun_out/rst/pytest_$t.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/rst/pytest_$t.log; exit $rc; }
done
out=gpurun_out/rst/kern.txt; : > $out
for r in 1 2 3; do
  for t in $T; do
    MGIC_RESTRICT_TILE=$t timeout -k 10 120 python tools/bench_kernels.py --size 512 --reps 30 --tag $t >> $out || exit 1
    MGIC_RESTRICT_TILE=$t timeout -k 10 120 python tools/bench_kernels.py --size 256 --reps 50 --tag $t >> $out || exit 1
  done
done
python3 - $out <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    j = json.loads(l); d[(j["tag"], j["size"])].append(j["restrict"]["ms"])
for k in sorted(d):
    v = sorted(d[k]); print(k, "median %.4f ms" % v[len(v) // 2], v)
PY
for t in $T; do
  timeout -s KILL 90 env MGIC_RESTRICT_TILE=$t rocprofv3 --pmc FETCH_SIZE --kernel-include-regex restrict -d "$R/gpurun_out/rst/f_$t" -o p --output-format csv -- python3 "$R/tools/bench_kernels.py" --size 512 --reps 5 > gpurun_out/rst/f_$t.log 2>&1 || { echo "pmc $t failed"; tail gpurun_out/rst/f_$t.log; exit 1; }
  f=$(find gpurun_out/rst/f_$t -name "*counter_collection.csv" | head -n 1)
  python3 - "$f" $t <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if r.get("Counter_Name") == "FETCH_SIZE"]
v = [float(r["Counter_Value"]) for r in rows]
big = [x for x in v if x > 0.5 * max(v)]
print("tile", sys.argv[2], "FETCH_SIZE x1024 x2 (GB, 512^3 launches):", round(sum(big) / len(big) * 2048 / 1e9, 3), "n", len(big))
PY
done
for r in 1 2; do
  for t in ${VTILES:-0}; do
    MGIC_RESTRICT_TILE=$t timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic --no-bottom > gpurun_out/rst/b.tmp 2> gpurun_out/rst/b_err.log || { tail gpurun_out/rst/b_err.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/rst/b.tmp').read().strip().splitlines()[-1]); print('tile $t vcycles', d['value'])"
  done
done
find gpurun_out/rst -name "*.csv" -size +5M -delete
echo "session done"
