#!/bin/bash
# round-5 GPU session sxcd: the LDS-staged residual and restriction in the
# XCD-aware tile order (MGIC_STREAM_XCD = band of S tiles) against the dispatch order (0):
# parity subset, FETCH_SIZE of both orders, three interleaved rounds of
# bench_kernels 512^3 / 256^3 and the V-cycle.  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sxcd
export TMPDIR=/tmp
R=$(pwd)
for S in 64 7; do
  MGIC_STREAM_XCD=$S timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_mixed.py -q -x \
    -k "residual or restrict or lds_staged or operator_methods or vcycle or multibox or agglomerat or periodic or mixed or fmg" --timeout 200 --timeout-method thread > gpurun_out/sxcd/pytest$S.log 2>&1; rc=$?
  echo "xcd=$S: $(tail -1 gpurun_out/sxcd/pytest$S.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/sxcd/pytest$S.log; exit $rc; }
done
for v in 0 64; do
  MGIC_STREAM_XCD=$v timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/sxcd/f$v" -o p --output-format csv -- python3 "$R/tools/bench_kernels.py" --size 512 --reps 5 > gpurun_out/sxcd/f$v.log 2>&1 || { tail gpurun_out/sxcd/f$v.log; exit 1; }
  echo "fetch xcd=$v"; PMC_KERNELS='k_restrict|k_residual' python3 tools/pmc_sq_summary.py gpurun_out/sxcd/f$v
done
o=gpurun_out/sxcd/ab.txt; : > $o
for r in 1 2 3; do
  for v in ${XS:-0 16 64 256}; do
    MGIC_STREAM_XCD=$v timeout -k 10 120 python tools/bench_kernels.py --size 512 --reps 30 --tag x$v >> $o || exit 1
    MGIC_STREAM_XCD=$v timeout -k 10 120 python tools/bench_kernels.py --size 256 --reps 50 --tag x$v >> $o || exit 1
    MGIC_STREAM_XCD=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-bottom > gpurun_out/sxcd/b.tmp 2> gpurun_out/sxcd/err.log || { tail gpurun_out/sxcd/err.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/sxcd/b.tmp').read().strip().splitlines()[-1]); print(json.dumps({'tag':'x$v','vcycles':d['value']}))" >> $o
  done
done
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
find gpurun_out/sxcd -name "*.csv" -size +20M -delete
echo "session done"
