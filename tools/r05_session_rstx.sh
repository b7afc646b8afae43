#!/bin/bash
# round-5 GPU session rstx: the restriction's z chunk (MGIC_RESTRICT_ZL)
# against its tile order (MGIC_RESTRICT_XCD bands): FETCH_SIZE per 512^3
# launch for each pair, then three interleaved rounds of bench_kernels
# 512^3 / 256^3.  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rstx
export TMPDIR=/tmp
R=$(pwd)
V="2 0;4 0;8 0;4 16;8 16;8 64"
IFS=';' read -ra VS <<< "$V"
MGIC_RESTRICT_ZL=8 MGIC_RESTRICT_XCD=16 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x \
  -k "restrict or lds_staged or vcycle_iterations or full_size_512_vcycle or multibox or agglomerat" --timeout 200 --timeout-method thread > gpurun_out/rstx/pytest.log 2>&1; rc=$?
echo "zl8 x16: $(tail -1 gpurun_out/rstx/pytest.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/rstx/pytest.log; exit $rc; }
for v in "${VS[@]}"; do
  set -- $v
  MGIC_RESTRICT_ZL=$1 MGIC_RESTRICT_XCD=$2 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_restrict -d "$R/gpurun_out/rstx/f$1_$2" -o p --output-format csv -- python3 "$R/tools/bench_kernels.py" --size 512 --reps 5 > gpurun_out/rstx/f.log 2>&1 || { tail gpurun_out/rstx/f.log; exit 1; }
  echo "fetch zl=$1 xcd=$2: $(PMC_KERNELS='k_restrict' python3 tools/pmc_sq_summary.py gpurun_out/rstx/f$1_$2 | grep FETCH_SIZE | head -1)"
done
o=gpurun_out/rstx/ab.txt; : > $o
for r in 1 2 3; do
  for v in "${VS[@]}"; do
    set -- $v
    MGIC_RESTRICT_ZL=$1 MGIC_RESTRICT_XCD=$2 timeout -k 10 120 python tools/bench_kernels.py --size 512 --reps 30 --tag "zl$1x$2" >> $o || exit 1
    MGIC_RESTRICT_ZL=$1 MGIC_RESTRICT_XCD=$2 timeout -k 10 120 python tools/bench_kernels.py --size 256 --reps 50 --tag "zl$1x$2" >> $o || exit 1
  done
done
python3 - $o <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    j = json.loads(l)
    d[(j["tag"], str(j["size"]))].append(j["restrict"]["ms"])
for k in sorted(d): print(k, d[k])
PY
find gpurun_out/rstx -name "*.csv" -size +20M -delete
echo "session done"
