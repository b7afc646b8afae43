#!/bin/bash
# rocprofv3 passes over a short bench run (kernel trace + stats, then PMC
# passes for HBM traffic of the smoother kernels; counters in their own runs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof}
TAG=${TAG:-r01}
KRE=${KRE:-k_gsrb}
BARGS=${BARGS:---steps 5 --warmup 1 --no-cpu-baseline}
mkdir -p "$OUT"
R=$(pwd)
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/$OUT/trace" -o "$TAG" --output-format csv -- python3 "$R/bench.py" $BARGS > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -d "$R/$OUT/pmc_fetch" -o "$TAG" --output-format csv -- python3 "$R/bench.py" $BARGS > "$OUT/pmc_fetch.log" 2>&1
rc=$?; echo "pmc fetch rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -d "$R/$OUT/pmc_write" -o "$TAG" --output-format csv -- python3 "$R/bench.py" $BARGS > "$OUT/pmc_write.log" 2>&1
rc=$?; echo "pmc write rc=$rc"; exit $rc
