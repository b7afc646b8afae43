#!/bin/bash
# rocprofv3 kernel trace of a short bench run -> gpurun_out/trace_<TAG>/ and a
# per-kernel summary (tools/trace_summary.py).  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-t}
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/trace_$TAG" -o "$TAG" --output-format csv -- python3 "$R/bench.py" --steps ${BSTEPS:-5} --warmup 1 --no-cpu-baseline --no-traffic --no-bottom > gpurun_out/trace_$TAG.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
f=$(find gpurun_out/trace_$TAG -name "*kernel_trace.csv" | head -n 1)
python3 tools/trace_summary.py "$f" > gpurun_out/trace_$TAG.txt 2>&1
st=$(find gpurun_out/trace_$TAG -name "*kernel_stats.csv" | head -n 1)
[ -n "$st" ] && cp "$st" gpurun_out/trace_${TAG}_kernel_stats.csv
rm -rf gpurun_out/trace_$TAG  # (the raw trace is too large to bring back)
sed -n 1,30p gpurun_out/trace_$TAG.txt
