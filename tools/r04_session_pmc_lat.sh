#!/bin/bash
# round-4 GPU session pmc_lat: mean VMEM / LDS / instruction-fetch latency of
# the plain two-sweep launch (rocprofv3 derived counters VmemLatency,
# LdsLatency, InstrFetchLatency, one pass each, on tools/bench_smoother.py at
# 512^3 and 256^3).  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out/pmclat
for n in 512 256; do
  for c in VmemLatency LdsLatency InstrFetchLatency MeanOccupancyPerActiveCU; do
    timeout -s KILL 120 rocprofv3 --pmc $c -d "$R/gpurun_out/pmclat/${c}_$n" -o p --output-format csv -- python3 "$R/tools/bench_smoother.py" --n $n --sweeps 8 > gpurun_out/pmclat/${c}_$n.log 2>&1
    rc=$?; echo "$c n=$n rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmclat/${c}_$n.log; exit $rc; }
  done
done
python3 tools/pmc_sq_summary.py gpurun_out/pmclat > gpurun_out/pmclat/summary.txt
cat gpurun_out/pmclat/summary.txt
echo "session done"
