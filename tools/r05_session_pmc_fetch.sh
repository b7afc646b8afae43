#!/bin/bash
# round-5 GPU session pmc_fetch: FETCH_SIZE / WRITE_SIZE / TCC hit counters of the streaming
# kernels (residual, restriction, prolongation) on tools/bench_kernels.py
# --size 512, one rocprofv3 --pmc pass per counter group, each under its own
# kill timeout.  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out/pmcf
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmcf/avail.txt 2>&1 || true
have() { grep -qw "$1" gpurun_out/pmcf/avail.txt; }
run_pass() {  # name counters...
  local name=$1; shift
  local cs=""
  for c in "$@"; do have "$c" && cs="$cs $c"; done
  echo "pass $name:$cs"
  [ -z "$cs" ] && return 0
  timeout -s KILL 120 rocprofv3 --pmc $cs -d "$R/gpurun_out/pmcf/$name" -o p --output-format csv -- python3 "$R/tools/bench_kernels.py" --size 512 --reps 5 > gpurun_out/pmcf/$name.log 2>&1
  local rc=$?; echo "  rc=$rc"; return $rc
}
run_pass e FETCH_SIZE || exit 1
run_pass f WRITE_SIZE || exit 1
run_pass g TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum || exit 1
PMC_KERNELS='k_restrict|k_residual|k_prolong' python3 tools/pmc_sq_summary.py gpurun_out/pmcf > gpurun_out/pmcf/summary.txt
cat gpurun_out/pmcf/summary.txt
find gpurun_out/pmcf -name "*.csv" -size +20M -delete
echo "session done"
