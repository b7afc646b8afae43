#!/bin/bash
# round-4 GPU session pmc_sq: where a two-sweep step's wave cycles go (SQ
# counters on tools/bench_smoother.py, 512^3, plain launches; one pass per
# counter group, each under its own kill timeout).  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out/pmcsq
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmcsq/avail.txt 2>&1 || true
have() { grep -qw "$1" gpurun_out/pmcsq/avail.txt; }
run_pass() {  # name counters...
  local name=$1; shift
  local cs=""
  for c in "$@"; do have "$c" && cs="$cs $c"; done
  echo "pass $name:$cs"
  [ -z "$cs" ] && return 0
  timeout -s KILL 120 rocprofv3 --pmc $cs -d "$R/gpurun_out/pmcsq/$name" -o p --output-format csv -- python3 "$R/tools/bench_smoother.py" --n ${N:-512} --sweeps 8 > gpurun_out/pmcsq/$name.log 2>&1
  local rc=$?; echo "  rc=$rc"; return $rc
}
run_pass a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
run_pass b SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA || exit 1
run_pass c SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_WAIT_INST_ANY || exit 1
python3 tools/pmc_sq_summary.py gpurun_out/pmcsq > gpurun_out/pmcsq/summary.txt
cat gpurun_out/pmcsq/summary.txt
find gpurun_out/pmcsq -name "*.csv" -size +20M -delete
echo "session done"
