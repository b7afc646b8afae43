#!/bin/bash
# round-5 GPU session pmc_stream: SQ / TA / TD counters of the streaming
# kernels (residual, restriction, prolongation) on tools/bench_kernels.py
# --size 512, one rocprofv3 --pmc pass per counter group, each under its own
# kill timeout.  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$(pwd)
mkdir -p gpurun_out/pmcst
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmcst/avail.txt 2>&1 || true
have() { grep -qw "$1" gpurun_out/pmcst/avail.txt; }
run_pass() {  # name counters...
  local name=$1; shift
  local cs=""
  for c in "$@"; do have "$c" && cs="$cs $c"; done
  echo "pass $name:$cs"
  [ -z "$cs" ] && return 0
  timeout -s KILL 120 rocprofv3 --pmc $cs -d "$R/gpurun_out/pmcst/$name" -o p --output-format csv -- python3 "$R/tools/bench_kernels.py" --size 512 --reps 5 > gpurun_out/pmcst/$name.log 2>&1
  local rc=$?; echo "  rc=$rc"; return $rc
}
run_pass a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE || exit 1
run_pass b SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_SCA || exit 1
run_pass c TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TD_SPI_STALL_sum GRBM_GUI_ACTIVE || exit 1
run_pass d TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum || exit 1
PMC_KERNELS='k_restrict|k_residual|k_prolong' python3 tools/pmc_sq_summary.py gpurun_out/pmcst > gpurun_out/pmcst/summary.txt
cat gpurun_out/pmcst/summary.txt
find gpurun_out/pmcst -name "*.csv" -size +20M -delete
echo "session done"
