#!/bin/bash
# Memory-side counters (DRAM vs Infinity-Cache reads, outstanding-read
# level, credit stalls, TCP->TCC latency) for smoother configurations in
# $VARIANTS (comma-separated VAR=value lists; "passes" = per-colour kernel).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$(pwd); OUT=$R/gpurun_out/pmc_mem; mkdir -p $OUT
j=0
for V in ${VARIANTS:-MGIC_FUSED_VARIANT=0}; do
  j=$((j+1)); i=0
  extra=""; [ "$V" = "passes" ] && extra="--no-fused" && V="X=1"
  for C in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" "TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum" "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum" "GRBM_GUI_ACTIVE TCC_EA0_WRREQ_sum"; do
    i=$((i+1))
    env ${V//,/ } timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "gsrb" -d $OUT/c$j.$i -o p --output-format csv -- python3 $R/tools/bench_smoother.py --n 512 --sweeps 2 --reps 1 $extra > $OUT/c$j.$i.log 2>&1 || { echo "pass $V $i failed"; tail -3 $OUT/c$j.$i.log; }
  done
done
echo done
