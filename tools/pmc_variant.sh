#!/bin/bash
# PMC passes (one counter group per run) on the smoother micro-benchmark for
# each configuration in $VARIANTS (comma-separated VAR=value lists).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$(pwd); OUT=$R/gpurun_out/pmc_var; mkdir -p $OUT
j=0
for V in ${VARIANTS:-MGIC_SWEEPS_PER_LAUNCH=2}; do
  j=$((j+1)); i=0
  for C in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" "SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU" "SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH"; do
    i=$((i+1))
    env ${V//,/ } timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "gsrb" -d $OUT/c$j.$i -o p --output-format csv -- python3 $R/tools/bench_smoother.py --n 512 --sweeps 2 --reps 1 > $OUT/c$j.$i.log 2>&1 || { echo "pass $V $i failed"; tail -3 $OUT/c$j.$i.log; }
  done
done
echo done
