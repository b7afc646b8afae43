#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$(pwd); OUT=$R/gpurun_out/pmc_sm; mkdir -p $OUT
KRE=${KRE:-gsrb}
ARGS=${ARGS:---n 512 --sweeps 4 --reps 1}
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "$KRE" -d $OUT/p$i -o p --output-format csv -- python3 $R/tools/bench_smoother.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
