#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$(pwd); OUT=$R/gpurun_out/pmc_cal; mkdir -p $OUT
i=0
for V in passes 1; do
  for C in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" ; do
    i=$((i+1))
    if [ $V = passes ]; then A="--no-fused"; else A=""; fi
    MGIC_FUSED_VARIANT=$V timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "gsrb" -d $OUT/$V$i -o p --output-format csv -- python3 $R/tools/bench_smoother.py --n 512 --sweeps 2 --reps 1 $A > $OUT/$V$i.log 2>&1 || { echo "pass $V $i failed"; tail -5 $OUT/$V$i.log; }
  done
done
echo done
