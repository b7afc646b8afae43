#!/bin/bash
# PMC passes (one counter group per run) over a short program for the kernels
# matching $KRE.  Output: gpurun_out/pmc_k/<i>/...counter_collection.csv and a
# per-kernel summary in gpurun_out/pmc_k/summary.txt.
#   KRE: kernel-name regex; CMD: the program after `python3` (default a
#   one-step bench.py); PASSES: counter groups separated by ';'
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$(pwd); OUT=$R/gpurun_out/${PMC_OUT:-pmc_k}; mkdir -p $OUT
KRE=${KRE:-k_restrict|k_prolong|k_residual|k_blas}
BARGS=${BARGS:---steps 1 --warmup 0 --no-cpu-baseline}
CMD=${CMD:-$R/bench.py $BARGS}
PASSES=${PASSES:-FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum;SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES;SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU}
IFS=';' read -r -a groups <<< "$PASSES"
i=0
for C in "${groups[@]}"; do
  i=$((i+1))
  # shellcheck disable=SC2086
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "$KRE" -d $OUT/$i -o p --output-format csv -- python3 $CMD > $OUT/$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/$i.log; exit 1; }
done
python3 tools/pmc_summary.py "$OUT/*/*/*counter_collection.csv" "$OUT/*/*counter_collection.csv" > $OUT/summary.txt 2>&1
echo done
