set -u
export TMPDIR=/tmp
R=$(pwd); OUT=$R/gpurun_out/pmc_rst; mkdir -p $OUT
i=0
for C in "SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU" "SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "k_gsrb_fused" -d $OUT/$i -o p --output-format csv -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu-baseline > $OUT/$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/$i.log; exit 1; }
done
echo done
