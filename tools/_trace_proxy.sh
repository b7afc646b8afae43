set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$(pwd)
for t in ${TRANSPORTS:-ipc}; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/tp_$t -o tp --output-format csv -- python3 $R/tools/rank_proxy.py --deep 1 --transport $t --steps 20 --warmup 2 > gpurun_out/tp_$t.log 2>&1 || exit 1
f=$(find gpurun_out/tp_$t -name "*kernel_trace.csv" | head -1)
python3 tools/trace_summary.py $f > gpurun_out/tp_$t.txt
done
