set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$(pwd)
for lv in 3 5; do
for ag in 0 65 33 17; do
  timeout -k 5 180 python tools/rank_proxy.py --size 512 --parts 2,2,2 --periodic 0,0,0 --deep 1 --transport ipc --levels $lv --agglomerate-below $ag --steps 20 || exit 1
done
done
for ag in 0 65; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/agg_$ag -o tp --output-format csv -- python3 $R/tools/rank_proxy.py --size 512 --parts 2,2,2 --periodic 0,0,0 --deep 1 --transport ipc --levels 3 --agglomerate-below $ag --steps 10 --warmup 2 > gpurun_out/agg_$ag.log 2>&1 || exit 1
f=$(find gpurun_out/agg_$ag -name "*kernel_trace.csv" | head -1)
python3 tools/trace_summary.py $f > gpurun_out/agg_$ag.txt
done
