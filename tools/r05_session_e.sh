#!/bin/bash
# round-5 GPU session e: conflict-free lanes for the rows' last pairs
# (TB2_XMAP, gpurun_ab/xmap) and with the plain launch's steady step (sx);
# parity subset, three interleaved A/B rounds against the in-tree library
# and sdy, then a rocprofv3 kernel trace of the bench for base, sdy, xmap.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="sdy xmap sx"
for v in xmap sx; do
  MGIC_LIB_PATH=gpurun_ab/$v/libmgic.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x \
    -k "two_sweep or full_size_512_vcycle or full_size_256 or deep_halo_vcycle or streaming_vcycle or vcycle_iterations" \
    --timeout 200 --timeout-method thread > gpurun_out/pytest_$v.log 2>&1; rc=$?
  echo "$v: $(tail -1 gpurun_out/pytest_$v.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/pytest_$v.log; exit $rc; }
done
out=gpurun_out/r05e_ab.txt; : > $out
for r in 1 2 3; do
  for v in base $V; do
    L=""; [ $v != base ] && L=gpurun_ab/$v/libmgic.so
    MGIC_LIB_PATH=$L timeout -k 10 120 python tools/bench_smoother.py --n 512 --sweeps 8 --tag $v >> $out || exit 1
    MGIC_LIB_PATH=$L timeout -k 10 120 python tools/bench_smoother.py --n 256 --sweeps 8 --tag $v >> $out || exit 1
    MGIC_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic --no-bottom > gpurun_out/ab_bench.tmp 2> gpurun_out/ab_err.log || { tail gpurun_out/ab_err.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_bench.tmp').read().strip().splitlines()[-1]); print(json.dumps({'variant':'$v','vcycles':d['value'],'ms':d['ms_per_step'],'launch_ms':d['roofline']['avg_launch_ms'],'frac':d['roofline']['frac']}))" >> $out
  done
done
python3 tools/ab_summary.py $out
for v in base sdy xmap; do
  if [ $v != base ]; then export MGIC_LIB_PATH=gpurun_ab/$v/libmgic.so; else unset MGIC_LIB_PATH; fi
  TAG=r05e_$v BSTEPS=10 bash tools/trace_bench.sh > /dev/null || exit 1
  grep -E "k_gsrb_tb2" gpurun_out/trace_r05e_$v.txt | head -8
done
echo "session done"
