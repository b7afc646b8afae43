#!/bin/bash
# round-5 GPU session c: (1) the new gathered-depth tests on the in-tree
# library (the BiCGStab bottom on rank 0 between 4 / 8 processes, C5's mixed
# FMG with agglomeration and deep halo); (2) four more load placements of the
# two-sweep launch (gpurun_ab/s4..s7) against s1 and the in-tree library;
# (3) the charged 8-GPU share proxy.  Measurement + tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
[ -z "${SKIP_NEW:-}" ] && timeout -k 10 900 python -u -m pytest tests/test_multiprocess.py tests/test_mixed.py -q -x -rf \
  -k "bicgstab or agglomerated or mixed_fmg" --timeout 400 --timeout-method thread > gpurun_out/pytest_new.log 2>&1; rc=$?
[ -z "${SKIP_NEW:-}" ] && tail -3 gpurun_out/pytest_new.log; [ -z "${SKIP_NEW:-}" ] && [ $rc -ne 0 ] && { tail -60 gpurun_out/pytest_new.log; exit $rc; }
V="s4 s5 s6 s7"
for v in ${TEST_V-$V}; do
  MGIC_LIB_PATH=gpurun_ab/$v/libmgic.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x \
    -k "two_sweep or full_size_512_vcycle or full_size_256 or deep_halo_vcycle or streaming_vcycle or vcycle_iterations" \
    --timeout 200 --timeout-method thread > gpurun_out/pytest_$v.log 2>&1; rc=$?
  echo "$v: $(tail -1 gpurun_out/pytest_$v.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/pytest_$v.log; exit $rc; }
done
out=gpurun_out/r05c_spread_ab.txt; : > $out
for r in 1 2 3; do
  for v in base s1 $V; do
    L=""; [ $v != base ] && L=gpurun_ab/$v/libmgic.so
    MGIC_LIB_PATH=$L timeout -k 10 120 python tools/bench_smoother.py --n 512 --sweeps 8 --tag $v >> $out || exit 1
    MGIC_LIB_PATH=$L timeout -k 10 120 python tools/bench_smoother.py --n 256 --sweeps 8 --tag $v >> $out || exit 1
    MGIC_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic --no-bottom > gpurun_out/ab_bench.tmp 2> gpurun_out/ab_err.log || { tail gpurun_out/ab_err.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_bench.tmp').read().strip().splitlines()[-1]); print(json.dumps({'variant':'$v','vcycles':d['value'],'ms':d['ms_per_step'],'launch_ms':d['roofline']['avg_launch_ms'],'frac':d['roofline']['frac']}))" >> $out
  done
done
for r in 1 2; do
  timeout -k 10 240 python3 tools/rank_proxy.py --transport ipc --deep 1 --steps 30 >> gpurun_out/r05c_proxy.txt 2> gpurun_out/proxy_err.log || { tail gpurun_out/proxy_err.log; exit 1; }
  MGIC_LIB_PATH=gpurun_ab/s1/libmgic.so timeout -k 10 240 python3 tools/rank_proxy.py --transport ipc --deep 1 --steps 30 >> gpurun_out/r05c_proxy_s1.txt 2> gpurun_out/proxy_err.log || { tail gpurun_out/proxy_err.log; exit 1; }
done
cat gpurun_out/r05c_proxy.txt gpurun_out/r05c_proxy_s1.txt
echo "session done"
