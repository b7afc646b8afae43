#!/bin/bash
# round-4 GPU session p: iterations() takes iteration i's norm while iteration i+1's V-cycle runs up to its phi += e launch (the GPU no longer idles between iterations); previous: results published into
# pinned host memory, the host spinning on a sequence word (no copy, no
# stream synchronisation per readback) -- the GPU suite, then the 1-GPU bench
# A/B against the previous library (gpurun_ab/prev), three interleaved
# rounds, and a kernel trace of the new library's bench (iteration gaps)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -rf -k "pipelined or iterations or multiprocess or process or full_size_512"  --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
out=gpurun_out/pipe_ab.txt; : > $out
for r in 1 2 3; do
  for v in prev new; do
    L=""; [ $v = prev ] && L=gpurun_ab/prev/libmgic.so
    MGIC_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic > gpurun_out/ab_bench.tmp 2> gpurun_out/ab_err.log || { tail gpurun_out/ab_err.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_bench.tmp').read().strip().splitlines()[-1]); print(json.dumps({'variant':'$v','vcycles':d['value'],'ms':d['ms_per_step'],'bottom_ms':d['bottom']['ms_per_vcycle'],'launch_ms':d['roofline']['avg_launch_ms']}))" >> $out
  done
done
cat $out
TAG=pipe BSTEPS=5 bash tools/trace_bench.sh > /dev/null || exit 1
grep -A90 "last launches" gpurun_out/trace_pipe.txt | grep -B1 -A1 "copyBuffer\|reduce_final" | head -30
echo "session done"
