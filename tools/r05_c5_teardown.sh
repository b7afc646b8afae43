#!/bin/bash
# round-5: the multi-rank C5 bench's exit-time heap error came from two HIP
# runtimes in one process (libmgic.so loaded before torch); torch first now
# (_lib.py): 2 ranks at 128^3, then the 8-rank one-GPU rehearsal of C5 at
# 1024^3 and bench.py --gpus 8's rehearsal (the rank-0 bottom solve timed).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
MGIC_BENCH_DEVICE=0 timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29631 tools/bench_c5.py --size 128 --levels 3 --vcycles 2 \
  --kinds fp64 --no-oracle-check > gpurun_out/c5td_2.log 2>&1
echo "2 ranks rc=$? double-free lines: $(grep -c 'double free' gpurun_out/c5td_2.log)"
STEPS_TO_RUN="c5_8 bench8" bash tools/gpu_session.sh
echo "session done"
