#!/bin/bash
# round-5 final GPU checkpoint at HEAD: tools/r05_session_final2.sh (suite,
# smoke, default bench line, kernel trace, share proxies, rank rehearsal),
# then C5: tools/bench_c5.py on one GPU (mixed and fp64) and on 8 ranks
# (mixed).  Measurement only; each step bounded.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/f3
export TMPDIR=/tmp
bash tools/r05_session_final2.sh || exit 1
timeout -k 10 600 python tools/bench_c5.py --vcycles 4 > gpurun_out/f3/c5.log 2>&1 || { tail gpurun_out/f3/c5.log; exit 1; }
tail -n 1 gpurun_out/f3/c5.log
timeout -k 10 600 env MGIC_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29651 tools/bench_c5.py --vcycles 4 --kinds mixed > gpurun_out/f3/c5_8.log 2>&1 || { tail gpurun_out/f3/c5_8.log; exit 1; }
tail -n 1 gpurun_out/f3/c5_8.log
echo "final session done"
