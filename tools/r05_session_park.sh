#!/bin/bash
# round-5 GPU session park: ranks that do not hold the gathered bottom wait for
# the scatter on the host (MGIC_PARK_SYNC=1) instead of queueing the rest of
# the V-cycle behind it; 8-rank one-GPU rehearsal, two interleaved rounds,
# the driver's --steps 20 --warmup 5.  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/park
export TMPDIR=/tmp
port=29591
for r in 1 2; do
  for p in 1 0; do
    timeout -k 10 300 env MGIC_PARK_SYNC=$p MGIC_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
      --master-addr 127.0.0.1 --master-port $port bench.py --gpus 8 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/park/b$p.log 2>&1 \
      || { tail gpurun_out/park/b$p.log; exit 1; }
    port=$((port + 1))
    grep -E '^\{"metric"' gpurun_out/park/b$p.log | tail -n 1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); b = d['bottom']
print(json.dumps({'park': $p, 'vcycles': d['value'], 'bottom_delta_ms': b['bottom_delta_ms'], 'bottom_solve_ms_rank0': b['bottom_solve_ms_rank0']}))"
  done
done
echo "session done"
