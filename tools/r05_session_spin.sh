#!/bin/bash
# round-5 GPU session spin: host waits that sleep after 1 ms of spinning
# (MGIC_HOST_SPIN_US=1000, the default) against spinning throughout (1e9):
# two interleaved rounds of the 8-rank one-GPU rehearsal and the 1-rank bench.
# Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/spin
export TMPDIR=/tmp
out=gpurun_out/spin/r.jsonl; : > $out
summ() {  # tag log
  grep -E '^\{"metric"' "$2" | tail -n 1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); b = d['bottom']
print(json.dumps({'case': '$1', 'n': d['n_gpus'], 'vcycles': d['value'], 'bottom_delta_ms': b['bottom_delta_ms'], 'bottom_solve_ms_rank0': b['bottom_solve_ms_rank0'], 'bicg_ms_per_vcycle': b['ms_per_vcycle']}))" >> $out
}
port=29561
for r in 1 2; do
  for s in 1000 1000000000; do
    timeout -k 10 400 env MGIC_HOST_SPIN_US=$s MGIC_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
      --master-addr 127.0.0.1 --master-port $port bench.py --gpus 8 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/spin/b8_$s.log 2>&1 \
      || { tail gpurun_out/spin/b8_$s.log; exit 1; }
    summ "8 ranks spin_us $s" gpurun_out/spin/b8_$s.log
    port=$((port + 1))
    timeout -k 10 300 env MGIC_HOST_SPIN_US=$s python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic > gpurun_out/spin/b1_$s.log 2>&1 || { tail gpurun_out/spin/b1_$s.log; exit 1; }
    summ "1 rank spin_us $s" gpurun_out/spin/b1_$s.log
  done
done
cat $out
echo "session done"
