#!/bin/bash
# round-5 GPU session hwq: is the 8-rank rehearsal's slow bottom solve the
# one GPU's queue sharing?  The 8-rank bench.py rehearsal with HIP's default
# hardware queues per process and with GPU_MAX_HW_QUEUES=1 (8 processes -> 8
# queues), then the 1-rank run with 7 idle processes holding a GPU context
# beside it.  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/hwq
export TMPDIR=/tmp
out=gpurun_out/hwq/r.jsonl; : > $out
summ() {  # tag log
  grep -E '^\{"metric"' "$2" | tail -n 1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); b = d['bottom']
print(json.dumps({'case': '$1', 'n': d['n_gpus'], 'vcycles': d['value'], 'bottom_delta_ms': b['bottom_delta_ms'], 'bottom_solve_ms_rank0': b['bottom_solve_ms_rank0'], 'bicg_ms_per_vcycle': b['ms_per_vcycle']}))" >> $out
}
port=29551
for q in default 1; do
  E=""; [ $q != default ] && E="GPU_MAX_HW_QUEUES=$q"
  timeout -k 10 400 env $E MGIC_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus 8 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/hwq/b8_$q.log 2>&1 \
    || { tail gpurun_out/hwq/b8_$q.log; exit 1; }
  summ "8 ranks, hw queues $q" gpurun_out/hwq/b8_$q.log
  port=$((port + 1))
done
# 1 rank with 7 idle GPU contexts beside it (each holds a context and sleeps)
pids=""
for i in 1 2 3 4 5 6 7; do
  timeout -k 5 200 python3 -c "import torch, time; torch.zeros(1, device='cuda'); torch.cuda.synchronize(); time.sleep(150)" > /dev/null 2>&1 &
  pids="$pids $!"
done
sleep 20
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic > gpurun_out/hwq/b1_idle7.log 2>&1; rc=$?
kill $pids 2>/dev/null; wait
[ $rc -ne 0 ] && { tail gpurun_out/hwq/b1_idle7.log; exit $rc; }
summ "1 rank + 7 idle contexts" gpurun_out/hwq/b1_idle7.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic > gpurun_out/hwq/b1.log 2>&1 || { tail gpurun_out/hwq/b1.log; exit 1; }
summ "1 rank" gpurun_out/hwq/b1.log
cat $out
echo "session done"
