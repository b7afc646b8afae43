#!/bin/bash
# round-5 GPU session: multi-rank evidence on one GPU at HEAD.  The charged
# 8-GPU share proxy (three runs), then bench.py at 1, 2, 4, 8 ranks with the
# owner-rank bottom-solve timer (profiles/r05_rank_rehearsal.jsonl), with the
# driver's --steps 20 --warmup 5 (WARM); SKIP_PROXY=1 skips the proxy.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
W=${WARM:-5}
: > gpurun_out/proxy_charged.txt
[ -z "${SKIP_PROXY:-}" ] && for r in 1 2 3; do
  timeout -k 10 180 python3 tools/rank_proxy.py --transport ipc --deep 1 --steps 30 --charge 1 >> gpurun_out/proxy_charged.txt 2> gpurun_out/proxy_err.log || { tail gpurun_out/proxy_err.log; exit 1; }
done
cat gpurun_out/proxy_charged.txt
out=gpurun_out/rank_rehearsal.jsonl; : > $out
timeout -k 10 300 python bench.py --steps 20 --warmup $W --no-cpu-baseline --no-traffic > gpurun_out/rb1.log 2>&1 || { tail gpurun_out/rb1.log; exit 1; }
tail -n 1 gpurun_out/rb1.log >> $out
port=29531
for n in 2 4 8; do
  timeout -k 10 400 env MGIC_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n --steps 20 --warmup $W > gpurun_out/rb$n.log 2>&1 \
    || { tail gpurun_out/rb$n.log; exit 1; }
  grep -E '^\{"metric"' gpurun_out/rb$n.log | tail -n 1 >> $out
  port=$((port + 1))
done
python3 -c "
import json
for l in open('$out'):
    d = json.loads(l); b = d.get('bottom', {})
    print(d['n_gpus'], d['value'], d['ms_per_step'], {k: b.get(k) for k in ('bottom_delta_ms', 'bottom_solve_ms_rank0', 'ms_per_vcycle')})
"
echo "session done"
