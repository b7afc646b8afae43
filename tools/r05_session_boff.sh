#!/bin/bash
# round-5 GPU session boff: polling back-off of the peer-mapped transport's
# waits (MGIC_IPC_BACKOFF, default 1) against the 64-clock poll
# (gpurun_ab/nobo): the multi-process tests, then two interleaved rounds of
# the 8-rank one-GPU rehearsal (bench.py with the owner-rank bottom timer)
# and the 8-GPU share proxy.  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/boff
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_multiprocess.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/boff/mp.log 2>&1; rc=$?
tail -1 gpurun_out/boff/mp.log; [ $rc -ne 0 ] && { tail -30 gpurun_out/boff/mp.log; exit $rc; }
out=gpurun_out/boff/r8.jsonl; : > $out
port=29541
for r in 1 2; do
  for v in base nobo; do
    L=""; [ $v != base ] && L=gpurun_ab/$v/libmgic.so
    timeout -k 10 400 env MGIC_LIB_PATH=$L MGIC_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
      --master-addr 127.0.0.1 --master-port $port bench.py --gpus 8 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/boff/b8_$v.log 2>&1 \
      || { tail gpurun_out/boff/b8_$v.log; exit 1; }
    port=$((port + 1))
    grep -E '^\{"metric"' gpurun_out/boff/b8_$v.log | tail -n 1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); b = d['bottom']
print(json.dumps({'variant': '$v', 'n': d['n_gpus'], 'vcycles': d['value'], 'ms': d['ms_per_step'], 'bottom_delta_ms': b['bottom_delta_ms'], 'bottom_solve_ms_rank0': b['bottom_solve_ms_rank0'], 'bicg_ms_per_vcycle': b['ms_per_vcycle']}))" >> $out
    MGIC_LIB_PATH=$L timeout -k 10 180 python3 tools/rank_proxy.py --transport ipc --deep 1 --steps 30 --charge 1 > gpurun_out/boff/p.tmp 2>> gpurun_out/boff/p_err.log || { tail gpurun_out/boff/p_err.log; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/boff/p.tmp')); print(json.dumps({'variant': '$v', 'proxy_ms': d['ms_per_vcycle'], 'charged_ms': d['charged_ms_per_vcycle']}))" >> $out
  done
done
cat $out
echo "session done"
