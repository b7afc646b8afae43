#!/bin/bash
# round-4 GPU session b: fast-reciprocal A/B (tb2_probe, old = HEAD~ kernel
# with the fp64 division), GPU suite, bench, interleaved 8-rank rehearsals
# with the coarsest depth distributed / on rank 0, the 8-GPU share proxy
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local name=$1 limit=$2; shift 2
  echo "== $name"
  timeout -k 10 "$limit" "$@" >> "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 2 "gpurun_out/$name.log"
  return $rc
}
for r in 1 2 3; do
  for v in old new; do
    b=tools/tb2_probe; [ $v = old ] && b=tools/tb2_probe_old
    for a in "512 0 0" "512 1 0" "256 0 1"; do
      run probe_$v 60 $b $a || exit $?
    done
  done
done
for r in 1 2; do
  for st in 0 1 5 37 301; do
    run stagger 60 tools/tb2_probe 512 0 0 1 $st || exit $?
  done
done
for st in 0 37; do
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex tb2 -d gpurun_out/pmc_st$st \
    -o p --output-format csv -- tools/tb2_probe 512 0 0 1 $st > gpurun_out/pmc_st$st.log 2>&1 \
    || { echo "pmc stagger $st failed"; exit 1; }
done
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 400 --timeout-method thread || exit $?
run bench 900 python bench.py --steps 20 --warmup 2 || exit $?
for r in 1 2; do
  for a in 0 65; do
    run reh_agg$a 400 env MGIC_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node 8 --master-addr 127.0.0.1 --master-port $((29600 + r * 10 + a % 7)) bench.py \
      --gpus 8 --steps 30 --warmup 2 --agglomerate-below $a --no-roofline-events --no-bottom || exit $?
  done
done
for r in 1 2; do
  run proxy 300 python tools/rank_proxy.py --transport ipc --deep 1 --steps 40 || exit $?
done
echo "session done"
