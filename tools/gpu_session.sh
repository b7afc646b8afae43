#!/bin/bash
# One GPU session of named steps, each under its own time limit; the first
# failing / timed-out / crashed step ends the session (no retries).
#   STEPS_TO_RUN="ipc_tests mp_tests pytest_gpu smoke bench bench2" bash tools/gpu_session.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PYT="python -u -m pytest -x -q -rf --timeout 300 --timeout-method thread"
run() {
  local name=$1 limit=$2; shift 2
  echo "== $name (limit ${limit}s)"
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -n 3 "gpurun_out/$name.log"
  return $rc
}
for s in ${STEPS_TO_RUN:-pytest_gpu smoke bench}; do
  case $s in
    ipc_tests) run ipc_tests 600 $PYT tests/test_gpu_parity.py -m gpu -k "self_messages or deep_halo or eight_boxes" || exit $? ;;
    mp_tests) run mp_tests 600 $PYT tests/test_multiprocess.py -m gpu || exit $? ;;
    pytest_gpu) run pytest_gpu 1200 $PYT tests -m gpu ${PYTEST_ARGS:-} || exit $? ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench) run bench 900 python bench.py --steps "${BSTEPS:-20}" --warmup 2 ${BENCH_ARGS:-} || exit $?
           tail -n 1 gpurun_out/bench.log > gpurun_out/bench_line.json ;;
    bench2) run bench2 600 env MGIC_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 \
              --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 \
              --steps "${BSTEPS:-20}" --warmup 2 ${BENCH2_ARGS:-} || exit $? ;;
    bench4) run bench4 600 env MGIC_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 \
              --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 4 \
              --steps "${BSTEPS:-20}" --warmup 2 ${BENCH2_ARGS:-} || exit $? ;;
    bench8) run bench8 600 env MGIC_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 \
              --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 8 \
              --steps "${BSTEPS:-20}" --warmup 2 ${BENCH2_ARGS:-} || exit $? ;;
    bench8_agg0) run bench8_agg0 600 env MGIC_BENCH_DEVICE=0 python -m torch.distributed.run \
              --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29520 bench.py \
              --gpus 8 --steps "${BSTEPS:-20}" --warmup 2 --agglomerate-below 0 ${BENCH2_ARGS:-} || exit $? ;;
    bench8_agg65) run bench8_agg65 600 env MGIC_BENCH_DEVICE=0 python -m torch.distributed.run \
              --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29521 bench.py \
              --gpus 8 --steps "${BSTEPS:-20}" --warmup 2 --agglomerate-below 65 ${BENCH2_ARGS:-} || exit $? ;;
    proxy) run proxy 600 python tools/rank_proxy.py ${PROXY_ARGS:-} || exit $? ;;
    c5) run c5 600 python tools/bench_c5.py --vcycles 4 || exit $? ;;
    c5_8) run c5_8 900 env MGIC_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 \
              --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29522 tools/bench_c5.py \
              --vcycles 4 || exit $? ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "session done"
