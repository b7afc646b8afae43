#!/bin/bash
# One GPU session: parity tests, smoke, a short bench.  Each GPU step has its
# own time limit; a crash / abort / timeout ends the session (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=${STEPS:-10}
run() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
run pytest_gpu 900 python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS:-}
rc=$?
if [ $rc -gt 1 ]; then echo "stopping: pytest rc=$rc"; exit $rc; fi
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
run bench 900 python bench.py --steps "$STEPS" --warmup 2 ${BENCH_ARGS:-} || exit $?
tail -n 1 gpurun_out/bench.log
