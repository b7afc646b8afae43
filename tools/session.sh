#!/bin/bash
# One GPU session of named steps, each under its own time limit; the first
# failing / timed-out / crashed step ends the session (no retries).  Output
# under gpurun_out/$TAG/.  Replaces the per-session scripts of rounds 4-5.
#   TAG=r06a STEPS="tests smoke bench" bash tools/session.sh
# Steps:
#   tests        pytest -m gpu (PYTEST_K: a -k expression; PYTEST_ARGS: more options)
#   smoke        __graft_entry__.smoke()
#   bench        the default bench.py line (BENCH_ARGS appended)
#   benchq       bench.py without the CPU baseline / PMC passes (BENCH_ARGS)
#   bottom       tools/bench_bottom.py (BOTTOM_ARGS); BOTTOM_ENVS="A=1 B=2,A=0" runs
#                one line per comma-separated env set, interleaved BOTTOM_REPS times
#   ab           bench.py interleaved over AB_ENVS ("X=1,X=0"), AB_REPS rounds (BENCH_ARGS)
#   trace        rocprofv3 kernel trace of benchq -> summary txt + kernel stats csv
#   trace_bottom rocprofv3 kernel trace of bench_bottom.py -> summary + timeline of its tail
#   proxy        tools/rank_proxy.py (PROXY_ARGS)
#   c5           tools/bench_c5.py (C5_ARGS)
#   c5ab         bench_c5.py interleaved over C5_ENVS ("X=1,X=0"), C5_REPS rounds (C5_ARGS)
#   kernels      tools/bench_kernels.py (KERNEL_ARGS)
#   pmc          tools/pmc_kernels.sh (KRE, CMD, PASSES) -> pmc_summary.txt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-s}
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
R=$(pwd)
PYT="python -u -m pytest -x -q -rf --timeout 300 --timeout-method thread"
run() {
  local name=$1 limit=$2; shift 2
  echo "== $name (limit ${limit}s) $(date +%T)"
  timeout -k 10 "$limit" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -n 4 "$O/$name.log"
  return $rc
}
envrun() {  # envrun NAME LIMIT "A=1 B=2" cmd...
  local name=$1 limit=$2 e=$3; shift 3
  # shellcheck disable=SC2086
  run "$name" "$limit" env $e "$@"
}
trace_sum() {  # trace_sum DIR NAME
  local f st
  f=$(find "$1" -name "*kernel_trace.csv" | head -n 1)
  python3 tools/trace_summary.py "$f" > "$O/$2.txt" 2>&1
  python3 -c "import sys; sys.path.insert(0, 'tools'); import trace_summary as t; print('\n'.join(t.timeline('$f', ${TIMELINE:-120})))" > "$O/$2_timeline.txt" 2>&1
  st=$(find "$1" -name "*kernel_stats.csv" | head -n 1)
  [ -n "$st" ] && cp "$st" "$O/$2_kernel_stats.csv"
  rm -rf "$1"
  sed -n 1,25p "$O/$2.txt"
}
BQ="--no-cpu-baseline --no-traffic"
for s in ${STEPS:-tests smoke bench}; do
  case $s in
    tests) if [ -n "${PYTEST_K:-}" ]; then
             run tests 1100 $PYT tests -m gpu -k "$PYTEST_K" ${PYTEST_ARGS:-} || exit $?
           else
             run tests 1100 $PYT tests -m gpu ${PYTEST_ARGS:-} || exit $?
           fi ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench) run bench 900 python bench.py ${BENCH_ARGS:-} || exit $?
           tail -n 1 "$O/bench.log" > "$O/bench_line.json" ;;
    benchq) run benchq 600 python bench.py $BQ ${BENCH_ARGS:-} || exit $?
            tail -n 1 "$O/benchq.log" > "$O/benchq_line.json" ;;
    bottom)
      IFS=',' read -r -a sets <<< "${BOTTOM_ENVS:-MGIC_NONE=1}"
      for rep in $(seq 1 "${BOTTOM_REPS:-1}"); do
        i=0
        for e in "${sets[@]}"; do
          envrun "bottom_${rep}_$i" 300 "$e" python tools/bench_bottom.py ${BOTTOM_ARGS:-} || exit $?
          tail -n 1 "$O/bottom_${rep}_$i.log" >> "$O/bottom.jsonl"
          i=$((i + 1))
        done
      done ;;
    ab)
      IFS=',' read -r -a sets <<< "${AB_ENVS:-MGIC_NONE=1}"
      for rep in $(seq 1 "${AB_REPS:-2}"); do
        i=0
        for e in "${sets[@]}"; do
          envrun "ab_${rep}_$i" 600 "$e" python bench.py $BQ ${BENCH_ARGS:-} || exit $?
          python3 -c "import json,sys; d=json.loads(open('$O/ab_${rep}_$i.log').read().strip().splitlines()[-1]); b=d.get('bottom') or {}; rp=b.get('replay') or {}; print(json.dumps({'env': '$e', 'round': $rep, 'value': d['value'], 'launch_ms': d['roofline']['avg_launch_ms'], 'bottom_ms_per_vcycle': b.get('ms_per_vcycle'), 'bottom_solve_ms': rp.get('ms_per_solve'), 'bottom_iters': rp.get('iterations_per_solve')}))" >> "$O/ab.jsonl"
          i=$((i + 1))
        done
      done
      cat "$O/ab.jsonl" ;;
    trace) run trace 600 rocprofv3 --kernel-trace --stats -d "$R/$O/tr" -o tr --output-format csv \
             -- python3 "$R/bench.py" --steps 5 --warmup 1 $BQ ${BENCH_ARGS:-} || exit $?
           trace_sum "$O/tr" trace ;;
    trace_bottom) run trace_bottom 600 rocprofv3 --kernel-trace --stats -d "$R/$O/tb" -o tb \
                    --output-format csv -- python3 "$R/tools/bench_bottom.py" --rounds 1 \
                    --replays 5 ${BOTTOM_ARGS:-} || exit $?
                  trace_sum "$O/tb" trace_bottom ;;
    proxy) run proxy 600 python tools/rank_proxy.py ${PROXY_ARGS:-} || exit $? ;;
    c5) run c5 600 python tools/bench_c5.py ${C5_ARGS:---vcycles 4} || exit $? ;;
    c5ab)
      IFS=',' read -r -a sets <<< "${C5_ENVS:-MGIC_NONE=1}"
      for rep in $(seq 1 "${C5_REPS:-2}"); do
        i=0
        for e in "${sets[@]}"; do
          envrun "c5_${rep}_$i" 400 "$e" python tools/bench_c5.py ${C5_ARGS:---vcycles 4} || exit $?
          echo "$e $(tail -n 1 "$O/c5_${rep}_$i.log")" >> "$O/c5ab.txt"
          i=$((i + 1))
        done
      done ;;
    kernels) run kernels 600 python tools/bench_kernels.py ${KERNEL_ARGS:-} || exit $? ;;
    pmc) run pmc 1000 bash tools/pmc_kernels.sh || exit $?
         cp gpurun_out/${PMC_OUT:-pmc_k}/summary.txt "$O/pmc_summary.txt" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "session done"
