#!/bin/bash
# Generic round-5 A/B session over library builds gpurun_ab/<v>/libmgic.so
# ("base" = the in-tree library): the two-sweep parity subset on each
# variant, ROUNDS interleaved rounds of [bench_smoother 512^3 / 256^3 unless
# NO_SMOOTHER] + bench.py, then (TRACE=1) a rocprofv3 kernel trace of the
# bench per variant.  VARIANTS="a1 a2" OUT=tag bash tools/ab_session.sh
# Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V="${VARIANTS}"
OUT=${OUT:-ab}
for v in $V; do
  MGIC_LIB_PATH=gpurun_ab/$v/libmgic.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x \
    -k "two_sweep or full_size_512_vcycle or full_size_256 or deep_halo_vcycle or streaming_vcycle or vcycle_iterations" \
    --timeout 200 --timeout-method thread > gpurun_out/pytest_$v.log 2>&1; rc=$?
  echo "$v: $(tail -1 gpurun_out/pytest_$v.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/pytest_$v.log; exit $rc; }
done
out=gpurun_out/${OUT}_ab.txt; : > $out
for r in $(seq ${ROUNDS:-3}); do
  for v in base $V; do
    L=""; [ $v != base ] && L=gpurun_ab/$v/libmgic.so
    if [ -z "${NO_SMOOTHER:-}" ]; then
      MGIC_LIB_PATH=$L timeout -k 10 120 python tools/bench_smoother.py --n 512 --sweeps 8 --tag $v >> $out || exit 1
      MGIC_LIB_PATH=$L timeout -k 10 120 python tools/bench_smoother.py --n 256 --sweeps 8 --tag $v >> $out || exit 1
    fi
    MGIC_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic --no-bottom > gpurun_out/ab_bench.tmp 2> gpurun_out/ab_err.log || { tail gpurun_out/ab_err.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_bench.tmp').read().strip().splitlines()[-1]); print(json.dumps({'variant':'$v','vcycles':d['value'],'ms':d['ms_per_step'],'launch_ms':d['roofline']['avg_launch_ms'],'frac':d['roofline']['frac']}))" >> $out
  done
done
python3 tools/ab_summary.py $out
if [ -n "${TRACE:-}" ]; then
  for v in base $V; do
    if [ $v != base ]; then export MGIC_LIB_PATH=gpurun_ab/$v/libmgic.so; else unset MGIC_LIB_PATH; fi
    TAG=${OUT}_$v BSTEPS=10 bash tools/trace_bench.sh > /dev/null || exit 1
    echo "== $v"; grep -E "k_gsrb_tb2|k_restrict|k_residual|k_prolong" gpurun_out/trace_${OUT}_$v.txt | head -12
  done
fi
echo "session done"
