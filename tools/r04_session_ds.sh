#!/bin/bash
# round-4 GPU session ds: LDS read merging in the two-sweep kernel.  hipcc
# merges the pass's xm / xp (adjacent 8-B elements) and ym / yp, zm / zp
# reads into ds_read2_b64, which the LDS services at half the rate of two
# ds_read_b64.  Variants (gpurun_ab/<name>, tools/ab_build.sh): xp = xp read
# from its own laundered lane offset (no xm / xp merge); nl = the
# load-store optimiser off for the sweep kernels (no ym / yp, zm / zp merge);
# xpnl = both.  Two-sweep parity tests on xpnl, then the interleaved A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in xpnl xp nl; do
  MGIC_LIB_PATH=gpurun_ab/$v/libmgic.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -rf -k "two_sweep or vcycle or fused" --timeout 200 --timeout-method thread > gpurun_out/pytest_$v.log 2>&1; rc=$?
  echo "$v: $(tail -1 gpurun_out/pytest_$v.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/pytest_$v.log; exit $rc; }
done
: > gpurun_out/ab.jsonl
VARIANTS="base xpnl xp nl" ROUNDS=3 bash tools/ab_run.sh || exit 1
echo "session done"
