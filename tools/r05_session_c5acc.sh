#!/bin/bash
# round-5 GPU session c5acc: the mixed V-cycle's last post-smoothing pair
# with phi += e folded into the fp32 two-sweep launch (two launches after the
# coarse correction instead of three) against HEAD before it (gpurun_ab/base0):
# the fp32 / mixed tests (bitwise against oracle/mixed.py), the 4-process
# mixed FMG test, then two interleaved rounds of tools/bench_c5.py (mixed,
# 1024^3, one GPU) and one 8-rank rehearsal.  Measurement only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/c5acc
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_mixed.py tests/test_multiprocess.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/c5acc/tests.log 2>&1; rc=$?
tail -1 gpurun_out/c5acc/tests.log; [ $rc -ne 0 ] && { tail -30 gpurun_out/c5acc/tests.log; exit $rc; }
out=gpurun_out/c5acc/ab.txt; : > $out
for r in 1 2; do
  for v in new base0; do
    L=""; [ $v != new ] && L=gpurun_ab/$v/libmgic.so
    MGIC_LIB_PATH=$L timeout -k 10 400 python tools/bench_c5.py --kinds mixed --vcycles 4 > gpurun_out/c5acc/c5.tmp 2> gpurun_out/c5acc/err.log || { tail gpurun_out/c5acc/err.log; exit 1; }
    echo "$v $(tail -n 1 gpurun_out/c5acc/c5.tmp)" >> $out
  done
done
python3 - $out <<'PY'
import json, sys
for l in open(sys.argv[1]):
    v, j = l.split(" ", 1); d = json.loads(j); m = d["mixed"]
    print(v, "fmg", m["ms_per_fmg"], "vcycle", m["ms_per_vcycle"], "sweep", m.get("fine_sweep_ms_events"), "oracle", d.get("oracle_check", {}).get("bit_identical"), "res", m["residual_max_norm"])
PY
timeout -k 10 600 env MGIC_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29641 tools/bench_c5.py --vcycles 4 --kinds mixed > gpurun_out/c5acc/c5_8.log 2>&1 || { tail gpurun_out/c5acc/c5_8.log; exit 1; }
tail -n 1 gpurun_out/c5acc/c5_8.log
echo "session done"
