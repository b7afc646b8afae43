#!/bin/bash
# round-4 GPU session d: FETCH_SIZE and time of the 512^3 plain two-sweep
# launch (tools/tb2_probe) against the z chunk (MGIC_TB2_KC): how much of the
# over-fetch is neighbour drift (one long chunk: all tiles start together and
# drift apart) vs round / band borders
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/kc
export TMPDIR=/tmp
R=$(pwd)
for kc in 512 256 128 64 32; do
  MGIC_TB2_KC=$kc timeout -k 10 60 tools/tb2_probe 512 0 0 1 >> gpurun_out/kc/time.log 2>&1 || exit 1
  MGIC_TB2_KC=$kc timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex tb2 -d "$R/gpurun_out/kc/f$kc" -o c --output-format csv -- "$R/tools/tb2_probe" 512 0 0 1 > gpurun_out/kc/f$kc.log 2>&1 || { echo "pmc $kc failed"; exit 1; }
  MGIC_TB2_KC=$kc timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex tb2 -d "$R/gpurun_out/kc/h$kc" -o c --output-format csv -- "$R/tools/tb2_probe" 512 0 0 1 > gpurun_out/kc/h$kc.log 2>&1 || { echo "pmc hit $kc failed"; exit 1; }
  python3 - <<PY
import csv,glob
out={}
for d in ("f$kc","h$kc"):
    for f in glob.glob("gpurun_out/kc/"+d+"/*counter_collection.csv"):
        rows=list(csv.DictReader(open(f)))
        for r in rows: out.setdefault(r["Counter_Name"],[]).append(float(r["Counter_Value"]))
print("kc=$kc", {k: round(sum(v)/len(v)) for k,v in out.items()}, "fetch GB", round(sum(out["FETCH_SIZE"])/len(out["FETCH_SIZE"])*2048/1e9,3))
PY
done
cat gpurun_out/kc/time.log
# neighbour-throttle experiment (tools/abtmp/smoother_tb_thr.hip, THR_D groups of tolerance)
for r in 1 2 3; do
  for b in tb2_probe tb2_probe_thr0 tb2_probe_thr1 tb2_probe_thr2; do
    echo -n "$b " >> gpurun_out/kc/thr.log
    timeout -k 10 60 tools/$b 512 0 0 1 >> gpurun_out/kc/thr.log 2>&1 || exit 1
  done
done
for b in tb2_probe_thr1 tb2_probe_thr2; do
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex tb2 -d "$R/gpurun_out/kc/$b" -o c --output-format csv -- "$R/tools/$b" 512 0 0 1 > gpurun_out/kc/$b.log 2>&1 || { echo "pmc $b failed"; exit 1; }
  python3 -c "
import csv,glob
v=[float(r['Counter_Value']) for f in glob.glob('gpurun_out/kc/$b/*counter_collection.csv') for r in csv.DictReader(open(f))]
print('$b fetch GB', round(sum(v)/len(v)*2048/1e9,3))"
done
cat gpurun_out/kc/thr.log
echo "session done"
