set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for C in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  n=$(echo $C | tr ' ' '_')
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex tb2 -d gpurun_out/pmc/$n -o p --output-format csv -- tools/tb2_probe 512 0 > gpurun_out/pmc/$n.log 2>&1 || { echo "pmc $C failed"; exit 1; }
done
echo ok
