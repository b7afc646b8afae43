#!/bin/bash
# builds the two-sweep kernel probe (diagnostics; see tools/tb2_probe.hip):
# tb2_probe (plain), tb2_probe_st (time stamps), tb2_probe_s<k> (bit mask
# TB2_PROBE_SKIP: 1 no loads, 2 no colour passes, 4 no stores)
set -e
cd "$(dirname "$0")"
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -I../mg_ic_code_amd/csrc"
S=../mg_ic_code_amd/csrc/smoother.hip
D=${DEFS:-}
$H $F $D -o tb2_probe tb2_probe.hip $S &
$H $F $D -DSTAMPS -o tb2_probe_st tb2_probe.hip $S &
$H $F $D -DDRIFT -o tb2_probe_drift tb2_probe.hip $S &
for k in ${SKIPS:-1 2 4}; do $H $F -DTB2_PROBE_SKIP=$k -o tb2_probe_s$k tb2_probe.hip $S & done
wait
