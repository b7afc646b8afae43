#!/bin/bash
# builds the two-sweep kernel timing harness (tools/tb2_probe.hip); DEFS adds
# compiler definitions (e.g. a candidate kernel variant)
set -e
cd "$(dirname "$0")"
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -I../mg_ic_code_amd/csrc"
S=../mg_ic_code_amd/csrc/smoother.hip
$H $F ${DEFS:-} -o tb2_probe tb2_probe.hip $S
