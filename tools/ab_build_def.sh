#!/bin/bash
# A/B build of the in-tree sources with extra defines for smoother_tb.hip
# (measurement only):  tools/ab_build_def.sh <name> -DX=1 ...
# -> gpurun_ab/<name>/libmgic.so (the other objects from the in-tree build)
set -e
name=$1; shift
cd "$(dirname "$0")/../mg_ic_code_amd/csrc"
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -fvisibility=hidden -I/opt/rocm/include -I. -x hip --offload-arch=gfx950 -munsafe-fp-atomics"
d=../../gpurun_ab/$name; mkdir -p $d
$H $F "$@" -c smoother_tb.hip -o $d/smoother_tb.o
objs=""; for o in kernels smoother transport level op mixed amr capi chf_dropin; do objs="$objs $o.o"; done
$H -shared -fPIC --offload-arch=gfx950 -o $d/libmgic.so $objs $d/smoother_tb.o \
   -L/opt/rocm/lib -lrccl -lamdhip64 -Wl,-rpath,/opt/rocm/lib
rm -f $d/*.o
echo "built $d/libmgic.so ($*)"
