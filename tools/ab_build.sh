#!/bin/bash
# A/B builds of the sweep kernels (measurement only): each argument is
# name:DEFS (DEFS comma-separated, e.g. rot:-DTB2_ROT=1); builds
# gpurun_ab/<name>/libmgic.so from the in-tree objects with smoother_tb.hip
# and smoother.hip recompiled under DEFS.  Select with MGIC_LIB_PATH.
set -e
cd "$(dirname "$0")/../mg_ic_code_amd/csrc"
make -s -j8 ../libmgic.so
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -fvisibility=hidden -I/opt/rocm/include -x hip --offload-arch=gfx950 -munsafe-fp-atomics"
for spec in "$@"; do
  (
    name=${spec%%:*}; defs=${spec#*:}; defs=${defs//,/ }
    d=../../gpurun_ab/$name; mkdir -p $d
    $H $F $defs -c smoother_tb.hip -o $d/smoother_tb.o
    $H $F $defs -c smoother.hip -o $d/smoother.o
    objs=""; for o in kernels transport level op mixed amr capi chf_dropin; do objs="$objs $o.o"; done
    $H -shared -fPIC --offload-arch=gfx950 -o $d/libmgic.so $objs $d/smoother_tb.o $d/smoother.o \
       -L/opt/rocm/lib -lrccl -lamdhip64 -Wl,-rpath,/opt/rocm/lib
    echo "built $d/libmgic.so ($defs)"
  ) &
done
wait
