#!/bin/bash
# A/B build from another revision of the sweep kernels (measurement only):
#   tools/ab_build_rev.sh <git-rev> <name>
# builds gpurun_ab/<name>/libmgic.so from the in-tree objects with
# smoother_tb.hip and smoother.hip taken from <git-rev>.
set -e
rev=$1; name=$2
cd "$(dirname "$0")/../mg_ic_code_amd/csrc"
make -s -j8 ../libmgic.so
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -fvisibility=hidden -I/opt/rocm/include -I. -x hip --offload-arch=gfx950 -munsafe-fp-atomics"
d=../../gpurun_ab/$name; mkdir -p $d
for f in smoother_tb smoother; do
  git show "$rev:mg_ic_code_amd/csrc/$f.hip" > $d/$f.hip
  $H $F -c $d/$f.hip -o $d/$f.o
done
objs=""; for o in kernels transport level op mixed amr capi chf_dropin; do objs="$objs $o.o"; done
$H -shared -fPIC --offload-arch=gfx950 -o $d/libmgic.so $objs $d/smoother_tb.o $d/smoother.o \
   -L/opt/rocm/lib -lrccl -lamdhip64 -Wl,-rpath,/opt/rocm/lib
rm -f $d/*.hip $d/*.o
echo "built $d/libmgic.so (sweep kernels of $rev)"
