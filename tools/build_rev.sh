#!/bin/bash
# Build the kernel library of a git revision's t2_kernels.hip (with the current host objects) for same-box A/B:
# tools/build_rev.sh NAME REV  ->  exp_ab/libNAME.so
set -e
cd "$(dirname "$0")/.."
name=$1; rev=$2
C=gr-dvbt2ll_amd/csrc
make -s -C $C
mkdir -p exp_build exp_ab
git show "$rev:$C/t2_kernels.hip" > exp_build/t2_kernels_$name.hip
/opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -I$C -c exp_build/t2_kernels_$name.hip -o exp_build/k_$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o exp_ab/lib$name.so $C/_obj/t2_plan.o exp_build/k_$name.o $C/_obj/t2_capi.o
echo built exp_ab/lib$name.so
