#!/bin/bash
# Build exp_build/libbase.so from the committed (HEAD, or $1) kernel / C-API / planner sources, for a
# same-box A/B of uncommitted product changes (tools/experiments/gpu_ab.sh TAG base); EXTRA_OBJ: objects
# linked in as well (e.g. a stub of a symbol the current Python binding expects)
set -e
REV=${1:-HEAD}
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
mkdir -p $T/include $T/a/b
cp $R/include/dvbt2ll_hip.h $T/include/
cd $T/a/b
for f in t2_kernels.hip t2_kernels.h t2_capi.cpp t2_plan.cpp t2_plan.h; do git -C $R show $REV:gr-dvbt2ll_amd/csrc/$f > $f; done
git -C $R show $REV:include/dvbt2ll_hip.h > $T/include/dvbt2ll_hip.h
cp -r $R/gr-dvbt2ll_amd/csrc/gen .
H=/opt/rocm/bin/hipcc
$H -x c++ -std=c++17 -O3 -fPIC -ffp-contract=off -D__HIP_PLATFORM_AMD__ -c t2_plan.cpp -o p.o
$H -std=c++17 -O3 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -c t2_kernels.hip -o k.o
$H -std=c++17 -O3 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -c t2_capi.cpp -o c.o
mkdir -p $R/exp_build
$H --offload-arch=gfx950 -shared -fPIC -o $R/exp_build/libbase.so p.o k.o c.o $EXTRA_OBJ
rm -rf $T
echo built $R/exp_build/libbase.so from $REV
