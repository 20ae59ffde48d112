# Build an experiment variant of the kernel library: tools/build_variant.sh <name> <-Dflags...>
# -> exp_build/lib<name>.so (same host objects as the product build; only t2_kernels.hip differs)
set -e
name=$1; shift
C=gr-dvbt2ll_amd/csrc
make -s -C $C
mkdir -p exp_build
/opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics "$@" -c $C/t2_kernels.hip -o exp_build/k_$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o exp_build/lib$name.so $C/_obj/t2_plan.o exp_build/k_$name.o $C/_obj/t2_capi.o
echo built exp_build/lib$name.so
