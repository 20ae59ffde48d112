# OFDM phase probes of several OFDM_VARIANT=8 builds: VARIANTS="p0 p1" bash tools/ofdm_phases_ab.sh
set -o pipefail
mkdir -p gpurun_out
LIB=gr-dvbt2ll_amd/dvbt2ll/libdvbt2ll_hip.so
cp $LIB /tmp/prod.so
for v in $VARIANTS; do
  cp exp_build/lib$v.so $LIB
  timeout -k 10 120 python tools/ofdm_phases.py ${CFG:-cfg3} > gpurun_out/phases_$v.txt 2>&1 || { echo "variant $v failed"; break; }
  echo "== $v"; grep -v amdgpu.ids gpurun_out/phases_$v.txt
done
cp /tmp/prod.so $LIB
