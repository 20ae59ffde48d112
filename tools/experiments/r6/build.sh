#!/bin/bash
# builds every r6 map-phase probe library into exp_ab/ (tools/exp_variant.py, then moved: exp_build/ is gpurun-ignored)
set -e
cd "$(dirname "$0")/../../.."
mkdir -p exp_ab
for f in "$@"; do
  n=$(basename $f .py)
  python tools/exp_variant.py $n tools/experiments/r6/$n.py > /dev/null
  cp exp_build/lib$n.so exp_ab/lib$n.so
  echo built $n
done
