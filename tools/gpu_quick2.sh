#!/bin/bash
# quick GPU iteration: parity tests, 32K phase probe, bench without PMC / CPU baseline
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-q}
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$O/pytest.log" 2>&1 && tail -2 "$O/pytest.log" \
  && bash tools/gpu_o32_phases.sh cfg3 > "$O/phases.txt" 2>&1 && cat "$O/phases.txt" \
  && timeout -k 10 300 python -u bench.py --no-pmc --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err" \
  && python -c "
import json;d=json.load(open('$O/bench.json'))
print('value', round(d['value']), 'serial', round(d['serial_1_stream']['value']), 'ms', round(d['ms_per_step'],4))
print({k: round(v['avg_launch_ms'],4) for k,v in d['stages'].items()})
print('sc16', round(d['iq_sc16_x0.2']['value']), 'lat', d['latency_1_frame']['median_ms'])"
