#!/bin/bash
# CU split: its GPU tests, the CU-mask scaling experiment, then the bench at several OFDM CU counts
set -o pipefail
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r4cu2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -k "cu_split or slots" -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 240 python -u tools/experiments/cu_split.py 192 5 > $O/cu_split.jsonl 2> $O/cu_split.err
rc=$?; cat $O/cu_split.jsonl; [ $rc = 0 ] || { tail -5 $O/cu_split.err; exit $rc; }
for a in "0" "160" "128" "192" "160 --slots 3"; do
  t=$(echo $a | tr -d ' -')
  timeout -k 10 200 python bench.py --no-pmc --no-cpu-baseline --no-latency --no-sc16 --no-blocks --no-mplp \
    --steps 10 --warmup 3 --cu-split $a > $O/b_$t.json 2> $O/b_$t.err || { tail -5 $O/b_$t.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_$t.json')); print('split $a', round(d['value']), round(d['ms_per_step'],3), {k: round(s['avg_launch_ms'],4) for k,s in d['stages'].items()})"
done
