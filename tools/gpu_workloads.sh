#!/bin/bash
# The other bench lines: configs[2] (batched), configs[1] and configs[4] (single streams), the C
# ABI and compression; one JSON line each under gpurun_out/<tag>_<workload>.json.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; TAG=${1:-w}; shift; mkdir -p "$OUT"; cd "$R" || exit 1
for w in ${@:-cfg2 cfg1 cfg4 capi}; do
  timeout -k 10 400 python bench.py --workload $w > "$OUT/${TAG}_$w.json" 2> "$OUT/${TAG}_$w.err" || { echo "$w failed"; tail -5 "$OUT/${TAG}_$w.err"; exit 1; }
  python3 -c "
import json,sys
d=json.load(open(sys.argv[1])); r=d.get('roofline') or {}; c=d.get('cpu_baseline') or {}
print(sys.argv[2], d['value'], d['unit'], 'us/launch', r.get('avg_launch_us'), 'frac', r.get('frac'), 'traffic', r.get('traffic_over_alg'), 'cpu', c.get('value'), d.get('capi',{}).get('encode_us',{}).get('p50'))
" "$OUT/${TAG}_$w.json" $w
done
