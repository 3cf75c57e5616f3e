#!/bin/bash
# One bench workload under two environment settings ("K=V,K=V" or "-"), alternated ROUNDS times
# on the same box: usage WORKLOAD A B.  Prints value and the C ABI's encode/decode percentiles.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; TAG=${TAG:-wab}; mkdir -p "$OUT"; cd "$R" || exit 1
w=$1; shift
for r in $(seq 1 ${ROUNDS:-2}); do
  for cfg in "$@"; do
    envs=(); [ "$cfg" != "-" ] && IFS=',' read -ra envs <<< "$cfg"
    f="$OUT/${TAG}_${w}_${r}_$(echo "$cfg" | tr -c 'A-Za-z0-9_\n' '_').json"
    env "${envs[@]}" timeout -k 10 400 python bench.py --workload $w > "$f" 2> "$f.err" || { echo "$cfg failed"; tail -5 "$f.err"; exit 1; }
    python3 -c "
import json,sys
d=json.load(open(sys.argv[1])); c=d.get('capi') or {}
print(sys.argv[2], d['value'], d['unit'], {k: c[k] for k in c if k.endswith('_us')})
" "$f" "$cfg"
  done
done
