#!/bin/bash
# Single-stream lines (bench.py --workload cfg1|cfg4) over programs of several sizes, each under
# the environment settings given ("K=V,K=V" or "-"): usage WORKLOAD "STEPS" SETTING...
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; TAG=${TAG:-ss}; mkdir -p "$OUT"; cd "$R" || exit 1
w=$1; steps=$2; shift 2
for st in $steps; do
  for cfg in "$@"; do
    envs=(); [ "$cfg" != "-" ] && IFS=',' read -ra envs <<< "$cfg"
    f="$OUT/${TAG}_${w}_${st}_$(echo "$cfg" | tr -c 'A-Za-z0-9_\n' '_').json"
    env "${envs[@]}" timeout -k 10 300 python bench.py --workload $w --step $st > "$f" 2> "$f.err" || { echo "$w $st $cfg failed"; tail -5 "$f.err"; exit 1; }
    python3 -c "
import json,sys
d=json.load(open(sys.argv[1])); p=d['per_program']; h=p['host_us_per_program']
print(sys.argv[2], sys.argv[3], d['value'], 'ref', (d.get('cpu_baseline') or {}).get('value'), 'programs', p['programs'], 'launches', p['launches'], 'wall/prog', p['wall_us_per_program'], 'kernel/prog', p['kernel_us_per_program'], 'control', h['control_sum'], 'launch', h.get('launch'))
" "$f" "$st" "$cfg"
  done
done
