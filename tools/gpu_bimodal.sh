#!/bin/bash
# The driver's bench command RUNS times per setting ("K=V,K=V" or "-"): per run the executor's
# us/launch and where the arena landed (is the 134 / 141 us split per process?).
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; TAG=${TAG:-bm}; mkdir -p "$OUT"; cd "$R" || exit 1
for cfg in "$@"; do
  envs=(); [ "$cfg" != "-" ] && IFS=',' read -ra envs <<< "$cfg"
  for r in $(seq 1 ${RUNS:-4}); do
    f="$OUT/${TAG}_$(echo "$cfg" | tr -c 'A-Za-z0-9_\n' '_')_$r.json"
    env TONK_AMD_DEBUG_ALLOC=1 "${envs[@]}" timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$f" 2> "$f.err" || { echo "$cfg failed"; tail -5 "$f.err"; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(sys.argv[2],d['value'],r['avg_launch_us'],r.get('traffic_over_alg'),r['device_busy_frac'])" "$f" "$cfg" | tr '\n' ' '
    grep -o "arena 0x[0-9a-f]*" "$f.err" | head -1
  done
done
