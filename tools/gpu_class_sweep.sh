#!/bin/bash
# The driver's bench command under TONK_AMD_CLASS settings (cost class thresholds), RUNS times each,
# interleaved: executor us/launch, frac, traffic.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; TAG=${TAG:-cs}; mkdir -p "$OUT"; cd "$R" || exit 1
for r in $(seq 1 ${RUNS:-2}); do
  for cfg in "$@"; do
    f="$OUT/${TAG}_$(echo "$cfg" | tr -c 'A-Za-z0-9_\n' '_')_$r.json"
    if [ "$cfg" = "-" ]; then e=(); else e=("TONK_AMD_CLASS=$cfg"); fi
    env "${e[@]}" timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline ${ARGS:-} > "$f" 2> "$f.err" || { echo "$cfg failed"; tail -5 "$f.err"; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(sys.argv[2],d['value'],r['avg_launch_us'],r['frac'],r.get('traffic_over_alg'))" "$f" "$cfg"
  done
done
