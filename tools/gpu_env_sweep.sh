#!/bin/bash
# The driver's bench command once per environment setting given as arguments (each "K=V,K=V" or
# "-" for none); prints value, us/launch, frac, traffic/alg, op bytes, control ms, device busy.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; TAG=${TAG:-sw}; mkdir -p "$OUT"; cd "$R" || exit 1
i=0
for cfg in "$@"; do
  i=$((i+1))
  envs=(); [ "$cfg" != "-" ] && IFS=',' read -ra envs <<< "$cfg"
  env "${envs[@]}" timeout -k 10 300 python bench.py --gpus 1 --steps ${STEPS:-20} --warmup 5 ${ARGS:-} > "$OUT/${TAG}_$i.json" 2> "$OUT/${TAG}_$i.err" || { echo "run $i failed"; tail -5 "$OUT/${TAG}_$i.err"; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(sys.argv[2],d['value'],r['avg_launch_us'],r['frac'],r.get('traffic_over_alg'),round(r.get('op_trace_bytes_per_launch',0)/1e6,1),d['host_ms_per_program']['control_sum'],r['device_busy_frac'])" "$OUT/${TAG}_$i.json" "$cfg"
done
