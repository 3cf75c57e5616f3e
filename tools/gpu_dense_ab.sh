#!/bin/bash
# -m gpu once, then the driver's bench command with grouped dense rows and without
# (TONK_AMD_NO_DENSE_GROUP=1), in both orders; outputs under gpurun_out/<tag>_*.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; TAG=${1:-dg}; mkdir -p "$OUT"; cd "$R" || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/${TAG}_gpu_tests.log" 2>&1 || { tail -30 "$OUT/${TAG}_gpu_tests.log"; exit 1; }
tail -2 "$OUT/${TAG}_gpu_tests.log"
for v in g n g n; do
  if [ $v = n ]; then export TONK_AMD_NO_DENSE_GROUP=1; else unset TONK_AMD_NO_DENSE_GROUP; fi
  i=$((i+1))
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/${TAG}_${v}${i}.json" 2> "$OUT/${TAG}_${v}${i}.err" || exit 1
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(sys.argv[1][-9:],d['value'],r['avg_launch_us'],r['frac'],r.get('traffic_over_alg'),r.get('alg_bytes_per_launch'),r.get('op_trace_bytes_per_launch'),d['host_ms_per_program']['control_sum'],r['device_busy_frac'])" "$OUT/${TAG}_${v}${i}.json"
done
