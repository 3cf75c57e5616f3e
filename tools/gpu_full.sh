#!/bin/bash
# -m gpu (as the driver runs it), smoke, the driver's bench command, and a rocprofv3 kernel-trace
# --stats pass over the same command; outputs under gpurun_out/<tag>_*.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; TAG=${1:-f}; mkdir -p "$OUT"; cd "$R" || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/${TAG}_gpu_tests.log" 2>&1 || { tail -30 "$OUT/${TAG}_gpu_tests.log"; exit 1; }
tail -1 "$OUT/${TAG}_gpu_tests.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/${TAG}_smoke.log" 2>&1 || { tail -20 "$OUT/${TAG}_smoke.log"; exit 1; }
tail -1 "$OUT/${TAG}_smoke.log"
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err" || { tail -20 "$OUT/${TAG}_bench.err"; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(d['value'],r['avg_launch_us'],r['frac'],r.get('traffic_over_alg'),round(r.get('op_trace_bytes_per_launch',0)/1e6,1),d['host_ms_per_program']['control_sum'],r['device_busy_frac'],d['cpu_baseline']['value'],d['checks']['digests_match'])" "$OUT/${TAG}_bench.json"
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_prof" -o run -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/${TAG}_bench_prof.json" 2> "$OUT/${TAG}_bench_prof.err"
