#!/bin/bash
# The driver's bench command on this tree, its rocprofv3 kernel trace (+ timed-region average), and cfg2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; TAG=${1:-fb}; mkdir -p "$OUT"; cd "$R" || exit 1
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err" &&
timeout -k 10 600 python bench.py --workload cfg2 --no-cpu-baseline --no-end-to-end > "$OUT/bench_cfg2_$TAG.json" 2> "$OUT/bench_cfg2_$TAG.err" &&
( cd /tmp && export TMPDIR=/tmp &&
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run -- python3 "$R/bench.py" --no-cpu-baseline --no-end-to-end --no-verify --no-pmc > "$OUT/bench_prof_$TAG.json" 2> "$OUT/bench_prof_$TAG.err" &&
  python3 "$R/tools/trace_region.py" "$OUT/prof_$TAG/run_kernel_trace.csv" > "$OUT/trace_region_$TAG.json" )
