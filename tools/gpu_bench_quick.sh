#!/bin/bash
# Bench line only (no CPU leg, no end-to-end), N repetitions: quick A/B of host/kernel changes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:-bq}
N=${2:-2}
mkdir -p "$OUT" && cd "$R" || exit 1
for i in $(seq 1 "$N"); do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end > "$OUT/${TAG}_$i.json" 2> "$OUT/${TAG}_$i.err" || exit 1
done
