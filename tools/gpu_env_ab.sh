#!/bin/bash
# A/B of environment settings on the default bench (short lines, no PMC / CPU leg / byte check):
# VARIANTS="NAME=VAL NAME=VAL ..." (use "-" for the default), REPS rounds, interleaved.
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-envab}
for i in $(seq 1 ${REPS:-2}); do
  for v in $VARIANTS; do
    n=$(echo "$v" | tr '=/' '__')
    if [ "$v" = "-" ]; then e=""; else e="$v"; fi
    env $e timeout -k 10 300 python bench.py ${BENCH_ARGS} --no-cpu-baseline --no-end-to-end --no-pmc --no-verify > "gpurun_out/${TAG}_${n}_$i.json" 2> "gpurun_out/${TAG}_${n}_$i.err" || exit 1
  done
done
