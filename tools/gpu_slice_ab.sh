#!/bin/bash
# Executor variant A/B on one box: GPU parity tests and the bench (no CPU leg, no host-staged
# leg) for each executor variant: TONK_AMD_SLICE=512|1024 (8 or 16 B per lane) x
# TONK_AMD_PREFETCH=0|1 (next-batch instruction prefetch), benches twice each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:-ab}
VARS=${2:-"512:0 512:1 1024:0 1024:1"}
mkdir -p "$OUT" && cd "$R" || exit 1
for v in $VARS; do
  TONK_AMD_SLICE=${v%:*} TONK_AMD_PREFETCH=${v#*:} timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/${TAG}_tests_${v%:*}_${v#*:}.log" 2>&1 || exit 1
done
for rep in 1 2; do
  for v in $VARS; do
    TONK_AMD_SLICE=${v%:*} TONK_AMD_PREFETCH=${v#*:} timeout -k 10 120 python bench.py --no-cpu-baseline --no-end-to-end > "$OUT/${TAG}_${v%:*}_${v#*:}_$rep.json" 2> "$OUT/${TAG}_${v%:*}_${v#*:}_$rep.err" || exit 1
  done
done
