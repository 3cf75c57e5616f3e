#!/bin/bash
# Environment-switch A/B on one box: for each variant "name:VAR=v,VAR=v" run the GPU parity
# tests once, then the bench (no CPU leg, no host-staged leg) twice per variant, interleaved.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:?tag}
shift
mkdir -p "$OUT" && cd "$R" || exit 1
envs() { local spec=${1#*:}; [ "$spec" = "$1" ] && return; echo "${spec//,/ }"; }
for v in "$@"; do
  env $(envs "$v") timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/${TAG}_tests_${v%%:*}.log" 2>&1 || exit 1
done
for rep in 1 2; do
  for v in "$@"; do
    env $(envs "$v") timeout -k 10 180 python bench.py --no-cpu-baseline --no-end-to-end ${BENCH_ARGS} > "$OUT/${TAG}_${v%%:*}_$rep.json" 2> "$OUT/${TAG}_${v%%:*}_$rep.err" || exit 1
  done
done
