#!/bin/bash
# Environment-switch A/B on one box, REPS interleaved bench runs per variant (no CPU leg, no
# host-staged leg); the GPU parity tests run once first with the default environment.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:?tag}
shift
REPS=${REPS:-4}
mkdir -p "$OUT" && cd "$R" || exit 1
envs() { local spec=${1#*:}; [ "$spec" = "$1" ] && return; echo "${spec//,/ }"; }
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/${TAG}_tests.log" 2>&1 || exit 1
fi
for rep in $(seq 1 $REPS); do
  for v in "$@"; do
    env $(envs "$v") timeout -k 10 180 python bench.py --no-cpu-baseline --no-end-to-end ${BENCH_ARGS} > "$OUT/${TAG}_${v%%:*}_$rep.json" 2> "$OUT/${TAG}_${v%%:*}_$rep.err" || exit 1
  done
done
