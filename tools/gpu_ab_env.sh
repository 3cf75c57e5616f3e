#!/bin/bash
# Environment A/B on one box: variants "name:VAR=v,VAR=v" (or "name:" for the defaults), REPS
# interleaved bench runs each, for every workload in WORKLOADS (default cfg3).  The GPU parity
# tests run first (NO_TESTS=1 skips them).  Bench runs skip the CPU leg, the host-staged leg and
# the PMC passes; they keep the byte check of the timed schedule unless NO_VERIFY=1.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:?tag}
shift
REPS=${REPS:-3}
WORKLOADS=${WORKLOADS:-cfg3}
mkdir -p "$OUT" && cd "$R" || exit 1
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${TEST_ARGS} > "$OUT/${TAG}_tests.log" 2>&1 || exit 1
fi
V=""; [ -n "$NO_VERIFY" ] && V="--no-verify"
for rep in $(seq 1 $REPS); do
  for w in $WORKLOADS; do
    for v in "$@"; do
      name=${v%%:*}; spec=${v#*:}
      env ${spec//,/ } timeout -k 10 240 python bench.py --workload $w --no-cpu-baseline --no-end-to-end --no-pmc $V ${BENCH_ARGS} > "$OUT/${TAG}_${w}_${name}_$rep.json" 2> "$OUT/${TAG}_${w}_${name}_$rep.err" || exit 1
    done
  done
done
