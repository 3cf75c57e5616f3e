#!/bin/bash
# The A/B runner (usage: tools/gpu_ab.sh TAG variant...) -- mixed A/B on one box: variants "name:LIB:VAR=v,VAR=v" (LIB = library file in tonk_amd/, or
# "-" for the default), REPS interleaved bench runs each (no CPU leg, no host-staged leg).  The
# GPU parity tests run first with the default library; the box's CPU limits are recorded.
# BENCH_ARGS: extra bench.py arguments (e.g. --workload cfg2).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:?tag}
shift
REPS=${REPS:-4}
mkdir -p "$OUT" && cd "$R" || exit 1
{ nproc; cat /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpuset.cpus.effective 2>&1; python3 -c "import os; print(len(os.sched_getaffinity(0)))"; } > "$OUT/${TAG}_cpu.txt" 2>&1
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${TEST_ARGS} > "$OUT/${TAG}_tests.log" 2>&1 || exit 1
fi
for rep in $(seq 1 $REPS); do
  for v in "$@"; do
    name=${v%%:*}; rest=${v#*:}; lib=${rest%%:*}; spec=${rest#*:}; [ "$spec" = "$rest" ] && spec=""
    e=""; [ "$lib" != "-" ] && e="TONK_AMD_LIB=$lib"
    env $e ${spec//,/ } timeout -k 10 180 python bench.py --no-cpu-baseline --no-end-to-end --steps 30 ${BENCH_ARGS} > "$OUT/${TAG}_${name}_$rep.json" 2> "$OUT/${TAG}_${name}_$rep.err" || exit 1
  done
done
