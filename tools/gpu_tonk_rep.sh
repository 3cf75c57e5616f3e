#!/bin/bash
# Tonk's unit_tests relink (unit_tests_amd) run REPS times (default 2), optionally under
# extra environment (TONK_ENV="K=V ..."), each run's start-up watchdog line and outcome summarised.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-rep}
CG=/sys/fs/cgroup
{ echo "cpu.max: $(cat $CG/cpu.max 2>/dev/null)"; grep Cpus_allowed_list /proc/self/status; } >> gpurun_out/tonk_${TAG}_summary.txt
for i in $(seq 1 ${REPS:-2}); do
  grep -E "usage_usec|nr_throttled|throttled_usec" $CG/cpu.stat 2>/dev/null | tr '\n' ' ' | sed "s/^/before run $i: /" >> gpurun_out/tonk_${TAG}_summary.txt; echo >> gpurun_out/tonk_${TAG}_summary.txt
  env $TONK_ENV TONK_AMD_TONK_BINARY=unit_tests_amd timeout -k 10 800 python -u -m pytest tests/test_tonk_unit_tests.py -m gpu -x -q --timeout 900 > gpurun_out/tonk_${TAG}_$i.txt 2>&1; echo "$TAG run $i rc=$?" >> gpurun_out/tonk_${TAG}_summary.txt
  grep -E "usage_usec|nr_throttled|throttled_usec" $CG/cpu.stat 2>/dev/null | tr '\n' ' ' | sed "s/^/after run $i: /" >> gpurun_out/tonk_${TAG}_summary.txt; echo >> gpurun_out/tonk_${TAG}_summary.txt
  cp gpurun_out/tonk_unit_tests_amd.log gpurun_out/tonk_${TAG}_$i.log
  grep -E "t=5.0s|SUCCESS|Failure|slow executor relaunch|executor stop" gpurun_out/tonk_${TAG}_$i.log | cut -c1-160 >> gpurun_out/tonk_${TAG}_summary.txt
done
