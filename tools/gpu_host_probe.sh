#!/bin/bash
# Host contention probe (profiling only): the bench three times with its host_env diagnostics,
# and what else runs on the box's CPUs before and after.
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
TAG=${1:-probe}
mkdir -p "$OUT"
{ cat /proc/loadavg; cat /sys/fs/cgroup/cpu.max; cat /sys/fs/cgroup/cpu.stat; ps -eo pid,psr,pcpu,comm --sort=-pcpu | head -25; } > "$OUT/host_before_$TAG.txt" 2>&1
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end --no-pmc --no-verify > "$OUT/hp_${TAG}_$i.json" 2> "$OUT/hp_${TAG}_$i.err" || exit 1
done
{ cat /proc/loadavg; cat /sys/fs/cgroup/cpu.stat; ps -eo pid,psr,pcpu,comm --sort=-pcpu | head -25; } > "$OUT/host_after_$TAG.txt" 2>&1
