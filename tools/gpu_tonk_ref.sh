#!/bin/bash
# Tonk's unit_tests with the REFERENCE codec (oracle/_ref/tonk/unit_tests_ref) REPS times on the GPU
# box's CPU quota (no GPU use), to compare its TestBandwidthControl behaviour with the relinks'.
mkdir -p gpurun_out
for i in $(seq 1 ${REPS:-3}); do
  s=$(date +%s)
  u0=$(awk '/usage_usec/{print $2}' /sys/fs/cgroup/cpu.stat 2>/dev/null); t0=$(awk '/throttled_usec/{print $2}' /sys/fs/cgroup/cpu.stat 2>/dev/null)
  timeout -k 10 400 oracle/_ref/tonk/unit_tests_ref < /dev/null > gpurun_out/tonk_ref_$i.log 2>&1
  rc=$?
  u1=$(awk '/usage_usec/{print $2}' /sys/fs/cgroup/cpu.stat 2>/dev/null); t1=$(awk '/throttled_usec/{print $2}' /sys/fs/cgroup/cpu.stat 2>/dev/null)
  echo "ref run $i cgroup cpu_s=$(( (${u1:-0} - ${u0:-0}) / 1000000 )) throttled_ms=$(( (${t1:-0} - ${t0:-0}) / 1000 ))" >> gpurun_out/tonk_ref_summary.txt
  echo "ref run $i rc=$rc seconds=$(( $(date +%s) - s )) $(grep -E 'SUCCESS|Failure' gpurun_out/tonk_ref_$i.log | tr '\n' ' ' | cut -c1-120)" >> gpurun_out/tonk_ref_summary.txt
done
