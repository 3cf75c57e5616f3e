#!/bin/bash
# Single-stream cold start: the control plane's first program on a fresh process (cp_bench,
# CPU only, on one core of the box) with glibc's default heap and with mmap/trim thresholds
# raised (no fresh pages per large vector growth), then the cfg1 / cfg4 bench lines both ways.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
CORE=$(python3 -c "import os; print(sorted(os.sched_getaffinity(0))[len(os.sched_getaffinity(0))//2])")
M="MALLOC_MMAP_THRESHOLD_=268435456 MALLOC_TRIM_THRESHOLD_=1073741824 MALLOC_TOP_PAD_=67108864"
{
for i in 1 2 3 4 5 6; do
  echo "cold $(taskset -c $CORE tools/_ab/cp_cold streams=1 n=4096 step=4096 warm=0)"
  echo "coldM $(env $M taskset -c $CORE tools/_ab/cp_cold streams=1 n=4096 step=4096 warm=0)"
  echo "warm $(taskset -c $CORE tools/_ab/cp_cold streams=1 n=16384 step=4096 warm=2)"
done
} > $OUT/cold_cp.txt 2>&1
for i in 1 2; do
  timeout -k 10 200 python bench.py --workload cfg1 --no-cpu-baseline > $OUT/cold_cfg1_base_$i.json 2>/dev/null || exit 1
  env $M timeout -k 10 200 python bench.py --workload cfg1 --no-cpu-baseline > $OUT/cold_cfg1_m_$i.json 2>/dev/null || exit 1
  timeout -k 10 200 python bench.py --workload cfg4 --no-cpu-baseline > $OUT/cold_cfg4_base_$i.json 2>/dev/null || exit 1
  env $M timeout -k 10 200 python bench.py --workload cfg4 --no-cpu-baseline > $OUT/cold_cfg4_m_$i.json 2>/dev/null || exit 1
done
