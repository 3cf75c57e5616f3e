#!/bin/bash
# Control plane with and without huge pages for glibc's heap (GLIBC_TUNABLES=glibc.malloc.hugetlb=1:
# madvise(MADV_HUGEPAGE) on the arenas), interleaved, on one core of the box; then the two-rank
# rehearsal (tools/gpu_multi_rehearsal.sh).
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
{ cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag; ldd --version | head -1; } > $OUT/thp_env.txt 2>&1
CORE=$(python3 -c "import os; print(sorted(os.sched_getaffinity(0))[len(os.sched_getaffinity(0))//2])")
for i in 1 2 3 4 5 6; do
  echo "base $(taskset -c $CORE tools/_ab/cp_cold streams=16 n=49152 step=4096 warm=2)"
  echo "thp $(GLIBC_TUNABLES=glibc.malloc.hugetlb=1 taskset -c $CORE tools/_ab/cp_cold streams=16 n=49152 step=4096 warm=2)"
done > $OUT/thp_cp.txt 2>&1
bash tools/gpu_multi_rehearsal.sh
