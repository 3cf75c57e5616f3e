#!/bin/bash
# Control-plane cost on the GPU box's CPU (no GPU use): cp_bench per-phase cycles (TAMD_PROF) of
# the headline shape, 4 streams on one pinned core as each bench worker runs them, with the
# decoder's direct eliminations on and off.
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
TAG=${1:-r06}
mkdir -p "$OUT"
make -C tests/native bench > /dev/null 2>&1 || exit 1
for d in 1 0; do
  TONK_AMD_DEC_DIRECT=$d timeout -k 5 120 taskset -c 2 tests/native/_build/cp_bench streams=16 n=262144 step=4096 warm=8 reps=3 > "$OUT/cp_${TAG}_d$d.txt" 2>&1 || exit 1
  TONK_AMD_DEC_DIRECT=$d timeout -k 5 120 taskset -c 2 tests/native/_build/cp_bench_prof streams=16 n=262144 step=4096 warm=8 > "$OUT/cpprof_${TAG}_d$d.txt" 2>&1 || exit 1
done
