#!/bin/bash
# Sampled control-plane profile on the GPU box's CPUs (no GPU use): tools/_ab/cp_np (non-PIE,
# frame pointers) with cp_bench's SIGPROF sampler; symbols are resolved where it was built.
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p "$OUT"
CORE=$(python3 -c "import os; print(sorted(os.sched_getaffinity(0))[len(os.sched_getaffinity(0))//2])")
timeout -k 10 300 taskset -c $CORE tools/_ab/cp_np ${ARGS:-streams=16 n=8388608 step=4096 warm=2} sample="$OUT/cp_samples_${1:-x}.txt" > "$OUT/cp_prof_${1:-x}.json" 2>&1
cat "$OUT/cp_prof_${1:-x}.json"
