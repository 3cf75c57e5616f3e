#!/bin/bash
# Control-plane A/B on the GPU box's CPUs (no GPU use): tools/_ab/cp_a vs cp_b, interleaved.
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p "$OUT"
cd tools/_ab && sed -i 's/"taskset", "-c", "2", //' cp_ab.py
CORE=$(python3 -c "import os; print(sorted(os.sched_getaffinity(0))[len(os.sched_getaffinity(0))//2])")
timeout -k 10 300 taskset -c $CORE python3 cp_ab.py ./cp_a ./cp_b rounds=${ROUNDS:-10} ${ARGS:-streams=16 n=49152 step=4096 warm=2} > "$OUT/cp_ab_${1:-x}.txt" 2>&1
cat "$OUT/cp_ab_${1:-x}.txt"
