#!/bin/bash
# Control-plane A/B/C on the box's cores (no GPU): tools/_ab/cp_a vs cp_b, then cp_a vs cp_c,
# interleaved runs on one core each (tests/native/cp_ab.py).
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p "$OUT"
cd tools/_ab && sed -i 's/"taskset", "-c", "2", //' cp_ab.py
CORE=$(python3 -c "import os; print(sorted(os.sched_getaffinity(0))[len(os.sched_getaffinity(0))//2])")
A=${ARGS:-streams=16 n=49152 step=4096 warm=2}
timeout -k 10 300 taskset -c $CORE python3 cp_ab.py ./cp_a ./cp_b rounds=${ROUNDS:-8} $A > "$OUT/cp_ab_${1:-x}_b.txt" 2>&1 &&
timeout -k 10 300 taskset -c $CORE python3 cp_ab.py ./cp_a ./cp_c rounds=${ROUNDS:-8} $A > "$OUT/cp_ab_${1:-x}_c.txt" 2>&1
cat "$OUT/cp_ab_${1:-x}_b.txt" "$OUT/cp_ab_${1:-x}_c.txt"
