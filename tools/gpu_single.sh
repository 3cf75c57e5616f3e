#!/bin/bash
# Single-stream configurations under different program sizes and slot counts (A/B, profiling).
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p $OUT
T=${1:-ss}
run() { local name=$1; shift; timeout -k 10 200 env "$@" > $OUT/${T}_$name.json 2> $OUT/${T}_$name.err || exit 1; }
run c4_512 python bench.py --workload cfg4 --step 512 --no-cpu-baseline
run c4_1024 python bench.py --workload cfg4 --step 1024 --no-cpu-baseline
run c4_256 python bench.py --workload cfg4 --step 256 --no-cpu-baseline
run c4_512_s16 TONK_AMD_SLOTS=16 python bench.py --workload cfg4 --step 512 --no-cpu-baseline
run c4_1024_s16 TONK_AMD_SLOTS=16 python bench.py --workload cfg4 --step 1024 --no-cpu-baseline
run c1_4096 python bench.py --workload cfg1 --step 4096 --no-cpu-baseline
run c1_1024 python bench.py --workload cfg1 --step 1024 --no-cpu-baseline
run c1_512 python bench.py --workload cfg1 --step 512 --no-cpu-baseline
run c1_1024_s16 TONK_AMD_SLOTS=16 python bench.py --workload cfg1 --step 1024 --no-cpu-baseline
