#!/bin/bash
# Control-plane A/B (CPU only), then single-stream level-count experiments on configs[1]/[4].
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p $OUT
T=${1:-ss2}
ROUNDS=10 bash tools/gpu_cp_ab.sh words || exit 1
run() { local name=$1; shift; timeout -k 10 300 env "$@" > $OUT/${T}_$name.json 2> $OUT/${T}_$name.err || exit 1; }
run c1_def python bench.py --workload cfg1 --no-cpu-baseline
run c1_inl TONK_AMD_EXPAND=4294967295 TONK_AMD_BACKSUB_ROWS=4294967295 python bench.py --workload cfg1 --no-cpu-baseline
run c1_nobs TONK_AMD_BACKSUB_ROWS=4294967295 python bench.py --workload cfg1 --no-cpu-baseline
run c4_def python bench.py --workload cfg4 --no-cpu-baseline
run c4_inl TONK_AMD_EXPAND=4294967295 python bench.py --workload cfg4 --no-cpu-baseline
