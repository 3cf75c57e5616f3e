#!/bin/bash
# GPU parity suite, then grouped Cauchy rows (MULTI runs) against one op per row on cfg2/cfg3,
# then the single-stream configurations under the free-running schedule against passes.
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p $OUT
T=${1:-ca}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/${T}_gpu_tests.log 2>&1 || exit 1
run() { local name=$1; shift; timeout -k 10 300 env "$@" > $OUT/${T}_$name.json 2> $OUT/${T}_$name.err || exit 1; }
for i in 1 2; do
  run cfg2_multi_$i python bench.py --workload cfg2 --no-cpu-baseline --no-end-to-end --no-verify
  run cfg2_single_$i TONK_AMD_NO_MULTI=1 python bench.py --workload cfg2 --no-cpu-baseline --no-end-to-end --no-verify
done
run cfg3_multi python bench.py --no-cpu-baseline --no-end-to-end --no-verify
run cfg3_single TONK_AMD_NO_MULTI=1 python bench.py --no-cpu-baseline --no-end-to-end --no-verify
for st in 512 1024; do
  run c4_fr_$st python bench.py --workload cfg4 --step $st --no-cpu-baseline
  run c4_pass_$st TONK_AMD_PASSES=1 python bench.py --workload cfg4 --step $st --no-cpu-baseline
  run c1_fr_$st python bench.py --workload cfg1 --step $st --no-cpu-baseline
  run c1_pass_$st TONK_AMD_PASSES=1 python bench.py --workload cfg1 --step $st --no-cpu-baseline
done
exit 0
