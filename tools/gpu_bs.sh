#!/bin/bash
# GPU parity suite, back-substitution over materialized rows A/B (configs[2], [4], [3]), then
# per-item stamps of configs[2] and configs[3].
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p $OUT
T=${1:-bs}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "not tonk_unit" > $OUT/${T}_gpu_tests.log 2>&1 || exit 1
run() { local name=$1; shift; timeout -k 10 300 env "$@" > $OUT/${T}_$name.json 2> $OUT/${T}_$name.err || exit 1; }
for i in 1 2; do
  run cfg2_mat_$i python bench.py --workload cfg2 --no-cpu-baseline --no-end-to-end --no-verify --no-pmc
  run cfg2_old_$i TONK_AMD_BACKSUB_ROWS=100000 python bench.py --workload cfg2 --no-cpu-baseline --no-end-to-end --no-verify --no-pmc
done
run cfg4_mat python bench.py --workload cfg4
run cfg4_old TONK_AMD_BACKSUB_ROWS=100000 python bench.py --workload cfg4
run cfg3_mat python bench.py --no-cpu-baseline --no-end-to-end --no-verify --no-pmc
run cfg3_old TONK_AMD_BACKSUB_ROWS=100000 python bench.py --no-cpu-baseline --no-end-to-end --no-verify --no-pmc
ARGS="--workload cfg2" bash tools/gpu_stamps.sh st_cfg2 9 && bash tools/gpu_stamps.sh st_cfg3 9
