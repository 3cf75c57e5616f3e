#!/bin/bash
# GPU parity suite, then the bench configs after the Cauchy-table / rolling-parity kernel change,
# with back-substitution thresholds and shared combines as A/B knobs.
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p $OUT
T=${1:-k1}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "not tonk_unit" > $OUT/${T}_gpu_tests.log 2>&1 || exit 1
run() { local name=$1; shift; timeout -k 10 300 env "$@" > $OUT/${T}_$name.json 2> $OUT/${T}_$name.err || exit 1; }
for i in 1 2; do
  run cfg3_$i python bench.py --no-cpu-baseline --no-end-to-end --no-verify --no-pmc
  run cfg2_$i python bench.py --workload cfg2 --no-cpu-baseline --no-end-to-end --no-verify --no-pmc
done
run cfg3_bs2 TONK_AMD_BACKSUB_ROWS=2 python bench.py --no-cpu-baseline --no-end-to-end --no-verify --no-pmc
run cfg2_bs2 TONK_AMD_BACKSUB_ROWS=2 python bench.py --workload cfg2 --no-cpu-baseline --no-end-to-end --no-verify --no-pmc
run cfg3_share TONK_AMD_SHARE=1 python bench.py --no-cpu-baseline --no-end-to-end --no-verify --no-pmc
run cfg2_share TONK_AMD_SHARE=1 python bench.py --workload cfg2 --no-cpu-baseline --no-end-to-end --no-verify --no-pmc
run cfg4 python bench.py --workload cfg4
ARGS="--workload cfg2" bash tools/gpu_stamps.sh st2_cfg2 9 && bash tools/gpu_stamps.sh st2_cfg3 9
