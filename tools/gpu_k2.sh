#!/bin/bash
# GPU parity suite, then every bench config once (device time per program is the comparison).
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p $OUT
T=${1:-k2}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "not tonk_unit" > $OUT/${T}_gpu_tests.log 2>&1 || exit 1
run() { local name=$1; shift; timeout -k 10 300 env "$@" > $OUT/${T}_$name.json 2> $OUT/${T}_$name.err || exit 1; }
for i in 1 2; do
  run cfg3_$i python bench.py --no-cpu-baseline --no-end-to-end --no-verify --no-pmc
  run cfg2_$i python bench.py --workload cfg2 --no-cpu-baseline --no-end-to-end --no-verify --no-pmc
done
run cfg4 python bench.py --workload cfg4
run cfg1 python bench.py --workload cfg1
