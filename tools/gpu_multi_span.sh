#!/bin/bash
# Grouped Cauchy/parity rows: window span limit A/B on configs[3] and configs[2].
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p $OUT
T=${1:-ms}
run() { local name=$1; shift; timeout -k 10 300 env "$@" > $OUT/${T}_$name.json 2> $OUT/${T}_$name.err || exit 1; }
for i in 1 2; do
  for sp in 32 64 256; do
    run cfg3_s${sp}_$i TONK_AMD_MULTI_SPAN=$sp python bench.py --no-cpu-baseline --no-end-to-end --no-verify --no-pmc
    run cfg2_s${sp}_$i TONK_AMD_MULTI_SPAN=$sp python bench.py --workload cfg2 --no-cpu-baseline --no-end-to-end --no-verify --no-pmc
  done
  run cfg3_none_$i TONK_AMD_NO_MULTI=1 python bench.py --no-cpu-baseline --no-end-to-end --no-verify --no-pmc
  run cfg2_none_$i TONK_AMD_NO_MULTI=1 python bench.py --workload cfg2 --no-cpu-baseline --no-end-to-end --no-verify --no-pmc
done
