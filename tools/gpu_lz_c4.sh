#!/bin/bash
# Compression (2-wave workgroups, large messages) tests and bench, grouped Cauchy rows A/B on
# cfg2/cfg3, decoder-stress program sizes, then Tonk relinked with the GPU compressor.
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p $OUT
T=${1:-lc}
timeout -k 10 300 python -u -m pytest tests/test_compress.py -x -v -m gpu --timeout 120 --timeout-method thread > $OUT/${T}_compress_tests.log 2>&1 || exit 1
run() { local name=$1; shift; timeout -k 10 300 env "$@" > $OUT/${T}_$name.json 2> $OUT/${T}_$name.err || exit 1; }
run compress python bench.py --workload compress
for i in 1 2; do
  run cfg2_multi_$i python bench.py --workload cfg2 --no-cpu-baseline --no-end-to-end --no-verify --no-pmc
  run cfg2_single_$i TONK_AMD_NO_MULTI=1 python bench.py --workload cfg2 --no-cpu-baseline --no-end-to-end --no-verify --no-pmc
  run cfg3_multi_$i python bench.py --no-cpu-baseline --no-end-to-end --no-verify --no-pmc
  run cfg3_single_$i TONK_AMD_NO_MULTI=1 python bench.py --no-cpu-baseline --no-end-to-end --no-verify --no-pmc
done
for st in 1024 2048 4096; do
  run c4_$st python bench.py --workload cfg4 --step $st
done
TONK_AMD_TONK_BINARY=unit_tests_amd_lz timeout -k 10 600 python -u -m pytest tests/test_tonk_unit_tests.py -x -v -m gpu --timeout 580 --timeout-method thread > $OUT/${T}_tonk_lz.log 2>&1
cp $OUT/tonk_unit_tests.log $OUT/${T}_tonk_lz_unit.log 2>/dev/null
exit 0
