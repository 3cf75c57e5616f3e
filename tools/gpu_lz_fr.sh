#!/bin/bash
# Compression drop-in (combined batches) under Tonk, and the free-running schedule's stealing A/B.
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p $OUT
T=${1:-lz1}
timeout -k 10 300 python -u -m pytest tests/test_compress.py -x -v -m gpu --timeout 120 --timeout-method thread > $OUT/${T}_compress_tests.log 2>&1 || exit 1
for i in 1 2 3; do
  TONK_AMD_STEAL=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end --no-pmc --no-verify > $OUT/${T}_steal1_$i.json 2>&1 || exit 1
  TONK_AMD_STEAL=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end --no-pmc --no-verify > $OUT/${T}_steal0_$i.json 2>&1 || exit 1
done
TONK_AMD_TONK_BINARY=unit_tests_amd_lz timeout -k 10 900 python -u -m pytest tests/test_tonk_unit_tests.py -x -v -m gpu --timeout 880 --timeout-method thread > $OUT/${T}_tonk_lz.log 2>&1
cp $OUT/tonk_unit_tests.log $OUT/${T}_tonk_lz_unit.log 2>/dev/null
exit 0
