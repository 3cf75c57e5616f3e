#!/bin/bash
# After the GPU tests (as the driver's round-end order has it): the headline bench alternating
# the huge-page heap on / off, twice each.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/to_tests.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 240 python bench.py --no-cpu-baseline --no-end-to-end --no-pmc --no-verify > $OUT/to_thp_$i.json 2>/dev/null || exit 1
  TONK_AMD_HUGEPAGE_HEAP=0 timeout -k 10 240 python bench.py --no-cpu-baseline --no-end-to-end --no-pmc --no-verify > $OUT/to_base_$i.json 2>/dev/null || exit 1
done
