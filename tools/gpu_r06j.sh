#!/bin/bash
# Round 6j: BAR staging under concurrency (which path differs), and the compression chain fix.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:-r06j}
mkdir -p "$OUT" && cd "$R" &&
{
for v in "8 16 TONK_AMD_CAPI_BAR=0" "8 16 TONK_AMD_CAPI_BAR=7" "1 16 TONK_AMD_CAPI_BAR=7" "8 16 TONK_AMD_CAPI_BAR=1" "8 16 TONK_AMD_CAPI_BAR=2" "8 16 TONK_AMD_CAPI_BAR=4" "8 16 TONK_AMD_CAPI_BAR=7 TONK_AMD_SERVE=0"; do
  timeout -k 10 300 python tools/capi_digest_check.py $v || exit 1
done
} > "$OUT/${TAG}_bar_matrix.txt" 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_compress.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/${TAG}_lz_tests.log" 2>&1 &&
for f in 1 0; do TONK_AMD_LZ_FIT=$f TONK_AMD_LZ_PROF=1 timeout -k 10 300 python bench.py --workload compress --no-cpu-baseline > "$OUT/${TAG}_lz_fit$f.json" 2> "$OUT/${TAG}_lz_fit$f.err" || exit 1; done
