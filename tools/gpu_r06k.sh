#!/bin/bash
# Round 6k: compression (tables side by side) tests + A/B; BAR placement matrix; C ABI tests;
# capi bench with BAR (default 7) vs none, interleaved; Tonk relink.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:-r06k}
mkdir -p "$OUT" && cd "$R" &&
timeout -k 10 300 python -u -m pytest tests/test_compress.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/${TAG}_lz_tests.log" 2>&1 &&
for f in 1 0; do TONK_AMD_LZ_FIT=$f TONK_AMD_LZ_PROF=1 timeout -k 10 300 python bench.py --workload compress --no-cpu-baseline > "$OUT/${TAG}_lz_fit$f.json" 2> "$OUT/${TAG}_lz_fit$f.err" || exit 1; done &&
{
for v in "8 16 TONK_AMD_CAPI_BAR=0" "8 16 TONK_AMD_CAPI_BAR=1" "8 16 TONK_AMD_CAPI_BAR=2" "8 16 TONK_AMD_CAPI_BAR=4" "8 16 TONK_AMD_CAPI_BAR=7" "1 16 TONK_AMD_CAPI_BAR=7" "8 16 TONK_AMD_CAPI_BAR=7 TONK_AMD_SERVE=0"; do
  timeout -k 10 300 python tools/capi_digest_check.py $v || exit 1
done
} > "$OUT/${TAG}_bar_matrix.txt" 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "capi" --timeout 300 --timeout-method thread > "$OUT/${TAG}_capi_tests.log" 2>&1 &&
for i in 1 2; do for b in 7 0; do TONK_AMD_CAPI_BAR=$b timeout -k 10 300 python bench.py --workload capi > "$OUT/${TAG}_capi_bar${b}_$i.json" 2> "$OUT/${TAG}_capi_bar${b}_$i.err" || exit 1; done; done &&
for b in 7 0; do TONK_AMD_CAPI_WATCH=100 TONK_AMD_CAPI_BAR=$b timeout -k 10 300 python bench.py --workload capi > "$OUT/${TAG}_capi_watch_bar$b.json" 2> "$OUT/${TAG}_capi_watch_bar$b.err" || exit 1; done &&
REPS=1 bash tools/gpu_tonk_rep.sh ${TAG}bar
