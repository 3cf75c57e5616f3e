#!/bin/bash
# Round 6i: compression phases with and without fitted tables (TONK_AMD_LZ_FIT), then the C ABI
# with BAR-written staging and commands: its GPU tests, the capi bench BAR vs pinned (interleaved),
# and Tonk's relink.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:-r06i}
mkdir -p "$OUT" && cd "$R" &&
timeout -k 10 300 python -u -m pytest tests/test_compress.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/${TAG}_lz_tests.log" 2>&1 &&
for f in 1 0; do TONK_AMD_LZ_FIT=$f TONK_AMD_LZ_PROF=1 timeout -k 10 300 python bench.py --workload compress --no-cpu-baseline > "$OUT/${TAG}_lz_fit$f.json" 2> "$OUT/${TAG}_lz_fit$f.err" || exit 1; done &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "capi" --timeout 300 --timeout-method thread > "$OUT/${TAG}_capi_tests.log" 2>&1 &&
for i in 1 2; do for b in 1 0; do TONK_AMD_CAPI_BAR=$b timeout -k 10 300 python bench.py --workload capi > "$OUT/${TAG}_capi_bar${b}_$i.json" 2> "$OUT/${TAG}_capi_bar${b}_$i.err" || exit 1; done; done &&
for b in 1 0; do TONK_AMD_CAPI_WATCH=100 TONK_AMD_CAPI_BAR=$b timeout -k 10 300 python bench.py --workload capi > "$OUT/${TAG}_capi_watch_bar$b.json" 2> "$OUT/${TAG}_capi_watch_bar$b.err" || exit 1; done &&
REPS=1 bash tools/gpu_tonk_rep.sh ${TAG}bar
