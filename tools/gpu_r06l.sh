#!/bin/bash
# Round 6l: compression sub-phases with and without fitted tables.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:-r06l}
mkdir -p "$OUT" && cd "$R" &&
timeout -k 10 300 python -u -m pytest tests/test_compress.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/${TAG}_lz_tests.log" 2>&1 &&
for f in 1 0; do TONK_AMD_LZ_FIT=$f TONK_AMD_LZ_PROF=1 timeout -k 10 300 python bench.py --workload compress --no-cpu-baseline > "$OUT/${TAG}_lz_fit$f.json" 2> "$OUT/${TAG}_lz_fit$f.err" || exit 1; done
