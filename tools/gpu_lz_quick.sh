#!/bin/bash
# Compression step quick pass: its -m gpu tests (every block through the reference decoder), the
# compress bench line twice, and once with per-job phase ticks (TONK_AMD_LZ_PROF=1).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:-lzq}
mkdir -p "$OUT" && cd "$R" &&
timeout -k 10 300 python -u -m pytest tests/test_compress.py -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/${TAG}_tests.log" 2>&1 &&
timeout -k 10 300 python bench.py --workload compress > "$OUT/${TAG}_bench_compress.json" 2> "$OUT/${TAG}_bench_compress.err" &&
timeout -k 10 300 python bench.py --workload compress --no-cpu-baseline > "$OUT/${TAG}_bench_compress2.json" 2> "$OUT/${TAG}_bench_compress2.err" &&
TONK_AMD_LZ_PROF=1 timeout -k 10 300 python bench.py --workload compress --no-cpu-baseline > "$OUT/${TAG}_bench_compress_prof.json" 2> "$OUT/${TAG}_bench_compress_prof.err"
