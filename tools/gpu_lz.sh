#!/bin/bash
# Compression step on the GPU: its -m gpu tests (every block through the reference decoder), the
# compress bench line (with the reference compressor's ratio and rate), a rocprofv3 kernel trace,
# and Tonk's unit_tests with the GPU compressor (unit_tests_amd_lz).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:-lz}
mkdir -p "$OUT" && cd "$R" &&
timeout -k 10 300 python -u -m pytest tests/test_compress.py -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/${TAG}_tests.log" 2>&1 &&
timeout -k 10 300 python bench.py --workload compress > "$OUT/${TAG}_bench_compress.json" 2> "$OUT/${TAG}_bench_compress.err" &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_prof" -o run -- python3 "$R/bench.py" --workload compress --no-cpu-baseline > "$OUT/${TAG}_bench_compress_prof.json" 2> "$OUT/${TAG}_bench_compress_prof.err" &&
cd "$R" &&
TONK_AMD_TONK_BINARY=unit_tests_amd_lz timeout -k 10 800 python -u -m pytest tests/test_tonk_unit_tests.py -m gpu -x -q --timeout 900 > "$OUT/${TAG}_tonk_lz.txt" 2>&1
