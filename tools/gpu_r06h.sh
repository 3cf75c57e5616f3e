#!/bin/bash
# Round 6h: the compression kernel's faster table choice (tests + bench), then the host-to-VRAM
# coherence probe (host rewrites fine-grained device memory, a polling kernel reads it).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:-r06h}
mkdir -p "$OUT" && cd "$R" &&
timeout -k 10 300 python -u -m pytest tests/test_compress.py -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/${TAG}_lz_tests.log" 2>&1 &&
timeout -k 10 300 python bench.py --workload compress > "$OUT/${TAG}_bench_compress.json" 2> "$OUT/${TAG}_bench_compress.err" &&
TONK_AMD_LZ_PROF=1 timeout -k 10 300 python bench.py --workload compress --no-cpu-baseline > "$OUT/${TAG}_bench_compress_lzprof.json" 2> "$OUT/${TAG}_bench_compress_lzprof.err" &&
timeout -k 10 90 tools/probe/bar_coherence > "$OUT/${TAG}_bar_coherence.txt" 2>&1
