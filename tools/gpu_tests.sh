#!/bin/bash
# GPU parity tests only (per-test timeouts), then the default bench line without the CPU leg.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:-t}
mkdir -p "$OUT" && cd "$R" &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/${TAG}_tests.log" 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err"
