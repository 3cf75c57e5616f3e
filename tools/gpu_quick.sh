#!/bin/bash
# Quick GPU iteration: parity tests, the bench line (no CPU leg) and a rocprofv3 kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:-q}
mkdir -p "$OUT" && cd "$R" &&
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/${TAG}_tests.log" 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err" &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_prof" -o run -- python3 "$R/bench.py" --no-cpu-baseline > "$OUT/${TAG}_bench_prof.json" 2> "$OUT/${TAG}_bench_prof.err"
