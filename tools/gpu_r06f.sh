#!/bin/bash
# Round 6f: the full -m gpu suite (compression blocks with fitted tables through the reference
# decoder; parked completion waits under the C ABI tests and both Tonk relinks), the compress bench
# line, and the C ABI bench with parked waits on and off.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:-r06f}
mkdir -p "$OUT" && cd "$R" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > "$OUT/${TAG}_gpu_tests.log" 2>&1 &&
timeout -k 10 300 python bench.py --workload compress > "$OUT/${TAG}_bench_compress.json" 2> "$OUT/${TAG}_bench_compress.err" &&
timeout -k 10 300 python bench.py --workload capi > "$OUT/${TAG}_bench_capi_park.json" 2> "$OUT/${TAG}_bench_capi_park.err" &&
TONK_AMD_WAIT_PARK=0 timeout -k 10 300 python bench.py --workload capi > "$OUT/${TAG}_bench_capi_poll.json" 2> "$OUT/${TAG}_bench_capi_poll.err" &&
timeout -k 10 300 python bench.py --workload capi > "$OUT/${TAG}_bench_capi_park2.json" 2> "$OUT/${TAG}_bench_capi_park2.err"
