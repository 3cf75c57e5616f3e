#!/bin/bash
# Round 6g: compression (tests + bench, faster table choice), C ABI waits with a yield phase before
# parking (bench park vs poll, interleaved), Tonk's relink, then the host-writable device memory
# probe (last: a host pointer that is not mapped ends the probe with SIGSEGV, nothing else).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:-r06g}
mkdir -p "$OUT" && cd "$R" &&
timeout -k 10 300 python -u -m pytest tests/test_compress.py -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/${TAG}_lz_tests.log" 2>&1 &&
timeout -k 10 300 python bench.py --workload compress > "$OUT/${TAG}_bench_compress.json" 2> "$OUT/${TAG}_bench_compress.err" &&
timeout -k 10 300 python bench.py --workload capi > "$OUT/${TAG}_capi_park1.json" 2> "$OUT/${TAG}_capi_park1.err" &&
TONK_AMD_WAIT_PARK=0 timeout -k 10 300 python bench.py --workload capi > "$OUT/${TAG}_capi_poll1.json" 2> "$OUT/${TAG}_capi_poll1.err" &&
timeout -k 10 300 python bench.py --workload capi > "$OUT/${TAG}_capi_park2.json" 2> "$OUT/${TAG}_capi_park2.err" &&
TONK_AMD_WAIT_PARK=0 timeout -k 10 300 python bench.py --workload capi > "$OUT/${TAG}_capi_poll2.json" 2> "$OUT/${TAG}_capi_poll2.err" &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "wait_modes or idle_exit or dead_server or stalled_post" --timeout 300 --timeout-method thread > "$OUT/${TAG}_wait_tests.log" 2>&1 &&
REPS=2 bash tools/gpu_tonk_rep.sh ${TAG}park &&
timeout -k 10 60 tools/probe/bar_probe > "$OUT/${TAG}_bar_probe.txt" 2>&1
