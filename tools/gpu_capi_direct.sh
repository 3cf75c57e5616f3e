#!/bin/bash
# C ABI: the capi tests, then the capi leg with direct dense reads (default) and through the lane
# sums (TONK_AMD_CAPI_DIRECT=0), twice each, interleaved.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; TAG=${1:-cd}; mkdir -p "$OUT"; cd "$R" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_capi.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu > "$OUT/${TAG}_tests.log" 2>&1 || { tail -30 "$OUT/${TAG}_tests.log"; exit 1; }
tail -1 "$OUT/${TAG}_tests.log"
ARGS=$(python3 -c "
import sys; sys.path.insert(0, '.')
import tonk_amd
print(' '.join(tonk_amd.WorkloadParams(n=4096, payload=1300, loss=0.02, ack=64).args()))")
run() { name=$1; shift; env "$@" timeout -k 5 120 tests/native/_build/capi_gen time threads=16 streams=64 reps=1 runs=2 lat=1 prof=1 $ARGS > "$OUT/${TAG}_$name.json" 2>&1 || { echo "$name failed"; tail -5 "$OUT/${TAG}_$name.json"; exit 1; }
  tail -1 "$OUT/${TAG}_$name.json" | python3 -c "
import json,sys; j=json.loads(sys.stdin.read()); print('$name', round(j['gib_per_s'],3), j['seconds'], j.get('encode_us',{}).get('p50'), j.get('decode_us',{}).get('p50'), j['slowest_stream'])"; }
run direct1 X=1 && run lanes1 TONK_AMD_CAPI_DIRECT=0 && run direct2 X=1 && run lanes2 TONK_AMD_CAPI_DIRECT=0
