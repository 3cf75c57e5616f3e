#!/bin/bash
# capi leg under TONK_AMD_SERVE_DEBUG variants: GiB/s, encode/decode p50, the slowest stream.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; TAG=${1:-var}; mkdir -p "$OUT"; cd "$R" || exit 1
ARGS=$(python3 -c "
import sys; sys.path.insert(0, '.')
import tonk_amd
print(' '.join(tonk_amd.WorkloadParams(n=4096, payload=1300, loss=0.02, ack=64).args()))")
for v in ${VARS:-0}; do
  TONK_AMD_SERVE_DEBUG=$v TONK_AMD_CAPI_WATCH=${WATCH:-} timeout -k 5 120 tests/native/_build/capi_gen time threads=16 streams=64 reps=1 runs=2 lat=1 prof=1 $ARGS > "$OUT/${TAG}_$v.json" 2> "$OUT/${TAG}_$v.err"
  echo "== $v rc=$?"; tail -1 "$OUT/${TAG}_$v.json" | python3 -c "
import json,sys; j=json.loads(sys.stdin.read()); ss=j['slowest_stream']
print(round(j['gib_per_s'],3), 'enc p50/p99', j['encode_us']['p50'], j['encode_us']['p99'], 'dec p50', j['decode_us']['p50'], 's56 encode ms', ss['encode'], 'decode ms', ss['decode'])"
  grep "server:" "$OUT/${TAG}_$v.err" | tail -1
done
