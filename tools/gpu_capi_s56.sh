#!/bin/bash
# The C ABI's slowest stream of configs[2] (stream 56: a serial flush of ~4,300 encodes and
# decodes) alone on one thread, ours with the executor's phase stamps and the reference build.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; TAG=${1:-s56}; mkdir -p "$OUT"; cd "$R" || exit 1
ARGS=$(python3 -c "
import sys; sys.path.insert(0, '.')
import tonk_amd
print(' '.join(tonk_amd.WorkloadParams(n=4096, payload=1300, loss=0.02, ack=64).args()))")
S=${STREAM:-56}
TONK_AMD_CAPI_WATCH=${WATCH:-0.05} timeout -k 5 120 tests/native/_build/capi_gen time threads=1 streams=1 reps=1 runs=3 lat=1 prof=1 stream=$S $ARGS > "$OUT/${TAG}_ours.json" 2> "$OUT/${TAG}_ours.err" || { echo "ours failed"; tail -5 "$OUT/${TAG}_ours.err"; exit 1; }
timeout -k 5 120 oracle/_ref/golden_gen time threads=1 streams=1 reps=1 runs=3 lat=1 prof=1 stream=$S $ARGS > "$OUT/${TAG}_ref.json" 2> "$OUT/${TAG}_ref.err" || { echo "ref failed"; tail -5 "$OUT/${TAG}_ref.err"; exit 1; }
for f in ours ref; do tail -1 "$OUT/${TAG}_$f.json" | python3 -c "
import json,sys; j=json.loads(sys.stdin.read()); print('$f', j['seconds'], j['encode_us'], j['decode_us'], j['slowest_stream'])"; done
grep "server phases" "$OUT/${TAG}_ours.err" | tail -1
