#!/bin/bash
# Round 6m: BAR placement for the C ABI -- per-call latency of ordinary streams alone (configs[2]
# streams 0 and 5, one thread) and the 64-stream capi bench, masks 0 / 6 (commands + ring) / 7.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:-r06m}
mkdir -p "$OUT" && cd "$R" || exit 1
args=$(python3 -c "import json; print(' '.join(json.load(open('tests/golden/scenarios.json'))['batches']['cfg2_64x4096_p2_ack64']['args']))")
for i in 1 2; do for b in 0 6 7; do for s in 0 5; do
  TONK_AMD_CAPI_BAR=$b TONK_AMD_CAPI_WATCH=100 timeout -k 10 200 tests/native/_build/capi_gen time threads=1 streams=1 stream=$s lat=1 runs=3 $args > "$OUT/${TAG}_ord_s${s}_bar${b}_$i.json" 2> "$OUT/${TAG}_ord_s${s}_bar${b}_$i.err" || exit 1
done; done; done
for i in 1 2; do for b in 0 6 7; do
  TONK_AMD_CAPI_BAR=$b timeout -k 10 300 python bench.py --workload capi > "$OUT/${TAG}_capi_bar${b}_$i.json" 2> "$OUT/${TAG}_capi_bar${b}_$i.err" || exit 1
done; done
