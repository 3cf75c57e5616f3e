#!/bin/bash
# Where a C ABI call's time goes, A/B over TONK_AMD_SERVE_DEBUG values (VARIANTS, "0" = default):
# configs[2]'s 64 streams through capi_gen on 16 threads with the watchdog's executor stamps.
set -o pipefail
mkdir -p gpurun_out
args=$(python3 -c "import json; print(' '.join(json.load(open('tests/golden/scenarios.json'))['batches']['cfg2_64x4096_p2_ack64']['args']))")
for i in 1 2; do for v in ${VARIANTS:-0}; do
  TONK_AMD_SERVE_DEBUG=$v TONK_AMD_CAPI_WATCH=100 timeout -k 10 200 tests/native/_build/capi_gen time threads=16 streams=64 stream=0 lat=1 $args > gpurun_out/phases_${v}_$i.json 2> gpurun_out/phases_${v}_$i.err || exit 1
done; done
