#!/bin/bash
# Tonk unit_tests against libtonk_amd.so up to N times (150 s each) with the C ABI watchdog and
# its encoder state dump, to catch an intermittent stall; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$PWD}" && mkdir -p gpurun_out || exit 1
for i in $(seq 1 "${1:-3}"); do
  { time TONK_AMD_CAPI_WATCH=5 TONK_AMD_CAPI_WATCH_STATE=1 timeout -k 10 150 ./oracle/_ref/tonk/unit_tests_amd < /dev/null > "gpurun_out/tonk_w$i.log" 2>&1 ; } 2> "gpurun_out/tonk_w$i.time" || exit 1
done
