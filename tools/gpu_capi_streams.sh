#!/bin/bash
# The GPU suite with the default C-ABI launch streams, then Tonk's unit_tests with one stream and
# with four (150 s each), for the C ABI's per-call latency under Tonk's load.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$PWD}" && mkdir -p gpurun_out || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/cs_tests.log 2>&1 || exit 1
for n in 1 4; do
  { time TONK_AMD_CAPI_STREAMS=$n TONK_AMD_CAPI_WATCH=5 timeout -k 10 150 ./oracle/_ref/tonk/unit_tests_amd < /dev/null > "gpurun_out/tonk_s$n.log" 2>&1 ; } 2> "gpurun_out/tonk_s$n.time" || exit 1
done
