#!/bin/bash
# Flakiness check of Tonk's unit_tests on the GPU box's host: the reference-codec build
# (unit_tests_ref, CPU only) N times, 150 s each; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$PWD}" && mkdir -p gpurun_out || exit 1
for i in $(seq 1 "${1:-3}"); do
  { time timeout -k 10 150 ./oracle/_ref/tonk/unit_tests_ref < /dev/null > "gpurun_out/tonk_ref_$i.log" 2>&1 ; } 2> "gpurun_out/tonk_ref_$i.time" || exit 1
done
