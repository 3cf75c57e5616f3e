#!/bin/bash
# Tonk unit_tests (relinked against libtonk_amd.so) with two builds of the engine on one box:
# $1 then $2 (library files in tonk_amd/), 150 s each; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$PWD}" && mkdir -p gpurun_out || exit 1
cp tonk_amd/libtonk_amd.so tonk_amd/libtonk_amd_default.so || exit 1
for lib in "$@"; do
  cp "tonk_amd/$lib" tonk_amd/libtonk_amd.so &&
  { time TONK_AMD_CAPI_WATCH=5 timeout -k 10 150 ./oracle/_ref/tonk/unit_tests_amd < /dev/null > "gpurun_out/tonk_$lib.log" 2>&1 ; } 2> "gpurun_out/tonk_$lib.time" || exit 1
done
