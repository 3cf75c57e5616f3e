#!/bin/bash
# gprof flat profile of the control plane on the GPU box's CPU (no GPU use): the headline shape
# (16 streams so dense ranges are chunked as in the bench), one pinned core.
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p "$OUT"
cd tests/native && g++ -std=c++14 -O2 -g -pg -march=x86-64-v3 -fno-inline-small-functions -o _build/cp_bench_pg cp_bench.cpp ../../tonk_amd/csrc/engine.cpp ../../tonk_amd/csrc/encoder.cpp ../../tonk_amd/csrc/decoder.cpp ../../tonk_amd/csrc/gf256.cpp || exit 1
cd /tmp && timeout -k 5 300 taskset -c 3 "$OLDPWD/_build/cp_bench_pg" streams=16 n=1048576 step=4096 warm=8 > "$OUT/cpgprof.json" 2>&1 || exit 1
gprof -b -p "$OLDPWD/_build/cp_bench_pg" gmon.out 2>/dev/null | head -70 > "$OUT/cpgprof_flat.txt"
