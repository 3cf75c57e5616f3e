#!/bin/bash
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p $OUT
T=${1:-fr2}
for i in 1 2 3 4; do timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end --no-pmc --no-verify > $OUT/${T}_bench_$i.json 2> $OUT/${T}_bench_$i.err || exit 1; done
for i in 1 2; do TONK_AMD_PASSES=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end --no-pmc --no-verify > $OUT/${T}_passes_$i.json 2> $OUT/${T}_passes_$i.err || exit 1; done
