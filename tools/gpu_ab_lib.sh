#!/bin/bash
# A/B of two builds of the engine on one box: bench.py (no CPU leg) alternately with the
# library tonk_amd/$2 (A) and tonk_amd/$3 (B), $4 rounds each.  Build B with
# `make -C tonk_amd LIB=libtonk_amd_b.so` after copying the A build aside.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:-abl}
A=${2:-libtonk_amd_a.so}
B=${3:-libtonk_amd.so}
N=${4:-3}
mkdir -p "$OUT" && cd "$R" || exit 1
for i in $(seq 1 "$N"); do
  TONK_AMD_LIB=$A timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end --steps 30 > "$OUT/${TAG}_A_$i.json" 2> "$OUT/${TAG}_A_$i.err" || exit 1
  TONK_AMD_LIB=$B timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end --steps 30 > "$OUT/${TAG}_B_$i.json" 2> "$OUT/${TAG}_B_$i.err" || exit 1
done
python3 tools/ab_report.py "$TAG"
