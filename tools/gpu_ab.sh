#!/bin/bash
# A/B of an environment switch on one box: bench.py (no CPU leg) alternately without (A) and
# with (B) the assignment given as $2 (e.g. TONK_AMD_SINGLE_ADDS=1), $3 rounds each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:-ab}
SW=${2:-TONK_AMD_SINGLE_ADDS=1}
N=${3:-3}
mkdir -p "$OUT" && cd "$R" || exit 1
for i in $(seq 1 "$N"); do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end --steps 30 > "$OUT/${TAG}_A_$i.json" 2> "$OUT/${TAG}_A_$i.err" || exit 1
  timeout -k 10 300 env "$SW" python bench.py --no-cpu-baseline --no-end-to-end --steps 30 > "$OUT/${TAG}_B_$i.json" 2> "$OUT/${TAG}_B_$i.err" || exit 1
done
