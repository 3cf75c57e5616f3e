#!/bin/bash
# A/B of a host-side switch on one box: bench without and with the environment setting, twice.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
VAR=${1:?env var}
cd "$R" && mkdir -p "$OUT" &&
for rep in 1 2; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-end-to-end > "$OUT/ab_base_$rep.json" 2>/dev/null &&
  env "$VAR=1" timeout -k 10 120 python bench.py --no-cpu-baseline --no-end-to-end > "$OUT/ab_var_$rep.json" 2>/dev/null || exit 1
done
