#!/bin/bash
# Per-item stamps of one bench program (TONK_AMD_STAMPS=<program>) and the per-level report.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:-st}
PROG=${2:-8}
mkdir -p "$OUT/$TAG" && cd "$OUT/$TAG" || exit 1
TONK_AMD_STAMPS=$PROG timeout -k 10 300 python "$R/bench.py" ${ARGS:-} --no-cpu-baseline --no-end-to-end --no-verify --no-pmc --steps 4 --warmup 2 > bench.json 2> stamps.err || exit 1
bases=$(grep "item_base" stamps.err | awk '{print $NF}' | paste -sd,)
python "$R/tools/stamps_report.py" "$bases" > report.txt 2>&1
rm -f tonk_amd_*.bin
