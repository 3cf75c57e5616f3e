#!/bin/bash
# Per-item stamps of one bench program (TONK_AMD_STAMPS=<program>) and the per-level report.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:-st}
PROG=${2:-8}
mkdir -p "$OUT/$TAG" && cd "$OUT/$TAG" || exit 1
TONK_AMD_STAMPS=$PROG timeout -k 10 300 python "$R/bench.py" --no-cpu-baseline --no-end-to-end --steps 10 --warmup 3 > bench.json 2> stamps.err || exit 1
ib=$(grep -o "n_instr_bytes [0-9]*" stamps.err | awk '{print $2}')
ob=$(grep -o "n_ops_bytes [0-9]*" stamps.err | awk '{print $2}')
ni=$(grep -o "n_items [0-9]*" stamps.err | awk '{print $2}')
bases=$(grep "item_base" stamps.err | awk '{print $NF}' | paste -sd,)
python "$R/tools/stamps_report.py" "$ib" "$ob" "$ni" "$bases" > report.txt 2>&1
rm -f tonk_amd_program.bin tonk_amd_stamps.bin
