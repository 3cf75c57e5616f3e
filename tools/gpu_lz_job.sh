#!/bin/bash
# Compression: messages per job (TONK_AMD_LZ_JOB) A/B on the compress line, interleaved.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; TAG=${1:-lzjob}; mkdir -p "$OUT"; cd "$R" || exit 1
for r in 1 2; do
  for j in ${JOBS:-16 32 8 24}; do
    f="$OUT/${TAG}_j${j}_$r.json"
    TONK_AMD_LZ_JOB=$j timeout -k 10 300 python bench.py --workload compress --no-cpu-baseline > "$f" 2> "$f.err" || exit 1
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],d['ratio'],d['kernel']['ms_per_step'])" "$f" "j$j"
  done
done
