#!/bin/bash
# Compression A/B: the compress -m gpu tests on this tree, then the compress bench line alternated
# between this tree's library and variant libraries (tools/build_lz_variant.sh), ROUNDS times.
#   bash tools/gpu_lz_ab.sh TAG libtonk_amd_x.so [libtonk_amd_y.so ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:-lzab}; shift
mkdir -p "$OUT" && cd "$R" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_compress.py -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/${TAG}_tests.log" 2>&1 || exit 1
for v in "$@"; do
  TONK_AMD_LIB=$v timeout -k 10 300 python -u -m pytest tests/test_compress.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/${TAG}_tests_$v.log" 2>&1 || exit 1
done
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in default "$@"; do
    f="$OUT/${TAG}_${v}_$r.json"
    if [ $v = default ]; then
      timeout -k 10 300 python bench.py --workload compress --no-cpu-baseline > "$f" 2> "$f.err" || exit 1
    else
      TONK_AMD_LIB=$v timeout -k 10 300 python bench.py --workload compress --no-cpu-baseline > "$f" 2> "$f.err" || exit 1
    fi
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],d['ratio'],d['kernel']['ms_per_step'])" "$f" $v
  done
done
TONK_AMD_LZ_PROF=1 timeout -k 10 300 python bench.py --workload compress --no-cpu-baseline > "$OUT/${TAG}_prof.json" 2> "$OUT/${TAG}_prof.err" || exit 1
for v in "$@"; do
  TONK_AMD_LIB=$v TONK_AMD_LZ_PROF=1 timeout -k 10 300 python bench.py --workload compress --no-cpu-baseline > "$OUT/${TAG}_prof_$v.json" 2> "$OUT/${TAG}_prof_$v.err" || exit 1
done
