set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; cd "$R" || exit 1
for i in 1 2; do
 for c in 64 16 8; do
  TONK_AMD_CHUNK=$c timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end --steps 30 > "$OUT/r02j_c${c}_$i.json" 2>/dev/null || exit 1
 done
done
