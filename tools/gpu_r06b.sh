#!/bin/bash
# Round 6 pass b: GPU parity tests, smoke, the default bench line, then an A/B of the decoder's
# direct eliminations (TONK_AMD_DEC_DIRECT) on the headline and configs[2].
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
TAG=${1:-r06b}
mkdir -p "$OUT"
{ [ -n "$SKIP_TESTS" ] || timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > "$OUT/gpu_tests_$TAG.log" 2>&1; } &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1 &&
{ [ -n "$SKIP_TESTS" ] || timeout -k 10 600 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"; } &&
for i in 1 2; do for d in 1 0; do
  TONK_AMD_DEC_DIRECT=$d timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end --no-pmc --no-verify > "$OUT/ab_${TAG}_d${d}_$i.json" 2> "$OUT/ab_${TAG}_d${d}_$i.err" || exit 1
done; done &&
for d in 1 0; do
  TONK_AMD_DEC_DIRECT=$d timeout -k 10 300 python bench.py --workload cfg2 --no-cpu-baseline --no-end-to-end --no-verify > "$OUT/cfg2_${TAG}_d${d}.json" 2> "$OUT/cfg2_${TAG}_d${d}.err" || exit 1
done
