#!/bin/bash
# One GPU-box pass (run via gpurun from the repo root), in parts that each fit one call:
#   PART=a  parity tests, smoke, the default bench line (its own PMC traffic passes, the byte check
#           of the timed schedule, the CPU baseline and the host-staged legs)
#   PART=b  the configs[2] / [1] / [4] and compression lines, rocprofv3 kernel traces of the
#           default bench and of the compressor (+ the timed-region average)
#   PART=c  the siamese.h C ABI line and the two-rank rehearsal
#   PART=d  part a without the tests (smoke and the default bench line)
# (no PART: all three in one go).  Every GPU step has its own time limit; a part stops at its first
# failure.
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:-r04}
PART=${PART:-abc}
mkdir -p "$OUT" && cd "$R" || exit 1
if [[ $PART == *a* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > "$OUT/gpu_tests_$TAG.log" 2>&1 &&
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1 &&
  timeout -k 10 900 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err" || exit 1
fi
if [[ $PART == *d* ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1 &&
  timeout -k 10 900 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err" || exit 1
fi
if [[ $PART == *b* ]]; then
  timeout -k 10 600 python bench.py --workload cfg2 --no-cpu-baseline --no-end-to-end > "$OUT/bench_cfg2_$TAG.json" 2> "$OUT/bench_cfg2_$TAG.err" &&
  timeout -k 10 300 python bench.py --workload cfg1 > "$OUT/bench_cfg1_$TAG.json" 2> "$OUT/bench_cfg1_$TAG.err" &&
  timeout -k 10 300 python bench.py --workload cfg4 > "$OUT/bench_cfg4_$TAG.json" 2> "$OUT/bench_cfg4_$TAG.err" &&
  timeout -k 10 300 python bench.py --workload compress > "$OUT/bench_compress_$TAG.json" 2> "$OUT/bench_compress_$TAG.err" &&
  ( cd /tmp && export TMPDIR=/tmp &&
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run -- python3 "$R/bench.py" --no-cpu-baseline --no-end-to-end --no-verify --no-pmc > "$OUT/bench_prof_$TAG.json" 2> "$OUT/bench_prof_$TAG.err" &&
    python3 "$R/tools/trace_region.py" "$OUT/prof_$TAG/run_kernel_trace.csv" > "$OUT/trace_region_$TAG.json" &&
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_lz_$TAG" -o run -- python3 "$R/bench.py" --workload compress --no-cpu-baseline > "$OUT/bench_compress_prof_$TAG.json" 2> "$OUT/bench_compress_prof_$TAG.err" ) || exit 1
fi
if [[ $PART == *c* ]]; then
  timeout -k 10 400 python bench.py --workload capi > "$OUT/bench_capi_$TAG.json" 2> "$OUT/bench_capi_$TAG.err" &&
  bash tools/gpu_multi_rehearsal.sh || exit 1
fi
