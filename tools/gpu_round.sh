#!/bin/bash
# One GPU-box pass (run via gpurun from the repo root): parity tests, smoke, the bench line with
# the CPU baseline, a rocprofv3 kernel trace of the bench, and the PMC traffic passes.  Every GPU
# step has its own time limit; the chain stops at the first failure.
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
R=${GRAFT_REPO_ROOT:-$PWD}
TAG=${1:-r01}
mkdir -p "$OUT" && cd "$R" && make -C tools > "$OUT/tools_build.log" 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
timeout -k 10 900 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 300 python bench.py --workload cfg2 --no-cpu-baseline --no-end-to-end > "$OUT/bench_cfg2.json" 2> "$OUT/bench_cfg2.err" &&
timeout -k 10 300 python bench.py --workload cfg1 > "$OUT/bench_cfg1.json" 2> "$OUT/bench_cfg1.err" &&
timeout -k 10 300 python bench.py --workload cfg4 > "$OUT/bench_cfg4.json" 2> "$OUT/bench_cfg4.err" &&
timeout -k 10 300 python bench.py --workload compress > "$OUT/bench_compress.json" 2> "$OUT/bench_compress.err" &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run -- python3 "$R/bench.py" --no-cpu-baseline --no-end-to-end > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" &&
python3 "$R/tools/trace_region.py" "$OUT/prof_$TAG/run_kernel_trace.csv" > "$OUT/trace_region_$TAG.json" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_lz_$TAG" -o run -- python3 "$R/bench.py" --workload compress --no-cpu-baseline > "$OUT/bench_compress_prof.json" 2> "$OUT/bench_compress_prof.err" &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch_$TAG" -o run -- python3 "$R/bench.py" --no-cpu-baseline --no-end-to-end --steps 3 --warmup 1 > "$OUT/pmc_fetch.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write_$TAG" -o run -- python3 "$R/bench.py" --no-cpu-baseline --no-end-to-end --steps 3 --warmup 1 > "$OUT/pmc_write.log" 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/calib_fetch_$TAG" -o run -- "$R/tools/pmc_calib" > "$OUT/calib_fetch.log" 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/calib_write_$TAG" -o run -- "$R/tools/pmc_calib" > "$OUT/calib_write.log" 2>&1 &&
cd "$R" && python tools/pmc_traffic.py "$OUT/pmc_fetch_$TAG" "$OUT/pmc_write_$TAG" "$OUT/calib_fetch_$TAG" "$OUT/calib_write_$TAG" "$OUT/pmc_traffic_$TAG.json" > "$OUT/pmc_traffic.log" 2>&1
