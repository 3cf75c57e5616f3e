set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 200 python bench.py --no-cpu-baseline --no-end-to-end --no-pmc --no-verify > $OUT/tr_a.json 2>/dev/null &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr_prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-end-to-end --no-verify --no-pmc > $OUT/tr_p.json 2>/dev/null &&
python3 $R/tools/trace_region.py $OUT/tr_prof/run_kernel_trace.csv > $OUT/tr_region.json && cd $R &&
timeout -k 10 200 python bench.py --no-cpu-baseline --no-end-to-end --no-pmc --no-verify > $OUT/tr_b.json 2>/dev/null
