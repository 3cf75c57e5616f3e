#!/bin/bash
# The executor's launch-time split across processes: N bench processes under rocprofv3 with L2
# hit / miss counters and the L2's fabric read requests, per timed executor dispatch.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for i in $(seq 1 ${N:-4}); do
  timeout -k 10 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --kernel-trace --output-format csv -d "$OUT/split_$i" -o run -- python3 "$R/bench.py" --no-cpu-baseline --no-end-to-end --no-pmc --no-verify --steps 10 > "$OUT/split_$i.json" 2> "$OUT/split_$i.err" || exit 1
done
