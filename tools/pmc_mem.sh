#!/bin/bash
# Memory-side counters of tamd_exec over a short bench (one rocprofv3 run per pass).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:-mem}
mkdir -p "$OUT" && cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 60 rocprofv3 -L > "$OUT/${TAG}_counters.txt" 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum --kernel-trace --output-format csv -d "$OUT/${TAG}_a" -o run -- python3 "$R/bench.py" --no-cpu-baseline --no-end-to-end --steps 3 --warmup 1 > "$OUT/${TAG}_a.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d "$OUT/${TAG}_b" -o run -- python3 "$R/bench.py" --no-cpu-baseline --no-end-to-end --steps 3 --warmup 1 > "$OUT/${TAG}_b.log" 2>&1
