#!/bin/bash
# Instruction/scalar cache counters of tamd_exec over a short bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:-ic}
mkdir -p "$OUT" && cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_DCACHE_HITS SQC_DCACHE_MISSES --kernel-trace --output-format csv -d "$OUT/${TAG}_a" -o run -- python3 "$R/bench.py" --no-cpu-baseline --no-end-to-end --steps 3 --warmup 1 > "$OUT/${TAG}_a.log" 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_IFETCH SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d "$OUT/${TAG}_b" -o run -- python3 "$R/bench.py" --no-cpu-baseline --no-end-to-end --steps 3 --warmup 1 > "$OUT/${TAG}_b.log" 2>&1
