#!/bin/bash
# SQ counter passes over the bench (kernel diagnosis): one rocprofv3 run per pass.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:-sq}
mkdir -p "$OUT" && cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace --output-format csv -d "$OUT/${TAG}_a" -o run -- python3 "$R/bench.py" --no-cpu-baseline --no-end-to-end --no-pmc --no-verify --steps 3 --warmup 1 > "$OUT/${TAG}_a.log" 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/${TAG}_b" -o run -- python3 "$R/bench.py" --no-cpu-baseline --no-end-to-end --no-pmc --no-verify --steps 3 --warmup 1 > "$OUT/${TAG}_b.log" 2>&1
