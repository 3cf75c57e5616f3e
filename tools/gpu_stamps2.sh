#!/bin/bash
# Per-item stamps of one program of configs[2] and of configs[3] (tools/gpu_stamps.sh).
set -o pipefail
ARGS="--workload cfg2" bash tools/gpu_stamps.sh st_cfg2 9 && bash tools/gpu_stamps.sh st_cfg3 9
