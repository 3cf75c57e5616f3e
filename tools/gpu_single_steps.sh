#!/bin/bash
# configs[1] / configs[4] lines over originals per program (--single-step).
set -o pipefail
mkdir -p gpurun_out
for s in ${CFG1_STEPS:-1024 2048 4096}; do
  timeout -k 10 300 python bench.py --workload cfg1 --step $s > gpurun_out/single_cfg1_$s.json 2> gpurun_out/single_cfg1_$s.err || exit 1
done
for s in ${CFG4_STEPS:-256 512 1024}; do
  timeout -k 10 300 python bench.py --workload cfg4 --step $s > gpurun_out/single_cfg4_$s.json 2> gpurun_out/single_cfg4_$s.err || exit 1
done
