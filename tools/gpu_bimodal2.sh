#!/bin/bash
# Executor launch time across processes (the 134 / 142 us split): N short bench runs, each
# reporting its average executor launch and where its arena landed.
set -o pipefail
mkdir -p gpurun_out
for i in $(seq 1 ${N:-6}); do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end --no-pmc --no-verify > gpurun_out/bimodal_$i.json 2> gpurun_out/bimodal_$i.err || exit 1
done
