#!/bin/bash
# C ABI pass: the siamese.h parity tests, then the capi bench line REPS times.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-capi}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_capi_boundary.py -m gpu -k "capi or boundary" -x -v --timeout 600 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 &&
for i in $(seq 1 ${REPS:-2}); do
  timeout -k 10 400 python bench.py --workload capi > gpurun_out/${TAG}_bench_$i.json 2> gpurun_out/${TAG}_bench_$i.err || exit 1
done
