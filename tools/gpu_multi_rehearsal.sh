#!/bin/bash
# Rehearsal of the N-rank bench path on a one-GPU box: two ranks, both on GPU 0
# (TONK_AMD_BENCH_DEVICE), each with 8 host threads on its own half of the GPU's cores -- once
# spawned by bench.py itself, once under torch.distributed.run as the driver launches it.  The
# ranks share one GPU and the box's 16-CPU quota: a functional check, not a scaling number.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
export TONK_AMD_BENCH_DEVICE=0 TONK_AMD_HOST_THREADS=8
timeout -k 10 300 python bench.py --gpus 2 --steps 10 --no-cpu-baseline --no-end-to-end --no-pmc > $OUT/multi_spawn.json 2> $OUT/multi_spawn.err &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 2 --steps 10 --no-cpu-baseline --no-end-to-end --no-pmc > $OUT/multi_torchrun.json 2> $OUT/multi_torchrun.err
