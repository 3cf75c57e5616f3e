#!/bin/bash
# capi leg variants (rusage + per-call-kind time): current, launch path, 8 threads, reference.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; TAG=${1:-ab}; mkdir -p "$OUT"; cd "$R" || exit 1
ARGS=$(python3 -c "
import sys; sys.path.insert(0, '.')
import tonk_amd
print(' '.join(tonk_amd.WorkloadParams(n=4096, payload=1300, loss=0.02, ack=64).args()))")
nproc; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max
run() { name=$1; shift; env "$@" timeout -k 5 120 $EXE time threads=${T:-16} streams=64 reps=1 runs=2 lat=1 prof=1 $ARGS > "$OUT/${TAG}_$name.json" 2>&1; echo "== $name rc=$?"; tail -1 "$OUT/${TAG}_$name.json" | python3 -c "
import json,sys; j=json.loads(sys.stdin.read()); print(round(j['gib_per_s'],3), j['seconds'], j['threads_ms'], j['slowest_stream'], j['call_ms'])"; }
EXE=tests/native/_build/capi_gen run serve X=1
#EXE=tests/native/_build/capi_gen run launch TONK_AMD_SERVE=0
#EXE=tests/native/_build/capi_gen T=8 run serve_t8 X=1
EXE=oracle/_ref/golden_gen run ref X=1
