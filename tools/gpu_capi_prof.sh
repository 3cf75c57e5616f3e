#!/bin/bash
# The capi bench leg (configs[2] through siamese.h, 16 threads) once, with the C ABI watchdog's
# per-site sums and the cgroup's CPU throttling around it.  Usage: tools/gpu_capi_prof.sh TAG [env...]
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:-cp}
mkdir -p "$OUT" && cd "$R" || exit 1
ARGS=$(python3 -c "
import sys; sys.path.insert(0, '.')
import tonk_amd
print(' '.join(tonk_amd.WorkloadParams(n=4096, payload=1300, loss=0.02, ack=64).args()))")
cat /sys/fs/cgroup/cpu.stat > "$OUT/${TAG}_cpustat0.txt" 2>/dev/null
TONK_AMD_CAPI_WATCH=${WATCH:-0.5} timeout -k 5 120 tests/native/_build/capi_gen time threads=16 streams=64 reps=1 runs=${RUNS:-3} lat=1 prof=${PROF:-0} $ARGS \
    > "$OUT/${TAG}.json" 2> "$OUT/${TAG}.err"
echo "rc=$?"
cat /sys/fs/cgroup/cpu.stat > "$OUT/${TAG}_cpustat1.txt" 2>/dev/null
paste "$OUT/${TAG}_cpustat0.txt" "$OUT/${TAG}_cpustat1.txt"
cat "$OUT/${TAG}.json"
if [ -n "$REF" ]; then
  timeout -k 5 120 oracle/_ref/golden_gen time threads=16 streams=64 reps=1 runs=${RUNS:-3} lat=1 prof=${PROF:-0} $ARGS > "$OUT/${TAG}_ref.json" 2>&1
  cat "$OUT/${TAG}_ref.json"
fi
