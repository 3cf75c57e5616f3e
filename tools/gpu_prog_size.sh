#!/bin/bash
# Headline: originals per stream per device program (TONK_AMD_BENCH_PROGRAM), interleaved, with the
# byte check of the timed schedule on; each line's launch time, frac, control and device busy.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; TAG=${1:-psize}; mkdir -p "$OUT"; cd "$R" || exit 1
for r in $(seq 1 ${ROUNDS:-2}); do
  for p in ${SIZES:-4096 8192 16384}; do
    f="$OUT/${TAG}_p${p}_$r.json"
    TONK_AMD_BENCH_PROGRAM=$p timeout -k 10 300 python bench.py ${BENCH_ARGS} --no-cpu-baseline --no-end-to-end --no-pmc > "$f" 2> "$f.err" || { tail -5 "$f.err"; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];h=d['host_ms_per_program'];print(sys.argv[2],d['value'],'launch',r['avg_launch_us'],'frac',r['frac'],'control/prog',h['control_sum'],'busy',r['device_busy_frac'],'digests',d['checks'].get('digests_match'))" "$f" "p$p"
  done
done
