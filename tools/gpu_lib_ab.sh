#!/bin/bash
# The driver's bench command, alternated between this tree and an older build in _old/ (bench.py
# and tonk_amd/ of that commit), ROUNDS times on one box.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; TAG=${TAG:-lab}; mkdir -p "$OUT"; cd "$R" || exit 1
for r in $(seq 1 ${ROUNDS:-2}); do
  for side in new old; do
    b=bench.py; [ $side = old ] && b=_old/bench.py
    f="$OUT/${TAG}_${side}_$r.json"
    timeout -k 10 300 python $b --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$f" 2> "$f.err" || { echo "$side failed"; tail -5 "$f.err"; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(sys.argv[2],d['value'],r['avg_launch_us'],d['host_ms_per_program']['control_sum'],r['device_busy_frac'],d['checks'].get('digests_match'))" "$f" $side
  done
done
