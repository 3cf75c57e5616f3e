#!/bin/bash
# Executor dynamic tail (TONK_AMD_TAIL=c): the session parity tests and the headline's byte check
# with it on, then interleaved A/B lines (headline and configs[2]) against the default.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; TAG=${1:-tail}; mkdir -p "$OUT"; cd "$R" || exit 1
TONK_AMD_TAIL=3 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "session" --timeout 300 --timeout-method thread > "$OUT/${TAG}_tests.log" 2>&1 || exit 1
TONK_AMD_TAIL=3 timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end > "$OUT/${TAG}_check3.json" 2> "$OUT/${TAG}_check3.err" || exit 1
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print('check3',d['value'],r['avg_launch_us'],r['frac'],r.get('traffic_over_alg'),d['checks'].get('digests_match'))" "$OUT/${TAG}_check3.json"
for i in $(seq 1 ${REPS:-2}); do
  for w in default cfg2; do
    for t in 0 3 2; do
      f="$OUT/${TAG}_${w}_t${t}_$i.json"
      a=""; [ $w = cfg2 ] && a="--workload cfg2"
      TONK_AMD_TAIL=$t timeout -k 10 300 python bench.py $a --no-cpu-baseline --no-end-to-end --no-pmc --no-verify > "$f" 2> "$f.err" || exit 1
      python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(sys.argv[2],d['value'],r['avg_launch_us'],r['frac'],d['host_ms_per_program']['control_sum'],r['device_busy_frac'])" "$f" "$w t$t"
    done
  done
done
