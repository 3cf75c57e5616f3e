#!/bin/bash
# The launch-free C-ABI path on the GPU: one transcript with the watchdog, the C-ABI parity
# tests, then the capi bench line.  Usage: tools/gpu_serve.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:-sv}
mkdir -p "$OUT" && cd "$R" || exit 1
ARGS=$(python3 -c "
import json; sc=json.load(open('tests/golden/scenarios.json'))['scenarios']['c2_4096_p1_ack64']
print(' '.join(sc['args'] + ['seed_data=%d' % (1000 + sc['stream']), 'seed_loss=%d' % (2000 + sc['stream'])]))")
TONK_AMD_CAPI_WATCH=1 timeout -k 5 60 tests/native/_build/capi_gen transcript "$OUT/${TAG}_one.txt" $ARGS \
    > "$OUT/${TAG}_one.out" 2> "$OUT/${TAG}_one.err" || { echo "one transcript failed rc=$?"; tail -5 "$OUT/${TAG}_one.err"; exit 1; }
python3 - "$OUT/${TAG}_one.txt" <<'PY' || exit 1
import gzip, sys
want = gzip.open('tests/golden/c2_4096_p1_ack64.txt.gz', 'rt').read()
got = open(sys.argv[1]).read()
print('one transcript', 'MATCH' if got == want else 'DIFFERS')
sys.exit(0 if got == want else 1)
PY
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k capi -x -v --timeout 120 --timeout-method thread \
    > "$OUT/${TAG}_capi_tests.log" 2>&1 || { echo "capi tests failed"; tail -30 "$OUT/${TAG}_capi_tests.log"; exit 1; }
tail -3 "$OUT/${TAG}_capi_tests.log"
timeout -k 10 300 python bench.py --workload capi > "$OUT/${TAG}_bench_capi.json" 2> "$OUT/${TAG}_bench_capi.err" || { echo "capi bench failed"; tail -5 "$OUT/${TAG}_bench_capi.err"; exit 1; }
cat "$OUT/${TAG}_bench_capi.json"
