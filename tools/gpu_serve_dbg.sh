#!/bin/bash
# Start-up probe of the persistent executor under diagnostic modes (TONK_AMD_SERVE_DEBUG).
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
TAG=${1:-dbg}
mkdir -p "$OUT" && cd "$R" || exit 1
ARGS=$(python3 -c "
import json; sc=json.load(open('tests/golden/scenarios.json'))['scenarios']['c1_256_p3']
print(' '.join(sc['args'] + ['seed_data=%d' % (1000 + sc['stream']), 'seed_loss=%d' % (2000 + sc['stream'])]))")
for m in ${MODES:-1 2 3 0}; do
  TONK_AMD_SERVE_DEBUG=$m timeout -k 5 20 tests/native/_build/capi_gen transcript /dev/null $ARGS > /dev/null 2> "$OUT/${TAG}_m$m.err"
  echo "mode $m rc=$? $(grep -c 'not completed' $OUT/${TAG}_m$m.err) $(grep 'not completed' $OUT/${TAG}_m$m.err | cut -c1-300)"
done
