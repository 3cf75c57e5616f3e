#!/bin/bash
# One golden scenario through the C ABI under several environments; prints MATCH/DIFFERS each.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; TAG=${1:-one}; SC=${SC:-c2_4096_p1_ack64}; mkdir -p "$OUT"; cd "$R" || exit 1
ARGS=$(python3 -c "
import json; sc=json.load(open('tests/golden/scenarios.json'))['scenarios']['$SC']
print(' '.join(sc['args'] + ['seed_data=%d' % (1000 + sc['stream']), 'seed_loss=%d' % (2000 + sc['stream'])]))")
i=0
for e in "${@:2}"; do
  i=$((i+1))
  env $e timeout -k 5 60 tests/native/_build/capi_gen transcript "$OUT/${TAG}_$i.txt" $ARGS > /dev/null 2> "$OUT/${TAG}_$i.err"
  rc=$?
  python3 - "$OUT/${TAG}_$i.txt" "$SC" "$e" "$rc" <<'PY'
import gzip, sys
want = gzip.open('tests/golden/%s.txt.gz' % sys.argv[2], 'rt').read().splitlines()
got = open(sys.argv[1]).read().splitlines()
d = next((k for k, (a, b) in enumerate(zip(want, got)) if a != b), None)
print(sys.argv[3], 'rc', sys.argv[4], 'MATCH' if want == got else 'DIFFERS at %s: want %r got %r' % (d, want[d] if d is not None else None, got[d] if d is not None else None))
PY
done
