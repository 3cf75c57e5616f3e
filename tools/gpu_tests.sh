#!/bin/bash
# The whole -m gpu suite once (as the driver runs it), then smoke(); logs under gpurun_out/.
R=${GRAFT_REPO_ROOT:-$PWD}; OUT=$R/gpurun_out; TAG=${1:-t}; mkdir -p "$OUT"; cd "$R" || exit 1
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 1500 --timeout-method thread > "$OUT/${TAG}_gpu_tests.log" 2>&1
rc=$?
tail -5 "$OUT/${TAG}_gpu_tests.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/${TAG}_smoke.log" 2>&1 && tail -1 "$OUT/${TAG}_smoke.log"
