#!/bin/bash
# Several short probes in one box call (each with its own time limit; stops at the first failure).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
for step in "$@"; do
  case "$step" in
    hp:*) timeout -k 10 600 bash tools/gpu_host_probe.sh "${step#hp:}" || exit 1 ;;
    prof:*) ARGS="streams=16 n=49152 step=4096 warm=2 reps=400" timeout -k 10 400 bash tools/gpu_cp_prof.sh "${step#prof:}" || exit 1 ;;
    ab:*) timeout -k 10 400 bash tools/gpu_cp_ab.sh "${step#ab:}" || exit 1 ;;
    round:*) timeout -k 10 1100 bash tools/gpu_round.sh "${step#round:}" || exit 1 ;;
  esac
done
