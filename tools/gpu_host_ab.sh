#!/bin/bash
# Host-side A/Bs in one box call: the control plane alone on one core (tools/gpu_cp_abc.sh:
# cp_a vs cp_b, cp_a vs cp_c), then the headline bench with and without glibc's huge-page heap.
R=${GRAFT_REPO_ROOT:-$PWD}; cd "$R"
bash tools/gpu_cp_abc.sh h1 && cd "$R" &&
NO_TESTS=1 WORKLOADS="cfg3" REPS=4 bash tools/gpu_ab_env.sh s6 base: thp:GLIBC_TUNABLES=glibc.malloc.hugetlb=1
