#!/bin/bash
# Sampled control-plane profile on the GPU box's CPU (no GPU use): cp_bench built without PIE,
# 4 streams on one pinned core (a bench worker's share), PC samples resolved per function and line.
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p "$OUT"
cd tests/native && g++ -std=c++14 -O3 -g -march=x86-64-v3 -no-pie -fno-omit-frame-pointer -o _build/cp_bench_s cp_bench.cpp ../../tonk_amd/csrc/engine.cpp ../../tonk_amd/csrc/encoder.cpp ../../tonk_amd/csrc/decoder.cpp ../../tonk_amd/csrc/gf256.cpp && cd ../.. || exit 1
timeout -k 5 300 taskset -c 3 tests/native/_build/cp_bench_s streams=4 n=2097152 step=4096 warm=8 sample=/tmp/samp.txt > "$OUT/cpsample.json" 2>&1 || exit 1
python3 tests/native/sample_report.py tests/native/_build/cp_bench_s /tmp/samp.txt 60 > "$OUT/cpsample_fn.txt" 2>&1
python3 - /tmp/samp.txt tests/native/_build/cp_bench_s > "$OUT/cpsample_lines.txt" <<'PY'
import collections, subprocess, sys
pcs = [l.strip() for l in open(sys.argv[1]) if l.strip()]
cnt = collections.Counter(pcs)
addrs = list(cnt)
out = subprocess.run(["addr2line", "-C", "-e", sys.argv[2]] + addrs, capture_output=True, text=True).stdout.splitlines()
by = collections.Counter()
for i, a in enumerate(addrs):
    by[out[i].split(" ")[0].split("/")[-1]] += cnt[a]
tot = sum(cnt.values())
for l, c in by.most_common(60):
    print(f"{100 * c / tot:5.1f}% {l}")
print("samples", tot)
PY
