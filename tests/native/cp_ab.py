"""Interleaved A/B of two cp_bench builds (the container's timing drifts: alternating runs
cancel the drift; min and median of each side are reported).

usage: python3 cp_ab.py BIN_A BIN_B [rounds=12] [cp_bench args...]"""
import json
import statistics
import subprocess
import sys

a, b = sys.argv[1], sys.argv[2]
rounds = 12
args = []
for x in sys.argv[3:]:
    if x.startswith("rounds="):
        rounds = int(x[7:])
    else:
        args.append(x)
if not args:
    args = ["streams=16", "n=49152", "step=4096", "warm=2"]
res = {a: [], b: []}
for i in range(rounds):
    for exe in ((a, b) if i % 2 == 0 else (b, a)):
        r = subprocess.run(["taskset", "-c", "2", exe] + args, capture_output=True, text=True)
        res[exe].append(json.loads(r.stdout.strip().splitlines()[-1])["ns_per_original"])
for exe in (a, b):
    v = res[exe]
    print(f"{exe}: min {min(v):.1f}  median {statistics.median(v):.1f} ns/original")
print(f"B/A: min {min(res[b]) / min(res[a]):.3f}  median {statistics.median(res[b]) / statistics.median(res[a]):.3f}")
