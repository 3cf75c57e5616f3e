"""Per-phase control-plane cycles (cp_bench_prof, prof.h scopes): the minimum over several runs
of each phase's cycles per original, and of ns per original (the container's timing is noisy).

usage: python3 cp_prof.py [runs=5] [cp_bench args...]"""
import json
import os
import subprocess
import sys

here = os.path.dirname(os.path.abspath(__file__))
runs = 5
args = []
for a in sys.argv[1:]:
    if a.startswith("runs="):
        runs = int(a[5:])
    else:
        args.append(a)
if not args:
    args = ["streams=16", "n=49152", "step=4096", "warm=2"]
# (the binary is not part of the Makefile's default target: rebuild it from the current sources)
subprocess.run(["make", "-s", "-C", here, "_build/cp_bench_prof"], check=True)
best, ns = {}, []
for _ in range(runs):
    r = subprocess.run([os.path.join(here, "_build", "cp_bench_prof")] + args, capture_output=True, text=True)
    ns.append(json.loads(r.stdout.strip().splitlines()[-1])["ns_per_original"])
    for line in r.stderr.splitlines():
        f = line.split()
        if len(f) >= 7 and f[1] == "calls/orig":
            v = float(f[6])
            best[f[0]] = min(best.get(f[0], v), v)
top = ["enc_add", "enc_encode", "enc_ack", "dec_add_orig", "dec_add_rec", "dec_decode", "dec_ack", "dec_is_ready",
       "prepare_flush", "finish_flush", "release"]
for k, v in sorted(best.items(), key=lambda kv: -kv[1]):
    print(f"{k:14s} {v:8.1f} cyc/orig{'  *' if k in top else ''}")
print(f"top-level sum  {sum(best.get(k, 0) for k in top):8.1f} cyc/orig;  min ns/original {min(ns)}")
