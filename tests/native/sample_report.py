"""Aggregate cp_bench PC samples by function (addr2line), for control-plane tuning."""
import collections
import subprocess
import sys

exe, samples = sys.argv[1], sys.argv[2]
pcs = [l.strip() for l in open(samples) if l.strip()]
# PIE: the binary is non-PIE when built with -no-pie, so addresses resolve directly
cnt = collections.Counter(pcs)
addrs = list(cnt)
out = subprocess.run(["addr2line", "-f", "-C", "-e", exe] + addrs, capture_output=True, text=True).stdout.splitlines()
byfn = collections.Counter()
for i, a in enumerate(addrs):
    fn = out[2 * i] if 2 * i < len(out) else "?"
    byfn[fn] += cnt[a]
tot = sum(cnt.values())
for fn, c in byfn.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 40):
    print(f"{100.0 * c / tot:6.2f}%  {fn[:150]}")
print("samples", tot)

# Samples outside the executable: resolve against the shared-library mappings (file offset ->
# symbol via nm -D), when the .maps file written by cp_bench is present.
import os
mp = samples + ".maps"
if os.path.exists(mp):
    maps = []
    for l in open(mp):
        f = l.split()
        if len(f) >= 6 and 'x' in f[1]:
            lo, hi = (int(x, 16) for x in f[0].split('-'))
            maps.append((lo, hi, int(f[2], 16), f[5]))
    syms = {}
    def symtab(path):
        if path not in syms:
            out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True).stdout
            t = sorted((int(a, 16), n) for a, _, n in (x.split()[:3] for x in out.splitlines() if len(x.split()) >= 3))
            syms[path] = t
        return syms[path]
    import bisect
    lib = collections.Counter()
    for a, c in cnt.items():
        x = int(a, 16)
        for lo, hi, off, path in maps:
            if lo <= x < hi and not path.endswith("cp_bench_s"):
                t = symtab(path)
                v = x - lo + off
                i = bisect.bisect_right([s[0] for s in t], v) - 1
                lib[(os.path.basename(path), t[i][1] if i >= 0 else "?")] += c
    for (p, n), c in lib.most_common(15):
        print(f"{100.0 * c / tot:6.2f}%  {p}:{n}")
