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
