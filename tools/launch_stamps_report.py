"""Per-launch item timing from TONK_AMD_LAUNCH_STAMPS (profiling only): span, item durations by
(level, class), and when the launch's last items started and ended."""
import sys
import numpy as np
rows = np.loadtxt(sys.argv[1] if len(sys.argv) > 1 else "tonk_amd_launch_stamps.txt", dtype=np.int64)
seg, lvl, cls, t0, t1 = rows[:, 0], rows[:, 1], rows[:, 2], rows[:, 3], rows[:, 4]
ok = t1 > 0
start = t0[ok].min()
a, b = (t0 - start) * 10 / 1000.0, (t1 - start) * 10 / 1000.0  # us
d = b - a
print(f"items {len(rows)} span {b[ok].max():.1f} us; busy {d[ok].sum():.0f} wave-us = {d[ok].sum() / 4096:.1f} us over 4096 wave slots")
for L in sorted(set(lvl.tolist())):
    for C in range(5):
        m = ok & (lvl == L) & (cls == C)
        if not m.any(): continue
        print(f"  level {L} class {C}: items {m.sum():5d} dur mean {d[m].mean():6.2f} p90 {np.percentile(d[m], 90):6.2f} max {d[m].max():6.2f}"
              f" | start p50 {np.percentile(a[m], 50):6.1f} max {a[m].max():6.1f} | end max {b[m].max():6.1f} us")
order = np.argsort(-b[ok])[:10]
print("last 10 items to end: (level, class, start, dur, end)")
for i in order:
    print(f"  L{lvl[ok][i]} c{cls[ok][i]} start {a[ok][i]:6.1f} dur {d[ok][i]:6.1f} end {b[ok][i]:6.1f}")
hist = np.histogram(a[ok], bins=10, range=(0, b[ok].max()))[0]
print("item starts per tenth of the span:", hist.tolist())
