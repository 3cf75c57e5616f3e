"""Per-item timing from TONK_AMD_STAMPS dumps (profiling only): per level, item duration vs op
composition, wave busy time and the level's span."""
import functools
import numpy as np, sys
print = functools.partial(print, flush=True)  # (progress reaches the file as it is made)
bases = [int(x) for x in sys.argv[1].split(',')]
# tables as Device::start_program dumps them: items index op records, ops index instructions
items = np.fromfile('tonk_amd_items.bin', dtype=np.uint32).reshape(-1, 2)
ops = np.fromfile('tonk_amd_ops.bin', dtype=np.uint32).reshape(-1, 4)
instr = np.fromfile('tonk_amd_instrs.bin', dtype=np.uint32).reshape(-1, 4)
st = np.fromfile('tonk_amd_stamps.bin', dtype=np.uint64).reshape(-1, 3)
kinds = instr[:, 0] & 0xff
for l in range(len(bases) - 1):
    a, b = bases[l], bases[l + 1]
    if a == b: continue
    s = st[a:b].astype(np.int64)
    dur = (s[:, 1] - s[:, 0]) * 10  # ns (100 MHz)
    t0 = s[:, 0].min()
    span = (s[:, 1].max() - t0) * 10
    # per-item loads: ACC/ACC3 count 1, ACCR count rows
    loads = np.zeros(b - a); ninstr = np.zeros(b - a); naccr = np.zeros(b - a)
    for i in range(a, b):
        op = ops[items[i, 0]]
        ks = kinds[op[0]:op[0] + op[1]]
        ii = instr[op[0]:op[0] + op[1]]
        loads[i - a] = ((ks == 1) | (ks == 5)).sum() + ii[ks == 7, 3].sum()
        ninstr[i - a] = op[1]
        naccr[i - a] = (ks == 7).sum()
    wave = s[:, 2]
    uw, inv = np.unique(wave, return_inverse=True)
    busy = np.bincount(inv, weights=dur)
    first = np.array([s[inv == k, 0].min() for k in range(len(uw))]); last = np.array([s[inv == k, 1].max() for k in range(len(uw))])
    print(f'level {l}: items {b-a} span {span/1e3:.1f} us; item dur median {np.median(dur)/1e3:.2f} p90 {np.percentile(dur,90)/1e3:.2f} max {dur.max()/1e3:.2f} us; waves {len(uw)} busy/wave mean {busy.mean()/1e3:.1f} max {busy.max()/1e3:.1f} us; wave start p50 {np.median(first-t0)*10/1e3:.1f} p99 {np.percentile(first-t0,99)*10/1e3:.1f} end p50 {np.median(last-t0)*10/1e3:.1f} us')
    # duration vs loads / instrs regression
    A = np.stack([np.ones_like(loads), loads, ninstr, naccr], 1)
    coef = np.linalg.lstsq(A, dur, rcond=None)[0]
    print(f'   dur ~ {coef[0]:.0f} ns + {coef[1]:.0f} ns/load + {coef[2]:.0f} ns/instr + {coef[3]:.0f} ns/accr;  loads mean {loads.mean():.1f} instrs mean {ninstr.mean():.1f}')
    # timeline: active items over time in 10 bins
    bins = np.linspace(0, span, 11)
    act = [((s[:, 0] - t0) * 10 <= x).sum() - ((s[:, 1] - t0) * 10 <= x).sum() for x in bins[:-1] + span / 20]
    print('   items in flight per tenth:', act)

# Busy time by op signature per level: (ACCR modes, ACC/ACC3/STOREC counts bucketed)
print()
for l in range(len(bases) - 1):
    a, b = bases[l], bases[l + 1]
    if a == b: continue
    s = st[a:b].astype(np.int64)
    dur = (s[:, 1] - s[:, 0]) * 10
    shared = (s[:, 2] & 0xffffffff) == 4
    groups = {}
    for i in range(a, b):
        op = ops[items[i, 0]]
        ks = kinds[op[0]:op[0] + op[1]]
        ii = instr[op[0]:op[0] + op[1]]
        modes = ((ii[ks == 7, 0] >> 8) & 0xff)
        sig = ('SH ' if shared[i - a] else '') + f"accr{sorted(set(modes.tolist()))} acc{int((ks == 1).sum()) // 8 * 8}+ acc3{int((ks == 5).sum())} storec{int((ks == 6).sum())}"
        g = groups.setdefault(sig, [0, 0.0, 0.0])
        g[0] += 1
        g[1] += dur[i - a]
        g[2] = max(g[2], dur[i - a])
    tot = sum(g[1] for g in groups.values())
    print(f'level {l}: busy by signature (items, share of busy, mean us, max us)')
    for sig, g in sorted(groups.items(), key=lambda kv: -kv[1][1])[:8]:
        print(f'   {sig:55s} {g[0]:6d} {100 * g[1] / tot:5.1f}% {g[1] / g[0] / 1e3:6.2f} {g[2] / 1e3:6.2f}')
