"""Summarize bench JSON lines (A/B runs): value, ms/step, executor us/launch, fractions, device
busy, control CPU per program, op-trace bytes, HBM traffic over B_alg, digest check."""
import glob
import json
import sys


def line(p):
    return json.loads([l for l in open(p).read().splitlines() if l.startswith('{')][-1])


for pat in sys.argv[1:]:
    for p in sorted(glob.glob(pat)):
        try:
            d = line(p)
        except (IndexError, ValueError):
            print(p, "no line")
            continue
        r, h = d["roofline"], d.get("host_ms_per_program") or {}
        print(f"{p.split('/')[-1]:28s} {d['value']:8.1f} GiB/s {d['ms_per_step']:7.3f} ms  {r.get('avg_launch_us')} us  "
              f"frac {r['frac']} fc {r.get('frac_counters')} busy {r.get('device_busy_frac')} ctl {h.get('control_sum')} "
              f"op {round((r.get('op_trace_bytes_per_launch') or 0) / 1e6, 1)} MB tr {r.get('traffic_over_alg')} "
              f"dig {d['checks'].get('digests_match')} cpu {(d.get('cpu_baseline') or {}).get('value')}")
