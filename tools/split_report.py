"""Per-process summary of tools/gpu_split_pmc.sh: the executor's average timed launch (from the
bench line) beside its L2 hit rate and fabric read requests per timed dispatch (PMC csv)."""
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import _timed_counter_values  # noqa: E402

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
for j in sorted(glob.glob(os.path.join(out, "split_*.json"))):
    d = os.path.splitext(j)[0]
    try:
        line = json.loads([l for l in open(j).read().splitlines() if l.startswith("{")][-1])
    except (IndexError, ValueError):
        print(j, "no bench line")
        continue
    r = line["roofline"]
    hit = _timed_counter_values(d, "TCC_HIT_sum")
    miss = _timed_counter_values(d, "TCC_MISS_sum")
    rd = _timed_counter_values(d, "TCC_EA0_RDREQ_sum")
    n = len(hit)
    if not n:
        print(j, "no counters")
        continue
    h, m, q = sum(hit) / n, sum(miss) / n, sum(rd) / max(1, len(rd))
    print(f"{os.path.basename(j)}: {r['avg_launch_us']} us/launch  L2 hit {h / (h + m):.4f}  hits {h / 1e6:.2f} M  "
          f"misses {m / 1e6:.2f} M  EA rdreq {q / 1e6:.2f} M (x128 B = {q * 128 / 1e6:.0f} MB)  dispatches {n}  "
          f"arena {r.get('arena', {}).get('base')}  value {line['value']}")
