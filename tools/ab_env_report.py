"""Summarise gpu_env_ab4.sh output per variant: value, ms/step, control wall/sum/max, fill, kernel."""
import glob, json, re, statistics, sys

tag = sys.argv[1]
rows = {}
for f in sorted(glob.glob(f"gpurun_out/{tag}_*_[0-9]*.json")):
    m = re.match(rf"gpurun_out/{tag}_(.+)_(\d+)\.json", f)
    j = json.load(open(f))
    h = j.get("host_ms_per_program") or j["host_ms_per_step"]
    rows.setdefault(m.group(1), []).append(
        (j["value"], j["ms_per_step"], h.get("control_wall", h.get("parts_wait")), h["control_sum"], h["control_max"],
              h.get("fill", h.get("stolen_steps")),
         j["roofline"]["avg_launch_us"]))
for v, rs in rows.items():
    for r in rs:
        print(v.ljust(10), " ".join(f"{x:9.3f}" for x in r))
    print(v.ljust(10), "median value", statistics.median(r[0] for r in rs))
