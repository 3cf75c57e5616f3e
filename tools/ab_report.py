"""Summarise gpu_ab.sh output: value, step, control wall/sum, fill, kernel per launch (A vs B)."""
import glob
import json
import sys

tag = sys.argv[1]
for side in ("A", "B"):
    for f in sorted(glob.glob(f"gpurun_out/{tag}_{side}_*.json")):
        j = json.load(open(f))
        h = j.get("host_ms_per_program") or j["host_ms_per_step"]
        print(side, j["value"], j["ms_per_step"], h.get("control_wall", h.get("parts_wait")), h["control_sum"], h["control_max"],
              h.get("fill", h.get("stolen_steps")),
              j["roofline"]["avg_launch_us"])
