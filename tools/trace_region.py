"""Average duration of a kernel's dispatches inside the bench's timed region, from a rocprofv3
kernel trace (--kernel-trace --output-format csv).  The region is delimited by the two
tamd_timed_region dispatches that Device::set_timing launches, so the figure covers the same
launches as the bench's own event timing (roofline.avg_launch_us).

usage: python tools/trace_region.py run_kernel_trace.csv [kernel=tamd_exec24]"""
import csv
import json
import sys


def region_stats(path: str, kernel: str = "tamd_exec24") -> dict:
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("tamd_timed_region")]
    if len(marks) < 2:
        raise SystemExit(f"{path}: expected two tamd_timed_region dispatches, found {len(marks)}")
    inside = rows[marks[0] + 1:marks[1]]
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in inside if r["Kernel_Name"] == kernel]
    allk = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows if r["Kernel_Name"] == kernel]
    return {"kernel": kernel, "timed_dispatches": len(d), "timed_avg_us": round(sum(d) / len(d) / 1e3, 3) if d else None,
            "all_dispatches": len(allk), "all_avg_us": round(sum(allk) / len(allk) / 1e3, 3) if allk else None}


if __name__ == "__main__":
    print(json.dumps(region_stats(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "tamd_exec24")))
