"""Per-launch HBM traffic of tamd_exec from rocprofv3 PMC passes (MI355X_MICROARCH.md, HBM).

usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR CALIB_FETCH_DIR CALIB_WRITE_DIR [out.json]

FETCH_SIZE and WRITE_SIZE are collected in separate passes (they do not fit one TCC pass).  Both
are in KiB.  The gfx950 correction is measured, not assumed: tools/pmc_calib.hip moves a known
byte count with the executor's access width (tamd_exec: 8 B per lane; tamd_exec16: 16 B per
lane), and the ratio known/counted scales the executor's counters.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys


def counters(d: str) -> dict:
    """{kernel: {counter: [value per dispatch]}} from a rocprofv3 csv output directory."""
    out: dict = {}
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get("Kernel_Name", "")
                name = row.get("Counter_Name", "")
                try:
                    v = float(row.get("Counter_Value", "nan"))
                except ValueError:
                    continue
                out.setdefault(k, {}).setdefault(name, []).append(v)
    return out


def pick(c: dict, prefix: str, counter: str) -> list:
    for k, v in c.items():
        if k.split("(")[0].strip() == prefix and counter in v:
            return v[counter]
    return []


def main() -> int:
    fetch, write, cfetch, cwrite = sys.argv[1:5]
    out_path = sys.argv[5] if len(sys.argv) > 5 else None
    F, W, CF, CW = counters(fetch), counters(write), counters(cfetch), counters(cwrite)
    read_known, write_known = 2 << 30, 1 << 30
    kernel = "tamd_exec16" if any(k.split("(")[0].strip() == "tamd_exec16" for k in F) else "tamd_exec"
    width = "16" if kernel == "tamd_exec16" else "8"
    cr = pick(CF, "calib_read" + width, "FETCH_SIZE")
    cw = pick(CW, "calib_write" + width, "WRITE_SIZE")
    read_scale = read_known / (sorted(cr)[len(cr) // 2] * 1024.0) if cr else 2.0
    write_scale = write_known / (sorted(cw)[len(cw) // 2] * 1024.0) if cw else 1.0
    fv = pick(F, kernel, "FETCH_SIZE")
    wv = pick(W, kernel, "WRITE_SIZE")
    res = {
        "kernel": kernel,
        "dispatches_fetch": len(fv),
        "dispatches_write": len(wv),
        "fetch_kib_avg": sum(fv) / len(fv) if fv else None,
        "write_kib_avg": sum(wv) / len(wv) if wv else None,
        "read_scale": read_scale,
        "write_scale": write_scale,
    }
    if fv and wv:
        res["traffic_bytes_per_launch"] = (sum(fv) / len(fv) * read_scale + sum(wv) / len(wv) * write_scale) * 1024.0
    js = json.dumps(res, indent=1)
    print(js)
    if out_path:
        with open(out_path, "w") as fh:
            fh.write(js + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
