"""Summarise tools/profile_configs.sh: per config, the average duration of each
step kernel over the timed passes (kernel trace) and, where counter passes ran,
HBM bytes per launch (FETCH_SIZE x 64 B read units + WRITE_SIZE x 64 B write
units as calibrated in profiles/pmc_latest.json when present) and SQ counters."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rows(pattern):
    out = []
    for f in sorted(glob.glob(pattern, recursive=True)):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def short(name):
    return name.split("(")[0].replace("void gr::", "")


def main(o):
    cal = {"read": 2048.0, "write": 1024.0}  # bytes per FETCH/WRITE_SIZE unit (tools/hbm_calib)
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_latest.json")) as fh:
            c = json.load(fh).get("calibration", {})
        cal["read"] = c.get("read_u64_bytes_per_unit", cal["read"])
        cal["write"] = c.get("write_u64_bytes_per_unit", cal["write"])
    except (OSError, ValueError):
        pass
    out = {"calibration": cal, "trace": {}, "pmc": {}}
    tr = defaultdict(list)
    for r in rows(os.path.join(o, "trace", "**", "*kernel_trace.csv")):
        n = short(r["Kernel_Name"])
        if n.startswith("gr_") and "kernel" in n:
            tr[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
    out["trace"] = {k: {"launches": len(v), "avg_us": sum(v) / len(v), "min_us": min(v)} for k, v in tr.items()}
    for d in sorted(x for x in glob.glob(os.path.join(o, "fetch*")) if os.path.isdir(x)):
        c = os.path.basename(d)[len("fetch"):]
        per = {}
        for sub, cnt, unit in (("fetch", "FETCH_SIZE", cal["read"]), ("write", "WRITE_SIZE", cal["write"])):
            agg = defaultdict(list)
            for r in rows(os.path.join(o, sub + c, "**", "*counter_collection.csv")):
                if r["Counter_Name"] == cnt:
                    agg[short(r["Kernel_Name"])].append(float(r["Counter_Value"]) * unit)
            for k, v in agg.items():
                per.setdefault(k, {})[sub + "_bytes_avg"] = sum(v) / len(v)
                per[k][sub + "_bytes_sum"] = sum(v)  # over the run's dispatches
                per[k][sub + "_dispatches"] = len(v)
        sq = defaultdict(lambda: defaultdict(list))
        for r in rows(os.path.join(o, "sq" + c, "**", "*counter_collection.csv")):
            sq[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, v in sq.items():
            per.setdefault(k, {})["sq"] = {cn: sum(x) / len(x) for cn, x in v.items()}
        out["pmc"]["config" + c] = per
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
