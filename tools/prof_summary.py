"""Summarise a tools/profile.sh run: per-kernel trace stats, HBM bytes per
launch of gr_step_kernel from FETCH_SIZE/WRITE_SIZE, calibrated against
tools/hbm_calib's known byte counts, and SQ occupancy counters."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def rows(pattern):
    out = []
    for f in sorted(glob.glob(pattern, recursive=True)):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def counters(d, kernel_sub):
    """{counter: [value per dispatch]} for kernels whose name contains kernel_sub."""
    per = defaultdict(lambda: defaultdict(float))
    for r in rows(os.path.join(d, "**", "*counter_collection.csv")):
        if kernel_sub not in r.get("Kernel_Name", ""):
            continue
        per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: [v[x] for x in sorted(v, key=int)] for k, v in per.items()}


# The lean kernels of one headline pass (gr_kernels.h, a split pass over
# loopback routes, RM = 3): the steady kernel, then the role instances over its
# wave lists, in one launch (gr_roles_kernel, round 4) or as <S, 2> (followers)
# and <S, 1> (leaders) with GR_ROLES_MERGED=0. A device pass's lean-kernel bytes
# are the sum over the kernels it ran.
ROLE_INSTANCES_MERGED = ("gr_steady_kernel<3, 3", "gr_roles_kernel<3, 3>")  # steady: <3, 3, LC>
ROLE_INSTANCES_SPLIT = ("gr_steady_kernel<3, 3", "gr_fast_kernel<3, 2, 3, true>", "gr_fast_kernel<3, 1, 3, true>")


def main(o):
    s = {}
    st = rows(os.path.join(o, "trace", "**", "*kernel_stats.csv"))
    s["kernel_stats"] = [{k: r[k] for k in r} for r in st[:8]]
    # calibration: bytes per FETCH_SIZE/WRITE_SIZE unit at our access widths
    cal = {}
    nbytes = 2 << 30
    for name in ("read_u64", "read_u8"):
        v = counters(os.path.join(o, "calib_fetch"), name).get("FETCH_SIZE", [])
        if v:
            cal[name + "_bytes_per_unit"] = nbytes / (sum(v) / len(v))
    for name in ("write_u64", "write_u8"):
        v = counters(os.path.join(o, "calib_write"), name).get("WRITE_SIZE", [])
        if v:
            cal[name + "_bytes_per_unit"] = nbytes / (sum(v) / len(v))
    s["calibration"] = cal
    kf = cal.get("read_u64_bytes_per_unit", 2048.0)
    kw = cal.get("write_u64_bytes_per_unit", 1024.0)
    s["kernels"] = {}
    for kname in ("gr_fast_kernel", "gr_step_kernel", "gr_tick_kernel"):
        f = counters(os.path.join(o, "fetch"), kname).get("FETCH_SIZE", [])
        w = counters(os.path.join(o, "write"), kname).get("WRITE_SIZE", [])
        f_ss, w_ss = f[3:] or f, w[3:] or w  # steady-state launches (after warm-up)
        k = {"launches": len(f)}
        if f_ss and w_ss:
            fu = sum(f_ss) / len(f_ss)
            wu = sum(w_ss) / len(w_ss)
            k.update({"fetch_size_units": fu, "write_size_units": wu, "read_bytes": fu * kf,
                      "write_bytes": wu * kw, "hbm_bytes_per_launch": fu * kf + wu * kw})
        for sub in ("sq", "sq2"):
            sq = counters(os.path.join(o, sub), kname)
            k.setdefault("sq", {}).update({c: sum(v[3:] or v) / len(v[3:] or v) for c, v in sq.items() if v})
        s["kernels"][kname] = k
    merged = bool(counters(os.path.join(o, "fetch"), "gr_roles_kernel<3, 3>").get("FETCH_SIZE"))
    ROLE_INSTANCES = ROLE_INSTANCES_MERGED if merged else ROLE_INSTANCES_SPLIT
    for kname in ROLE_INSTANCES:  # per instance, for the per-pass sum below
        f = counters(os.path.join(o, "fetch"), kname).get("FETCH_SIZE", [])
        w = counters(os.path.join(o, "write"), kname).get("WRITE_SIZE", [])
        f_ss, w_ss = f[3:] or f, w[3:] or w
        if f_ss and w_ss:
            fu, wu = sum(f_ss) / len(f_ss), sum(w_ss) / len(w_ss)
            s["kernels"][kname] = {"launches": len(f), "read_bytes": fu * kf, "write_bytes": wu * kw,
                                   "hbm_bytes_per_launch": fu * kf + wu * kw}
            sqk = {}
            for sub in ("sq", "sq2"):
                sq = counters(os.path.join(o, sub), kname)
                sqk.update({c: sum(v[3:] or v) / len(v[3:] or v) for c, v in sq.items() if v})
            s["kernels"][kname]["sq"] = sqk
    fk = s["kernels"].get("gr_fast_kernel", {})
    if all(k in s["kernels"] for k in ROLE_INSTANCES):  # split passes: one pass = both instances
        fk = {key: sum(s["kernels"][k][key] for k in ROLE_INSTANCES)
              for key in ("read_bytes", "write_bytes", "hbm_bytes_per_launch")}
        s["lean_kernel_bytes_per_pass"] = fk
    if "hbm_bytes_per_launch" in fk:
        groups = int(os.environ.get("GROUPS", "1000000"))
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from dragonboat_amd.build import source_digest
        with open(os.path.join(o, "pmc_latest.json"), "w") as fh:
            json.dump({"kernel": " + ".join(k + (", LC>" if k.endswith(", 3") else "") for k in ROLE_INSTANCES) + " (the lean kernels of one pass)", "groups": groups, "replicas": 3,
                       "source_digest": source_digest(),
                       "hbm_bytes_per_launch": fk["hbm_bytes_per_launch"],
                       "read_bytes": fk["read_bytes"], "write_bytes": fk["write_bytes"],
                       "calibration": cal, "source": os.path.basename(o)}, fh, indent=1)
    json.dump(s, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
