"""Summarise a rocprofv3 kernel trace database (the .db rocprofv3 writes when no
-f csv is given): per kernel, calls / average / min duration, and for the step
kernels the gaps between consecutive dispatches on the same queue.

    python tools/trace_db.py gpurun_out/trace_t0 [--match gr_] [--last N]
"""
import argparse
import glob
import os
import sqlite3


def load(path):
    if not os.path.exists(path):
        raise SystemExit(f"{path}: no such trace")
    dbs = glob.glob(os.path.join(path, "**", "*.db"), recursive=True) if os.path.isdir(path) else [path]
    rows = []
    for db in dbs:
        c = sqlite3.connect(f"file:{db}?mode=ro", uri=True)  # never creates a file
        rows += c.execute("select name, start, end, duration, queue_id, grid_x, workgroup_x, vgpr_count, "
                          "accum_vgpr_count, scratch_size from kernels order by start").fetchall()
    return rows


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").replace("gr::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--match", default="gr_")
    ap.add_argument("--last", type=int, default=0, help="only the last N matching dispatches")
    a = ap.parse_args()
    rows = [r for r in load(a.path) if a.match in r[0]]
    if a.last:
        rows = rows[-a.last:]
    agg = {}
    for name, s, e, d, q, gx, wx, vg, ag, sc in rows:
        k = short(name)
        x = agg.setdefault(k, [0, 0, 1 << 62, gx // max(wx, 1), vg, ag, sc])
        x[0] += 1
        x[1] += d
        x[2] = min(x[2], d)
    print(f"{'kernel':48s} {'calls':>6s} {'avg us':>8s} {'min us':>8s} {'wgs':>6s} {'vgpr':>5s} {'agpr':>5s} {'scratch':>7s}")
    for k, (n, tot, mn, wg, vg, ag, sc) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{k[:48]:48s} {n:6d} {tot / n / 1e3:8.2f} {mn / 1e3:8.2f} {wg:6d} {vg:5d} {ag:5d} {sc:7d}")
    gaps = [rows[i + 1][1] - rows[i][2] for i in range(len(rows) - 1) if rows[i + 1][4] == rows[i][4]]
    if gaps:
        gaps.sort()
        print(f"gaps between consecutive {a.match}* dispatches: median {gaps[len(gaps) // 2] / 1e3:.2f} us, "
              f"p90 {gaps[int(len(gaps) * 0.9)] / 1e3:.2f} us (n={len(gaps)})")


if __name__ == "__main__":
    main()
