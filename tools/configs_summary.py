"""Per-config evidence on one build: from a
tools/profile_configs.sh output directory (the configs' bench_configs.py line,
a kernel trace, calibrated FETCH_SIZE / WRITE_SIZE passes per config), one
summary per BASELINE config: pass time, HBM bytes per pass by PMC, SURVEY.md
8(d)'s canonical bytes per pass, their ratio, and the canonical fraction of the
8 TB/s spec. bench.py reports it beside the headline (never as `value`) when
its source digest is the build's.

    python tools/configs_summary.py gpurun_out/cfgprof_r06 [untraced_configs.json] > profiles/r06_configs/summary.json

The pass times come from the untraced run when one is given (tools/bench_configs.py
without the profiler: the kernel trace slows every launch), the bytes from the
counter passes.
"""
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
HBM_PEAK = 8000.0  # GB/s (MI355X_MICROARCH.md)


def b_round(R):  # (R-1)(69 + 65 + 138) + 8R + 48
    return (R - 1) * (69 + 65 + 138) + 8 * R + 48


def canonical(cfg):
    """SURVEY.md 8(d) bytes per pass: configs 2 and 5 G x B_round(R) (config 5
    at the steady group-round; its rejects and catch-ups move more), config 3
    100k x 62 (B_tick) + 10k x 145 (B_ri at R = 5)."""
    name, G, R = cfg["config"], cfg["groups"], cfg["replicas"]
    if name.startswith("3"):
        return G * 62 + int(G * 0.1) * (49 + 24 * (R - 1))
    return G * b_round(R)


def load_lines(path):
    out = []
    with open(path) as fh:
        for ln in fh:
            ln = ln.strip()
            if ln.startswith("{"):
                out.append(json.loads(ln))
    return out


def main(d, untraced=None):
    from dragonboat_amd.build import source_digest
    cfgs = load_lines(untraced) if untraced else load_lines(os.path.join(d, "configs.json"))
    summ = {}
    pmc_path = os.path.join(d, "summary.json")
    pmc = json.load(open(pmc_path)) if os.path.exists(pmc_path) else {}
    out = {"source_digest": source_digest(), "hbm_peak_GBs": HBM_PEAK, "configs": {},
           "times_from": "untraced tools/bench_configs.py" if untraced else "the traced run"}
    for c in cfgs:
        key = c["config"].split(":")[0]
        ms = c["device_ms_per_pass"]
        row = {"config": c["config"], "groups": c["groups"], "replicas": c["replicas"],
               "device_ms_per_pass": ms, "general_lanes_per_pass": c.get("general_lanes_per_pass"),
               "escalations_per_pass": c.get("escalations_per_pass")}
        if "stream" in c:
            row["stream_ms_per_pass"] = c["stream"]["ms_per_pass"]
        if "graph" in c:
            row["graph_ms_per_pass"] = c["graph"]["ms_per_pass"]
        canon = canonical(c)
        row["canonical_bytes_per_pass"] = canon
        t = row.get("stream_ms_per_pass", ms)
        row["canonical_GBs"] = canon / (t * 1e-3) / 1e9
        row["canonical_frac"] = row["canonical_GBs"] / HBM_PEAK
        per = pmc.get("pmc", {}).get("config" + key)
        if per:
            # per pass: every dispatch's bytes over the run's passes (the kernel
            # launched every pass sets the count), so kernels a pass may skip (the
            # role instances) or alternatives (the steady kernel's LC and plain
            # instances) count by how often they ran, not once each
            npass = max((v.get("fetch_dispatches", 0) for v in per.values()), default=0)
            if npass and all("fetch_bytes_sum" in v for v in per.values()):
                hb = sum(v.get("fetch_bytes_sum", 0) + v.get("write_bytes_sum", 0) for v in per.values()) / npass
            else:  # summaries without sums (before round 6's LC instance): one launch of each per pass
                hb = sum(v.get("fetch_bytes_avg", 0) + v.get("write_bytes_avg", 0) for v in per.values())
            row["pmc_bytes_per_pass"] = hb
            row["pmc_by_kernel"] = {k: {"fetch": v.get("fetch_bytes_avg"), "write": v.get("write_bytes_avg"),
                                        "dispatches": v.get("fetch_dispatches")}
                                    for k, v in per.items()}
            row["pmc_passes"] = npass
            row["pmc_over_canonical"] = hb / canon
            row["pmc_GBs"] = hb / (ms * 1e-3) / 1e9
        row["fast_ms"], row["general_ms"] = c.get("fast_ms"), c.get("general_ms")
        out["configs"][key] = row
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
