"""Parity helpers: compare engine outputs (GPU kernel or the test-only host-lane
build of the same code) with the oracle, field by field, bit-exact.

States are compared on every field of gr_peer except the term-run window,
which is checked semantically: every device run must describe the oracle's log
exactly over [run_start[0], last_index] (the device may know fewer old runs
than the oracle after dropping its oldest run, never a different term).
Messages are compared per (sender, target slot) as ordered lists: the
reference orders broadcasts by Go map iteration, so only per-target order is
defined.
"""
import numpy as np

from dragonboat_amd import abi

SCALARS = ["term", "vote", "committed", "applied", "last_index", "first_index_m1", "leader_id",
           "leader_transfer_target", "node_id", "election_tick", "heartbeat_tick",
           "randomized_election_timeout", "election_timeout", "heartbeat_timeout", "entry_size_ub",
           "state", "self_slot", "flags", "read_index_count", "saved_to", "marker_index", "log_applied"]
MSG_FIELDS = ["type", "slot", "reject", "term", "log_index", "log_term", "commit", "hint", "hint_high",
              "n_entries", "n_runs", "run2_offset"]


def oracle_runs(o):
    return [(int(o["run_start"][k]), int(o["run_term"][k])) for k in range(int(o["n_runs"]))]


def term_at(runs, lo, hi, idx):
    if idx < lo or idx > hi:
        return 0
    t = None
    for s, tt in runs:
        if s <= idx:
            t = tt
    return t


def window_consistent(g, o):
    """Device window g agrees with oracle export o wherever g claims knowledge."""
    gr_ = oracle_runs(g)
    orr = oracle_runs(o)
    lo, hi = int(o["first_index_m1"]), int(o["last_index"])
    if int(g["last_index"]) != hi:
        return False, "last_index"
    if not gr_:
        return True, ""
    if orr and gr_[0][0] < orr[0][0]:
        return False, f"device window starts below oracle window {gr_[0][0]} < {orr[0][0]}"
    for k, (s, t) in enumerate(gr_):
        end = gr_[k + 1][0] - 1 if k + 1 < len(gr_) else hi
        if s > end:
            return False, f"empty run {k}"
        if term_at(orr, lo, hi, s) != t or term_at(orr, lo, hi, end) != t:
            return False, f"run {k} ({s},{t}) disagrees with oracle {orr}"
        if k > 0 and term_at(orr, lo, hi, s - 1) == t:
            return False, f"run boundary {s} is not a term change in {orr}"
    return True, ""


def compare_peer(g, o, S):
    diffs = []
    for f in SCALARS:
        if g[f] != o[f]:
            diffs.append(f"{f}: engine={g[f]} oracle={o[f]}")
    for j in range(S):
        for f in ["match", "next", "snapshot_index", "state", "active", "kind"]:
            if g["remotes"][j][f] != o["remotes"][j][f]:
                diffs.append(f"remotes[{j}].{f}: engine={g['remotes'][j][f]} oracle={o['remotes'][j][f]}")
        if g["remote_id"][j] != o["remote_id"][j]:
            diffs.append(f"remote_id[{j}]")
    for q in range(int(o["read_index_count"])):
        for f in ["index", "ctx_low", "ctx_high", "from_slot", "ack_bits"]:
            if g["read_index"][q][f] != o["read_index"][q][f]:
                diffs.append(f"read_index[{q}].{f}: engine={g['read_index'][q][f]} oracle={o['read_index'][q][f]}")
    ok, why = window_consistent(g, o)
    if not ok:
        diffs.append("window: " + why)
    return diffs


def _exact_equal(eng, orc, S):
    """Vectorised screen: True where a peer equals the oracle on every compared
    field with an identical window (then compare_peer finds nothing)."""
    ok = np.ones(len(eng), bool)
    for f in SCALARS:
        ok &= eng[f] == orc[f]
    for f in ["match", "next", "snapshot_index", "state", "active", "kind"]:
        ok &= np.all(eng["remotes"][:, :S][f] == orc["remotes"][:, :S][f], axis=1)
    ok &= np.all(eng["remote_id"][:, :S] == orc["remote_id"][:, :S], axis=1)
    q = np.arange(abi.GR_Q)[None, :] < orc["read_index_count"][:, None].astype(np.int64)
    for f in ["index", "ctx_low", "ctx_high", "from_slot", "ack_bits"]:
        ok &= np.all((eng["read_index"][f] == orc["read_index"][f]) | ~q, axis=1)
    k = np.arange(abi.GR_K)[None, :] < orc["n_runs"][:, None].astype(np.int64)
    ok &= eng["n_runs"] == orc["n_runs"]
    ok &= np.all(((eng["run_start"] == orc["run_start"]) & (eng["run_term"] == orc["run_term"])) | ~k, axis=1)
    return ok


def normalize_marks(recs):
    """gr_peer.marker_index == 0 means a freshly loaded group (gpuraft.h): the
    engine and the oracle take marker = last + 1, saved_to = last, log_applied =
    first_index_m1. Returns a copy with those values filled in."""
    recs = recs.copy()
    fresh = recs["marker_index"] == 0
    recs["marker_index"] = np.where(fresh, recs["last_index"] + np.uint64(1), recs["marker_index"])
    recs["saved_to"] = np.where(fresh, recs["last_index"], recs["saved_to"])
    recs["log_applied"] = np.where(fresh, recs["first_index_m1"], recs["log_applied"])
    return recs


def compare_states(eng, orc, S, peers=None, limit=20):
    idx = np.arange(len(eng)) if peers is None else np.asarray(peers, np.int64)
    if len(idx) == 0:
        return []
    eng, orc = normalize_marks(eng), normalize_marks(orc)
    same = _exact_equal(eng[idx], orc[idx], S)
    bad = []
    for p in idx[~same]:  # field by field (the window compared semantically)
        d = compare_peer(eng[p], orc[p], S)
        if d:
            bad.append((int(p), d))
            if len(bad) >= limit:
                break
    return bad


def _norm(m):
    row = [int(m[f]) for f in MSG_FIELDS]
    nr = int(m["n_runs"])
    return tuple(row) + (int(m["run_term"][0]) if nr >= 1 else 0, int(m["run_term"][1]) if nr == 2 else 0)


def group_msgs(msgs):
    d = {}
    for m in msgs:
        d.setdefault((int(m["peer"]), int(m["slot"])), []).append(_norm(m))
    return d


def _norm_table(msgs):
    """_norm for every record at once: one uint64 row per message, ordered by
    (peer, slot) with arrival order kept inside a (peer, slot)."""
    order = np.lexsort((np.arange(len(msgs)), msgs["slot"], msgs["peer"]))
    m = msgs[order]
    nr = m["n_runs"].astype(np.int64)
    cols = [m["peer"].astype(np.uint64)] + [m[f].astype(np.uint64) for f in MSG_FIELDS]
    cols += [np.where(nr >= 1, m["run_term"][:, 0], 0).astype(np.uint64),
             np.where(nr == 2, m["run_term"][:, 1], 0).astype(np.uint64)]
    return np.stack(cols, axis=1) if len(m) else np.zeros((0, len(cols)), np.uint64)


def compare_msgs(eng_msgs, orc_msgs, limit=20):
    a, b = _norm_table(eng_msgs), _norm_table(orc_msgs)
    if a.shape == b.shape and np.array_equal(a, b):
        return []
    a, b = group_msgs(eng_msgs), group_msgs(orc_msgs)
    bad = []
    for k in sorted(set(a) | set(b)):
        if a.get(k, []) != b.get(k, []):
            bad.append((k, a.get(k, []), b.get(k, [])))
            if len(bad) >= limit:
                break
    return bad


RESULT_FIELDS = ["propose_result", "propose_first", "append_from", "n_ready", "n_forwarded", "forwarded_entries",
                 "committed", "last_index", "save_from", "term", "vote"]


def compare_results(eng_res, orc_res, limit=20, fields=None):
    """eng_res: results per lane (peer field); orc_res: per peer (prefix results)."""
    fields = fields or RESULT_FIELDS
    all_fields = fields
    if len(eng_res):
        o = orc_res[eng_res["peer"].astype(np.int64)]
        same = np.ones(len(eng_res), bool)
        for f in fields:
            same &= eng_res[f] == o[f]
        q = np.arange(abi.GR_Q)[None, :] < np.minimum(eng_res["n_ready"], abi.GR_Q)[:, None].astype(np.int64)
        for f in ["index", "ctx_low", "ctx_high"]:
            same &= np.all((eng_res["ready"][f] == o["ready"][f]) | ~q, axis=1)
        eng_res = eng_res[~same]
    bad = []
    for r in eng_res:
        p = int(r["peer"])
        o = orc_res[p]
        fields = all_fields
        d = [f"{f}: engine={r[f]} oracle={o[f]}" for f in fields if r[f] != o[f]]
        for q in range(min(int(r["n_ready"]), abi.GR_Q)):
            if tuple(r["ready"][q]) != tuple(o["ready"][q]):
                d.append(f"ready[{q}]: engine={r['ready'][q]} oracle={o['ready'][q]}")
        if d:
            bad.append((p, d))
            if len(bad) >= limit:
                break
    return bad


def limits_from(results, n):
    lim = np.full(n, 0xFFFFFFFF, np.uint32)
    for r in results:
        if r["escalation"]:
            lim[int(r["peer"])] = r["esc_item"]
    return lim


def prefix_msgs(orc, limits):
    """Oracle messages emitted by items the engine applied (item < limit of their sender)."""
    m, it = orc["msgs"], orc["items"]
    if len(m) == 0:
        return m
    keep = it < limits[m["peer"].astype(np.int64)]
    return m[keep]


def check_escalations(results, esc_mask, limit=20):
    """Every escalation the engine reported must be one the oracle's own execution
    of that item justifies (oracle.pyoracle step(..)["esc_mask"], bit = reason):
    an item handed to the host too early, or for a reason the reference behaviour
    does not show, fails. Returns [(peer, item, reason, justified reasons)]."""
    bad = []
    for r in results[results["escalation"] != 0]:
        p, why = int(r["peer"]), int(r["escalation"])
        m = int(esc_mask[p])
        if not (m >> why) & 1:
            bad.append((p, int(r["esc_item"]), abi.ESC_NAMES[why],
                        [abi.ESC_NAMES[b] for b in range(len(abi.ESC_NAMES)) if (m >> b) & 1]))
            if len(bad) >= limit:
                break
    return bad


def update_commits(recs):
    """The pb.UpdateCommit a host sends back after persisting and applying
    everything a pass left (oracle commit_all: entriesToSave -> LogDB, AppliedTo =
    committed), from exported records: abi.UPDATE_COMMIT per record."""
    r = normalize_marks(recs)
    last, mk, sv = r["last_index"], r["marker_index"], r["saved_to"]
    idx = sv + np.uint64(1)
    nothing = (idx - mk) > (last + np.uint64(1) - mk)  # uint64 wrap, inmemory.go:101-108
    has = ~nothing & (idx <= last)
    nr = r["n_runs"].astype(np.int64)
    last_term = r["run_term"][np.arange(len(r)), np.maximum(nr - 1, 0)]
    uc = np.zeros(len(r), abi.UPDATE_COMMIT)
    uc["stable_log_to"] = np.where(has, last, 0)
    uc["stable_log_term"] = np.where(has, last_term, 0)
    uc["applied_to"] = np.where(r["committed"] > r["log_applied"], r["committed"], 0)
    return uc
