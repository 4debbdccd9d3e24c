"""Workloads that reach every branch of the lane code (gr_cover.h ids), run
through an engine backend against the oracle (simulate.Lockstep checks state,
messages, results and escalations every pass). Used by tests/test_coverage.py
with the coverage builds (the host lane on the CPU, libgpuraft_cover.so on the
GPU): the blind-spot and network workloads, a message fuzz, and targeted
single-pass states for the rare escalations."""
import numpy as np

from dragonboat_amd import abi, populations as P
import simulate as SIM
from network import Net
import test_blindspots as BS
import test_network_kat as KAT

FUZZ_TYPES = [abi.UNREACHABLE, abi.SNAPSHOT_STATUS, abi.LEADER_HEARTBEAT, abi.CHECK_QUORUM, abi.ELECTION,
              abi.NOOP, abi.READ_INDEX, abi.LEADER_TRANSFER, abi.PROPOSE, abi.TIMEOUT_NOW,
              abi.INSTALL_SNAPSHOT, abi.REQUEST_VOTE, abi.REQUEST_VOTE_RESP, abi.HEARTBEAT,
              abi.HEARTBEAT_RESP, abi.REPLICATE_RESP, abi.REPLICATE, abi.READ_INDEX_RESP, abi.PING]


def fuzz(backend, G=200, passes=10, seed=7):
    """Random message types at random members (3 voters + 1 observer, some
    followers turned candidates), terms one below / equal / above / zero, on
    top of steady proposals, ticks and ReadIndex."""
    R, obs = 3, 1
    M = R + obs
    peers = P.make_groups(G, R, seed=seed, observers=obs, check_quorum=True)
    cand = np.random.default_rng(seed).random(G) < 0.1
    f = peers[G:2 * G]
    f["state"][cand] = abi.CANDIDATE
    f["vote"][cand] = 2
    topo = P.Topology(G, M)

    def extra(k, state):
        rng = np.random.default_rng([seed, 100, k])
        n = G // 2
        m = np.zeros(n, abi.MESSAGE)
        at = rng.integers(0, M, n)
        g = rng.integers(0, G, n)
        m["peer"] = at * G + g
        frm = (at + rng.integers(1, M, n)) % M
        local = rng.random(n) < 0.25
        m["slot"] = np.where(local, at, frm)
        m["type"] = rng.choice(FUZZ_TYPES, n)
        term = state["term"][m["peer"]].astype(np.int64)
        dt = rng.choice([-1, 0, 0, 0, 1, 2], n)
        t = np.maximum(term + dt, 0)
        t = np.where(rng.random(n) < 0.15, 0, t)
        m["term"] = t.astype(np.uint64)
        hi = state["last_index"][m["peer"]].astype(np.int64)
        com = state["committed"][m["peer"]].astype(np.int64)
        li = np.maximum(hi - rng.integers(-1, 4, n), 0)
        m["log_index"] = li
        m["log_term"] = np.where(rng.random(n) < 0.7, t, np.maximum(t - 1, 0)).astype(np.uint64)
        m["commit"] = np.minimum(com + rng.integers(0, 2, n), hi)
        m["reject"] = rng.random(n) < 0.3
        m["hint"] = np.where(rng.random(n) < 0.5, rng.integers(1, 2**40, n), hi)
        m["hint_high"] = rng.integers(0, 3, n)
        ne = np.where(np.isin(m["type"], [abi.REPLICATE, abi.PROPOSE]), rng.integers(0, 3, n), 0)
        m["n_entries"] = ne
        m["n_runs"] = (ne > 0).astype(np.uint8)
        m["run_term"][:, 0] = np.where(ne > 0, np.where(m["type"] == abi.PROPOSE, 0, t), 0)
        # two runs (t-1, t): a leader never sends an entry above its own term, so the
        # message stays one a real leader could send (the checked build's
        # BAD_LAST_TERM_ABOVE_TERM counts what the device does to valid input)
        two = (ne == 2) & (rng.random(n) < 0.3) & (m["type"] == abi.REPLICATE) & (t >= 1)
        m["n_runs"] = np.where(two, 2, m["n_runs"])
        m["run2_offset"] = np.where(two, 1, 0)
        m["run_term"][:, 1] = np.where(two, t, 0)
        m["run_term"][:, 0] = np.where(two, t - 1, m["run_term"][:, 0])
        return m
    return SIM.simulate(backend, peers, topo, passes, BS._locals(M, G, seed + 1, tick=0.4, ri=0.2,
                                                                 prop_everywhere=0.1),
                        slots=M, extra_fn=extra, allow_error=True)


def _one_pass(backend, peers, slots, msgs=None, loc=None, max_entry_size=abi.MAX_ENTRY_SIZE):
    ls = SIM.Lockstep(backend, peers, slots, max_entry_size=max_entry_size, allow_error=True)
    try:
        out, res = ls.step(msgs, loc)
        return res
    finally:
        ls.close()


def targeted(backend):
    """Single-pass states for the rare escalations and drops; returns {name: escalation reasons}."""
    G, R = 64, 3
    got = {}

    def esc(res):
        return {abi.ESC_NAMES[int(r["escalation"])] for r in res if r["escalation"]}

    lead = np.arange(G)
    # ENTRY_SIZE: a follower 4 entries behind with MaxEntrySize fitting one entry
    p = P.make_groups(G, R, seed=1)
    hi = p["last_index"][lead]
    p["remotes"]["next"][lead, 1] = hi - np.uint64(3)
    p["remotes"]["match"][lead, 1] = hi - np.uint64(4)
    got["entry_size"] = esc(_one_pass(backend, p, R, loc=P.propose_locals(R * G, lead), max_entry_size=200))
    # MSG_RUNS: the follower's next entries span three term runs
    p = P.make_groups(G, R, seed=2, term_lo=5, term_hi=5)
    lo = p["first_index_m1"]
    p["n_runs"] = 3
    p["run_start"][:, 0], p["run_term"][:, 0] = lo, 3
    p["run_start"][:, 1], p["run_term"][:, 1] = lo + np.uint64(10), 4
    p["run_start"][:, 2], p["run_term"][:, 2] = lo + np.uint64(20), 5
    p["remotes"]["next"][lead, 1] = lo[lead] + np.uint64(5)
    p["remotes"]["match"][lead, 1] = lo[lead] + np.uint64(4)
    got["msg_runs"] = esc(_one_pass(backend, p, R, loc=P.propose_locals(R * G, lead)))
    # TERM_WINDOW: the window starts above firstIndex-1 and a follower's next is below it
    p = P.make_groups(G, R, seed=3)
    lo = p["first_index_m1"]
    p["run_start"][:, 0] = lo + np.uint64(50)
    p["remotes"]["next"][lead, 2] = lo[lead] + np.uint64(10)
    p["remotes"]["match"][lead, 2] = lo[lead] + np.uint64(9)
    got["term_window"] = esc(_one_pass(backend, p, R, loc=P.propose_locals(R * G, lead)))
    # SNAPSHOT: a follower's next at or below firstIndex-1 (InstallSnapshot path)
    p = P.make_groups(G, R, seed=4)
    p["remotes"]["next"][lead, 1] = p["first_index_m1"][lead]
    p["remotes"]["match"][lead, 1] = p["first_index_m1"][lead] - np.uint64(1)
    got["snapshot"] = esc(_one_pass(backend, p, R, loc=P.propose_locals(R * G, lead)))
    # NONMEMBER: followers forward a proposal to a leader id outside their slot table
    p = P.make_groups(G, R, seed=5)
    fol = np.arange(G, 2 * G)
    p["leader_id"][fol] = 99
    got["nonmember"] = esc(_one_pass(backend, p, R, loc=P.propose_locals(R * G, fol)))
    # PANIC: a Heartbeat committing past the follower's lastIndex (commitTo panics)
    p = P.make_groups(G, R, seed=6)
    hb = np.zeros(G, abi.MESSAGE)
    hb["peer"], hb["type"], hb["slot"] = fol, abi.HEARTBEAT, 0
    hb["term"] = p["term"][fol]
    hb["commit"] = p["last_index"][fol] + np.uint64(5)
    got["panic"] = esc(_one_pass(backend, p, R, msgs=hb))
    # RANDOM: two term bumps in one pass need two random draws
    p = P.make_groups(G, R, seed=7)
    two = np.zeros(2 * G, abi.MESSAGE)
    two["peer"] = np.repeat(fol, 2)
    two["type"], two["slot"] = abi.HEARTBEAT, 0
    two["term"] = np.repeat(p["term"][fol], 2) + np.tile(np.array([1, 2], np.uint64), G)
    got["random"] = esc(_one_pass(backend, p, R, msgs=two))
    # CONFIG_CHANGE: a leader's local proposal carries a ConfigChangeEntry
    p = P.make_groups(G, R, seed=8)
    loc = P.propose_locals(R * G, lead)
    loc["propose_has_config_change"][lead] = 1
    got["config_change"] = esc(_one_pass(backend, p, R, loc=loc))
    # selfRemoved leader drops its proposal (raft.go:1126-1129)
    p = P.make_groups(G, R, seed=9)
    for f in ("kind", "match", "next", "state", "active"):
        p["remotes"][f][lead, 0] = 0  # slot 0 (the leader itself) left the membership
    p["self_slot"][lead] = abi.GR_SLOT_NONE
    loc = P.propose_locals(R * G, lead, ticks=1)  # with a tick: the general lane, not the lean one
    got["self_removed"] = esc(_one_pass(backend, p, R, loc=loc))
    # a response from an empty slot is dropped (Peer.Handle, peer.go:199-209)
    p = P.make_groups(G, R, seed=10, slots=4)
    rs = np.zeros(G, abi.MESSAGE)
    rs["peer"], rs["type"], rs["slot"] = lead, abi.HEARTBEAT_RESP, 3
    rs["term"] = p["term"][lead]
    got["nonmember_resp"] = esc(_one_pass(backend, p, 4, msgs=rs))
    # a duplicate ReadIndex context (readIndex.addRequest ignores it, readindex.go:44-46):
    # a follower's forwarded request and the leader's own with the same context
    p = P.make_groups(G, R, seed=11)
    ri = np.zeros(G, abi.MESSAGE)
    ri["peer"], ri["type"], ri["slot"], ri["hint"], ri["hint_high"] = lead, abi.READ_INDEX, 1, 777, 1
    loc = P.propose_locals(R * G, [])
    loc["read_index"][lead] = 1
    loc["read_ctx_low"][lead], loc["read_ctx_high"][lead] = 777, 1
    got["ri_dup"] = esc(_one_pass(backend, p, R, msgs=ri, loc=loc))
    # QuiescedTick: alone (the lean lane) and after a message (the general lane)
    p = P.make_groups(G, R, seed=12)
    loc = P.propose_locals(R * G, [], quiesced=3)
    hb = np.zeros(G, abi.MESSAGE)
    hb["peer"], hb["type"], hb["slot"] = np.arange(G, 2 * G), abi.HEARTBEAT, 0
    hb["term"] = p["term"][G:2 * G]
    hb["commit"] = p["committed"][G:2 * G]
    got["qtick"] = esc(_one_pass(backend, p, R, msgs=hb, loc=loc))
    return got


def quiesced(backend, G=256, passes=6, seed=13):
    """A quiesced population (QuiescedTick only) between steady passes: the lean
    lane's quiesced path and, on split passes, the steady kernel's quiet_step."""
    R = 3
    peers = P.make_groups(G, R, seed=seed)
    topo = P.Topology(G, R)

    def lf(k):
        if k % 3 == 2:
            return P.propose_locals(R * G, np.arange(G), pass_index=k)
        return P.propose_locals(R * G, [], pass_index=k, quiesced=1 + k % 2)
    return SIM.simulate(backend, peers, topo, passes, lf)


def device_battery(lib_path):
    """The device-resident split schedule (devsim.DeviceLockstep, split forced on
    a small population): the steady kernel's closed-form leader and follower
    lanes and quiet_step, the role instances, staggered acks, leader changes; oracle
    every pass. Returns the stats of each run."""
    import os
    import devsim
    out = {}
    saved = {k: os.environ.get(k) for k in ("GR_SPLIT_MIN_LANES", "GR_SMALL_BLOCKS", "GR_TAIL_MODE")}
    os.environ["GR_SPLIT_MIN_LANES"] = "1"  # all three read at gr_create
    os.environ["GR_SMALL_BLOCKS"] = "0"     # not the fused small-pass kernel
    os.environ["GR_TAIL_MODE"] = "1"        # the role instances every pass
    try:
        G, R = 1024, 3
        topo = P.Topology(G, R)
        rng = np.random.default_rng(17)
        ls = devsim.DeviceLockstep(P.make_groups(G, R, seed=17), G, R, lib_path=lib_path)
        try:
            for k in range(15):
                if k in (11, 13):
                    cur = ls.export()
                    ch = P.inject_leader_change(cur, topo, 0.2, rng)
                    ls.inject(ch, cur[ch])
                if 3 <= k <= 9:  # quiesced passes; once the messages die out, waves lose
                    # their hints (FastLane's quiesced path) and the steady kernel's quiet_step runs
                    loc = P.propose_locals(R * G, [], pass_index=k, quiesced=1)
                else:
                    loc = P.propose_locals(R * G, P.current_leaders(ls.export(), topo), pass_index=k)
                ls.step(loc)
            out["device_split"] = dict(ls.stats)
        finally:
            ls.close()
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return out


def battery(backend):
    """Everything above plus the blind-spot and network workloads (small sizes)."""
    class Req:  # the tests' fixture lookup, satisfied by the caller
        def getfixturevalue(self, name):
            return None
    out = {"fuzz": fuzz(backend)["esc_reasons"], "targeted": targeted(backend),
           "quiesced": quiesced(backend)["commits"]}
    be = "gpu" if backend is SIM.GpuBackend else "cpu"
    req = Req()
    for R, obs in [(2, 1), (3, 2)]:
        BS.test_observers(be, R, obs, req)
    for obs in (0, 1):
        BS.test_single_voter(be, obs, req)
    BS.test_leader_transfer(be, req)
    BS.test_snapshot_state_remotes(be, req)
    BS.test_terms_straddling_2_32(be, req)
    for ht in (1, 2):
        BS.test_check_quorum_step_down(be, ht, req)
    KAT.test_log_replication(be, 1, req)
    KAT.test_cannot_commit_without_new_term_entry(be, req)
    KAT.test_bcast_beat(be, req)
    KAT.test_leader_transfer_timeout(be, req)
    KAT.test_read_index_leader_can_be_confirmed(be, req)
    KAT.test_observer_can_read_index(be, [1], req)
    KAT.test_observer_can_read_index(be, [1, 2], req)
    KAT.test_leader_read_index_committed_at_term(be, True, req)
    KAT.test_leader_read_index_committed_at_term(be, False, req)
    return out
