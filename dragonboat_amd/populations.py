"""Synthetic Raft group populations and replica topologies (BASELINE.json configs).

Peers are laid out replica-major: engine slot p = r * G + g holds replica r of
group g, so the followers of 64 consecutive groups are 64 consecutive slots and
every per-field access of a wave stays contiguous. Replica r of a group has
node id r + 1 and remote slot r in every member's slot table; replica 0 is the
leader unless a generator says otherwise.
"""
import numpy as np

from . import abi

NOPOS = 0xFFFFFFFF


def make_groups(G, R=3, seed=2, term_lo=1, term_hi=5, base_index=2**32, spread=2**20,
                election=10, heartbeat=1, check_quorum=False, payload=16, slots=None,
                log_span=1024, observers=0):
    """Steady-state groups: leader at term T, followers caught up, all committed.

    BASELINE config 2/4: T ~ U[term_lo, term_hi] and lastIndex = 2^32 + U[0, 2^20)
    (exercises the upper 32 bits of every index). A group has R voters (node ids
    1..R, replica 0 leads) and `observers` observers (node ids R+1..R+observers,
    raft.observers): M = R + observers members in slots 0..M-1 of every member."""
    M = R + observers
    S = slots or M
    assert S >= M
    rng = np.random.default_rng(seed)
    T = rng.integers(term_lo, term_hi + 1, G).astype(np.uint64)
    hi = (np.uint64(base_index) + rng.integers(0, spread, G).astype(np.uint64))
    lo = hi - np.uint64(log_span)
    peers = np.zeros(M * G, abi.PEER)
    for r in range(M):
        v = peers[r * G:(r + 1) * G]
        v["term"] = T
        v["vote"] = 1 if r < R else 0
        v["committed"] = hi
        v["applied"] = hi
        v["last_index"] = hi
        v["first_index_m1"] = lo
        v["leader_id"] = 1
        v["node_id"] = r + 1
        v["election_timeout"] = election
        v["heartbeat_timeout"] = heartbeat
        v["randomized_election_timeout"] = election + rng.integers(0, election, G)
        v["election_tick"] = 0 if r == 0 else rng.integers(0, election, G)
        v["entry_size_ub"] = 128 + payload
        two = T > 1
        v["n_runs"] = np.where(two, 2, 1)
        v["run_start"][:, 0] = lo
        v["run_term"][:, 0] = np.where(two, T - np.uint64(1), T)
        v["run_start"][:, 1] = np.where(two, hi, 0)
        v["run_term"][:, 1] = np.where(two, T, 0)
        for j in range(M):
            v["remote_id"][:, j] = j + 1
            v["remotes"][:, j]["kind"] = abi.SLOT_VOTER if j < R else abi.SLOT_OBSERVER
            if r == 0:  # leader: followers in Replicate state, caught up
                v["remotes"][:, j]["match"] = hi
                v["remotes"][:, j]["next"] = hi + np.uint64(1)
                v["remotes"][:, j]["state"] = abi.RETRY if j == 0 else abi.REPLICATE_ST
                v["remotes"][:, j]["active"] = 0 if j == 0 else 1
            else:  # follower / observer: remotes as reset() leaves them
                v["remotes"][:, j]["match"] = hi if j == r else 0
                v["remotes"][:, j]["next"] = hi + np.uint64(1)
                v["remotes"][:, j]["state"] = abi.RETRY
        v["state"] = abi.LEADER if r == 0 else (abi.FOLLOWER if r < R else abi.OBSERVER)
        v["self_slot"] = r
        v["flags"] = abi.F_CHECK_QUORUM if check_quorum else 0
    for j in range(M, S):
        peers["remotes"][:, j]["kind"] = abi.SLOT_EMPTY
    return peers


class Topology:
    """Replica-major topology: slot j of peer p talks to replica j of the same group."""

    def __init__(self, G, R):
        self.G, self.R = G, R
        p = np.arange(R * G, dtype=np.int64)
        self.group = p % G
        self.replica = p // G

    def dest(self, peer, slot):
        """Engine slot of the remote in `slot` of `peer`, and the sender's slot at the receiver."""
        peer = np.asarray(peer, np.int64)
        slot = np.asarray(slot, np.int64)
        return slot * self.G + peer % self.G, peer // self.G

    def route_messages(self, out):
        """Outbox records (peer = sender, slot = target) -> inbox records of the next pass.
        Records addressed outside the group (no remote slot) are dropped, as a
        transport drops messages to an unknown node."""
        out = out[out["slot"] < self.R]
        nxt = out.copy()
        dp, ds = self.dest(out["peer"], out["slot"])
        nxt["peer"] = dp.astype(np.uint32)
        nxt["slot"] = ds.astype(np.uint8)
        # stable order: by receiver, then sender slot, then arrival
        order = np.lexsort((np.arange(len(nxt)), nxt["slot"], nxt["peer"]))
        return nxt[order]

    def route_unsorted(self, out):
        """route_messages without the sort: gr_step groups the records by mailbox on
        the device (stable), so only the relative order of one sender's records to
        one target matters, and it is kept."""
        nxt = out.copy()
        dp, ds = self.dest(out["peer"], out["slot"])
        nxt["peer"] = dp.astype(np.uint32)
        nxt["slot"] = ds.astype(np.uint8)
        return nxt

    def loopback_routes(self, S):
        """in_pos/out_pos tables [S][n] for a one-space loopback.

        Mailbox (receiver q, sender slot j) sits at position j*n + q (slot-major),
        so the 64 lanes of a wave read and write 64 consecutive positions of
        every message field array (coalesced), receivers and senders alike."""
        n = self.R * self.G
        p = np.arange(n, dtype=np.int64)
        in_pos = np.full((S, n), NOPOS, np.uint32)
        out_pos = np.full((S, n), NOPOS, np.uint32)
        for j in range(self.R):
            other = self.replica != j
            in_pos[j, other] = (j * n + p[other]).astype(np.uint32)
            dp = j * self.G + self.group
            out_pos[j, other] = (self.replica[other] * n + dp[other]).astype(np.uint32)
        return in_pos, out_pos


def propose_locals(n_peers, leaders, entries=1, seed=0, pass_index=0, ticks=0, quiesced=None):
    """Per-pass local inputs: `entries` proposals on each leader slot, random draws for all."""
    loc = np.zeros(n_peers, abi.LOCAL)
    loc["peer"] = np.arange(n_peers, dtype=np.uint32)
    loc["propose_entries"][leaders] = entries
    loc["ticks"] = ticks
    if quiesced is not None:
        loc["quiesced_ticks"] = quiesced
    rng = np.random.default_rng([seed, pass_index])
    loc["rand"] = rng.integers(0, 2**63, n_peers, dtype=np.uint64)
    return loc


def _push_run(rec, start, term):
    n = int(rec["n_runs"])
    if n and int(rec["run_term"][n - 1]) == int(term):
        return
    if n < abi.GR_K:
        rec["run_start"][n] = start
        rec["run_term"][n] = term
        rec["n_runs"] = n + 1
    else:
        rec["run_start"][:-1] = rec["run_start"][1:].copy()
        rec["run_term"][:-1] = rec["run_term"][1:].copy()
        rec["run_start"][-1] = start
        rec["run_term"][-1] = term


def _last_term(rec):
    n = int(rec["n_runs"])
    return int(rec["run_term"][n - 1]) if n else 0


def inject_leader_change(state, topo, p, rng, max_div=8, max_extra=4):
    """BASELINE config 5 fault injection on settled groups (one leader, all at term T).

    The old leader L appended d+e entries at term T and replicated the first d
    only to follower F; F then wins an election for term T+1 (becomeLeader,
    raft.go:689-702: reset remotes, append a no-op). The third replica keeps its
    log. Next passes exercise rejects (Hint = lastIndex), decreaseTo/becomeRetry
    and getConflictIndex truncation of L's divergent suffix. Returns changed slots.
    """
    G, R = topo.G, topo.R
    st = state.reshape(R, G)
    terms = st["term"]
    leaders = st["state"] == abi.LEADER
    settled = (leaders.sum(0) == 1) & np.all(terms == terms[0], axis=0) & \
        np.all((st["state"] == abi.LEADER) | (st["state"] == abi.FOLLOWER) | (st["state"] == abi.OBSERVER), axis=0)
    cand = np.nonzero(settled & (rng.random(G) < p))[0]
    changed = []
    for g in cand:
        a = int(np.argmax(leaders[:, g]))
        voters = [r for r in range(R) if r != a and st["state"][r, g] == abi.FOLLOWER]
        if not voters:
            continue
        b = int(rng.choice(voters))
        L = state[a * G + g]
        F = state[b * G + g]
        T = int(L["term"])
        if _last_term(L) != T or _last_term(F) != T:
            continue
        d = int(rng.integers(1, max_div + 1))
        e = int(rng.integers(1, max_extra + 1))
        hi_a = int(L["last_index"])
        if int(F["last_index"]) > hi_a:
            continue
        L["last_index"] = hi_a + d + e
        hf = hi_a + d
        F["last_index"] = hf
        # F becomes leader for T+1
        F["term"] = T + 1
        F["vote"] = F["node_id"]
        F["state"] = abi.LEADER
        F["leader_id"] = F["node_id"]
        F["election_tick"] = 0
        F["heartbeat_tick"] = 0
        et = int(F["election_timeout"])
        F["randomized_election_timeout"] = et + int(rng.integers(0, et))
        F["read_index_count"] = 0
        F["read_index"] = np.zeros(abi.GR_Q, abi.READ_STATUS)
        F["leader_transfer_target"] = 0
        F["flags"] = int(F["flags"]) & ~abi.F_PENDING_CONFIG_CHANGE
        me = int(F["self_slot"])
        for j in range(R):
            F["remotes"][j]["next"] = hf + 1
            F["remotes"][j]["match"] = 0
            F["remotes"][j]["state"] = abi.RETRY
            F["remotes"][j]["active"] = 0
            F["remotes"][j]["snapshot_index"] = 0
        F["last_index"] = hf + 1
        _push_run(F, hf + 1, T + 1)
        F["remotes"][me]["match"] = hf + 1
        F["remotes"][me]["next"] = hf + 2
        changed += [a * G + g, b * G + g]
    return np.array(sorted(changed), np.int64)


def current_leaders(state, topo):
    """Slots of all peers in the leader state (proposal targets)."""
    return np.nonzero(state["state"] == abi.LEADER)[0]


def config3(G, R=5, seed=3, active_frac=0.1, election=10, heartbeat=1):
    """BASELINE config 3: G groups x R replicas, 90% quiesced, 10% active with a
    ReadIndex pending each pass; electionTick uniform in [0, ET), ET=10, HT=1,
    checkQuorum on for half of the groups (seed 3). Returns (peers, active[G])."""
    peers = make_groups(G, R, seed=seed, election=election, heartbeat=heartbeat)
    rng = np.random.default_rng([seed, 1])
    cq = rng.random(G) < 0.5
    active = rng.random(G) < active_frac
    for r in range(R):
        v = peers[r * G:(r + 1) * G]
        v["flags"] = np.where(cq, v["flags"] | abi.F_CHECK_QUORUM, v["flags"])
        v["election_tick"] = rng.integers(0, election, G)
    return peers, active


def config3_locals(G, R, active, pass_index, seed=3):
    """Per-pass inputs of config 3: quiesced groups get one QuiescedTick per
    replica; active groups one Tick per replica and a ReadIndex on the leader."""
    n = R * G
    rng = np.random.default_rng([seed, 2, pass_index])
    act = np.tile(active, R)
    loc = np.zeros(n, abi.LOCAL)
    loc["peer"] = np.arange(n, dtype=np.uint32)
    loc["quiesced_ticks"] = np.where(act, 0, 1)
    loc["ticks"] = np.where(act, 1, 0)
    lead = act & (np.arange(n) < G)
    loc["read_index"] = lead
    loc["read_ctx_low"] = np.where(lead, rng.integers(1, 2**63, n, dtype=np.uint64), 0)
    loc["read_ctx_high"] = np.where(lead, pass_index + 1, 0)
    loc["rand"] = rng.integers(0, 2**63, n, dtype=np.uint64)
    return loc


def drop_acks(msgs, p, rng):
    """Drop each HeartbeatResp with probability p (config 3: followers ack with 1 - p)."""
    if len(msgs) == 0:
        return msgs
    keep = ~((msgs["type"] == abi.HEARTBEAT_RESP) & (rng.random(len(msgs)) < p))
    return msgs[keep]


def inject_leader_transfer(state, topo, p, rng, lag_frac=0.5):
    """Leader transfer in flight (raft.go:1242-1262 handleLeaderLeaderTransfer):
    with probability p a settled group's leader gets leaderTransferTarget = a
    follower's node id, the target is flagged isLeaderTransferTarget, and for
    `lag_frac` of them the target lags (its match one below the leader's log, so
    the next ack that catches it up sends TimeoutNow, raft.go:1216-1219; a
    caught-up target gets TimeoutNow on its next ack). electionTick is reset as
    the handler does. Returns the changed slots."""
    G, M = topo.G, topo.R
    st = state.reshape(M, G)
    changed = []
    for g in np.nonzero(rng.random(G) < p)[0]:
        lead = np.nonzero(st["state"][:, g] == abi.LEADER)[0]
        if len(lead) != 1:
            continue
        a = int(lead[0])
        L = state[a * G + g]
        if int(L["leader_transfer_target"]):
            continue
        cands = [r for r in range(M) if r != a and int(L["remotes"][r]["kind"]) == abi.SLOT_VOTER]
        if not cands:
            continue
        b = int(rng.choice(cands))
        L["leader_transfer_target"] = int(L["remote_id"][b])
        L["election_tick"] = 0
        if rng.random() < lag_frac and int(L["remotes"][b]["match"]) > 0:
            L["remotes"][b]["match"] = int(L["remotes"][b]["match"]) - 1
        F = state[b * G + g]
        F["flags"] = int(F["flags"]) | abi.F_IS_LEADER_TRANSFER_TARGET
        changed += [a * G + g, b * G + g]
    return np.array(sorted(changed), np.int64)


def inject_snapshot_state(state, topo, p, rng):
    """Leader remotes in Snapshot state (remote.go:98-106 becomeSnapshot) with a
    Replicate already in flight to them: with probability p per group one of the
    leader's remotes gets state Snapshot and snapshotIndex at or below its match
    (the next accepted ack runs respondedTo -> becomeRetry, remote.go:130-138) or
    above it (the remote stays paused). Returns the changed slots."""
    G, M = topo.G, topo.R
    st = state.reshape(M, G)
    changed = []
    for g in np.nonzero(rng.random(G) < p)[0]:
        lead = np.nonzero(st["state"][:, g] == abi.LEADER)[0]
        if len(lead) != 1:
            continue
        a = int(lead[0])
        L = state[a * G + g]
        js = [j for j in range(M) if j != int(L["self_slot"]) and int(L["remotes"][j]["kind"]) != abi.SLOT_EMPTY]
        if not js:
            continue
        j = int(rng.choice(js))
        m = int(L["remotes"][j]["match"])
        L["remotes"][j]["state"] = abi.SNAPSHOT_ST
        L["remotes"][j]["snapshot_index"] = max(1, m - int(rng.integers(0, 3))) if rng.random() < 0.7 else m + 3
        changed.append(a * G + g)
    return np.array(sorted(changed), np.int64)
