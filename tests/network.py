"""The reference's in-memory test network (internal/raft/raft_etcd_test.go:2803-2938)
over the engine, for its multi-node known-answer tests and BASELINE config 1.

Nodes 1..N of one group sit in engine slots (node - 1) * copies + c: `copies`
identical copies of the group are stepped side by side (one lane each), so
every known answer is checked on all of them. Each pass runs through
simulate.Lockstep: engine and oracle on identical inputs, compared bit-exactly,
escalations checked by the oracle's predicate, escalated items run by the
oracle (the host) and the group reloaded.

send(m...) mirrors network.send: it delivers the messages and runs passes until
nothing is in flight. The reference's FIFO hands one message at a time to
p.Handle; here every message in flight is delivered in the next pass (level by
level, each receiver in slot then arrival order). Messages that ticks produce
stay with their node until the next send, as in the reference, where a direct
r.tick() leaves them in r.msgs until the network reads them. drop/cut/isolate/
ignore/recover filter what the network carries (:2880-2927); the messages given
to send() are not filtered. The host applies what is committed after every pass
(raft.applied = committed), standing in for testOnlyHasConfigChangeToApply.
"""
import numpy as np

from dragonboat_amd import abi
import simulate as SIM


def node_records(ids, voters, copies=1, election=10, heartbeat=1, check_quorum=False, payload=8, rand_timeout=None):
    """newTestRaft / newTestObserver (raft_etcd_test.go:2955-2990) as engine
    records: term 0, empty log (marker 0), every remote next = 1, follower (or
    observer), randomizedElectionTimeout = election unless given."""
    M = len(ids)
    peers = np.zeros(M * copies, abi.PEER)
    for r, nid in enumerate(ids):
        v = peers[r * copies:(r + 1) * copies]
        v["node_id"] = nid
        v["election_timeout"] = election
        v["heartbeat_timeout"] = heartbeat
        v["randomized_election_timeout"] = rand_timeout or election
        v["entry_size_ub"] = 128 + payload
        v["n_runs"] = 1  # the marker (0, term 0)
        v["state"] = abi.FOLLOWER if nid in voters else abi.OBSERVER
        v["self_slot"] = r
        v["flags"] = abi.F_CHECK_QUORUM if check_quorum else 0
        for j, oid in enumerate(ids):
            v["remote_id"][:, j] = oid
            v["remotes"][:, j]["kind"] = abi.SLOT_VOTER if oid in voters else abi.SLOT_OBSERVER
            v["remotes"][:, j]["next"] = 1
    return peers


class Net:
    def __init__(self, backend, ids, voters=None, copies=1, records=None, max_entry_size=abi.MAX_ENTRY_SIZE, **kw):
        self.ids = list(ids)
        self.voters = set(voters if voters is not None else ids)
        self.G = copies
        self.M = len(self.ids)
        peers = records if records is not None else node_records(self.ids, self.voters, copies, **kw)
        self.ls = SIM.Lockstep(backend, peers, self.M, max_entry_size=max_entry_size)
        self.drops = set()
        self.ignored = set()
        self.held = np.zeros(0, abi.MESSAGE)  # produced by ticks, not yet read by the network
        self.passes = 0
        self.ready = {}  # node id -> ReadyToRead of copy 0, accumulated
        self.sent = []   # engine outbox records of every pass (device prefix)

    # ---- addressing
    def slot(self, nid):
        return self.ids.index(nid)

    def peer(self, nid, c=0):
        return self.slot(nid) * self.G + c

    def state(self, nid=None, c=0):
        st = self.ls.export()
        return st if nid is None else st[self.peer(nid, c)]

    def all_copies(self, nid):
        st = self.ls.export()
        return st[self.slot(nid) * self.G:(self.slot(nid) + 1) * self.G]

    def msg(self, frm, to, mtype, entries=0, **fields):
        """A message from node `frm` to node `to` (every copy); local messages have frm == to."""
        m = np.zeros(self.G, abi.MESSAGE)
        m["peer"] = [self.peer(to, c) for c in range(self.G)]
        m["slot"] = self.slot(frm)
        m["type"] = mtype
        if entries:
            m["n_entries"] = entries
            m["n_runs"] = 1
        for k, v in fields.items():
            m[k] = v
        return m

    # ---- network filters
    def cut(self, a, b):
        self.drops |= {(a, b), (b, a)}

    def isolate(self, nid):
        for o in self.ids:
            if o != nid:
                self.cut(nid, o)

    def ignore(self, mtype):
        self.ignored.add(mtype)

    def recover(self):
        self.drops = set()
        self.ignored = set()

    def _route(self, out):
        """Outbox records (sender peer, target slot) -> inbox records, filtered."""
        if len(out) == 0:
            return out
        sender_slot = out["peer"].astype(np.int64) // self.G
        copy = out["peer"].astype(np.int64) % self.G
        to_slot = out["slot"].astype(np.int64)
        keep = np.ones(len(out), bool)
        for k in range(len(out)):
            a, b = self.ids[sender_slot[k]], self.ids[to_slot[k]]
            if (a, b) in self.drops or int(out["type"][k]) in self.ignored:
                keep[k] = False
        nxt = out[keep].copy()
        nxt["peer"] = (to_slot[keep] * self.G + copy[keep]).astype(np.uint32)
        nxt["slot"] = sender_slot[keep].astype(np.uint8)
        return nxt

    def _pass(self, msgs, loc=None):
        out, res = self.ls.step(msgs, loc)
        self.ls.apply_all()
        self.passes += 1
        self.sent.append(self.ls.last_out)
        for p, lst in self.ls.last_ready.items():
            if p % self.G == 0:
                self.ready.setdefault(self.ids[p // self.G], []).extend(lst)
        return out

    def send(self, *msgs, max_passes=100):
        inflight = np.concatenate([self.held] + [np.asarray(m, abi.MESSAGE) for m in msgs])
        self.held = np.zeros(0, abi.MESSAGE)
        for _ in range(max_passes):
            if len(inflight) == 0:
                return
            inflight = self._route(self._pass(inflight))
        raise AssertionError("network did not quiesce")

    def locals_(self, per_node):
        """Local inputs: per_node = {nid: dict(ticks=.., read_index=.., ...)} for every copy."""
        loc = np.zeros(self.M * self.G, abi.LOCAL)
        loc["peer"] = np.arange(self.M * self.G)
        for nid, f in per_node.items():
            s = slice(self.slot(nid) * self.G, (self.slot(nid) + 1) * self.G)
            for k, v in f.items():
                loc[k][s] = v
        return loc

    def tick(self, nid, n=1):
        """r.tick() n times on node nid: its messages wait for the next send()."""
        for _ in range(n):
            out = self._pass(None, self.locals_({nid: {"ticks": 1}}))
            self.held = np.concatenate([self.held, self._route(out)])

    def local(self, per_node, deliver=True):
        """One pass with local inputs (ReadIndex, proposals); deliver = send() what it produced."""
        out = self._pass(None, self.locals_(per_node))
        self.held = np.concatenate([self.held, self._route(out)])
        if deliver:
            self.send()

    def close(self):
        self.ls.close()
