"""Multi-pass simulations of replicated groups: the engine (GPU kernel, or the
test-only host build of the same lane code) against the oracle, compared
bit-exactly after every pass.

Escalation protocol (what the Go host does in production): a group that
escalates at item i keeps the device's state after items < i; the host runs
items >= i with the reference code and reloads the group. Here the oracle plays
the host: its prefix snapshot is compared with the device, its full-pass state
is what both sides continue from, and its full message list is routed. Every
escalation must be one the oracle's own execution of that item justifies
(parity.check_escalations).

A peer whose full state no longer fits a gr_peer record (e.g. more than GR_Q
pending ReadIndex requests) is "parked": the host steps it alone (the engine
gets no input for it) until it fits again, then it is reloaded.
"""
import os

import numpy as np

from dragonboat_amd import abi
from oracle.pyoracle import OraclePopulation, hostlane_step
import parity


class HostlaneBackend:
    def __init__(self, peers, slots, max_entry_size=abi.MAX_ENTRY_SIZE):
        self.state = np.array(peers, abi.PEER, copy=True)
        self.slots = slots
        self.max_entry_size = max_entry_size

    def step(self, msgs, loc):
        self.state, out, res = hostlane_step(self.state, msgs, loc, self.slots, self.max_entry_size)
        return out, res

    def sync(self):
        return self.state.copy()

    def load(self, idx, recs):
        self.state[idx] = recs

    def notify_applied(self, idx, applied):
        self.state["applied"][idx] = applied

    def commit_update(self, idx, uc):
        from oracle.pyoracle import hostlane_commit_update
        rc, st = hostlane_commit_update(self.state, idx, uc, self.slots)
        assert rc == 0, (rc, st[st != 0][:5])

    def close(self):
        pass


class GpuBackend:
    lib_path = None  # a different build of libgpuraft (e.g. the coverage build)

    def __init__(self, peers, slots, max_entry_size=abi.MAX_ENTRY_SIZE):
        from dragonboat_amd.engine import Engine
        self.eng = Engine(len(peers), slots, max_entry_size=max_entry_size, lib_path=self.lib_path)
        self.eng.load(peers)
        self.n = len(peers)

    def step(self, msgs, loc):
        return self.eng.step(msgs, loc)

    def sync(self):
        return self.eng.sync(self.n)

    def load(self, idx, recs):
        self.eng.load_peers(np.asarray(idx, np.uint32), np.asarray(recs, abi.PEER))  # one call, scattered slots

    def notify_applied(self, idx, applied):
        self.eng.notify_applied(np.asarray(idx, np.uint32), np.asarray(applied, np.uint64))

    def commit_update(self, idx, uc):
        rc, st = self.eng.commit_update(np.asarray(idx, np.uint32), uc)
        assert rc == 0, (rc, st[st != 0][:5])

    def close(self):
        self.eng.close()


class GpuCompactBackend(GpuBackend):
    """The compact boundary (gr_step_compact): records packed with
    gr_pack_messages/gr_pack_locals, outputs expanded back to full records so the
    Lockstep compares them with the oracle like any other backend. A compact
    result carries no append_from (save_from replaces it for persistence); its
    term/vote are the synced state's (a change would have made it an ext record)."""
    result_fields = [f for f in parity.RESULT_FIELDS if f != "append_from"]

    halves = False  # GpuCompactHalvesBackend: gr_step_compact_begin + _end

    def step(self, msgs, loc):
        cm, xm = self.eng.pack_messages(msgs)
        cm = self.eng.pair_messages(cm)  # the device takes GR_CM_PAIR records as two messages
        cl, xl = self.eng.pack_locals(loc)
        om, ox, cr, rx = self.eng.step_compact(cm, xm, cl, xl, halves=self.halves)
        return self.expand(om, ox, cr, rx, loc)

    def expand(self, om, ox, cr, rx, loc):
        """Compact outputs -> full outbox and result records (the Lockstep's form)."""
        out = self.eng.unpack_messages(om, ox)
        res = np.zeros(len(cr), abi.RESULT)
        for f in ("peer", "escalation", "propose_result", "last_index"):
            res[f] = cr[f]
        # gpuraft.h gr_cresult: indexes relative to last_index, aux = esc_item (not EXT)
        res["esc_item"] = cr["aux"]
        res["committed"] = cr["last_index"] - cr["commit_lag"]
        sc = cr["save_count"].astype(np.uint64)
        res["save_from"] = np.where(sc > 0, cr["last_index"] - sc + np.uint64(1), 0)
        st = self.eng.sync(self.n)
        p = cr["peer"].astype(np.int64)
        res["term"], res["vote"] = st["term"][p], st["vote"][p]
        nprop = np.zeros(self.n, np.uint64)
        if len(loc):
            nprop[loc["peer"].astype(np.int64)] = loc["propose_entries"]
        app = cr["propose_result"] == abi.PROP_APPENDED
        res["propose_first"] = np.where(app, cr["last_index"] - nprop[p] + np.uint64(1), 0)
        x = (cr["flags"] & abi.CR_EXT) != 0
        if x.any():
            res[x] = rx[cr["aux"][x].astype(np.int64)]
        return out, res


class GpuCompactHalvesBackend(GpuCompactBackend):
    """gr_step_compact as its two halves (the pipelined host path)."""
    halves = True


class GpuWireBackend(GpuBackend):
    """The wire path (gr_step_wire): the inbox records become MessageBatch frames
    (tests/wirefeed.py, the senders' transports), the frames are the only inbox
    bytes uploaded, libgrwire decodes them in HBM, and the engine routes the
    decoded records straight into the pass. Every message must route (the
    populations' messages are all between members)."""
    cluster_of = None  # slot -> cluster id; default: replica-major groups (slot % G) + 1

    def __init__(self, peers, slots, max_entry_size=abi.MAX_ENTRY_SIZE):
        super().__init__(peers, slots, max_entry_size=max_entry_size)
        import wirefeed
        n = len(peers)
        cl = self.cluster_of
        if cl is None:
            G = n // slots if slots and n % slots == 0 else n
            cl = (np.arange(n) % G) + 1
        self.feed = wirefeed.WireFeed(peers, cl)
        self.eng.bind_nodes(cl, np.asarray(peers["node_id"], np.uint64))

    def step(self, msgs, loc):
        dm, nm, de, ne, keep = self.feed.decode(msgs)
        out, res, idx, why = self.eng.step_wire(dm, nm, de, ne, loc)
        assert len(idx) == 0, [abi.WIRE_REASONS[w] for w in why[:4]]
        return out, res

    def close(self):
        self.feed.close()
        super().close()


class GpuWireCompactBackend(GpuWireBackend):
    """The wire path with the compact outbox (gr_step_wire_compact): frames in,
    24-B gr_cmsg / gr_cresult records (ext records where they do not fit) out,
    expanded as GpuCompactBackend expands gr_step_compact's."""
    result_fields = GpuCompactBackend.result_fields
    expand = GpuCompactBackend.expand

    def step(self, msgs, loc):
        dm, nm, de, ne, keep = self.feed.decode(msgs)
        got, idx, why = self.eng.step_wire(dm, nm, de, ne, loc, compact=True)
        assert len(idx) == 0, [abi.WIRE_REASONS[w] for w in why[:4]]
        om, ox, cr, rx = got
        return self.expand(om, ox, cr, rx, loc)


def res_esc_free(res, n):
    """Peers that did not escalate this pass (their device state is the pass's)."""
    ok = np.ones(n, bool)
    esc = res[res["escalation"] != 0]
    ok[esc["peer"].astype(np.int64)] = False
    return ok


def _threads():
    return min(16, os.cpu_count() or 1)


class Lockstep:
    """The engine and the oracle stepped pass by pass on identical inputs.

    step(msgs, loc) runs one pass over inbox records `msgs` (receiver peer,
    sender slot) and local inputs `loc` on both sides, checks state, messages,
    results and escalations, reloads escalated peers from the oracle (the host's
    role) and returns (oracle outbox records, engine results). The oracle's full
    outbox is what the network delivers next."""

    def __init__(self, backend, peers, slots, max_entry_size=abi.MAX_ENTRY_SIZE, check=True, max_report=3,
                 allow_error=False):
        self.pop = OraclePopulation(peers, slots, max_entry_size=max_entry_size)
        self.eng = backend(peers, slots, max_entry_size=max_entry_size)
        self.n = len(peers)
        self.slots = slots
        self.check = check
        self.max_report = max_report
        self.allow_error = allow_error  # reference panics (and records the network cannot carry) tolerated
        self.errors = 0
        self.parked = np.zeros(self.n, bool)
        self.k = 0
        self.stats = {"msgs": 0, "escalations": 0, "esc_reasons": {}, "commits": 0, "ready": 0, "forwarded": 0,
                      "parked": 0, "snapshot_left": 0}
        self.last_out = np.zeros(0, abi.MESSAGE)  # the engine's outbox of the last pass (device prefix)
        self.last_ready = {}                      # peer -> [(index, ctx_low, ctx_high)] of the last pass

    def export(self):
        return self.pop.export()

    def reload(self, idx, recs):
        """Host-side state edits (fault injection): both sides."""
        idx = np.asarray(idx, np.int64)
        if len(idx):
            self.pop.reload(idx, recs)
            self.eng.load(idx, recs)

    def apply_all(self):
        """The host applies what is committed (node.handleEvents ->
        Peer.NotifyRaftLastApplied, peer.go:282-284): raft.applied = committed."""
        keep = np.nonzero(~self.parked)[0]
        uc = parity.update_commits(self.pop.export()[keep])  # what the host persisted and applied
        self.pop.commit_all()
        cur = self.pop.export()
        self.eng.commit_update(keep, uc)  # entryLog.commitUpdate on the device
        self.eng.notify_applied(keep, cur["committed"][keep])

    def step(self, msgs, loc):
        msgs = np.zeros(0, abi.MESSAGE) if msgs is None else np.asarray(msgs, abi.MESSAGE)
        loc = np.zeros(0, abi.LOCAL) if loc is None else np.asarray(loc, abi.LOCAL)
        st, parked = self.stats, self.parked
        dev0 = self.eng.sync() if self.check else None
        before = dev0["committed"] if self.check else None
        emsgs = msgs[~parked[msgs["peer"]]] if len(msgs) else msgs
        eloc = loc[~parked[loc["peer"]]] if len(loc) else loc
        out, res = self.eng.step(emsgs, eloc)
        if len(out):  # the engine's outbox is valid gr_step input (gr_host.h validate_msg)
            nr, ne = out["n_runs"], out["n_entries"]
            assert np.all(nr <= 2) and np.all((ne == 0) == (nr == 0)), "invalid outbox record"
            assert np.all(out["type"] <= abi.TIMEOUT_NOW)
        lim = parity.limits_from(res, self.n)
        o = self.pop.step(msgs, loc, lim, threads=_threads(), dev_before=dev0, allow_error=self.allow_error)
        self.errors += bool(o["error"])
        esc = res[res["escalation"] != 0]
        st["ready"] += int(res["n_ready"].sum())
        st["forwarded"] += int(res["n_forwarded"].sum())
        st["escalations"] += len(esc)
        for r in esc:
            nm = abi.ESC_NAMES[r["escalation"]]
            st["esc_reasons"][nm] = st["esc_reasons"].get(nm, 0) + 1
        st["msgs"] += len(msgs)
        if self.check:
            dev = self.eng.sync()
            keep = np.nonzero(~parked)[0]
            bad_s = parity.compare_states(dev, o["mid"], self.slots, peers=keep)
            om = parity.prefix_msgs(o, lim)
            bad_m = parity.compare_msgs(out, om[~parked[om["peer"]]])
            bad_r = parity.compare_results(res, o["results"], fields=getattr(self.eng, "result_fields", None))
            bad_e = parity.check_escalations(res, o["esc_mask"])
            if bad_s or bad_m or bad_r or bad_e:
                mr = self.max_report
                raise AssertionError(
                    f"pass {self.k}: state {bad_s[:mr]} msgs {bad_m[:mr]} results {bad_r[:mr]}"
                    f" unjustified escalations {bad_e[:mr]}")
            st["commits"] += int(np.sum(dev["committed"] > before))
            # remotes a leader moved out of the Snapshot state this pass on the
            # device (respondedTo -> becomeRetry, remote.go:130-138)
            lead = (dev0["state"] == abi.LEADER) & (dev["state"] == abi.LEADER) & (res_esc_free(res, self.n))
            rs0, rs1 = dev0["remotes"]["state"], dev["remotes"]["state"]
            st["snapshot_left"] += int(np.sum(lead[:, None] & (rs0 == abi.SNAPSHOT_ST) & (rs1 != abi.SNAPSHOT_ST)))
        self.last_out = out
        # ReadyToRead of the whole pass (device prefix + host suffix): the oracle's
        self.last_ready = {}
        for p in np.nonzero(o["results"]["n_ready"])[0]:
            r = o["results"][p]
            self.last_ready[int(p)] = [tuple(int(x) for x in r["ready"][q]) for q in range(min(int(r["n_ready"]),
                                                                                                abi.GR_Q))]
        full = self.pop.export()
        fits = self.pop.representable()
        reload = np.zeros(self.n, bool)
        reload[esc["peer"].astype(np.int64)] = True
        reload |= parked & fits  # back on the device
        self.parked = ~fits
        st["parked"] += int(self.parked.sum())
        idx = np.nonzero(reload & fits)[0]
        if len(idx):
            self.eng.load(idx, full[idx])
        self.k += 1
        return o["msgs"], res

    def close(self):
        self.eng.close()


def simulate(backend, peers, topo, passes, locals_fn, slots=3, inject_fn=None, check=True,
             max_report=3, drop_fn=None, threads=None, extra_fn=None, max_entry_size=abi.MAX_ENTRY_SIZE,
             allow_error=False):
    """Run `passes` passes; returns a dict of counters. Raises AssertionError on divergence.

    inject_fn(k, state) -> changed slots (state edited in place, reloaded on both sides);
    extra_fn(k, state) -> gr_message records appended to pass k's inbox (local
    messages such as LeaderTransfer, or messages from outside the population)."""
    ls = Lockstep(backend, peers, slots, max_entry_size=max_entry_size, check=check, max_report=max_report,
                  allow_error=allow_error)
    msgs = np.zeros(0, abi.MESSAGE)
    try:
        for k in range(passes):
            if inject_fn is not None:
                cur = ls.export()
                changed = inject_fn(k, cur)
                if changed is not None and len(changed):
                    ls.reload(changed, cur[changed])
            # locals_fn(k) or locals_fn(k, state): the second form sees the pass's
            # starting state (e.g. to propose on the current leaders)
            loc = locals_fn(k, ls.export()) if locals_fn.__code__.co_argcount == 2 else locals_fn(k)
            if extra_fn is not None:
                ext = extra_fn(k, ls.export())
                if ext is not None and len(ext):
                    msgs = np.concatenate([msgs, np.asarray(ext, abi.MESSAGE)])
            out, _ = ls.step(msgs, loc)
            msgs = topo.route_messages(out)
            if drop_fn is not None:
                msgs = drop_fn(k, msgs)
        ls.stats["final"] = ls.export()
        ls.stats["oracle_errors"] = ls.errors
        return ls.stats
    finally:
        ls.close()
