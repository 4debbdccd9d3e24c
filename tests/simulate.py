"""Multi-pass simulations of replicated groups: the engine (GPU kernel, or the
test-only host build of the same lane code) against the oracle, compared
bit-exactly after every pass.

Escalation protocol (what the Go host does in production): a group that
escalates at item i keeps the device's state after items < i; the host runs
items >= i with the reference code and reloads the group. Here the oracle plays
the host: its prefix snapshot is compared with the device, its full-pass state
is what both sides continue from, and its full message list is routed.

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
    def __init__(self, peers, slots):
        self.state = np.array(peers, abi.PEER, copy=True)
        self.slots = slots

    def step(self, msgs, loc):
        self.state, out, res = hostlane_step(self.state, msgs, loc, self.slots)
        return out, res

    def sync(self):
        return self.state.copy()

    def load(self, idx, recs):
        self.state[idx] = recs


class GpuBackend:
    def __init__(self, peers, slots):
        from dragonboat_amd.engine import Engine
        self.eng = Engine(len(peers), slots)
        self.eng.load(peers)
        self.n = len(peers)

    def step(self, msgs, loc):
        return self.eng.step(msgs, loc)

    def sync(self):
        return self.eng.sync(self.n)

    def load(self, idx, recs):
        self.eng.load_peers(np.asarray(idx, np.uint32), np.asarray(recs, abi.PEER))  # one call, scattered slots


def simulate(backend, peers, topo, passes, locals_fn, slots=3, inject_fn=None, check=True,
             max_report=3, drop_fn=None, threads=None, extra_fn=None):
    """Run `passes` passes; returns a dict of counters. Raises AssertionError on divergence.

    inject_fn(k, state) -> changed slots (state edited in place, reloaded on both sides);
    extra_fn(k, state) -> gr_message records appended to pass k's inbox (local
    messages such as LeaderTransfer, or messages from outside the population)."""
    pop = OraclePopulation(peers, slots)
    eng = backend(peers, slots)
    n = len(peers)
    msgs = np.zeros(0, abi.MESSAGE)
    stats = {"msgs": 0, "escalations": 0, "esc_reasons": {}, "commits": 0, "ready": 0, "forwarded": 0}
    parked = np.zeros(n, bool)
    for k in range(passes):
        if inject_fn is not None:
            cur = pop.export()
            changed = inject_fn(k, cur)
            if changed is not None and len(changed):
                pop.reload(changed, cur[changed])
                eng.load(changed, cur[changed])
        # locals_fn(k) or locals_fn(k, state): the second form sees the pass's
        # starting state (e.g. to propose on the current leaders)
        loc = locals_fn(k, pop.export()) if locals_fn.__code__.co_argcount == 2 else locals_fn(k)
        if extra_fn is not None:
            ext = extra_fn(k, pop.export())
            if ext is not None and len(ext):
                msgs = np.concatenate([msgs, np.asarray(ext, abi.MESSAGE)])
        dev0 = eng.sync() if check else None
        before = dev0["committed"] if check else None
        emsgs = msgs[~parked[msgs["peer"]]] if len(msgs) else msgs
        eloc = loc[~parked[loc["peer"]]]
        out, res = eng.step(emsgs, eloc)
        if len(out):  # the engine's outbox is valid gr_step input (gr_host.h validate_msg)
            nr, ne = out["n_runs"], out["n_entries"]
            assert np.all(nr <= 2) and np.all((ne == 0) == (nr == 0)), "invalid outbox record"
            assert np.all(out["type"] <= abi.TIMEOUT_NOW)
        lim = parity.limits_from(res, n)
        o = pop.step(msgs, loc, lim, threads=threads or min(16, os.cpu_count() or 1), dev_before=dev0)
        esc = res[res["escalation"] != 0]
        stats["ready"] += int(res["n_ready"].sum())
        stats["forwarded"] += int(res["n_forwarded"].sum())
        stats["escalations"] += len(esc)
        for r in esc:
            nm = abi.ESC_NAMES[r["escalation"]]
            stats["esc_reasons"][nm] = stats["esc_reasons"].get(nm, 0) + 1
        stats["msgs"] += len(msgs)
        if check:
            dev = eng.sync()
            keep = np.nonzero(~parked)[0]
            bad_s = parity.compare_states(dev, o["mid"], slots, peers=keep)
            om = parity.prefix_msgs(o, lim)
            bad_m = parity.compare_msgs(out, om[~parked[om["peer"]]])
            bad_r = parity.compare_results(res, o["results"])
            bad_e = parity.check_escalations(res, o["esc_mask"])
            if bad_s or bad_m or bad_r or bad_e:
                raise AssertionError(
                    f"pass {k}: state {bad_s[:max_report]} msgs {bad_m[:max_report]} results {bad_r[:max_report]}"
                    f" unjustified escalations {bad_e[:max_report]}")
            stats["commits"] += int(np.sum(dev["committed"] > before))
        full = pop.export()
        fits = pop.representable()
        reload = np.zeros(n, bool)
        reload[esc["peer"].astype(np.int64)] = True
        reload |= parked & fits  # back on the device
        parked = ~fits
        stats["parked"] = stats.get("parked", 0) + int(parked.sum())
        idx = np.nonzero(reload & fits)[0]
        if len(idx):
            eng.load(idx, full[idx])
        msgs = topo.route_messages(o["msgs"])
        if drop_fn is not None:
            msgs = drop_fn(k, msgs)
    stats["final"] = pop.export()
    return stats
