"""Device-resident message exchange between passes (the transport's role).

In the reference every Replicate/ReplicateResp leaves a node through
``transport.Send`` (plugin/transport) and is delivered to the receiving
node's ``Peer.Handle`` on the next step. Here the engines of all GPUs write
their outgoing messages straight into mailbox "spaces" in HBM:

* ``local`` placement — all replicas of a group on one GPU: two spaces,
  ping-ponged; the kernel of pass k reads space k%2 and writes space (k+1)%2.
  No copy, no collective.
* ``spread`` placement — replica r of the groups homed on rank h lives on
  rank (h + r) % N, so replica r talks to replica j only across the rank
  offset (j - r) % N. The out space has one chunk per destination rank that
  some pair reaches (ordered by rank), the in space one per source rank, and
  one RCCL ``all_to_all_single`` with split sizes (0 for ranks no pair
  reaches) moves every mailbox across xGMI once per pass. At R = 3 that is
  4 of N chunks for N ≥ 5, and the spaces hold depth-3 mailboxes (the steady
  state's two Replicates per follower per pass plus a heartbeat on a tick; a
  fourth message escalates CAPACITY). What crosses (``codec``):
  - ``cx`` (round 5, the default): the compact exchange (gr_space_cx_pack /
    _unpack): per chunk one fixed-size buffer holding only the mailboxes with
    messages, a 12-byte record for the steady state's uniform mailboxes and a
    full entry for the rest, one bit for an empty one (63 MB per GPU per pass
    designed at N = 8 and 1M groups per GPU, against 0.33 GB for ``dense``;
    31.5 MB against 186 MB measured in the N = 2 rehearsal);
  - ``dense`` (round 4): the hot region (counts + compact Replicates +
    non-reject acks, 41 B per depth-3 mailbox) every pass, the cold fields of
    the mailboxes that need them compacted into a fixed-capacity side buffer per
    chunk (gr_space_side_pack / _unpack).
  Either way the all-to-all sizes are fixed and the host never waits on the
  device inside the pass loop. A mailbox that does not fit escalates CAPACITY
  at its reader (detected one pass later, never silently lost). The compact
  buffers are sized for the steady state (records for the mailboxes that hold
  messages, full entries for 1/256 of the positions); a pass the caller knows to
  be heavy -- a tick pass and the pass after it (every leader's heartbeats,
  then every follower's ack, are full entries) or a burst of leader changes
  larger than the side capacity -- exchanges ``dense`` instead (``heavy=True``,
  the same on every rank: ``codec="cx"`` keeps both forms' buffers).

Peers on a rank are laid out replica-major: peer r*G + g is replica r of the
group (home = (rank - r) % N, index g), so a wave's accesses stay contiguous.
"""
import numpy as np

from . import abi, populations as P

NOPOS = 0xFFFFFFFF


def count_bytes(hot, n_chunks, hot_chunk, hot_tile, positions):
    """The mailbox count bytes of a hot region, [n_chunks, tiles, W] (gr_layout.h:
    a chunk's positions are tiled by W, each tile starting with its W count bytes;
    W = hot_tile / hot bytes per position). Works on a torch tensor or a numpy array."""
    w = TILE_W
    tiles = pad_positions(positions) // w
    return hot.reshape(n_chunks, hot_chunk)[:, :tiles * hot_tile].reshape(n_chunks, tiles, hot_tile)[:, :, :w]


TILE_W = 256  # gr_layout.h kTileW (GR_TILE_SHIFT = 8); Exchange checks it against the library
SIDE_DIV, SIDE_MIN = 32, 1024  # side-buffer capacity per chunk: positions / SIDE_DIV, at least SIDE_MIN
# compact exchange capacities per chunk: records for the share of a chunk's
# positions that hold messages in the steady state, whichever replica leads
# (cx_fill_max), plus CX_MARGIN for the pack's record regions (gr_io.h
# cx_region: each region holds its workgroups' share of the capacity, and the
# workgroups' fills differ by a few workgroups' worth between regions: at a
# chunk filled to its capacity, 0 % margin sent 3 % of the records to full
# entries), full entries for 1/CX_SIDE_DIV of them (at least CX_SIDE_MIN).
# A chunk carries the replica pairs (r -> j) of one rank offset; only the pairs
# with the leader on one end hold messages (a leader's Replicates, its
# followers' acks).
CX_MARGIN, CX_SIDE_DIV, CX_SIDE_MIN = 0.04, 256, 256
CX_MAX_CHUNKS = 8  # gr_io.h kCxMaxChunks: a rank's destination chunks in one compact buffer set
CX_SUB, CX_CTR = 16, 16  # gr_io.h kCxSub record regions, their counters kCxCtr words apart; then the side counter
CX_HDR = (CX_SUB + 1) * CX_CTR * 4


def cx_counts(hdr):
    """(records, full entries) a compact-exchange chunk's packer took, from its
    header (bytes or a uint8 array of at least CX_HDR bytes): the region
    counters' sum (records past a region's capacity included) and the side
    counter."""
    import numpy as _np
    w = _np.frombuffer(bytes(hdr[:CX_HDR]), _np.uint32)
    return int(w[0:CX_SUB * CX_CTR:CX_CTR].sum()), int(w[CX_SUB * CX_CTR])


def cx_fill(R, N, offset, leader=0):
    """Steady-state share of a chunk's positions (rank offset `offset`) that hold
    messages when replica `leader` of every group leads."""
    pairs = offset_pairs(R, N)
    per = max(len(v) for v in pairs.values())
    return sum(1 for r, j in pairs[offset] if leader in (r, j)) / per


def cx_fill_max(R, N, offset):
    """The largest steady-state share over leader placements: leaders move
    (config 5's churn, elections), and a chunk's fill depends on which replica
    leads. With every group led by replica 1 at N = 8 the offset-1 and offset-7
    chunks are full; with leaders spread evenly they are two thirds full. Sized
    by this, the records of a steady state never overflow wherever leaders sit
    (ADVICE r05): 3.0 vs 2.0 chunk-fills per rank at N = 8."""
    return max(cx_fill(R, N, offset, leader) for leader in range(R))


def cx_capacities(positions, fill, frac=None, side=None):
    """(record capacity, full-entry capacity) of one compact-exchange chunk whose
    steady-state fill is `fill` (frac: a fixed share instead of fill + margin;
    side: the full-entry share of the positions instead of 1/CX_SIDE_DIV, for
    callers whose passes are seldom steady, e.g. ticks on every pass; Exchange's
    cx_side also sizes the dense form's side buffers)."""
    pc = pad_positions(positions)
    share = frac if frac is not None else fill + CX_MARGIN
    cap = min(pc, (int(pc * share) + 63) // 64 * 64)
    scap = max(CX_SIDE_MIN, pc // CX_SIDE_DIV) if side is None else max(64, min(pc, int(pc * side)))
    return cap, scap


def pad_positions(positions):
    """gr_layout.h space_pad_positions: chunks hold a multiple of TILE_W mailboxes."""
    return (positions + TILE_W - 1) & ~(TILE_W - 1)


def offset_pairs(R, N):
    """(sender replica r, receiver replica j) pairs per rank offset (j - r) % N."""
    pairs = {o: [] for o in range(N)}
    for r in range(R):
        for j in range(R):
            if j != r:
                pairs[(j - r) % N].append((r, j))
    return pairs


def spread_peer_ranks(R, N, rank):
    """(destination ranks, source ranks) of `rank`'s chunks, each sorted: the
    ranks some (r -> j) pair reaches at offset (j - r) % N, and back."""
    offs = [o for o, lst in offset_pairs(R, N).items() if lst]
    return sorted({(rank + o) % N for o in offs}), sorted({(rank - o) % N for o in offs})


def spread_routes(G, R, S, N, rank):
    """Route tables for spread placement on `rank`.

    Returns (in_pos [S][R*G], out_pos [S][R*G], positions per chunk). The
    sender on rank a writes its mailbox for (r -> j, group g) into the chunk
    of destination d = (a - r + j) % N (chunk index = d's place among a's
    destinations), position pair_index * G + g; all_to_all delivers it into
    the chunk of source a on rank d (a's place among d's sources), where the
    receiver (replica j, same group) reads the same position."""
    pairs = offset_pairs(R, N)
    per = max(len(v) for v in pairs.values())
    positions = per * G
    pc = pad_positions(positions)
    index = {}
    for o, lst in pairs.items():
        for k, rj in enumerate(lst):
            index[rj] = k
    dests, srcs = spread_peer_ranks(R, N, rank)
    dslot = {d: c for c, d in enumerate(dests)}
    sslot = {a: c for c, a in enumerate(srcs)}
    n = R * G
    g = np.arange(G, dtype=np.int64)
    in_pos = np.full((S, n), NOPOS, np.uint32)
    out_pos = np.full((S, n), NOPOS, np.uint32)
    for r in range(R):
        for j in range(R):
            if j == r:
                continue
            k = index[(r, j)]
            # sender: local replica r, slot j -> chunk d
            d = (rank - r + j) % N
            out_pos[j, r * G + g] = (dslot[d] * pc + k * G + g).astype(np.uint32)
            # receiver: local replica j, slot r <- chunk a (sender rank)
            a = (rank - j + r) % N
            in_pos[r, j * G + g] = (sslot[a] * pc + k * G + g).astype(np.uint32)
    return in_pos, out_pos, positions


def group_seed(seed, home):
    return [seed, home]


def spread_peers(G, R, N, rank, seed=2, **kw):
    """Peer records for `rank`: replica r of the G groups homed on (rank - r) % N.
    Every rank regenerates a home's groups from the same seed, so the replicas
    of one group agree wherever they are placed."""
    out = np.zeros(R * G, dtype=P.make_groups(1, R).dtype)
    for r in range(R):
        h = (rank - r) % N
        grp = P.make_groups(G, R, seed=int(np.random.SeedSequence(group_seed(seed, h)).generate_state(1)[0]), **kw)
        out[r * G:(r + 1) * G] = grp[r * G:(r + 1) * G]
    return out


class Exchange:
    """Spaces + routes for one rank; `step` launches one pass and exchanges."""

    def __init__(self, G, R, S, world, rank, placement, seed=2, exchange=None, codec="cx", cx_frac=None,
                 cx_side=None, depth=None, collective=None):
        """exchange=True keeps the one-rank spread exchange (pack, move, unpack)
        that a one-rank run otherwise skips (tests of the N > 1 code on one GPU).
        collective: move the buffers with the process group's all_to_all_single
        (RCCL: async on the pass's stream, waited on as a stream wait) even with
        one rank, where a device copy would do (default: only with N > 1); the
        one-GPU test of the N = 8 exchange path (tests/test_pipeline_rccl.py).
        codec: "cx" (compact exchange) or "dense" (hot region + side buffers).
        depth: messages per mailbox of a spread space (default 3; a fuller one
        escalates CAPACITY at its writer)."""
        assert codec in ("cx", "dense")
        self.codec, self.cx_frac, self.cx_side = codec, cx_frac, cx_side
        self.last_cx = codec == "cx"  # the form of the last exchange (unpack reads it)
        self.G, self.R, self.S = G, R, S
        self.world, self.rank, self.placement = world, rank, placement
        self.n_peers = R * G
        self.leader_slots = np.arange(G)  # replica 0 of every hosted group leads
        if placement == "local":
            self.peers = P.make_groups(G, R, seed=int(np.random.SeedSequence(group_seed(seed, rank)).generate_state(1)[0]))
            self.in_pos, self.out_pos = P.Topology(G, R).loopback_routes(S)
            self.n_chunks = 1
            self.positions = self.n_peers * S
            self.depth = abi.GR_C  # nothing crosses a link, keep the full mailbox
            self.in_chunks = self.out_chunks = 1
        elif placement == "spread":
            self.peers = spread_peers(G, R, world, rank, seed=seed)
            self.in_pos, self.out_pos, self.positions = spread_routes(G, R, S, world, rank)
            self.dests, self.srcs = spread_peer_ranks(R, world, rank)
            self.n_chunks = len(self.dests)
            assert len(self.srcs) == self.n_chunks
            self.depth = depth or 3  # two Replicates (or acks) + a heartbeat (or its ack) per pass
        else:
            raise ValueError(placement)
        # one rank: every mailbox is the rank's own, at the same position on both
        # sides (the one chunk's sender and receiver positions coincide), so the
        # exchange is no copy at all: the two spaces ping-pong as in local placement
        self.pingpong = placement == "local" or (world == 1 and not exchange and not collective)
        self.collective = placement == "spread" and (world > 1 or bool(collective))
        if codec == "cx" and not self.pingpong and self.n_chunks > CX_MAX_CHUNKS:
            import warnings
            warnings.warn(f"spread placement with {self.n_chunks} peer chunks exceeds the compact exchange's "
                          f"{CX_MAX_CHUNKS}: exchanging the dense form")
            self.codec = codec = "dense"
            self.last_cx = False
        if placement == "spread" and world == 1:
            assert self.n_chunks == 1 and np.array_equal(np.sort(self.in_pos[self.in_pos != NOPOS]),
                                                         np.sort(self.out_pos[self.out_pos != NOPOS]))

    def allocate(self, eng, device):
        import torch
        assert int(eng.lib.gr_space_tile_positions()) == TILE_W, "library tile width differs from TILE_W"
        nbytes = eng.space_bytes(self.n_chunks, self.positions, self.depth)
        cb = eng.chunk_bytes(self.positions, self.depth)
        hb = eng.hot_chunk_bytes(self.positions, self.depth)
        assert nbytes == self.n_chunks * cb and 0 < hb < cb
        self.hot_region = self.n_chunks * hb  # hot chunks first, then the cold chunks
        self.hot_tile = eng.hot_tile_bytes(self.depth)  # positions tiled by 64, counts first in a tile
        if not self.pingpong:  # both forms' buffers: a heavy pass exchanges dense
            self._alloc_dense(eng, device, hb)
        if not self.pingpong and self.codec == "cx":
            # one fixed-size compact buffer per chunk, sent and received; a chunk's
            # record capacity follows its rank offset (cx_fill), the same on the
            # sender (destination d: offset d - rank) and the receiver (source a:
            # offset rank - a)
            N = self.world
            cap_of = lambda o: cx_capacities(self.positions, cx_fill_max(self.R, N, o), self.cx_frac, self.cx_side)
            self.cx_send_caps = [cap_of((d - self.rank) % N)[0] for d in self.dests]
            self.cx_recv_caps = [cap_of((self.rank - a) % N)[0] for a in self.srcs]
            self.cx_scap = cap_of(0)[1]
            sb = [eng.cx_bytes(1, self.positions, self.depth, [c], self.cx_scap) for c in self.cx_send_caps]
            rb = [eng.cx_bytes(1, self.positions, self.depth, [c], self.cx_scap) for c in self.cx_recv_caps]
            self.cx_splits = ([sb[self.dests.index(d)] if d in self.dests else 0 for d in range(self.world)],
                              [rb[self.srcs.index(a)] if a in self.srcs else 0 for a in range(self.world)])
            self.cx = [torch.zeros(sum(sb), dtype=torch.uint8, device=device),
                       torch.zeros(sum(rb), dtype=torch.uint8, device=device)]
        a = torch.zeros(nbytes, dtype=torch.uint8, device=device)
        b = torch.zeros(nbytes, dtype=torch.uint8, device=device)
        return [a, b]

    def _alloc_dense(self, eng, device, hb):
        import torch
        # all_to_all split sizes, bytes per peer rank
        self.hot_splits = ([hb if d in self.dests else 0 for d in range(self.world)],
                           [hb if a in self.srcs else 0 for a in range(self.world)])
        # side buffers: the cold fields of up to 1/32 of a chunk's mailboxes
        # (at least 1024), a fixed size every pass
        pc = pad_positions(self.positions)  # cx_side sizes the dense form's side buffers too
        self.side_cap = max(SIDE_MIN, pc // SIDE_DIV) if self.cx_side is None else \
            max(SIDE_MIN, min(pc, int(pc * self.cx_side)))
        sb = eng.side_bytes(1, self.depth, self.side_cap)
        self.side_splits = ([sb if d in self.dests else 0 for d in range(self.world)],
                            [sb if a in self.srcs else 0 for a in range(self.world)])
        self.side = [torch.zeros(self.n_chunks * sb, dtype=torch.uint8, device=device) for _ in range(2)]

    def exchange(self, eng, spaces, h, heavy=False):
        """Spread placement, after a pass on stream handle h: pack the out space
        (compact buffers, or for a heavy pass / the dense codec: its cold fields
        into the side buffers) and move it (fixed sizes). Returns the pending
        collective work (empty with one rank or a host backend); unpack() then
        writes what arrived into the in space. The copies and collectives run on
        torch's current stream, which the caller makes the stream of h
        (Exchange.step, Pipeline.step)."""
        inp, out = spaces
        self.last_cx = self.codec == "cx" and not heavy
        if self.last_cx:
            send, recv = self.cx
            eng.cx_pack(out.data_ptr(), self.n_chunks, self.positions, self.depth, send.data_ptr(),
                        self.cx_send_caps, self.cx_scap, h)
            if not self.collective:
                recv.copy_(send)
                return []
            return [_all_to_all(recv, send, self.cx_splits[1], self.cx_splits[0])]
        side_out, side_in = self.side
        eng.side_pack(out.data_ptr(), self.n_chunks, self.positions, self.depth, side_out.data_ptr(),
                      self.side_cap, h)
        hr = self.hot_region
        if not self.collective:
            inp[:hr].copy_(out[:hr])
            side_in.copy_(side_out)
            work = []
        else:
            work = [_all_to_all(inp[:hr], out[:hr], self.hot_splits[1], self.hot_splits[0]),
                    _all_to_all(side_in, side_out, self.side_splits[1], self.side_splits[0])]
        return work

    def unpack(self, eng, spaces, h):
        """Write what the exchange received into the in space (after its work has
        completed on stream h)."""
        if self.last_cx:
            eng.cx_unpack(spaces[0].data_ptr(), self.n_chunks, self.positions, self.depth, self.cx[1].data_ptr(),
                          self.cx_recv_caps, self.cx_scap, h)
            return
        eng.side_unpack(spaces[0].data_ptr(), self.n_chunks, self.positions, self.depth, self.side[1].data_ptr(),
                        self.side_cap, h)

    def step(self, eng, spaces, k, stream, events=None, heavy=False):
        """One pass: kernel (optionally bracketed by `events`), then the exchange
        (heavy: the dense form, for a pass with ticks or leader changes)."""
        h = stream.cuda_stream
        if self.pingpong:
            src, dst = spaces[k % 2], spaces[(k + 1) % 2]
        else:
            src, dst = spaces[0], spaces[1]
        if events is not None:
            events[0].record(stream)
        eng.step_device(src.data_ptr(), dst.data_ptr(), self.n_chunks, self.positions,
                        self.n_chunks, self.positions, self.n_peers, h, depth=self.depth)
        if events is not None:
            events[1].record(stream)
        if not self.pingpong:
            import torch
            # exchange() copies (one rank) and issues RCCL on torch's current
            # stream: make that the pass's stream, so they follow the pack
            with torch.cuda.stream(stream):
                for w in self.exchange(eng, spaces, h, heavy=heavy):
                    w.wait()
            self.unpack(eng, spaces, h)


def build_exchange(G, R, S, world, rank, placement, seed=2):
    return Exchange(G, R, S, world, rank, placement, seed=seed)


class Pipeline:
    """BASELINE config 4 across GPUs: the rank's groups in
    `banks` independent engines, each with its own spaces and HIP stream, so
    one bank's all-to-all over xGMI overlaps the other bank's pass.

    Per pass k, for every bank b on its stream s_b: wait for bank b's exchange
    of pass k-1 (the RCCL work handle: a stream wait, not a host wait) -> write
    its side buffers into the in space -> gr_step_device -> compact the out
    space's cold fields into the side buffers -> all_to_all_single of the hot
    region and of the side buffers, async on s_b. Every size is fixed, so the
    host issues the whole pass without reading anything back from the device.
    RCCL waits only on s_b, so bank 0's exchange runs beside bank 1's kernel and
    vice versa. With one rank the exchange is a device copy. `local` placement
    is one bank whose two spaces ping-pong (no exchange).
    """

    def __init__(self, G, R, S, world, rank, placement="spread", banks=None, seed=2, exchange=None, codec="cx",
                 cx_frac=None, cx_side=None, depth=None, collective=None, verify_heavy=None):
        """verify_heavy: check on every pass that all ranks passed the same
        `heavy` (one 2-element all_reduce; a disagreement would pair buffers of
        different sizes in the all-to-all). Default: on when GR_VERIFY_HEAVY=1."""
        import os
        self.verify_heavy = (os.environ.get("GR_VERIFY_HEAVY") == "1") if verify_heavy is None else verify_heavy
        if banks is None:  # banks overlap one another's exchange: only with one to overlap
            banks = 2 if placement == "spread" and world > 1 and G >= 128 else 1
        # bank sizes a multiple of 64 but the last: a wave's lanes then share a
        # replica block (StepParams::route_wu, scalar route arithmetic)
        base = (G // banks) // 64 * 64 if G // banks >= 64 else G // banks
        sizes = [base] * (banks - 1) + [G - base * (banks - 1)]
        self.R, self.S, self.world, self.rank, self.placement = R, S, world, rank, placement
        self.ex = [Exchange(Gb, R, S, world, rank, placement, seed=seed + 7919 * b, exchange=exchange, codec=codec,
                            cx_frac=cx_frac, cx_side=cx_side, depth=depth, collective=collective)
                   for b, Gb in enumerate(sizes)]
        self.groups = G
        self.engines, self.spaces, self.streams = [], [], []
        self.work = [[] for _ in self.ex]

    @property
    def n_peers(self):
        return sum(ex.n_peers for ex in self.ex)

    def setup(self, engine_cls, device, ordinal, locals_fn=None):
        """Engines (loaded, routes bound, locals bound), spaces, streams, pinned flags."""
        import torch
        from . import populations as P
        for ex in self.ex:
            eng = engine_cls(ex.n_peers, self.S, device=ordinal)
            eng.load(ex.peers)
            eng.bind_routes(ex.in_pos, ex.out_pos)
            loc = locals_fn(ex) if locals_fn else P.propose_locals(ex.n_peers, ex.leader_slots, pass_index=0)
            eng.set_locals(loc)
            self.engines.append(eng)
            self.spaces.append(ex.allocate(eng, device))
            self.streams.append(torch.cuda.Stream(device=device))

    def step(self, k, heavy=False):
        """Pass k of every bank (heavy: the pass's exchange in the dense form,
        Exchange.exchange; it must be the same on every rank)."""
        import torch
        if self.verify_heavy and any(ex.collective for ex in self.ex):
            self._check_heavy(bool(heavy))
        for b, (ex, eng) in enumerate(zip(self.ex, self.engines)):
            s = self.streams[b]
            with torch.cuda.stream(s):
                for w in self.work[b]:
                    w.wait()  # s waits for this bank's previous exchange
                self.work[b] = []
                if ex.pingpong:
                    src, dst = self.spaces[b][k % 2], self.spaces[b][(k + 1) % 2]
                else:
                    src, dst = self.spaces[b][0], self.spaces[b][1]
                    ex.unpack(eng, self.spaces[b], s.cuda_stream)
                eng.step_device(src.data_ptr(), dst.data_ptr(), ex.n_chunks, ex.positions, ex.n_chunks,
                                ex.positions, ex.n_peers, s.cuda_stream, depth=ex.depth)
                if not ex.pingpong:
                    self.work[b] = ex.exchange(eng, self.spaces[b], s.cuda_stream, heavy=heavy)

    def _check_heavy(self, heavy):
        """All ranks agree on `heavy` (max of (h, -h) over ranks: h and -h agree
        iff every rank passed the same flag); raises before any buffer moves."""
        import torch
        import torch.distributed as dist
        dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([int(heavy), -int(heavy)], dtype=torch.int32, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        hi, lo = int(t[0]), -int(t[1])
        if hi != lo:
            raise RuntimeError(f"Pipeline.step: ranks disagree on heavy (rank {self.rank}: {heavy})")

    def graph_ready(self):
        """Graph mode applies: every bank's spaces ping-pong (no exchange step)."""
        return all(ex.pingpong for ex in self.ex)

    def graph_steps(self, k0, K):
        """Passes k0 .. k0 + K - 1 (k0 and K even) as replays of each bank's
        two-pass HIP graph (gr_graph_capture over the ping-pong spaces, captured on
        first use): the launch model of SURVEY.md §7(d), no CPU launch per kernel.
        The bound locals are the same every pass, so a replay does a pass's work."""
        assert k0 % 2 == 0 and K % 2 == 0 and self.graph_ready()
        if not getattr(self, "graphs", None):
            self.graphs = []
            for ex, eng, sp in zip(self.ex, self.engines, self.spaces):
                self.graphs.append(eng.graph_capture(sp[0].data_ptr(), sp[1].data_ptr(), ex.n_chunks, ex.positions,
                                                     ex.n_peers, n_passes=2, depth=ex.depth))
        for _ in range(K // 2):
            for b, (eng, g) in enumerate(zip(self.engines, self.graphs)):
                eng.graph_replay(g, self.streams[b].cuda_stream)

    def exchange_bytes_per_pass(self, heavy=False):
        """Bytes this rank sends to other ranks per pass (its buffers for the
        chunks of other ranks: compact, or hot regions + side buffers for the
        dense form and heavy passes; 0 for local placement)."""
        tot = 0
        for ex in self.ex:
            if ex.pingpong:
                continue
            if ex.codec == "cx" and not heavy:
                tot += sum(n for d, n in zip(range(self.world), ex.cx_splits[0]) if d != self.rank)
            else:
                tot += sum(n for d, n in zip(range(self.world), ex.hot_splits[0]) if d != self.rank)
                tot += sum(n for d, n in zip(range(self.world), ex.side_splits[0]) if d != self.rank)
        return tot

    def synchronize(self):
        import torch
        for b, s in enumerate(self.streams):
            with torch.cuda.stream(s):
                for w in self.work[b]:
                    w.wait()
            self.work[b] = []
        torch.cuda.synchronize()

    def stats(self):
        tot = {}
        for eng in self.engines:
            for f, v in eng.stats().items():
                tot[f] = tot.get(f, 0) + v
        return tot

    def reset_stats(self):
        for eng in self.engines:
            eng.reset_stats()

    def timing_begin(self):
        for eng in self.engines:
            eng.timing_begin()

    def timing_end(self):
        tot = {"passes": 0, "fast_ms": 0.0, "general_ms": 0.0, "bailed_lanes": 0}
        for eng in self.engines:
            for f, v in eng.timing_end().items():
                tot[f] += v
        return tot

    def close(self):
        for eng, g in zip(self.engines, getattr(self, "graphs", None) or []):
            eng.graph_destroy(g)
        self.graphs = []
        for eng in self.engines:
            eng.close()
        self.engines = []


def _all_to_all(inp, out, in_splits, out_splits):
    """One all_to_all_single of byte ranges, async on the current stream (RCCL);
    over gloo (CPU rehearsal of the N > 1 path) through host tensors."""
    import torch.distributed as dist
    if dist.get_backend() == "nccl":
        return dist.all_to_all_single(inp, out, output_split_sizes=in_splits, input_split_sizes=out_splits,
                                      async_op=True)
    o, i = out.cpu(), inp.cpu()
    dist.all_to_all_single(i, o, output_split_sizes=in_splits, input_split_sizes=out_splits)
    inp.copy_(i)

    class _Done:
        def wait(self):
            pass
    return _Done()
