"""Test infrastructure for the wire path (gr_step_wire): what the senders'
transports put on the wire for an inbox of gr_message records.

Each record (receiving slot `peer`, sender remote slot `slot`) becomes a
raftpb.Message with To = the receiver's node id, From = its remote's node id,
ClusterID = the receiver's cluster, the record's values, and its entries (the
term runs made explicit: a Replicate's entries are LogIndex+1.., a forwarded
Propose's are unstamped, index and term 0, its first one a ConfigChangeEntry
when the record's reject bit says so), each with a 16-byte Cmd. Messages are
packed into MessageBatch frames in record order, so a mailbox's arrival order
is the frames' order, as a TCP connection delivers it (tcp.go:416-426).
"""
import numpy as np

from dragonboat_amd import abi, wire as W

CMD = np.arange(16, dtype=np.uint8)  # every entry's 16-byte Cmd (payload offset 0)


def to_wire(msgs, node_id, remote_id, cluster_of, per_frame=128, deployment=7, bin_ver=210):
    """(batches, wire messages, wire entries, payload) for inbox records `msgs`.

    node_id[p], remote_id[p, j], cluster_of[p]: the receiving slot's node id,
    its remote slot j's node id, its cluster id."""
    msgs = np.asarray(msgs, abi.MESSAGE)
    n = len(msgs)
    p = msgs["peer"].astype(np.int64)
    wm = np.zeros(n, W.WMESSAGE)
    wm["to"] = node_id[p]
    wm["from"] = remote_id[p, msgs["slot"].astype(np.int64)]
    wm["cluster_id"] = cluster_of[p]
    for f in ("term", "log_term", "log_index", "commit", "hint", "hint_high"):
        wm[f] = msgs[f]
    wm["type"] = msgs["type"].astype(np.int32)
    prop = msgs["type"] == abi.PROPOSE
    wm["reject"] = np.where(prop, 0, msgs["reject"])  # a Propose's reject bit is its config change entry
    ne = msgs["n_entries"].astype(np.int64)
    wm["n_entries"] = ne
    first = np.concatenate([[0], np.cumsum(ne)[:-1]]) if n else np.zeros(0, np.int64)
    wm["first_entry"] = first
    tot = int(ne.sum())
    we = np.zeros(tot, W.WENTRY)
    if tot:
        owner = np.repeat(np.arange(n), ne)
        k = np.arange(tot) - first[owner]
        m = msgs[owner]
        second = (m["n_runs"] == 2) & (k >= m["run2_offset"])
        we["term"] = np.where(second, m["run_term"][:, 1], m["run_term"][:, 0])
        rep = m["type"] == abi.REPLICATE
        we["index"] = np.where(rep, m["log_index"] + 1 + k, 0)
        we["type"] = np.where((m["type"] == abi.PROPOSE) & (m["reject"] != 0) & (k == 0), 1, 0)
        we["cmd_off"] = 0
        we["cmd_len"] = len(CMD)
    nb = (n + per_frame - 1) // per_frame
    batches = np.zeros(nb, W.BATCH)
    batches["first_msg"] = np.arange(nb) * per_frame
    batches["n_msgs"] = np.minimum(per_frame, n - np.arange(nb) * per_frame)
    batches["deployment_id"] = deployment
    batches["bin_ver"] = bin_ver
    return batches, wm, we, CMD.copy()


class WireFeed:
    """Frames for an engine: encode (the senders' side, libgrwire host API),
    upload the frames, decode them in HBM (grw_decode_device); the decoded
    records stay on the device for gr_step_wire."""

    def __init__(self, peers, cluster_of):
        import torch
        self.torch = torch
        self.node_id = np.asarray(peers["node_id"], np.uint64)
        self.remote_id = np.asarray(peers["remote_id"], np.uint64)
        self.cluster_of = np.asarray(cluster_of, np.uint64)
        self.codec = W.WireCodec(0)
        self.frame_bytes = 0

    def decode(self, msgs):
        """Returns (d_msgs, n_msgs, d_ents, n_ents, keep): device pointers of the
        decoded records and the tensors that own them."""
        torch = self.torch
        batches, wm, we, payload = to_wire(msgs, self.node_id, self.remote_id, self.cluster_of)
        if len(wm) == 0:
            return 0, 0, 0, 0, ()
        frames = self.codec.marshal(payload, batches, wm, we)
        self.frame_bytes += len(frames)
        table = W.frames_table(batches["frame_off"], batches["frame_len"])
        d_buf = torch.from_numpy(frames).cuda()
        d_bat = torch.from_numpy(table.view(np.uint8)).cuda()
        d_msgs = torch.empty(len(wm) * W.WMESSAGE.itemsize, dtype=torch.uint8, device="cuda")
        d_ents = torch.empty(max(1, len(we)) * W.WENTRY.itemsize, dtype=torch.uint8, device="cuda")
        nm, ne = self.codec.unmarshal_device(d_buf.data_ptr(), len(frames), d_bat.data_ptr(), len(table),
                                             d_msgs.data_ptr(), len(wm), d_ents.data_ptr(), max(1, len(we)))
        st = d_bat.cpu().numpy().view(W.BATCH)["status"]
        assert np.all(st == W.OK), st[st != W.OK][:4]
        assert nm == len(wm) and ne == len(we), (nm, len(wm), ne, len(we))
        return d_msgs.data_ptr(), nm, d_ents.data_ptr(), ne, (d_buf, d_bat, d_msgs, d_ents)

    def close(self):
        self.codec.close()
