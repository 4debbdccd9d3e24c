"""The drop-in boundary: include/gpuraft.h's layout matches the Python
mirror, libgpuraft.so loads and exports every declared symbol (no GPU calls)."""
import ctypes
import os
import re
import subprocess

import numpy as np

from dragonboat_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "gpuraft.h")


def _declared():
    src = open(HDR).read()
    return sorted(set(re.findall(r"^[A-Za-z_][\w \*]*?\b(gr_\w+)\(", src, re.M)))


def test_header_declarations_match_exports_list():
    assert _declared() == sorted(abi.EXPORTS)


def test_library_exports_every_symbol(built):
    from dragonboat_amd.engine import LIB_PATH
    lib = ctypes.CDLL(LIB_PATH)
    missing = [s for s in abi.EXPORTS if not hasattr(lib, s)]
    assert not missing
    # pure functions are callable without a device
    lib.gr_strerror.restype = ctypes.c_char_p
    assert lib.gr_strerror(-5) == b"mailbox capacity exceeded"
    lib.gr_space_chunk_bytes.restype = ctypes.c_uint64
    assert lib.gr_space_chunk_bytes(1, 4) % 256 == 0
    assert lib.gr_space_chunk_bytes(1, 0) == 0
    assert lib.gr_space_chunk_bytes(64, 2) < lib.gr_space_chunk_bytes(64, 4)


def _c_layout(tmp_path):
    checks = {
        "gr_peer": abi.PEER, "gr_message": abi.MESSAGE, "gr_local_input": abi.LOCAL,
        "gr_peer_result": abi.RESULT, "gr_remote": abi.REMOTE, "gr_read_status": abi.READ_STATUS,
    }
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HDR}"', "int main(void){"]
    for t, dt in checks.items():
        lines.append(f'printf("{t} sizeof %zu\\n", sizeof({t}));')
        for f in dt.names:
            if f.startswith("pad"):
                continue
            lines.append(f'printf("{t} {f} %zu\\n", offsetof({t}, {f}));')
    lines.append("return 0;}")
    c = tmp_path / "layout.c"
    c.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-o", str(exe), str(c)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout
    got = {}
    for line in out.splitlines():
        t, f, v = line.split()
        got[(t, f)] = int(v)
    return checks, got


def test_struct_layout_matches_numpy_mirror(tmp_path):
    checks, got = _c_layout(tmp_path)
    for t, dt in checks.items():
        assert got[(t, "sizeof")] == dt.itemsize, t
        for f in dt.names:
            if f.startswith("pad"):
                continue
            assert got[(t, f)] == dt.fields[f][1], (t, f)


def test_message_type_numbering():
    # raftpb.MessageType values (reference raftpb/raft.pb.go) used on the wire
    assert abi.REPLICATE == 12 and abi.REPLICATE_RESP == 13 and abi.HEARTBEAT == 17
    assert abi.READ_INDEX == 19 and abi.TIMEOUT_NOW == 24 and abi.PROPOSE == 7
