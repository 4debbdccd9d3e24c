"""The oracle's own gate: the known-answer tests transcribed from the
reference's internal/raft tests (oracle/kat_tests.cpp cites each test's
file:line). The oracle is trusted as the parity checker only because these pass."""
import subprocess

from oracle.pyoracle import KAT_BIN


def test_oracle_known_answer_tests(built):
    p = subprocess.run([KAT_BIN], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout[-4000:] + p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith(("PASS", "FAIL"))]
    assert len(lines) >= 39, p.stdout[-2000:]
    assert not [l for l in lines if l.startswith("FAIL")]
