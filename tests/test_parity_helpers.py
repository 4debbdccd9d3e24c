"""The parity helpers catch what they must: a one-field change in a state,
message or result record is reported (the vectorised screens only skip
records that are exactly equal)."""
import numpy as np

from dragonboat_amd import abi, populations as P
import parity


def test_state_field_change_is_reported():
    a = P.make_groups(50, 3, seed=1)
    b = a.copy()
    assert parity.compare_states(a, b, 3) == []
    b["committed"][7] += 1
    b["remotes"][11]["next"][2] += 1
    bad = parity.compare_states(a, b, 3)
    assert [p for p, _ in bad] == [7, 11]


def test_message_order_within_mailbox_matters():
    m = np.zeros(4, abi.MESSAGE)
    m["peer"] = [1, 1, 2, 1]
    m["slot"] = [0, 0, 1, 2]
    m["log_index"] = [10, 11, 5, 7]
    shuffled = m[[2, 3, 0, 1]]  # other mailboxes interleaved: same per-mailbox order
    assert parity.compare_msgs(m, shuffled) == []
    swapped = m[[1, 0, 2, 3]]   # two messages of mailbox (1, 0) swapped
    assert parity.compare_msgs(m, swapped)


def test_result_field_change_is_reported():
    r = np.zeros(5, abi.RESULT)
    r["peer"] = np.arange(5)
    o = r.copy()
    assert parity.compare_results(r, o) == []
    o["n_ready"][3] = 1
    o["ready"][3][0]["index"] = 9
    assert [p for p, _ in parity.compare_results(r, o)] == [3]
