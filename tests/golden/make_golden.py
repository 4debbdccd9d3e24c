"""Transcribe golden tables from the reference's own raft tests into JSON
fixtures (tests/golden/raft_tables.json). Run: python tests/golden/make_golden.py

The tables are data copied from the reference test sources (cited per table);
the cases are the reference's, unchanged. Entries are [index, term] pairs.
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))

# internal/raft/raft_etcd_test.go:1106-1158 (TestCommit): matches, logs, smTerm -> committed
TEST_COMMIT = [
    ([1], [[1, 1]], 1, 1),
    ([1], [[1, 1]], 2, 0),
    ([2], [[1, 1], [2, 2]], 2, 2),
    ([1], [[1, 2]], 2, 1),
    ([2, 1, 1], [[1, 1], [2, 2]], 1, 1),
    ([2, 1, 1], [[1, 1], [2, 1]], 2, 0),
    ([2, 1, 2], [[1, 1], [2, 2]], 2, 2),
    ([2, 1, 2], [[1, 1], [2, 1]], 2, 0),
    ([2, 1, 1, 1], [[1, 1], [2, 2]], 1, 1),
    ([2, 1, 1, 1], [[1, 1], [2, 1]], 2, 0),
    ([2, 1, 1, 2], [[1, 1], [2, 2]], 1, 1),
    ([2, 1, 1, 2], [[1, 1], [2, 1]], 2, 0),
    ([2, 1, 2, 2], [[1, 1], [2, 2]], 2, 2),
    ([2, 1, 2, 2], [[1, 1], [2, 1]], 2, 0),
]

# internal/raft/logentry_etcd_test.go:40-72 (TestFindConflict): previous log
# (1,1) (2,2) (3,3); ents -> wconflict
FIND_CONFLICT_PREV = [[1, 1], [2, 2], [3, 3]]
TEST_FIND_CONFLICT = [
    ([], 0),
    ([[1, 1], [2, 2], [3, 3]], 0),
    ([[2, 2], [3, 3]], 0),
    ([[3, 3]], 0),
    ([[1, 1], [2, 2], [3, 3], [4, 4], [5, 4]], 4),
    ([[2, 2], [3, 3], [4, 4], [5, 4]], 4),
    ([[3, 3], [4, 4], [5, 4]], 4),
    ([[4, 4], [5, 4]], 4),
    ([[1, 4], [2, 4]], 1),
    ([[2, 1], [3, 4], [4, 4]], 2),
    ([[3, 1], [4, 2], [5, 4], [6, 4]], 3),
]

# internal/raft/logentry_etcd_test.go:172-297 (TestLogMaybeAppend): previous
# log (1,1) (2,2) (3,3), committed 1; (logTerm, index, committed, ents) ->
# (wlasti, wappend, wcommit, wpanic)
MAYBE_APPEND_PREV = [[1, 1], [2, 2], [3, 3]]
MAYBE_APPEND_COMMIT = 1
_li, _lt, _c = 3, 3, 1
TEST_LOG_MAYBE_APPEND = [
    (_lt - 1, _li, _li, [[_li + 1, 4]], 0, False, _c, False),
    (_lt, _li + 1, _li, [[_li + 2, 4]], 0, False, _c, False),
    (_lt, _li, _li, [], _li, True, _li, False),
    (_lt, _li, _li + 1, [], _li, True, _li, False),
    (_lt, _li, _li - 1, [], _li, True, _li - 1, False),
    (_lt, _li, 0, [], _li, True, _c, False),
    (0, 0, _li, [], 0, True, _c, False),
    (_lt, _li, _li, [[_li + 1, 4]], _li + 1, True, _li, False),
    (_lt, _li, _li + 1, [[_li + 1, 4]], _li + 1, True, _li + 1, False),
    (_lt, _li, _li + 2, [[_li + 1, 4]], _li + 1, True, _li + 1, False),
    (_lt, _li, _li + 2, [[_li + 1, 4], [_li + 2, 4]], _li + 2, True, _li + 2, False),
    (_lt - 1, _li - 1, _li, [[_li, 4]], _li, True, _li, False),
    (_lt - 2, _li - 2, _li, [[_li - 1, 4]], _li - 1, True, _li - 1, False),
    (_lt - 3, _li - 3, _li, [[_li - 2, 4]], _li - 2, True, _li - 2, True),
    (_lt - 2, _li - 2, _li, [[_li - 1, 4], [_li, 4]], _li, True, _li, False),
]


def main():
    out = {
        "TestCommit": {"source": "internal/raft/raft_etcd_test.go:1106-1158",
                       "cases": [{"matches": m, "logs": l, "term": t, "want_committed": w}
                                 for m, l, t, w in TEST_COMMIT]},
        "TestFindConflict": {"source": "internal/raft/logentry_etcd_test.go:40-72",
                             "previous": FIND_CONFLICT_PREV,
                             "cases": [{"ents": e, "want_conflict": w} for e, w in TEST_FIND_CONFLICT]},
        "TestLogMaybeAppend": {"source": "internal/raft/logentry_etcd_test.go:172-297",
                               "previous": MAYBE_APPEND_PREV, "committed": MAYBE_APPEND_COMMIT,
                               "cases": [{"log_term": a, "index": b, "committed": c, "ents": d,
                                          "want_lasti": e, "want_append": f, "want_commit": g,
                                          "want_panic": h}
                                         for a, b, c, d, e, f, g, h in TEST_LOG_MAYBE_APPEND]},
    }
    with open(os.path.join(HERE, "raft_tables.json"), "w") as fh:
        json.dump(out, fh, indent=1)
        fh.write("\n")


if __name__ == "__main__":
    main()
