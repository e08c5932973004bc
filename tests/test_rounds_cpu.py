"""RoundExecutor's scheduling without a GPU (dasklearn_amd/rounds.py): waves,
placeholder resolution, and the release of results once every reader has
run (the broker clears a completed task's data, broker.py:221). A DAG of
non-aggregate tasks needs no device."""
from __future__ import annotations

import pytest

from dasklearn_amd.rounds import RoundExecutor


def _add(settings, params):
    return [sum(params["xs"]) + params.get("k", 0)]


TASKS = [
    ("a", "add", {"xs": [("init", 0)], "k": 1}),
    ("b", "add", {"xs": [("a", 0), ("init", 0)]}),
    ("c", "add", {"xs": [("a", 0), ("a", 0)]}),  # reads a twice in one task
    ("d", "add", {"xs": [("b", 0), ("c", 0)]}),
    ("e", "add", {"xs": [("b", 0)], "k": 10}),
]


def test_results_released_after_last_reader():
    ex = RoundExecutor({"add": _add}, settings=None)
    got = ex.run(TASKS, seed={"init": [2], "unused": [7]})
    # a = 3, b = 5, c = 6, d = 11, e = 15
    assert got == {"d": [11], "e": [15], "unused": [7]}
    assert ex.waves == [["a"], ["b", "c"], ["d", "e"]]


def test_keep_all_keeps_every_result():
    ex = RoundExecutor({"add": _add}, settings=None, keep_all=True)
    got = ex.run(TASKS, seed={"init": [2]})
    assert got == {"init": [2], "a": [3], "b": [5], "c": [6], "d": [11], "e": [15]}


def test_unresolvable_inputs_are_reported():
    ex = RoundExecutor({"add": _add}, settings=None)
    with pytest.raises(RuntimeError, match="unresolvable"):
        ex.run([("a", "add", {"xs": [("missing", 0)]})])
