"""bench.py's host-side machinery (CPU): the timed window, rank launch and
input-set rotation. The GPU leg itself runs on the box (bench.py, -m gpu)."""
from __future__ import annotations

import json
import os
import sys
import textwrap
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


class _ClockEvent:
    def record(self):
        self.t = time.perf_counter()

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3


def test_barriers_are_outside_the_timed_window():
    """A 0.3 s barrier on both sides of 5 x 2 ms launches: both clocks see
    only the launches."""
    calls = []

    def barrier():
        calls.append("barrier")
        time.sleep(0.3)

    def launch(k):
        calls.append(k)
        time.sleep(0.002)

    ev_ms, wall_ms = bench.time_steps(launch, 5, lambda: calls.append("sync"), barrier, _ClockEvent)
    assert 9.0 <= ev_ms < 100.0
    assert 9.0 <= wall_ms < 100.0
    assert calls[0] == "barrier" and calls[-1] == "barrier"
    assert calls[1:-1] == ["sync", 0, 1, 2, 3, 4, "sync"]


def test_input_sets_cover_the_infinity_cache():
    # the north star (402.5 MB a step): 3 sets; its 8-rank slice (50.3 MB): 22
    assert bench.n_sets(402_539_112) == 3
    assert bench.n_sets(50_319_360) == 22
    assert bench.n_sets(50_319_360) * 50_319_360 >= bench.MIN_SET_FOOTPRINT


def test_strong_split_is_the_default_for_several_gpus():
    a = bench.parse(["--gpus", "4"])
    assert not a.weak
    assert bench.parse(["--gpus", "4", "--weak"]).weak


_RANK_SCRIPT = textwrap.dedent("""
    import json, os, sys
    import torch, torch.distributed as dist
    dist.init_process_group("gloo")
    r, w = dist.get_rank(), dist.get_world_size()
    assert os.environ["MASTER_ADDR"] == "127.0.0.1" and int(os.environ["LOCAL_RANK"]) == r
    t = torch.tensor([float(r + 1)])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if "--fail" in sys.argv and r == 1:
        sys.exit(3)
    if r == 0:
        print(json.dumps({"world": w, "max": t.item(), "argv": sys.argv[1:]}), flush=True)
    dist.destroy_process_group()
""")


@pytest.mark.parametrize("n", [2, 3])
def test_spawn_ranks_runs_one_process_per_rank(tmp_path, capfd, n):
    script = tmp_path / "rank.py"
    script.write_text(_RANK_SCRIPT)
    rc = bench.spawn_ranks(n, ["--gpus", str(n)], script=str(script))
    assert rc == 0
    line = json.loads(capfd.readouterr().out.strip().splitlines()[-1])
    assert line == {"world": n, "max": float(n), "argv": ["--gpus", str(n)]}


def test_spawn_ranks_reports_a_failing_rank(tmp_path):
    script = tmp_path / "rank.py"
    script.write_text(_RANK_SCRIPT)
    assert bench.spawn_ranks(2, ["--fail"], script=str(script)) == 3


def test_rank_stdout_carries_only_the_result_line(tmp_path):
    """After _stdout_for_result_only, whatever a library writes to fd 1 (gloo
    prints its rendezvous to stdout) lands on stderr; the result line alone
    reaches stdout."""
    import subprocess
    script = tmp_path / "child.py"
    script.write_text(textwrap.dedent(f"""
        import os, sys, json
        sys.path.insert(0, {ROOT!r})
        import bench
        bench._stdout_for_result_only()
        os.write(1, b"[Gloo] Rank 0 is connected to 1 peer ranks\\n")
        print("a stray print")
        print(json.dumps({{"value": 1}}), file=bench._RESULT_OUT, flush=True)
    """))
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.splitlines() == ['{"value": 1}']
    assert "[Gloo] Rank 0" in r.stderr and "a stray print" in r.stderr


def test_guarded_returns_or_prints_and_exits_on_timeout(tmp_path):
    """bench._guarded: a call that returns in time gives its value; one that
    hangs past the timeout runs on_timeout (rank 0 prints its line) and the
    process exits with bench.WATCHDOG_EXIT (non-zero: the run is reported as
    failed) instead of holding the multi-GPU bench hostage."""
    import subprocess
    assert bench._guarded(lambda: 42, 5.0, lambda: None) == 42
    script = tmp_path / "child.py"
    script.write_text(textwrap.dedent(f"""
        import sys, time
        sys.path.insert(0, {ROOT!r})
        import bench
        bench._guarded(lambda: time.sleep(30), 0.5, lambda: print('{{"value": 7}}', flush=True))
        print("not reached", flush=True)
    """))
    t0 = time.perf_counter()
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, timeout=120)
    assert r.returncode == bench.WATCHDOG_EXIT != 0, r.stderr
    assert r.stdout.splitlines() == ['{"value": 7}']
    assert time.perf_counter() - t0 < 25


def test_pmc_traffic_takes_the_newest_round(tmp_path, monkeypatch):
    """with several PMC summaries for one config the
    newest round/session wins (r01 < r01_s4 < r02 < r02s2 < r03)."""
    prof = tmp_path / "profiles"
    (prof / "r03_sub").mkdir(parents=True)
    for name, val in [("r02s2_pmc_traffic.json", 2), ("r01_s4_pmc_traffic.json", 1), ("r02_pmc_traffic.json", 3),
                      ("r03_sub/r03_pmc_traffic.json", 4)]:
        (prof / name).write_text(json.dumps({"north_star": {"exact": {"hbm_bytes_per_launch": val}}}))
    (prof / "r03_other_pmc.json").write_text(json.dumps({"cfg2": {"exact": {"hbm_bytes_per_launch": 9}}}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    b, src = bench.pmc_traffic("north_star", "exact", 1)
    assert b == 4 and src.startswith("profiles/r03_sub/r03_pmc_traffic.json")
    assert bench.pmc_traffic("cfg3", "exact", 1)[0] is None


def test_box_info_names_the_host():
    info = bench.box_info()
    assert info["host_cpus"] >= 1 and info["threads_usable"] >= 1
    assert "cgroup_cpu_quota" in info and "omp_num_threads" in info
