"""The sharded path with the HIP kernel as the local reduce in more than one
process (GPU).

Two or four fresh rank processes (tests/_sharded_hip_child.py) share the one
MI355X of the box with a gloo control plane: each runs
aggregate_param_sharded (gathered and not), a plan's repeated runs,
aggregate_model_sharded(exact=True) and (round 5) its FAST form (partial
sums, reduce-scatter, all-gather; SURVEY §8e's tolerance) with
ShardedAggregator's default local reduce, the HIP kernel, on fp32 and bf16 models; the gathers go through host
tensors (gloo). Every rank's assembled output must be bit-identical to the
oracle's single fold ("results are bit-identical to 1 GPU").
The ranks are started as fresh interpreters, as bench.py starts its ranks:
this pytest process has used the GPU and forks nothing that uses it."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_ranks(world, script, *args, timeout=180):
    """Start `world` rank processes of `script`, wait, and return each rank's
    last JSON line (asserting every rank exited 0 and printed one)."""
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, script), *args], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    try:
        for pr in procs:
            out, err = pr.communicate(timeout=timeout)
            outs.append((pr.returncode, out, err))
    finally:
        for pr in procs:
            if pr.poll() is None:
                pr.kill()
                pr.wait()
    results = []
    for r, (rc, out, err) in enumerate(outs):
        lines = [ln for ln in out.splitlines() if ln.startswith("{")]
        assert rc == 0 and lines, f"rank {r}: rc={rc}\n{out[-2000:]}\n{err[-3000:]}"
        res = json.loads(lines[-1])
        assert res["rank"] == r and res["world"] == world
        results.append(res)
    return results


@pytest.mark.parametrize("world", [2, 4])
def test_processes_hip_local_reduce_bit_exact(world):
    for r, res in enumerate(_run_ranks(world, "_sharded_hip_child.py")):
        assert res["checks"] and all(res["checks"].values()), (r, res["checks"])


@pytest.mark.parametrize("config,world", [("cfg4", 4), ("cfg5", 8)])
def test_baseline_sharded_configs_full_size_bit_exact(config, world):
    """BASELINE.json's parameter-sharded configs at their
    real geometry -- cfg4, 2 x 125,000,000 bf16 over 4 ranks; cfg5, 100 x
    11,181,642 fp32 over 8 ranks -- each rank reducing its real slice with the
    HIP kernel; every rank's slice and rank 0's assembled output bit-exact
    against the oracle (tests/_sharded_full_child.py)."""
    results = _run_ranks(world, "_sharded_full_child.py", config, timeout=240)
    for r, res in enumerate(results):
        assert res["config"] == config and all(res["checks"].values()), (r, res["checks"])
    assert "assembled_full_bit_exact" in results[0]["checks"]
    assert [tuple(res["slice"]) for res in results][-1][1] == (125_000_000 if config == "cfg4" else 11_181_642)
