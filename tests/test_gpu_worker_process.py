"""The reference's process model around the HIP aggregate (GPU).

dasklearn/broker.py imports the task functions at top level (broker.py:16),
sets the file_system sharing strategy (broker.py:26) and starts its workers
with multiprocessing.Process under the default start method — fork on Linux
(broker.py:227-233); each worker runs worker.py:21-38's loop, host models
crossing the process boundary through shared memory. With INTEGRATION.md's
hook the top-level import is `from dasklearn_amd.functions import *`, so the
package must import in the broker WITHOUT initialising the GPU, and a forked
worker must run the HIP aggregate.

tests/_broker_child.py is that broker, started here as a fresh interpreter
(this pytest process has used the GPU, so it must not be the one that forks;
and torch's shm-manager helper then belongs to the broker and leaves with it,
not with pytest). Its worker runs the restated loop (tests/_worker_child.py):
results are checked against the oracle bit for bit, buffers come from
models[0], and a failing task comes back as ("error", task, None) and ends the
worker, as in the reference. Both start methods are covered."""
from __future__ import annotations

import json
import os
import subprocess
import sys
import time

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _wait_gone(pids, seconds):
    import psutil
    deadline = time.monotonic() + seconds
    alive = list(pids)
    while True:
        alive = [p for p in alive if psutil.pid_exists(p) and psutil.Process(p).status() != psutil.STATUS_ZOMBIE]
        if not alive or time.monotonic() > deadline:
            return alive
        time.sleep(0.1)


@pytest.mark.parametrize("method", ["fork", "spawn"])
def test_broker_worker_round_trip(method):
    r = subprocess.run([sys.executable, os.path.join(HERE, "_broker_child.py"), method], capture_output=True,
                       text=True, timeout=240)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines, r.stdout[-2000:] + r.stderr[-3000:]
    out = json.loads(lines[-1])
    assert out["start_method"] == method
    assert out["gpu_initialised_before_fork"] is False  # importing the hook does not touch the GPU
    assert out["checks"] == {"agg_0": True, "agg_1": True, "agg_2": True, "error_protocol": True}, out
    assert out["worker_exitcode"] == 0 and out["ok"] and r.returncode == 0, out
    # torch's helpers (the file_system strategy's shm manager) leave with their
    # last client; none may outlive the broker for long
    left = _wait_gone([h["pid"] for h in out["helpers"]], 15)
    assert not left, f"helper processes still alive: {out['helpers']}"
