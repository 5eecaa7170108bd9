"""The N > 1 exchange over the nccl (= RCCL) backend on the MI355X, at world
size 1 (a one-GPU box cannot hold two RCCL ranks): process-group init, the
all-reduce of θ.grad run eagerly between the split window graphs and captured
into the window graph, against the same engine with a no-op exchange — θ,
θ.grad, weights and scalars bit-identical every window (tests/rccl_worker.py,
run in its own process under a time limit so that an RCCL hang cannot take
the suite with it).  SURVEY §8(e); bench.py uses the captured exchange at
N > 1 when every rank's capture probe succeeds."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_world_size_1_exchange_eager_and_captured():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", LOCAL_RANK="0",
               WORLD_SIZE="1")
    proc = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "rccl_worker.py")], env=env,
                          capture_output=True, text=True, timeout=280)
    assert proc.returncode == 0, proc.stdout[-2000:] + proc.stderr[-4000:]
    res = json.loads(proc.stdout.strip().splitlines()[-1])
    assert res["backend"] == "nccl" and res["world"] == 1
    assert res["capturable"] and res["probe"], res
    assert res["capture_is_one_graph"], res
    assert res["theta_moved"], res
    for w, row in enumerate(res["bit_identical_per_window"]):
        assert row["eager"] and row["capture"], (w, res)
    assert res["group_replay_identical"], res
    assert res["band_sharded_rccl_identical"], res  # (the config-5 sharded exchange's RCCL collectives)
