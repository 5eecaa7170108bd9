"""bench.py end to end on the GPU, as the driver runs it: the one-GPU line
(prefetched draws, four windows per graph) and the N > 1 path rehearsed with
two ranks over gloo on the one card (the exchange, the replica check and the
strong-scaling leg) — the driver's 8-GPU run takes the same code path over
RCCL.  Short runs: the numbers are not checked, the line's contract is."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]


def _line(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert lines, out[-2000:]
    return json.loads(lines[-1])


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_one_gpu_line():
    r = subprocess.run([sys.executable, "bench.py", "--steps", "10", "--warmup", "5", "--no-cpu-baseline",
                        "--no-breakdown"], cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r.stdout)
    assert d["metric"] == METRIC and d["n_gpus"] == 1 and d["steps"] == 10 and d["value"] > 0
    assert d["config"]["prefetched_draw"] is True and d["config"]["windows_per_graph"] == 4


def test_bench_two_ranks_gloo():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2", "--backend", "gloo",
           "--steps", "10", "--warmup", "5", "--strong-steps", "5", "--no-cpu-baseline", "--no-breakdown"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert d["config"]["replicas_in_sync"] is True and d["config"]["prefetched_draw"] is True
    s = d["strong_scaling"]
    assert s["samples_total"] == 64 and s["samples_per_rank"] == 32 and s["speedup_vs_1gpu"] > 0


def test_bench_two_ranks_gloo_config5_sharded():
    """BASELINE config 5 at N > 1, rehearsed: the synthetic N = 20 000 dense-θ
    line on two gloo ranks takes the band-sharded exchange by default
    (factor all-gather, band update, band draws + all-to-all) and
    ends with θ identical on both ranks after the bands are gathered."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2", "--backend", "gloo",
           "--dataset", "synthetic20k", "--steps", "5", "--warmup", "5", "--no-cpu-baseline", "--no-breakdown"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert d["config"]["workload"] == "synthetic20k-lds-S1-tau5"
    assert d["config"]["exchange"] == "band-sharded-gloo" and d["config"]["replicas_in_sync"] is True
