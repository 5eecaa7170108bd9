"""Dump the engine's config-2 hypergradients at the golden's sampled entries
(gpurun_out/config2_grads.npz) for offline comparison with the reference
golden and its rounding probe."""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "lds-gnn_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ldsgnn  # noqa: E402
from ldsgnn.fused import engine_from_trainers  # noqa: E402
from tests.test_workloads_gpu import _trainers  # noqa: E402

g = np.load(os.path.join(ROOT, "tests/golden/hypergrad_cora_real.npz"))
seed = int(g["seed"])
data, inner, outer, gm = _trainers("cora", g, seed)
eng = engine_from_trainers(inner, outer, tau=5, generator=ldsgnn.rng.default_generator)
eng.inner_step()
eng.hyper_step()
torch.cuda.synchronize()
g0 = eng.grad.double().cpu().numpy()[g["idx"]]
eng.capture_window(5)
eng.replay(1)
torch.cuda.synchronize()
g1 = eng.grad.double().cpu().numpy()[g["idx"]]
p = eng.get_params()
flat = np.concatenate([p[k].detach().cpu().numpy().ravel() for k in p])
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", "config2_grads.npz"), grad0=g0, grad1=g1, params=flat)
