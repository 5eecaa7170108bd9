"""Debug helper: run the Cora-shaped τ-window of tests/golden/hypergrad_cora on
the GPU product and dump per-step details for comparison with the oracle."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lds-gnn_amd")]
import ldsgnn  # noqa: E402
from ldsgnn.models.gcn import MetaDenseGCN  # noqa: E402
from ldsgnn.models.graph import BernoulliGraphModel  # noqa: E402
from ldsgnn.trainers.bilevel import BilevelProblemRunner  # noqa: E402
from ldsgnn.trainers.inner import InnerProblemTrainer  # noqa: E402
from ldsgnn.trainers.outer import OuterProblemTrainer  # noqa: E402

g = np.load(os.path.join(ROOT, "tests/golden/hypergrad_cora.npz"))
seed = int(g["seed"])
from tests.test_oracle_golden import cora_golden_problem  # noqa: E402
from ldsgnn.utils.graph import DenseData  # noqa: E402
d, opt, seed = cora_golden_problem(g)
data = DenseData(x=d.x, y=d.y, dense_adj=d.dense_adj, train_mask=d.train_mask, val_mask=d.val_mask & ~opt,
                 test_mask=d.test_mask, num_classes=7).to("cuda")
ldsgnn.rng.manual_seed(seed, 0)
torch.manual_seed(seed)
gcn = MetaDenseGCN(data.num_features, 16, 7, dropout=0.5).to("cuda")
inner = InnerProblemTrainer(gcn, data, lr=0.01, weight_decay=5e-4)
gm = BernoulliGraphModel(data.dense_adj)
outer = OuterProblemTrainer(torch.optim.SGD(gm.parameters(), lr=0.1), data, opt.to("cuda"), gm, lr_decay=0.99)
runner = BilevelProblemRunner(inner, outer, data)
nnz, losses, grads, thetas, params = [], [], [], [], []
orig_sample = gm.sample


def spy_sample():
    gr = orig_sample()
    nnz.append(gr.nnz())
    return gr


gm.sample = spy_sample
for step in range(6):
    losses.append(runner.inner_opt_step().loss)
    params.append(np.concatenate([p.detach().cpu().numpy().ravel() for p in inner.model_params.values()]))
    if step % 5 == 0:
        runner.hyper_opt_step(step)
        grads.append(gm.probs.grad.detach().cpu().numpy())
        thetas.append(gm.probs.detach().cpu().numpy())
os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed("gpurun_out/cora_window.npz", nnz=np.array(nnz), losses=np.array(losses),
                    grad0=grads[0], theta0=thetas[0], grad1=grads[1], params=np.stack(params))
print("nnz", nnz, "losses", losses)
