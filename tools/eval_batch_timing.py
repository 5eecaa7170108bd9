"""empirical_mean on the fused engine at Cora shape: the batched evaluation
(16 graphs in one sampler launch set, one eval forward with grid.y = sample)
against the one-graph-at-a-time form.  Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "lds-gnn_amd")):
    sys.path.insert(0, p)
import torch  # noqa: E402

import ldsgnn  # noqa: E402
from ldsgnn.data.synthetic import knn_init, make_dataset  # noqa: E402
from ldsgnn.engine import LdsEngine  # noqa: E402
from ldsgnn.models.gcn import MetaDenseGCN  # noqa: E402
from oracle import lds_oracle as O  # noqa: E402


def main(dataset="cora", n_samples=16, reps=20):
    dev = torch.device("cuda:0")
    data = knn_init(make_dataset(dataset, seed=1), k=10).to(dev)
    torch.manual_seed(0)
    gcn = MetaDenseGCN(data.num_features, 16, data.num_classes, dropout=0.5).to(dev)
    params = {k: v.detach() for k, v in gcn.named_parameters()}
    theta = O.get_triu_values(data.dense_adj).contiguous()
    eng = LdsEngine(data.x, data.y, data.train_mask, data.val_mask, theta, data.num_classes, outer_lr=0.1, tau=5,
                    generator=ldsgnn.rng.Generator(1, 0), params=params)
    eng.run_window(5)
    flat = eng.flat_params().clone()
    out = {"workload": f"{dataset} empirical_mean, {n_samples} samples", "nodes": data.num_nodes}
    for name, fn in (("batched", eng._empirical_mean_batched), ("sequential", eng._empirical_mean_seq)):
        fn(flat, n_samples, data.val_mask, data.test_mask)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            res = fn(flat, n_samples, data.val_mask, data.test_mask)
        torch.cuda.synchronize()
        out[name] = {"ms_per_call": 1000.0 * (time.perf_counter() - t0) / reps, "val_loss": res[0],
                     "val_acc": res[1]}
    out["speedup"] = out["sequential"]["ms_per_call"] / out["batched"]["ms_per_call"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
