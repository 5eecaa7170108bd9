"""Build tests/golden/planetoid_{cora,citeseer}.npz from the reference's own
test resources (/root/reference/tst/res/<name>/raw/ind.*) with the data-only
pickle reader (ldsgnn.data.planetoid; nothing is unpickled).  Run in the
development container only — the GPU box reads the committed .npz."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lds-gnn_amd"))
import numpy as np  # noqa: E402

from ldsgnn.data.planetoid import read_planetoid_raw  # noqa: E402

for name in ("cora", "citeseer"):
    d = read_planetoid_raw(f"/root/reference/tst/res/{name}/raw", name)
    x = d["x"]
    rows, cols = np.nonzero(x)
    indptr = np.zeros(x.shape[0] + 1, dtype=np.int32)
    np.add.at(indptr, rows + 1, 1)
    indptr = np.cumsum(indptr).astype(np.int32)
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", f"planetoid_{name}.npz"),
                        x_shape=np.array(x.shape, dtype=np.int64), x_indptr=indptr,
                        x_indices=cols.astype(np.int32), x_data=x[rows, cols].astype(np.float32),
                        y=d["y"], edge_index=d["edge_index"].astype(np.int32),
                        train_mask=d["train_mask"], val_mask=d["val_mask"], test_mask=d["test_mask"])
    print(name, x.shape, "x nnz", len(rows), "edges", d["edge_index"].shape[1],
          "train/val/test", int(d["train_mask"].sum()), int(d["val_mask"].sum()), int(d["test_mask"].sum()))
