import sys; sys.path[:0]=['.','lds-gnn_amd']
import torch, numpy as np
from ldsgnn import ops
from ldsgnn.data.workloads import load_workload
data = load_workload("cora-given")
adj = data.dense_adj.clone(); adj[3,3]=1.0
g = ops.csr_graph_from_dense(adj.to("cuda"))
a = g.to_dense().cpu(); deg = a.sum(1)
s1 = g.s.cpu(); s2 = 1.0/deg.float().sqrt()
bad = (s1 != s2).nonzero().squeeze(1)
print("bad", bad.numel(), bad[:10].tolist(), deg[bad[:10]].tolist(), s1[bad[:10]].tolist(), s2[bad[:10]].tolist(), g.deg.cpu()[bad[:10]].tolist())
