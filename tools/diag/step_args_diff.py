"""Which launch argument of an inner step changes between windows although the
step-graph key does not?  The fused runner (Cora, tau = 20) runs with eager
steps; every C-ABI call of every inner step is recorded with the step's
graph key, and the calls of steps that share a key are compared argument by
argument.  A captured step graph bakes the arguments of its capture, so any
difference here is a stale argument in a replay."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lds-gnn_amd"), os.path.join(ROOT, "tools")]
import torch  # noqa: E402

import ldsgnn  # noqa: E402,F401
from ldsgnn import _native as nat  # noqa: E402
from ldsgnn import engine as E  # noqa: E402
from ldsgnn import fused as F  # noqa: E402
from ldsgnn.ops import theta_grad_form  # noqa: E402

MAX_STEPS = int(os.environ.get("MAX_STEPS", "64"))
rec = {"cur": None}
by_key = {}
real_call = nat.call


def call(name, *a):
    if rec["cur"] is not None:
        rec["cur"].append((name, a[:-1]))  # the stream handle is the capture's own
    return real_call(name, *a)


nat.call = call


class Stop(Exception):
    pass


def wrap(kind, orig):
    def step(self, *a, **k):
        key = (kind, self.t, self.pending_graph, self.pending_fwd, self.train_flag, self._tab_count(),
               theta_grad_form(), self.keep_grad, self._layout_version)
        n = sum(len(v) for v in by_key.values())
        if n >= MAX_STEPS:
            raise Stop()
        rec["cur"] = []
        try:
            return orig(self, *a, **k)
        finally:
            by_key.setdefault(key, []).append((n, rec["cur"]))
            rec["cur"] = None
    return step


E.LdsEngine.inner_step = wrap("inner", E.LdsEngine.inner_step)
E.LdsEngine.hyper_step = wrap("hyper", E.LdsEngine.hyper_step)
_init = F.FusedBilevelRunner.__init__


def _init_eager(self, *a, **k):
    k["step_graphs"] = False
    _init(self, *a, **k)


F.FusedBilevelRunner.__init__ = _init_eager
import accuracy_run  # noqa: E402

try:
    accuracy_run.run_lds("cora", 597905255 % (2 ** 31), torch.device("cuda:0"), pretrain=True, tau=20, fused=True)
except Stop:
    pass
torch.cuda.synchronize()
diffs = 0
for key, runs in by_key.items():
    if len(runs) < 2:
        continue
    n0, first = runs[0]
    for n, calls in runs[1:]:
        if [c[0] for c in calls] != [c[0] for c in first]:
            diffs += 1
            print(f"key {key}: call {n} launches {[c[0] for c in calls]} vs call {n0} {[c[0] for c in first]}")
            continue
        for (name, a), (_, b) in zip(calls, first):
            idx = [i for i, (x, y) in enumerate(zip(a, b)) if x != y]
            if idx:
                diffs += 1
                print(f"key {key}: call {n} vs {n0}: {name} args {idx}: "
                      f"{[a[i] for i in idx]} vs {[b[i] for i in idx]}", flush=True)
print(f"keys {len(by_key)}, repeated {sum(len(r) > 1 for r in by_key.values())}, differing calls {diffs}", flush=True)
