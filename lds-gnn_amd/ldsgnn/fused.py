"""Build the fused engine from the drop-in trainers (same problem, same state).

`engine_from_trainers(inner, outer)` maps an InnerProblemTrainer
(MetaDenseGCN + differentiable Adam) and an OuterProblemTrainer
(BernoulliGraphModel + plain SGD, optional StepLR) onto an LdsEngine that
updates the graph model's θ in place and continues the trainers' RNG stream.
"""
from __future__ import annotations

from . import replicas as _replicas
from . import rng as _rng
from .engine import LdsEngine, capture_into


def engine_from_trainers(inner, outer, tau: int = 5, generator: "_rng.Generator" = None,
                         samples: int = 1) -> LdsEngine:
    """samples > 1: S replica chains (replicas generator.replica + b) batched
    in one engine; θ moves by their mean hypergradient.
    The embedding model (PairwiseEmbeddingSampler, src/models/graph.py:81-112)
    runs the inner loop and the hypergradient dθ on the engine with θ = the
    upper triangle of P = σ(E·Eᵀ)^pow; its outer step (OuterProblemTrainer.
    train_step after the backward: optimizer, StepLR, projection) runs on E
    from dθ by autograd through P, and rewrites θ (`LdsEngine.outer_update`)."""
    from .models.graph import BernoulliGraphModel, GraphProposalNetwork, PairwiseEmbeddingSampler
    gm = outer.model
    gcn = inner.model
    data = inner.data
    if isinstance(gm, PairwiseEmbeddingSampler):
        return _param_theta_engine(inner, outer, tau, generator, samples)
    if isinstance(gm, GraphProposalNetwork):
        return _param_theta_engine(inner, outer, tau, generator, samples)
    if not isinstance(gm, BernoulliGraphModel) or gm.directed:
        raise NotImplementedError("the fused engine implements the undirected LDS Bernoulli model, "
                                  "the embedding model and the GAE model")
    opt = outer.optimizer
    if len(opt.param_groups) != 1:
        raise NotImplementedError("one θ parameter group expected")
    grp = opt.param_groups[0]
    if grp.get("momentum", 0) or grp.get("weight_decay", 0) or grp.get("nesterov", False) or \
            grp.get("dampening", 0):
        raise NotImplementedError("the fused engine implements plain SGD on θ")
    if outer.lr_decay is not None and outer.lr_decay_step_size != 1:
        raise NotImplementedError("StepLR with step_size 1 only")
    eng = LdsEngine(data.x, data.y, data.train_mask, outer.opt_mask, gm.probs.data, data.num_classes,
                    dropout=gcn.dropout, gcn_lr=inner.lr, gcn_wd=inner.weight_decay, outer_lr=grp["lr"],
                    lr_decay=outer.lr_decay, tau=tau, generator=generator or gcn.generator or _rng.default_generator,
                    params=inner.model_params, samples=samples)
    # θ.grad is the engine's dθ buffer, as after the reference's backward
    # (src/trainers/outer.py:77), so a grad_reducer written for the drop-in
    # trainer (e.g. ldsgnn.replicas.allreduce_mean(model)) sees the engine's
    # hypergradient; with one set, every hyper step runs dθ → reducer → SGD
    gm.probs.grad = eng.grad
    if outer.grad_reducer is not None:
        reducer, model = outer.grad_reducer, gm

        def reduce_engine_grad(grad, prescaled=False):
            # prescaled (the engine assembled dθ / world, see `prescale`): the
            # mean is the all-reduce SUM alone, no division pass over θ.grad
            if prescaled:
                _replicas.allreduce_sum_(grad)
                return
            # re-bind on every call: a zero_grad(set_to_none=True) in between
            # would otherwise leave θ.grad None, the reducer would skip it and
            # each rank would apply only its own dθ
            model.probs.grad = grad
            reducer(model)
            if model.probs.grad is not grad:  # a reducer that rebinds .grad
                grad.copy_(model.probs.grad)
                model.probs.grad = grad

        # graph-capturable exactly when the trainer's reducer is (RCCL all-reduce)
        reduce_engine_grad.capturable = getattr(reducer, "capturable", False)
        # the package's all-reduce mean: the engine may scale dθ by 1/world in
        # the assembly (a power-of-two world: the same bits as sum-then-divide
        # for every dθ entry above the subnormal range; entries near FLT_MIN
        # may differ by up to world subnormal ulps, world · 2^-149 —
        # tests/test_replicas_gloo.py)
        if reducer is _replicas.allreduce_mean:
            reduce_engine_grad.prescale = _replicas.mean_prescale
        eng.grad_reducer = reduce_engine_grad
    return eng


def _param_theta_engine(inner, outer, tau, generator, samples) -> LdsEngine:
    """Engine for a graph model whose θ is a function of its own parameters
    (embedding, GAE): θ = triu(P(params)), and the model's outer step, by
    autograd through P, runs as LdsEngine.outer_update.

    A GAE proposal GCN with dropout makes every sample() a new P
    (src/models/graph.py:167-186: the proposal forward runs in training mode
    once per draw, src/trainers/bilevel.py:103-106, outer.py:61-63), so the
    engine runs per-draw θ (LdsEngine.set_theta_fn): draw t of a window is
    sampled from θ_t = triu(P) of the proposal forward at the forward counter
    the drop-in's sample() would take (one before the classifier forward of
    the same step), the hyper step assembles one dθ_t per draw, and the outer
    step sums Σ_t ⟨triu(P_t), dθ_t⟩ through each draw's own P_t (same
    dropout masks, same counters).  θ for evaluation is the eval-mode P."""
    import torch

    from .models.graph import GraphProposalNetwork
    from .models.sampling import Sampler
    gm, gcn, data = outer.model, inner.model, inner.data
    if samples != 1:
        raise NotImplementedError("the embedding model runs single-sample on the engine")
    cfg = Sampler.config
    if not cfg.get("undirected", True) or str(cfg.get("sparsification", "NONE")).upper() != "NONE" or \
            cfg.get("dense", False):
        raise NotImplementedError("the engine draws undirected, unsparsified graphs")
    if outer.refine_embeddings:
        raise NotImplementedError("refine_embeddings changes the GAE inputs per sample")
    n = data.num_nodes
    iu = torch.triu_indices(n, n, device=data.x.device)

    def theta_of_model() -> torch.Tensor:
        # eval-mode P: what empirical_mean_loss samples from (src/utils/evaluation.py:66-72)
        was = gm.training
        gm.eval()
        try:
            with torch.no_grad():
                return gm.forward()[iu[0], iu[1]].contiguous()
        finally:
            gm.train(was)

    per_draw = isinstance(gm, GraphProposalNetwork) and gm.gcn.dropout != 0.0

    eng = LdsEngine(data.x, data.y, data.train_mask, outer.opt_mask, theta_of_model(), data.num_classes,
                    dropout=gcn.dropout, gcn_lr=inner.lr, gcn_wd=inner.weight_decay, outer_lr=0.0,
                    lr_decay=None, tau=tau, generator=generator or gcn.generator or _rng.default_generator,
                    params=inner.model_params, samples=1)

    def proposal_at(counter: int, grad: bool) -> torch.Tensor:
        """triu(P) of the proposal forward (training mode) at a forward counter."""
        was = gm.training
        gm.train()
        try:
            with torch.set_grad_enabled(grad):
                p, _ = gm.calculate_edges_and_embeddings(dropout_counter=counter)
            return p[iu[0], iu[1]]
        finally:
            gm.train(was)

    if per_draw:
        if (gm.gcn.generator or _rng.default_generator) is not eng.gen:
            raise NotImplementedError("per-draw θ needs the proposal GCN and the engine on one generator "
                                      "(one forward-counter sequence)")
        eng.set_theta_fn(lambda counter: proposal_at(counter, False))

    def outer_update(grad: torch.Tensor) -> None:
        # OuterProblemTrainer.train_step (src/trainers/outer.py:57-87) from the backward on:
        # dθ -> E through P's upper triangle, optimizer, StepLR, projection
        outer.optimizer.zero_grad()
        if per_draw:  # grad: [draws, n(n+1)/2], draw t through its own P_t
            for t in range(grad.size(0)):
                (proposal_at(eng.theta_counters[t], True) * grad[t]).sum().backward()
        else:
            gm.forward()[iu[0], iu[1]].backward(grad)
        if outer.grad_reducer is not None:
            outer.grad_reducer(gm)
        outer.optimizer.step()
        if outer.lr_decayer is not None:
            outer.lr_decayer.step()
        gm.project_parameters()
        eng.theta.copy_(theta_of_model())

    eng.outer_update = outer_update
    return eng


class FusedBilevelRunner:
    """BilevelProblemRunner.train / evaluate (src/trainers/bilevel.py:34-145)
    driven by the fused engine: the same loop, counters, early-stopping rules
    and reset / detach points, with every inner step, hyper step and the
    16-sample empirical evaluation running as fused HIP kernels.  The trainers
    supply the initial state and the weight re-initialisation
    (MetaDenseGCN.reset_weights consumes the torch RNG exactly as there); the
    per-step train loss is read back for the inner early stopping (one sync per
    inner step, as the reference's `.item()`), so the unit of replay is the
    step.  With `step_graphs` (default) every inner step position and hyper
    step length is captured as a HIP graph at its second use and replayed
    after that (LdsEngine.inner_step_graphed / hyper_step_graphed), with
    results identical to eager steps (`step_graphs=False`).  A captured step
    holds kernel nodes only: a memset node in the per-step draw faulted on
    its replay after a τ = 20 window."""

    def __init__(self, inner_trainer, outer_trainer, data, n_samples_empirical_mean: int = 16,
                 generator: "_rng.Generator" = None, step_graphs: bool = True):
        self.inner_trainer = inner_trainer
        self.outer_trainer = outer_trainer
        self.data = data
        self.n_samples_empirical_mean = n_samples_empirical_mean
        self.generator = generator
        self.step_graphs = step_graphs
        self.engine = None
        self.gcn_params = None
        self.graph_state_dict = None
        self.inner_steps = 0

    def train(self, patience: int, hyper_gradient_interval: int, inner_loop_max_epochs: int = 400,
              outer_loop_max_epochs: int = 400, sacred_runner=None):
        from copy import deepcopy

        from .utils.early_stopping import EarlyStopping
        tau = hyper_gradient_interval
        eng = self.engine = engine_from_trainers(self.inner_trainer, self.outer_trainer, tau=max(1, tau),
                                                 generator=self.generator)
        log = sacred_runner
        outer_stop = EarlyStopping(patience=patience, max_epochs=outer_loop_max_epochs)
        step = 0
        while not outer_stop.abort:
            inner_stop = EarlyStopping(patience=patience, max_epochs=inner_loop_max_epochs)
            self.inner_trainer.reset_weights()       # torch RNG draws as in the reference
            eng.reset_optimizer()                    # cuts the tape (new leaves), Adam state / step 0
            eng.set_params(self.inner_trainer.model_params)
            while not inner_stop.abort:
                t = eng.t
                if self.step_graphs:
                    eng.inner_step_graphed()
                else:
                    eng.inner_step()
                loss, acc = eng.inner_metrics(t)
                inner_stop.update(loss, model_params=eng.flat_params())
                if log is not None:
                    log("loss.train", loss, step)
                    log("acc.train", acc, step)
                if tau == 0 or step % tau == 0:
                    if self.step_graphs:
                        eng.hyper_step_graphed()
                    else:
                        eng.hyper_step()
                    if log is not None:
                        ol, oa = eng.outer_metrics()
                        log("loss.outer", ol, step)
                        log("acc.outer", oa, step)
                        self._log_model_statistics(eng, log, step)
                step += 1
            self.inner_steps = step
            vl, va, tl, ta = eng.empirical_mean(inner_stop.model_params, self.n_samples_empirical_mean,
                                                self.data.val_mask, self.data.test_mask)
            if log is not None:
                log("loss.val.empirical", vl, None)
                log("acc.val.empirical", va, None)
                log("loss.test.empirical", tl, None)
                log("acc.test.empirical", ta, None)
            # the reference stores the graph model's state_dict(): views of the
            # live θ, so evaluate() sees the final θ (kept)
            outer_stop.update(vl, model_params=[deepcopy(inner_stop.model_params), eng.theta])
        self.gcn_params, self.graph_state_dict = outer_stop.model_params
        eng.sync_generator()

    def _log_model_statistics(self, eng, log, step):
        """BilevelProblemRunner.hyper_opt_step logs the graph model's
        statistics() after a hyper step (src/trainers/bilevel.py:117-120).  A
        GAE proposal with dropout runs a training-mode forward there and takes
        a forward counter, which the engine's sequence skips likewise (per-draw
        θ); the other models' statistics draw nothing and are not logged here."""
        if getattr(eng, "theta_fn", None) is None:
            return
        for name, value in self.outer_trainer.model.statistics(dropout_counter=eng.take_forward_counter()).items():
            log(name, value, step)

    def evaluate(self):
        assert self.gcn_params is not None, "Models need to be trained before evaluation."
        vl, va, tl, ta = self.engine.empirical_mean(self.gcn_params, self.n_samples_empirical_mean,
                                                    self.data.val_mask, self.data.test_mask)
        return {"loss.val.final": vl, "acc.val.final": va, "loss.test.final": tl, "acc.test.final": ta}


class FixedGraphGcn:
    """BASELINE config 1 — fixed-adjacency GCN training, src/scripts/gcn.py:
    56-99 — on the fused engine.  θ is the given 0/1 adjacency's upper
    triangle, whose Bernoulli draws are exactly that graph (u ∈ [0, 1): u < 1
    always, u < 0 never), drawn once; there is no hyper step.  One epoch is the
    reference's train step (training-mode forward with dropout, NLL on the
    train rows, backward, Adam with weight decay on layer_in only,
    src/scripts/gcn.py:62-67,75-83) and evaluate() (eval-mode forward, NLL and
    accuracy on the validation and test rows, src/utils/evaluation.py:25-48),
    with one host read of the epoch's metrics (the reference's `.item()`s).
    From the second epoch on, train step and evaluation replay as one HIP
    graph.

    gcn: the MetaDenseGCN whose initial weights and dropout rate are used;
    data: DenseData with the fixed dense_adj (any symmetric 0/1 matrix)."""

    def __init__(self, gcn, data, lr: float = 0.01, weight_decay: float = 5e-4,
                 generator: "_rng.Generator" = None, graphs: bool = True):
        import numpy as np
        import torch

        from .engine import _Slot
        n = data.num_nodes
        iu = torch.triu_indices(n, n, device=data.x.device)
        theta = data.dense_adj[iu[0], iu[1]].float().contiguous()
        if not bool(((theta == 0) | (theta == 1)).all()):
            raise NotImplementedError("FixedGraphGcn takes a 0/1 adjacency (the graph the reference normalises)")
        params = gcn.model_params if hasattr(gcn, "model_params") else dict(gcn.named_parameters())
        from collections import OrderedDict
        params = OrderedDict((k, v.detach()) for k, v in params.items())
        self.eng = eng = LdsEngine(data.x, data.y, data.train_mask, data.val_mask, theta, data.num_classes,
                                   dropout=gcn.dropout, gcn_lr=lr, gcn_wd=weight_decay, outer_lr=0.0,
                                   lr_decay=None, tau=1, generator=generator or gcn.generator or _rng.default_generator,
                                   params=params, samples=1)
        if eng.long_rows:
            raise NotImplementedError("FixedGraphGcn: short-row graphs (the engine's in-kernel aggregation)")
        self.gcn, self.data = gcn, data
        self.use_graphs = graphs
        self._graph = None
        self._drawn = False
        self.vm = data.val_mask.to(device=eng.dev, dtype=torch.uint8).contiguous()
        self.tm = data.test_mask.to(device=eng.dev, dtype=torch.uint8).contiguous()
        self.inv_v = float(np.float32(1.0) / np.float32(int(data.val_mask.sum())))
        self.inv_t = float(np.float32(1.0) / np.float32(int(data.test_mask.sum())))
        # evaluation slot reading the training graph (no draw)
        self._ev = _Slot(n, eng.cap, eng.dev, x_nnz=0, samples=1, bptr_len=eng.bptr_len, words=eng.words)
        self._test_rows = torch.zeros((2, n), dtype=torch.float32, device=eng.dev)

    def _train_step(self):
        eng = self.eng
        if not self._drawn:
            eng.inner_step()  # draws the graph (deterministic) into slot 0
            self._drawn = True
        else:
            eng.inner_step(presampled=True)
        eng.detach()

    def _evaluate(self):
        """evaluate() launches: eval-mode forward on the fixed graph, NLL /
        correct sums of the val and test rows, and the train step's metrics,
        into self._res (6 floats on device)."""
        import torch

        from . import _native as nat
        eng, ev = self.eng, self._ev
        ev.g = eng.slots[0].g  # the fixed graph
        st, n, c = eng._stream(), eng.n, eng.c
        eng._forward(ev, eng.w[0], self.vm, self.inv_v, 0, 0)  # eval mode: val rows -> ev.lossrow / corrrow
        g = ev.g
        nat.call("lds_engine_fwd_layer2", nat.ptr(g.row_ptr), nat.ptr(g.col), nat.ptr(g.s), nat.ptr(g.ell), n,
                 nat.ptr(ev.h2), 0, 0, 0, nat.ptr(eng.label), nat.ptr(self.tm), self.inv_t,
                 nat.ptr(self._test_rows[0]), nat.ptr(self._test_rows[1]), c, 0, eng.bt, st)
        r = self._res
        torch.mul(eng.metrics[0][0], 1.0, out=r[0:2])  # a kernel: captured graphs hold kernel nodes only
        for i, t in enumerate((ev.lossrow[0], ev.corrrow[0], self._test_rows[0], self._test_rows[1])):
            torch.sum(t, dim=0, keepdim=True, out=r[2 + i:3 + i])

    def epoch(self):
        """train step + evaluate(); returns (train loss, train acc, val loss,
        val acc, test loss, test acc) of the epoch (one host sync).  With
        graphs, from the second epoch on both run as one HIP graph replay."""
        import torch

        from . import _native as nat
        eng = self.eng
        if getattr(self, "_res", None) is None:
            self._res = torch.zeros(6, dtype=torch.float32, device=eng.dev)
        if not self.use_graphs or not self._drawn:
            self._train_step()
            self._evaluate()
        else:
            if self._graph is None:
                s = torch.cuda.Stream(eng.dev)
                s.wait_stream(torch.cuda.current_stream(eng.dev))
                g = nat.new_graph()

                def body():
                    self._train_step()
                    self._evaluate()
                try:  # (an error inside the capture is raised alone, the stream left usable)
                    capture_into(g, s, body, joins=(eng.side,))
                finally:
                    torch.cuda.current_stream(eng.dev).wait_stream(s)
                self._graph = nat.seal_graph(g, "fixed-graph epoch")
            self._graph.replay()
        host = self._res.double().cpu().numpy()
        return (float(host[0] * eng.inv_train), float(host[1] * eng.inv_train), float(host[2] * self.inv_v),
                float(host[3] * self.inv_v), float(host[4] * self.inv_t), float(host[5] * self.inv_t))

    def params(self):
        """Current weights in the reference layout (layer_in.fc.weight, ...)."""
        return self.eng.get_params()

    def sync_generator(self):
        self.eng.sync_generator()
