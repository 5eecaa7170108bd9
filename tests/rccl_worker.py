"""World-size-1 RCCL rehearsal of the N > 1 exchange (run by
tests/test_rccl_gpu.py in its own process, under a time limit): a process
group on the nccl (= RCCL) backend, then three engines on the real Cora
workload with two replica samples each, identical but for the exchange:

  noop    the exchange point with no collective (two graphs per window);
  eager   the RCCL all-reduce (SUM, ÷ world) run eagerly between the two
          graphs of each window (the round-4 N > 1 path);
  capture the same all-reduce captured INTO the window graph, two windows per
          replayed graph (ldsgnn.replicas: capturable under nccl).

At world size 1 the all-reduce leaves θ.grad as it is, so θ, θ.grad, the
weights and the scalars must be bit-identical across the three after every
replay.  Prints one JSON line (and writes gpurun_out/rccl_ws1.json when that
directory exists)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lds-gnn_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

SEED, WINDOWS, SAMPLES = 23, 4, 2


def trainers(reducer):
    import numpy as np

    import ldsgnn
    from ldsgnn.data.workloads import load_workload
    from ldsgnn.fused import engine_from_trainers
    from ldsgnn.models.gcn import MetaDenseGCN
    from ldsgnn.models.graph import BernoulliGraphModel
    from ldsgnn.trainers.inner import InnerProblemTrainer
    from ldsgnn.trainers.outer import OuterProblemTrainer
    from ldsgnn.utils.graph import split_mask
    data = load_workload("cora")
    np.random.seed(SEED)
    data.val_mask, opt = split_mask(data.val_mask, 0.5, shuffle=True)
    data = data.to("cuda")
    ldsgnn.rng.manual_seed(SEED, 0)
    torch.manual_seed(SEED)
    gcn = MetaDenseGCN(data.num_features, 16, data.num_classes, dropout=0.5).to("cuda")
    inner = InnerProblemTrainer(gcn, data, lr=0.01, weight_decay=5e-4)
    gm = BernoulliGraphModel(data.dense_adj)
    outer = OuterProblemTrainer(torch.optim.SGD(gm.parameters(), lr=0.1), data, opt.to("cuda"), gm,
                                lr_decay=0.99, grad_reducer=reducer)
    return engine_from_trainers(inner, outer, tau=5, generator=ldsgnn.rng.default_generator, samples=SAMPLES)


def band_sharded_rccl() -> bool:
    """The band-sharded exchange's collectives on the nccl backend with
    device tensors (factor all-gather, the band rows' all-to-all with split
    sizes, θ's band gather), forced to run at world size 1: a long-row engine
    with them against one whose world-size-1 collectives are identities —
    θ, bits, s and weights bit-identical over a step-0 window and two τ = 5
    windows."""
    from ldsgnn.replicas import BandShards
    from tests.parity_harness import run_engine_and_oracle
    engs = []
    for always in (True, False):
        e = run_engine_and_oracle(n=700, f_in=24, classes=5, steps=1, tau=5, dropout=0.5, seed=31,
                                  theta_uniform=1.0, long_rows=True)["engine"]
        e.set_band_shards(BandShards(e.n, world=1, rank=0, always=always))
        assert e.shards.always == always
        for _ in range(2):
            e.run_window(5)
        e.sync_theta()
        engs.append(e)
    torch.cuda.synchronize()
    a, b = engs
    nbw = (a.n + 63) // 64
    return bool(torch.equal(a.theta, b.theta) and torch.equal(a.gbatch.bits[..., :nbw], b.gbatch.bits[..., :nbw])
                and torch.equal(a.gbatch.s, b.gbatch.s)
                and all(torch.equal(v, b.get_params()[k]) for k, v in a.get_params().items()))


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    t0 = time.time()
    dist.init_process_group("nccl", device_id=dev)
    from ldsgnn import _native as nat
    from ldsgnn.replicas import allreduce_mean_always, collective_capture_probe, exchange_capturable
    out = {"backend": dist.get_backend(), "world": dist.get_world_size(), "init_s": time.time() - t0,
           "capturable": exchange_capturable(), "probe": collective_capture_probe(dev)}

    def noop(model):
        return None

    engines = {"noop": trainers(noop), "eager": trainers(allreduce_mean_always),
               "capture": trainers(allreduce_mean_always)}
    census = {}
    real_seal = nat.seal_graph

    def seal(graph, what, exchange=False):  # record what the captures hold
        census[what] = nat.graph_census(graph)
        return real_seal(graph, what, exchange=exchange)

    nat.seal_graph = seal
    try:
        for name, eng in engines.items():
            eng.inner_step()
            eng.hyper_step()  # step 0 (its own window)
            if name == "capture":
                eng.capture_window(5, windows=2, prefetch=True)
            else:
                eng.capture_window(5, prefetch=True, capture_exchange=False)
    finally:
        nat.seal_graph = real_seal
    out["census"] = census
    out["capture_is_one_graph"] = engines["capture"]._graph_capture[2] is None
    same = []
    for w in range(WINDOWS):
        for eng in engines.values():
            eng.replay(1)
        torch.cuda.synchronize()
        ref = engines["noop"]
        row = {}
        for name in ("eager", "capture"):
            e = engines[name]
            row[name] = bool(torch.equal(e.theta, ref.theta) and torch.equal(e.grad, ref.grad) and
                             all(torch.equal(v, ref.get_params()[k]) for k, v in e.get_params().items()) and
                             e.scalars_host() == ref.scalars_host())
        same.append(row)
    out["bit_identical_per_window"] = same
    out["theta_moved"] = bool(not torch.equal(engines["noop"].theta, trainers(noop).theta))
    # replays of two windows per graph: the same as two single replays
    eng = engines["capture"]
    eng.replay(2)
    for name in ("noop", "eager"):
        engines[name].replay(1)
        engines[name].replay(1)
    torch.cuda.synchronize()
    out["group_replay_identical"] = bool(torch.equal(eng.theta, engines["noop"].theta) and
                                         torch.equal(eng.theta, engines["eager"].theta))
    out["band_sharded_rccl_identical"] = band_sharded_rccl()
    dist.destroy_process_group()
    line = json.dumps(out)
    print(line)
    if os.path.isdir(os.path.join(ROOT, "gpurun_out")):
        with open(os.path.join(ROOT, "gpurun_out", "rccl_ws1.json"), "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
