"""Benchmark: LDS inner-loop steps/s on Cora-sized LDS (BASELINE.json metric).

Workload (BASELINE.json configs[1]): Cora-shaped LDS bilevel, kNN-initialised
θ (k=10, cosine, symmetrised), 1 sampled graph per inner step, hidden 16,
dropout 0.5, Adam 0.01 / wd 5e-4, hyper step every τ=5 inner steps (SGD
lr 0.1, decay 0.99), fp32.  Early stopping disabled: W untimed warm-up inner
steps, then exactly K timed inner steps with their hyper steps inside the
timed region.  Synthetic data of Cora's shape (no network).

N>1 (torchrun, one process per GPU): every rank runs its own Monte-Carlo
replica (keyed RNG stream = rank) and the ranks all-reduce θ.grad once per
hyper step over RCCL — per-GPU work fixed ("weak"); value = inner steps of all
ranks / max-over-ranks wall time.

Also reported: `roofline` of the dominant kernel (HIP-event average launch
time over a second, instrumented pass of the same K steps) and
`cpu_baseline` — the CPU oracle (dense PyTorch restatement of the reference)
timed on this host over a bounded sample (rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "lds-gnn_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0     # MI355X HBM3E peak (MI355X_MICROARCH.md)
FP32_PEAK_TFLOPS = 157.3  # MI355X fp32 vector/MFMA peak
BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 MFMA peak (no sparsity)
INT8_PEAK_TOPS = 5000.0    # dense int8 MFMA: 2x the bf16 rate (MI355X_MICROARCH.md, I8 row)


def build(args, rank, device):
    import ldsgnn
    from ldsgnn.data.synthetic import knn_init, make_dataset
    from ldsgnn.models.gcn import MetaDenseGCN
    from ldsgnn.models.graph import BernoulliGraphModel
    from ldsgnn.replicas import allreduce_mean
    from ldsgnn.trainers.bilevel import BilevelProblemRunner
    from ldsgnn.trainers.inner import InnerProblemTrainer
    from ldsgnn.trainers.outer import OuterProblemTrainer
    from ldsgnn.utils.graph import split_mask

    data = make_dataset(args.dataset, seed=args.seed)
    if args.dataset == "synthetic20k":  # config 5: dense θ_ij ~ U(0, 1) i.i.d. (seed 20000), no kNN graph
        g = torch.Generator(device=device).manual_seed(20000)
        data.dense_adj = torch.rand((data.num_nodes, data.num_nodes), generator=g, device=device)
    else:
        data = knn_init(data, k=10)
    np.random.seed(args.seed)
    data.val_mask, opt_mask = split_mask(data.val_mask, 0.5, shuffle=True)
    data = data.to(device)
    opt_mask = opt_mask.to(device)
    ldsgnn.rng.manual_seed(args.seed, replica=rank * args.samples)  # rank r: replicas r·S .. r·S+S-1
    torch.manual_seed(args.seed)
    gcn = MetaDenseGCN(data.num_features, 16, data.num_classes, dropout=0.5).to(device)
    inner = InnerProblemTrainer(gcn, data, lr=0.01, weight_decay=5e-4)
    if args.graph_model == "lds":
        gm = BernoulliGraphModel(data.dense_adj)
        opt = torch.optim.SGD(gm.parameters(), lr=0.1)
    else:  # the embedding / GAE models: drop-in trainers only
        from ldsgnn.models.factory import GraphGenerativeModelFactory
        fac = GraphGenerativeModelFactory(data)
        gm = fac.create(args.graph_model)
        opt = fac.optimizer(gm)
    outer = OuterProblemTrainer(opt, data, opt_mask, gm, lr_decay=0.99, grad_reducer=allreduce_mean)
    return data, BilevelProblemRunner(inner, outer, data), opt_mask


def make_engine(runner, tau, world, samples=1):
    import ldsgnn
    from ldsgnn.fused import engine_from_trainers
    eng = engine_from_trainers(runner.inner_trainer, runner.outer_trainer, tau=tau,
                               generator=ldsgnn.rng.default_generator, samples=samples)
    reducer = None
    if world > 1:
        def reducer(grad):
            dist.all_reduce(grad, op=dist.ReduceOp.SUM)
            grad.div_(world)
    return eng, reducer


def run_engine_windows(eng, reducer, windows, tau, use_graph):
    """`windows` τ-windows (τ inner steps + hyper step each)."""
    if use_graph:
        eng.replay(windows)
        return
    for _ in range(windows):
        eng.run_window(tau, grad_reducer=reducer)


def run_steps(runner, start: int, count: int, tau: int) -> int:
    step = start
    for _ in range(count):
        runner.inner_opt_step()
        if tau == 0 or step % tau == 0:
            runner.hyper_opt_step(step)
        step += 1
    return step


# entry point -> HIP kernel symbol (for the PMC traffic record)
KERNEL_SYMBOL = {"lds_theta_grad_ex": "lds::theta_grad_mfma_kernel", "lds_theta_grad_sgd": "lds::theta_grad_mfma_kernel", "lds_theta_grad": "lds::theta_grad_mfma_kernel",
                 "lds_theta_grad_sgd_accum": "lds::theta_grad_mfma_kernel", "lds_spmm_norm": "lds::spmm_norm_group_kernel",
                 "lds_sample_bitmask": "lds::sample_tiles_kernel"}
PMC_RECORD = os.path.join(ROOT, "profiles", "r01_pmc_traffic.json")


def pmc_traffic(kernel, use_engine, world, args):
    """HBM bytes per launch of the roofline kernel from the committed rocprofv3
    PMC record (tools/gpu_pmc.sh + tools/pmc_summary.py: 2 x FETCH_SIZE +
    WRITE_SIZE, separate passes, gfx950 read correction), measured on this
    default workload (Cora-shaped, S = 1, τ = 5); None for any other."""
    default = args.dataset == "cora" and args.samples == 1 and args.tau == 5
    if not (default and use_engine and world == 1 and kernel == "lds_theta_grad_sgd") or \
            not os.path.exists(PMC_RECORD):
        return None, None
    with open(PMC_RECORD) as f:
        recs = json.load(f)
    if "theta_grad" in kernel:  # whichever θ-grad kernel the form in force launched (one per record)
        names = [k for k in recs if "theta_grad" in k]
        rec = recs[names[0]] if len(names) == 1 else None
    else:
        rec = recs.get(KERNEL_SYMBOL[kernel])
    if rec is None:
        return None, None
    return rec["traffic_bytes"], os.path.relpath(PMC_RECORD, ROOT)


def cpu_baseline(args, data, opt_mask):
    """The oracle (dense CPU restatement of the reference) on a bounded sample:
    `cpu_steps` inner steps incl. their τ-hyper steps, host threads."""
    from oracle import lds_oracle as O
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    cpu = data.to("cpu")
    theta = O.get_triu_values(cpu.dense_adj)
    prob = O.LdsProblem(cpu.x, cpu.y, cpu.train_mask, cpu.val_mask, cpu.test_mask, opt_mask.cpu(), theta,
                        hidden=16, dropout_p=0.5, gcn_lr=0.01, gcn_wd=5e-4, outer_lr=0.1, lr_decay=0.99,
                        rnd=O.Randomness(args.seed, 0), init_generator=torch.Generator().manual_seed(args.seed))
    prob.run_steps(1, args.tau)  # warm-up (allocations, first hyper step)
    t0 = time.perf_counter()
    prob.run_steps(args.cpu_steps, args.tau)
    dt = time.perf_counter() - t0
    return {"value": args.cpu_steps / dt, "unit": "steps/s", "cores": threads, "kind": "port",
            "sample": f"{args.cpu_steps} inner steps incl. hyper steps every tau={args.tau} "
                      f"(oracle/lds_oracle.py, dense torch-CPU fp32, {threads} threads), "
                      f"{dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--tau", type=int, default=5)
    ap.add_argument("--dataset", default="cora")
    ap.add_argument("--seed", type=int, default=597905255 % (2 ** 31))
    ap.add_argument("--cpu-steps", type=int, default=11)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--theta-form", default=None, help="θ-grad assembly form (ldsgnn.ops.THETA_GRAD_FORMS; "
                    "default: bf16x3, the split-bf16 MFMA form picked by shape)")
    ap.add_argument("--kernel", default="auto", help="entry point for the roofline leg (auto: the θ-grad "
                    "assembly the path uses)")
    ap.add_argument("--split", action="store_true", help="engine: per-graph dθ chunks on a side stream beside "
                    "the reverse pass instead of one assembly launch per window (measured slower on MI355X)")
    ap.add_argument("--samples", type=int, default=1, help="Monte-Carlo replica samples per GPU, batched in "
                    "every launch (BASELINE configs 3/4); value is then sample-steps/s")
    ap.add_argument("--eager", action="store_true", help="engine: launch windows eagerly (no HIP graph)")
    ap.add_argument("--backend", default="nccl", help="process group backend for N>1 (nccl = RCCL; gloo only "
                    "for rehearsing several ranks on one device)")
    ap.add_argument("--graph-model", default="lds", choices=["lds", "embedding", "gae"],
                    help="graph generative model (embedding / gae: P from node embeddings, autograd path)")
    ap.add_argument("--path", default="engine", choices=["engine", "autograd"],
                    help="engine: fused HIP engine (HIP-graph replayed tau-windows); autograd: drop-in trainers")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dev_index = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(args.backend)

    import ldsgnn
    from ldsgnn import _native as nat
    if args.theta_form is not None:
        from ldsgnn import ops as ldsops
        ldsops.theta_grad_form(args.theta_form)

    data, runner, opt_mask = build(args, rank, device)
    n = data.num_nodes

    def barrier_sync():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    use_engine = args.path == "engine"
    # embedding / GAE on the engine: θ = P(model parameters), the outer step
    # (autograd through P + the model's optimizer) runs eagerly between the
    # two replayed graphs of a window, where N>1 runs the all-reduce
    param_theta = args.graph_model != "lds"
    if param_theta and use_engine and (world > 1 or args.samples > 1):
        raise SystemExit("--graph-model embedding/gae on the engine: one GPU, one sample")
    if args.kernel == "auto":
        if use_engine and param_theta:
            args.kernel = "lds_theta_grad"
        elif use_engine and args.samples > 1:
            args.kernel = "lds_theta_grad_ex"
        elif use_engine and world == 1:
            args.kernel = "lds_theta_grad_sgd_accum" if args.split else "lds_theta_grad_sgd"
        else:
            args.kernel = "lds_theta_grad"
    if use_engine:
        assert args.steps % args.tau == 0 and args.warmup % args.tau == 0, "steps, warmup: multiples of tau"
        eng, reducer = make_engine(runner, args.tau, world, args.samples)
        eng.split_theta_grad = args.split
        # step 0 is its own window (hyper step at step 0, src/trainers/bilevel.py:70-71)
        eng.inner_step()
        eng.hyper_step(grad_reducer=reducer)
        if param_theta:  # the model's outer step runs eagerly between graph A and graph B
            reducer = eng.outer_update
        use_graph = not args.eager
        if use_graph:  # N>1: split at the all-reduce (graph A, RCCL, graph B)
            eng.capture_window(args.tau, grad_reducer=reducer)
        run_engine_windows(eng, reducer, args.warmup // args.tau, args.tau, use_graph)
    else:
        step = run_steps(runner, 0, args.warmup, args.tau)
    barrier_sync()
    t0 = time.perf_counter()
    if use_engine:
        run_engine_windows(eng, reducer, args.steps // args.tau, args.tau, use_graph)
    else:
        step = run_steps(runner, step, args.steps, args.tau)
    barrier_sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    value = world * args.samples * args.steps / elapsed
    in_sync = None
    if world > 1:  # replicas must hold bit-identical θ after every update
        th = eng.theta if use_engine else runner.outer_trainer.model.probs.data
        mine = torch.tensor([th.double().sum().item(), th.double().square().sum().item()], dtype=torch.float64)
        allv = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allv, mine.to(device) if args.backend == "nccl" else mine)
        in_sync = all(torch.equal(v.cpu(), allv[0].cpu()) for v in allv)

    # roofline leg: the same K steps again with HIP events around the kernel
    nat.timer.enable(args.kernel)
    if use_engine:
        run_engine_windows(eng, reducer, args.steps // args.tau, args.tau, False)
    else:
        step = run_steps(runner, step, args.steps, args.tau)
    ksum = nat.timer.summary()[args.kernel]
    nat.timer.disable()
    if use_engine:
        nnz = eng.sampled_nnz()
    else:
        g = runner.outer_trainer.model.sample()  # a representative graph for byte counts
        nnz = g.nnz()
    tri = n * (n + 1) // 2
    if args.kernel in ("lds_spmm_norm", "lds_spmm_norm_blocked"):
        f = 16
        algo = 4 * (n + 1) + 4 * nnz + 4 * n + 8 * n * f
        achieved = algo / (ksum["avg_us"] * 1e-6) / 1e9
        roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": None}
    elif args.kernel == "lds_aggregate_bitmask":  # int8 MFMA: 4 limbs x 2 ops per (row, column, feature)
        rows, cols = -(-n // 256) * 256, -(-n // 512) * 512
        ops = 2.0 * rows * cols * 16 * 4
        achieved = ops / (ksum["avg_us"] * 1e-6) / 1e12
        roof = {"bound": "mfma", "achieved": achieved, "peak": INT8_PEAK_TOPS, "unit": "TOP/s",
                "frac": achieved / INT8_PEAK_TOPS, "traffic": None,
                "hbm_algorithmic_GBs": (8 * n * nat.lib.lds_bitmask_words(n) + 4 * n + 8 * n * 16)
                / (ksum["avg_us"] * 1e-6) / 1e9}
    elif args.kernel == "lds_sample_bitmask":
        words = nat.lib.lds_bitmask_words(n)
        algo = 4 * tri + 8 * n * words
        achieved = algo / (ksum["avg_us"] * 1e-6) / 1e9
        roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": None}
    else:  # lds_theta_grad[_sgd]: rank-2k update of the packed triangle
        from ldsgnn.engine import LdsEngine
        if use_engine and args.kernel == "lds_theta_grad_ex":  # S factor blocks of ldk columns
            k = eng.S * eng.ldk
        elif use_engine and args.kernel in ("lds_theta_grad_sgd", "lds_theta_grad"):  # one launch per window
            k = LdsEngine.window_columns(args.tau, data.num_classes)
        elif use_engine:  # split assembly: the timed launch is one graph's chunk (+ R, SGD)
            k = LdsEngine.window_columns(1, data.num_classes) - LdsEngine.window_columns(0, data.num_classes)
        else:  # one launch per graph: 4 uses (16 + 8 + 8 + 16 columns)
            k = 16 + 8 + 8 + 16
        flops = 4.0 * k * tri
        fp32_equiv = flops / (ksum["avg_us"] * 1e-6) / 1e12
        from ldsgnn import ops as ldsops
        form = ldsops.theta_grad_form()
        if form == "fp32":
            roof = {"bound": "mfma", "achieved": fp32_equiv, "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": fp32_equiv / FP32_PEAK_TFLOPS, "traffic": None}
        else:  # split-bf16: six bf16 MFMA products per fp32 product, priced against the bf16 dense peak
            achieved = 6.0 * fp32_equiv
            roof = {"bound": "mfma", "achieved": achieved, "peak": BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": achieved / BF16_PEAK_TFLOPS, "traffic": None}
        roof.update(form=form, fp32_equiv_tflops=fp32_equiv)
    roof.update(kernel=args.kernel, avg_us=ksum["avg_us"], launches=ksum["launches"])
    roof["traffic"], roof["traffic_source"] = pmc_traffic(args.kernel, use_engine, world, args)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, data, opt_mask)

    if rank == 0:
        out = {
            "metric": "inner-loop GCN steps/sec on Cora-sized LDS at 1/2/4/8 MI355X",
            "value": value, "unit": "steps/s" if args.samples == 1 else "sample-steps/s", "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1000.0 * elapsed / args.steps,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
            "data": f"synthetic {args.dataset}-shaped (N={n}, F_in={data.num_features}, "
                    f"C={data.num_classes}), " + ("theta ~ U(0,1)" if args.dataset == "synthetic20k"
                                                  else "kNN-initialised theta"),
            "config": {"workload": f"{args.dataset}-lds-" + ("uniform" if args.dataset == "synthetic20k" else
                                                               "knn-init") + f"-S{args.samples}-tau{args.tau}", "path": args.path, "nodes": n,
                       "features": data.num_features, "classes": data.num_classes, "hidden": 16,
                       "tau": args.tau, "samples_per_rank": args.samples, "parallelism": f"replicas{world}",
                       "sampled_nnz": nnz, "replicas_in_sync": in_sync, "graph_model": args.graph_model,
                       "aggregation": (("bitmask x fixed-point s*Z on int8 MFMA (pre-pass)" if eng.bitmask_agg
                                        else "column-blocked LDS SpMM pre-pass")
                                       if use_engine and eng.long_rows else "in-kernel CSR")},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
