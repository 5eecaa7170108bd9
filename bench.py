"""Benchmark: LDS inner-loop steps/s on Cora-sized LDS (BASELINE.json metric).

Workload (BASELINE.json configs[1], the default): the real Cora Planetoid split
(NormalizeFeatures), θ₀ = the symmetrised cosine kNN graph (k = 10) from the
reference's own sklearn call, committed as tests/golden/knn_cora.npz so every
machine samples the same workload; 1 sampled graph per inner step, hidden 16,
dropout 0.5, Adam 0.01 / wd 5e-4, hyper step every τ = 5 inner steps (SGD lr
0.1, decay 0.99), fp32 (the θ-grad assembly in split bf16, fp32-accurate:
DESIGN §4c).  Early stopping disabled: W untimed warm-up inner steps, then
exactly K timed inner steps with their hyper steps inside the timed region
(SURVEY §8(d)); the fused engine replays captured τ-windows.

N > 1 (torchrun, one process per GPU): every rank runs S Monte-Carlo replicas
(keyed RNG streams rank·S … rank·S+S−1) and the ranks all-reduce θ.grad
(mean) once per hyper step over RCCL — per-GPU work fixed ("weak"); value =
inner steps of all ranks ÷ max-over-ranks wall time.  The line also carries
`strong_scaling` (BASELINE config 4): S_total = 64 samples split over the
ranks, timed against rank 0 running all 64 alone on its GPU first.

Also reported:
  * `window`: per-entry-point GPU time of one τ-window: every C-ABI call of
    one window replayed as a dependent chain of itself from a HIP graph (HIP
    events on the launch stream), with algorithmic bytes / flops and rates;
  * `roofline`: the entry point with the most GPU time per window, against
    its bound (HBM for the memory kernels, MFMA for the θ-grad assembly);
  * `cpu_baseline`: the CPU oracle (dense PyTorch restatement of the
    reference) on this host over a bounded sample (rank 0, N = 1 only).

`--model gcn` (BASELINE config 1): fixed-adjacency GCN training epochs/s on
the real Cora graph (src/scripts/gcn.py:75-91: train step + evaluate).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
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
ELL_W = 64              # ELL head width, neighbours per row (csrc/common.hpp kEllWidth)
FP32_PEAK_TFLOPS = 157.3  # MI355X fp32 vector/MFMA peak
BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 MFMA peak (no sparsity)
INT8_PEAK_TOPS = 5000.0    # dense int8 MFMA: 2x the bf16 rate (MI355X_MICROARCH.md, I8 row)
METRIC = "inner-loop GCN steps/sec on Cora-sized LDS at 1/2/4/8 MI355X"
# committed rocprofv3 PMC records (2 x FETCH_SIZE + WRITE_SIZE per launch, separate passes) by workload
PMC_RECORDS = {"cora-lds-S1-tau5": os.path.join(ROOT, "profiles", "r06b_pmc_traffic.json"),
               "synthetic20k-lds-S1-tau5": os.path.join(ROOT, "profiles", "r06b_pmc_traffic_config5.json")}


def world_info():
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def build(args, rank, device, samples=None, exchange=None):
    """The drop-in trainers of the workload (src/scripts/bilevel.py:74-99).
    exchange: give the outer trainer the all-reduce reducer (default: when a
    process group of more than one rank is up); False for a run on this rank
    alone inside a multi-rank job (the strong-scaling leg's T1)."""
    import ldsgnn
    from ldsgnn.data.workloads import load_workload
    from ldsgnn.models.gcn import MetaDenseGCN
    from ldsgnn.models.graph import BernoulliGraphModel
    from ldsgnn.replicas import allreduce_mean
    from ldsgnn.trainers.bilevel import BilevelProblemRunner
    from ldsgnn.trainers.inner import InnerProblemTrainer
    from ldsgnn.trainers.outer import OuterProblemTrainer
    from ldsgnn.utils.graph import split_mask

    S = args.samples if samples is None else samples
    data = load_workload(args.dataset, seed=args.seed, device=device)
    np.random.seed(args.seed)
    data.val_mask, opt_mask = split_mask(data.val_mask.cpu(), 0.5, shuffle=True)
    data = data.to(device)
    opt_mask = opt_mask.to(device)
    ldsgnn.rng.manual_seed(args.seed, replica=rank * S)  # rank r: replicas r·S .. r·S+S-1
    torch.manual_seed(args.seed)
    gcn = MetaDenseGCN(data.num_features, 16, data.num_classes, dropout=0.5).to(device)
    inner = InnerProblemTrainer(gcn, data, lr=0.01, weight_decay=5e-4)
    if args.graph_model == "lds":
        gm = BernoulliGraphModel(data.dense_adj)
        opt = torch.optim.SGD(gm.parameters(), lr=0.1)
    else:  # the embedding / GAE models
        from ldsgnn.models.factory import GraphGenerativeModelFactory
        fac = GraphGenerativeModelFactory(data)
        fac.gae_config = dict(fac.gae_config, dropout=args.gae_dropout)
        gm = fac.create(args.graph_model)
        opt = fac.optimizer(gm)
    multi = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    if exchange is not None:
        multi = multi and bool(exchange)
    outer = OuterProblemTrainer(opt, data, opt_mask, gm, lr_decay=0.99,
                                grad_reducer=allreduce_mean if multi else None)
    return data, BilevelProblemRunner(inner, outer, data), opt_mask


def make_engine(runner, tau, world, samples=1):
    """Fused engine over the trainers; with world > 1 the exchange is the
    trainer's reducer (all-reduce mean of θ.grad over RCCL), set on the engine
    by engine_from_trainers."""
    import ldsgnn
    from ldsgnn.fused import engine_from_trainers
    eng = engine_from_trainers(runner.inner_trainer, runner.outer_trainer, tau=tau,
                               generator=ldsgnn.rng.default_generator, samples=samples)
    return eng, eng.grad_reducer if world > 1 else None


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


# ---------------------------------------------------------------------------
# algorithmic bytes / flops per launch
# ---------------------------------------------------------------------------

def algo_cost(name, eng, n_calls_per_window):
    """(bound, algorithmic bytes or flops of ONE launch) of an engine entry
    point: every array the launch must touch, counted once."""
    from ldsgnn import _native as nat
    n, S = eng.n, eng.S
    nnz = eng.sampled_nnz_mean()
    xnnz = int(eng.xcol.numel())
    act = 4 * 16 * n * S                      # one n × 16 fp32 activation array (all samples)
    if eng.bitmask_agg:  # long rows, bitmask aggregation: the kernels read s and Â·Z's split partials, no CSR
        graph = S * (4 * n + 4 * 16 * n * eng.agg_splits)
    elif eng.long_rows:  # long rows, column-blocked pre-pass: s and Â·Z
        graph = S * (4 * n + 4 * 16 * n)
    else:
        graph = S * (4 * (n + 1) + 4 * nnz + 4 * n + 8 * ELL_W * n)  # row_ptr, col, s, ELL head
    tri = n * (n + 1) // 2
    P = eng.np
    words = nat.lib.lds_bitmask_words(n)
    if name in ("lds_theta_grad_sgd", "lds_theta_grad", "lds_theta_grad_ex", "lds_theta_grad_sgd_draw",
                "lds_theta_grad_direct"):
        # (_draw: the next window's graph draw rides in the epilogue; priced on the θ-grad's flops)
        k = eng.S * eng.ldk if eng.S > 1 else eng.window_columns(eng.tau, eng.c)
        return "mfma", 6.0 * 4.0 * k * tri   # split bf16: six bf16 MFMA products per fp32 product
    if name == "lds_sample_graphs_multi":
        g = eng.tau + 1
        if eng.bitmask_agg:  # bits written, read by the popcount pass, degrees and s written
            return "hbm", 4 * tri + g * S * (2 * 8 * n * words + 8 * n)
        per = S * (3 * 8 * n * words + 4 * (n + 1) + 4 * nnz + 4 * n + 8 * ELL_W * n)  # bits w/r/r, CSR, s, ELL
        return "hbm", 4 * tri + g * per      # θ read once per window
    if name == "lds_sample_fill_csr":  # the fill alone: bits read, CSR / s / ELL written
        g = eng.tau + 1
        if eng.bitmask_agg:  # col = NULL: s from the drawn degree counts only
            return "hbm", g * S * 8 * n
        return "hbm", g * S * (8 * n * words + 4 * n + 4 * (n + 1) + 4 * nnz + 4 * n + 8 * ELL_W * n)
    if name == "lds_engine_x_linear":
        return "hbm", S * (4 * (n + 1) + 8 * xnnz + 8 * xnnz) + 4 * 16 * eng.fin + act
    if name == "lds_engine_fill_x_linear":  # the window fill and the first X product in one launch
        g = eng.tau + 1
        return "hbm", (g * S * (8 * n * words + 4 * n + 4 * (n + 1) + 4 * nnz + 4 * n + 8 * ELL_W * n)
                       + S * (4 * (n + 1) + 8 * xnnz + 8 * xnnz) + 4 * 16 * eng.fin + act)
    if name == "lds_aggregate_bitmask_partials":
        chunks = (n + 511) // 512
        return "mfma_i8", 2.0 * n * chunks * 512 * 16 * 4
    if name == "lds_engine_xt_adam":
        return "hbm", S * (4 * (eng.fin + 1) + 8 * xnnz) + act + S * 28 * P + 4 * eng.nred * 304 * S
    if name in ("lds_engine_fwd_layer1", "lds_engine_rev_a", "lds_engine_rev_c"):
        return "hbm", graph + 5 * act
    if name in ("lds_engine_fwd2_bwd2", "lds_engine_rev_bc"):  # two hops over one graph read
        return "hbm", graph + 7 * act
    if name in ("lds_engine_fwd_layer2", "lds_engine_bwd_layer2", "lds_engine_rev_b"):
        return "hbm", graph + 4 * act
    if name in ("lds_engine_bwd1_reduce", "lds_engine_rev_d_reduce"):
        return "hbm", graph + 7 * act + 4 * eng.nred * 304 * S
    if name in ("lds_engine_sgd_clamp",):
        return "hbm", 12 * tri
    if name == "lds_engine_end_window":
        return "hbm", S * 24 * P
    if name == "lds_aggregate_bitmask":  # int8 MFMA: 0/1 mask x 4 base-256 digits of s*Z, 16 features
        chunks = (n + 511) // 512
        return "mfma_i8", 2.0 * n * chunks * 512 * 16 * 4
    if name == "lds_spmm_norm_blocked":
        return "hbm", 4 * (n + 1) + 4 * nnz + 4 * n + 8 * ELL_W * n
    if name == "lds_engine_xt_partials":
        return "hbm", 8 * xnnz + act
    return "hbm", 0


def theta_grad_hbm_bytes(name, eng):
    """Algorithmic HBM bytes of one θ-grad launch of the window (beside its
    MFMA flops): θ read and written, dθ written (when kept), the factor
    columns read once (U, V fp32; the direct form's planes are 3 × bf16), and,
    for the drawing forms, the next window's bit graphs written."""
    from ldsgnn import _native as nat
    n = eng.n
    tri = n * (n + 1) // 2
    k = eng.S * eng.ldk if eng.S > 1 else eng.window_columns(eng.tau, eng.c)
    fac = 2 * n * k * (6 if name == "lds_theta_grad_direct" else 4)
    out = 8 * tri + (4 * tri if eng.keep_grad else 0) + fac
    if name in ("lds_theta_grad_sgd_draw", "lds_theta_grad_direct") and eng.prefetch_draw:
        out += eng.gbatch.count * eng.S * 8 * n * nat.lib.lds_bitmask_words(n)
    return out


def bitagg_hbm_bytes(n):
    """Algorithmic HBM bytes of one lds_aggregate_bitmask call (csrc/bitagg.hip):
    the mask, s and Z once, the int8 digits written once and read once (the
    row groups' re-reads of them are tiling, served from L2 / MALL), the split
    partials written and read once (none with one split), Y written."""
    from ldsgnn import _native as nat
    words = nat.lib.lds_bitmask_words(n)
    chunks, groups = (n + 511) // 512, (n + 255) // 256
    splits = max(1, min(chunks, 512 // groups))
    part = 2 * splits * 64 * n if splits > 1 else 0
    return 8 * n * words + 4 * n + 64 * n + 2 * chunks * 32768 + part + 64 * n


def pmc_traffic(name, args):
    """HBM bytes per launch of an entry point from the committed rocprofv3 PMC
    record of THIS workload (tools/gpu.sh pmc / pmc5 + tools/pmc_summary.py:
    2 x FETCH_SIZE + WRITE_SIZE in separate passes, gfx950 read correction)."""
    path = PMC_RECORDS.get(f"{args.dataset}-lds-S{args.samples}-tau{args.tau}")
    if args.model != "lds" or path is None or not os.path.exists(path):
        return None, None
    with open(path) as f:
        recs = json.load(f)
    rec = recs.get(name)
    if rec is None:
        return None, None
    return rec["traffic_bytes"], os.path.relpath(path, ROOT)


def chain_us(fn, dev, k, reps=3):
    """µs per launch of `fn` (one C-ABI call) as a dependent chain of k copies
    captured in one HIP graph, timed with HIP events recorded on the stream
    the graph is replayed on (the stream the kernels run on)."""
    from ldsgnn import _native as nat
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(k):
                fn(nat.stream_of(dev))
        g.replay()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(reps):
            g.replay()
        b.record(s)
    b.synchronize()
    torch.cuda.current_stream(dev).wait_stream(s)
    return 1000.0 * a.elapsed_time(b) / (reps * k)


def _window_state(eng):
    """The device tensors one τ-window reads before it writes them (and
    changes): the scalars (counters, error word), θ, the prefetched graphs'
    bits and degree counts, the window-start weights / Adam state and the Adam
    table.  Everything else a window reads it wrote itself first."""
    ts = [eng.scalars, eng.theta, eng.gbatch.bits, eng.gbatch.deg, eng.w[0], eng.m[0], eng.v[0], eng.adam_tab]
    if eng._deg_next is not None:
        ts.append(eng._deg_next)
    return ts


def window_breakdown(eng, reducer, args, device, k=20, reps=10, rounds=5):
    """Where one τ-window's GPU time goes.  The C-ABI calls of one eager
    window are recorded.  Two measurements per entry point:

      * in-window (the table's us_per_window / avg_us): HIP graphs of the
        window's first j calls, j = 0 … all, each preceded by the same
        restore of the window-start state (kernel copies: θ, the prefetched
        bits and degree counts, scalars, the window-start weights), are
        replayed (HIP events on the replay stream, median of `rounds` rounds
        of `reps` replays); call j's cost is T(j) − T(j − 1): its own duration
        plus the dependent-launch gap it pays in the real sequence, on the
        window's real state.  The entries sum to the replayed window.
      * isolated (chain_avg_us): the call replayed as a dependent chain of k
        copies of itself from one HIP graph (round 2-4's method; a call whose
        inputs its own copies disturb — e.g. the fill of prefetched graphs —
        reads differently there).

    Per entry point: launches and µs per window, the average launch, its
    algorithmic cost and rate.  Runs after every timed leg: the replays
    re-apply θ / Adam updates, so the engine's state is not used afterwards."""
    from ldsgnn import _native as nat
    calls = []
    real = nat.call

    def rec(name, *a):
        # with the window's degree counts as this call found them (the chain
        # leg: a chain of a drawing launch accumulates into them k times over)
        calls.append((name, a, eng.gbatch.deg.clone()))
        real(name, *a)

    state = [t.clone() for t in _window_state(eng)]
    nat.call = rec
    try:
        run_engine_windows(eng, reducer, 1, args.tau, False)
    finally:
        nat.call = real
    torch.cuda.synchronize()
    live = _window_state(eng)

    def restore():  # kernel copies (x · 1 is exact for every dtype here): no memcpy node in the graphs
        for dst, src in zip(live, state):
            torch.mul(src, 1, out=dst)

    cur = torch.cuda.current_stream(device)

    def prefix_graph(j):
        g = torch.cuda.CUDAGraph()
        st = torch.cuda.Stream(device=device)
        st.wait_stream(cur)
        with torch.cuda.stream(st):
            with torch.cuda.graph(g, stream=st):
                restore()
                for name, a, _ in calls[:j]:
                    real(name, *(a[:-1] + (nat.stream_of(device),)))
        cur.wait_stream(st)
        return g

    graphs = [prefix_graph(j) for j in range(len(calls) + 1)]
    st = torch.cuda.Stream(device=device)
    samples = [[] for _ in graphs]
    for _ in range(rounds):
        for j, g in enumerate(graphs):
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                g.replay()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                for _ in range(reps):
                    g.replay()
                b.record(st)
            b.synchronize()
            samples[j].append(1000.0 * a.elapsed_time(b) / reps)
    t = [float(np.median(x)) for x in samples]
    restore()
    torch.cuda.synchronize()
    inwin = {}
    for j, (name, _, _) in enumerate(calls):
        inwin.setdefault(name, []).append(t[j + 1] - t[j])
    chain = {}
    for name, a, deg in calls:
        if name == "lds_sample_graphs_multi":  # repeated draws clear their own workspace (ws_zeroed = 0)
            a = a[:-3] + (0,) + a[-2:]
        eng.gbatch.deg.copy_(deg)
        us = chain_us(lambda s_, name=name, a=a: real(name, *(a[:-1] + (s_,))), device, k)
        chain.setdefault(name, []).append(us)
    rows = []
    for name, ts in inwin.items():
        calls_w = len(ts)
        avg = sum(ts) / calls_w
        bound, cost = algo_cost(name, eng, calls_w)
        row = {"entry": name, "launches_per_window": calls_w, "us_per_window": sum(ts), "avg_us": avg,
               "chain_avg_us": sum(chain[name]) / len(chain[name]), "bound": bound}
        if cost:
            if bound == "mfma_i8":
                row["algorithmic_int8_ops"] = cost
                row["achieved_tops"] = cost / (avg * 1e-6) / 1e12
                row["algorithmic_bytes"] = bitagg_hbm_bytes(eng.n)
                row["achieved_GBs"] = row["algorithmic_bytes"] / (avg * 1e-6) / 1e9
            elif bound == "mfma":
                row["algorithmic_flop"] = cost
                row["achieved_tflops"] = cost / (avg * 1e-6) / 1e12
                row["algorithmic_bytes"] = theta_grad_hbm_bytes(name, eng)
                row["achieved_GBs"] = row["algorithmic_bytes"] / (avg * 1e-6) / 1e9
            else:
                row["algorithmic_bytes"] = cost
                row["achieved_GBs"] = cost / (avg * 1e-6) / 1e9
        # HBM bytes per launch from the committed rocprofv3 PMC record of this
        # workload (FETCH_SIZE + WRITE_SIZE, profiles/r04_pmc_traffic*.json)
        tr, _src = pmc_traffic(name, args)
        if tr:
            row["pmc_traffic_bytes"] = tr
            row["pmc_GBs"] = tr / (avg * 1e-6) / 1e9
        rows.append(row)
    rows.sort(key=lambda r: -r["us_per_window"])
    return rows, len(calls), {"restore_us": t[0], "window_us": t[-1] - t[0]}


def roofline_of(row, args):
    """The roofline entry of the window's dominant kernel.  Its duration is the
    call's time as a dependent chain of copies in one HIP graph (HIP events on
    the launch stream: the kernel plus the graph's launch gap, the figure a
    rocprofv3 --kernel-trace --stats average of the same launch matches); the
    in-window marginal cost, which also carries the wait for the previous
    launch's writes, is kept beside it (in_window_us)."""
    us = row["chain_avg_us"]
    scale = row["avg_us"] / us  # in-window rates -> chain rates
    row = dict(row)
    for key in ("achieved_tops", "achieved_tflops", "achieved_GBs"):
        if key in row:
            row[key] = row[key] * scale
    if row["bound"] == "mfma_i8":  # the config-5 bitmask aggregation: int8 MFMA, HBM fraction alongside
        achieved = row["achieved_tops"]
        roof = {"bound": "mfma", "achieved": achieved, "peak": INT8_PEAK_TOPS, "unit": "TOP/s (int8)",
                "frac": achieved / INT8_PEAK_TOPS, "hbm_GBs": row["achieved_GBs"],
                "hbm_frac": row["achieved_GBs"] / HBM_PEAK_GBS}
    elif row["bound"] == "mfma":
        achieved = row["achieved_tflops"]
        from ldsgnn import ops as ldsops
        roof = {"bound": "mfma", "achieved": achieved, "peak": BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": achieved / BF16_PEAK_TFLOPS, "form": ldsops.theta_grad_form(),
                "fp32_equiv_tflops": achieved / 6.0, "hbm_GBs": row.get("achieved_GBs"),
                "hbm_frac": row["achieved_GBs"] / HBM_PEAK_GBS if "achieved_GBs" in row else None}
    else:
        achieved = row.get("achieved_GBs", 0.0)
        roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS}
    roof.update(kernel=row["entry"], avg_us=us, in_window_us=row["avg_us"],
                launches_per_window=row["launches_per_window"], share_of_window=None)
    if row["entry"] in ("lds_theta_grad_sgd_draw", "lds_theta_grad_direct"):  # priced on the assembly's flops alone
        roof["includes"] = "the next window's graph draw (tau+1 graphs, Philox VALU) in the epilogue"
    if row["entry"] == "lds_theta_grad_direct":
        roof["form"] = "bf16x3-direct (form 10: pre-split planes staged by direct global->LDS loads)"
    roof["traffic"], roof["traffic_source"] = pmc_traffic(row["entry"], args)
    return roof


def host_info():
    model = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    # the GPU box's share of its host is 16 cores (OMP_NUM_THREADS there);
    # nproc / os.cpu_count() report the whole machine
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(avail, cap) if cap > 0 else avail
    return model, threads, avail


def cpu_baseline(args, data, opt_mask):
    """The oracle (dense CPU restatement of the reference) on a bounded sample:
    `cpu_steps` inner steps incl. their τ-hyper steps, all host threads this
    process may use."""
    from oracle import lds_oracle as O
    model, threads, avail = host_info()
    torch.set_num_threads(threads)
    cpu = data.to("cpu")
    theta = O.get_triu_values(cpu.dense_adj)
    prob = O.LdsProblem(cpu.x, cpu.y, cpu.train_mask, cpu.val_mask, cpu.test_mask, opt_mask.cpu(), theta,
                        hidden=16, dropout_p=0.5, gcn_lr=0.01, gcn_wd=5e-4, outer_lr=0.1, lr_decay=0.99,
                        rnd=O.Randomness(args.seed, 0), init_generator=torch.Generator().manual_seed(args.seed))
    n = cpu.x.size(0)
    big = n > 8000  # config 5: one dense N x N normalisation is ~10^13 flop on the CPU
    steps, tau = (max(1, min(args.cpu_steps, 2)), 1) if big else (args.cpu_steps, args.tau)
    if not big:
        prob.run_steps(1, tau)  # warm-up (allocations, first hyper step)
    t0 = time.perf_counter()
    prob.run_steps(steps, tau)
    dt = time.perf_counter() - t0
    what = (f"{steps} inner steps, each with a hyper step (tau=1: the bounded config-5 sample of SURVEY "
            f"8(d); the GPU line runs tau={args.tau})" if big else
            f"{steps} inner steps incl. hyper steps every tau={tau}")
    unit = "steps/s"
    if args.samples > 1:  # one replica chain: the S chains of a step are independent (S x the work)
        unit = "sample-steps/s"
        what += f"; one replica chain of the S={args.samples} (each sample-step is one chain's step)"
    return {"value": steps / dt, "unit": unit, "cores": threads, "kind": "port",
            "cpu_model": model, "cpus_visible": avail,
            "sample": f"{what} (oracle/lds_oracle.py, dense torch-CPU fp32, {threads} threads, n={n}), {dt:.1f} s"}


def cpu_baseline_gcn(args, data, epochs):
    """Config 1 on the CPU: the reference's fixed-graph GCN epoch
    (src/scripts/gcn.py:75-91) as the oracle's dense torch-CPU restatement."""
    from oracle import lds_oracle as O
    model, threads, avail = host_info()
    torch.set_num_threads(threads)
    cpu = data.to("cpu")
    run = O.FixedGcnTraining(cpu.x, cpu.y, cpu.dense_adj, cpu.train_mask, cpu.val_mask, cpu.test_mask,
                             hidden=16, dropout_p=0.5, lr=0.01, wd=5e-4, rnd=O.Randomness(args.seed, 0),
                             init_generator=torch.Generator().manual_seed(args.seed))
    run.epoch()
    t0 = time.perf_counter()
    for _ in range(epochs):
        run.epoch()
    dt = time.perf_counter() - t0
    return {"value": epochs / dt, "unit": "epochs/s", "cores": threads, "kind": "port", "cpu_model": model,
            "cpus_visible": avail,
            "sample": f"{epochs} epochs (train step + evaluate, oracle/lds_oracle.py FixedGcnTraining, dense "
                      f"torch-CPU fp32, {threads} threads), {dt:.1f} s"}


def strong_scaling_leg(args, world, rank, device, barrier_sync):
    """BASELINE config 4: S_total samples per hyper step split over the
    ranks (S_total / world each).  Rank 0 first times S_total alone on its GPU
    (T1), then all ranks time their shards with the all-reduce (TN)."""
    total = args.strong_total
    if total % world:
        raise SystemExit(f"--strong-total {total} must divide by the world size {world}")
    windows = max(1, args.strong_steps // args.tau)

    def timed(S, reducer_world):
        # the single-GPU reference time runs on rank 0 alone: no exchange in
        # its engine (capture_window / hyper_step fall back to the engine's
        # own reducer, which would all-reduce with ranks waiting at a barrier)
        data, runner, _ = build(args, rank, device, samples=S, exchange=reducer_world > 1)
        eng, reducer = make_engine(runner, args.tau, reducer_world, S)
        eng.inner_step()
        eng.hyper_step(grad_reducer=reducer)
        # T1 replays whole groups of windows per graph as the N = 1 line does, and
        # so does TN when the all-reduce is captured into the window graph
        cap = reducer is not None and args.capture_exchange
        eng.capture_window(args.tau, grad_reducer=reducer,
                           windows=args.graph_windows if (reducer is None or cap) else 1,
                           prefetch=not args.no_prefetch_draw,
                           capture_exchange=cap if reducer is not None else None)
        eng.replay(1)
        if reducer_world > 1:
            barrier_sync()
        else:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.replay(windows)
        if reducer_world > 1:
            barrier_sync()
        else:
            torch.cuda.synchronize()
        el = time.perf_counter() - t0
        del eng, runner, data
        torch.cuda.empty_cache()
        return el

    t1 = None
    if rank == 0:  # the single-GPU time of the whole S_total, before the group syncs
        t1 = timed(total, 1)
    if world > 1:
        dist.barrier()
    tn = timed(total // world, world)
    if world > 1:
        t = torch.tensor([tn], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        tn = float(t.item())
    steps = windows * args.tau
    out = {"samples_total": total, "samples_per_rank": total // world, "steps": steps,
           "t1_ms_per_step": None if t1 is None else 1000.0 * t1 / steps,
           "tN_ms_per_step": 1000.0 * tn / steps,
           "value": total * steps / tn, "unit": "sample-steps/s"}
    if t1 is not None:
        out["speedup_vs_1gpu"] = t1 / tn
    return out


def bench_gcn(args, world, rank, device, barrier_sync):
    """BASELINE config 1: fixed-graph GCN epochs/s on the real Cora graph:
    the fused engine (default; ldsgnn.fused.FixedGraphGcn) or, with --path
    autograd, the drop-in API (MetaDenseGCN on a hot-path CSR graph, the
    reference's Adam groups, evaluate() per epoch)."""
    import torch.nn.functional as F
    import ldsgnn
    from ldsgnn.data.workloads import load_workload
    from ldsgnn.models.gcn import MetaDenseGCN
    from ldsgnn.utils.evaluation import evaluate
    data = load_workload("cora-given", device=device)
    ldsgnn.rng.manual_seed(args.seed, replica=rank)
    torch.manual_seed(args.seed)
    gcn = MetaDenseGCN(data.num_features, 16, data.num_classes, dropout=0.5).to(device)
    if args.path == "engine":  # the fused engine: the given graph as a 0/1 θ, no hyper steps
        from ldsgnn.fused import FixedGraphGcn
        run = FixedGraphGcn(gcn, data, lr=0.01, weight_decay=5e-4)

        def epoch():
            tl, ta, vl, va, sl, sa = run.epoch()  # one host read, as the reference's .item()s
            return {"val.loss": vl, "val.accuracy": va, "test.loss": sl, "test.accuracy": sa}
        path = "fused engine (ldsgnn.fused.FixedGraphGcn: train step + evaluate as one HIP graph, one host read per epoch)"
    else:
        opt = torch.optim.Adam([{"params": gcn.layer_in.parameters(), "weight_decay": 5e-4},
                                {"params": gcn.layer_out.parameters()}], lr=0.01)

        def epoch():
            opt.zero_grad()
            gcn.train()
            out = gcn(data.x, data.dense_adj)
            loss = F.nll_loss(out[data.train_mask], data.y[data.train_mask])
            loss.backward()
            opt.step()
            return evaluate(gcn, data)
        path = "drop-in MetaDenseGCN + torch Adam"

    for _ in range(args.warmup):
        epoch()
    barrier_sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        m = epoch()
    barrier_sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_gcn(args, data, args.cpu_gcn_epochs)
    if rank == 0:
        print(json.dumps({
            "metric": "fixed-adjacency GCN training epochs/sec on Cora (BASELINE config 1)",
            "value": world * args.steps / elapsed, "unit": "epochs/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1000.0 * elapsed / args.steps, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
            "data": "real Cora Planetoid split, given graph (tests/golden/planetoid_cora.npz)",
            "config": {"workload": "cora-gcn-fixed-adjacency", "path": path,
                       "val_acc_last_epoch": m["val.accuracy"]},
            "roofline": None, "cpu_baseline": cpu}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--tau", type=int, default=5)
    ap.add_argument("--graph-windows", type=int, default=4,
                    help="τ-windows per captured HIP graph (N=1, engine path): replays run whole groups, "
                         "the remainder one window at a time")
    ap.add_argument("--no-prefetch-draw", action="store_true",
                    help="N=1 engine: each window draws its own graphs (default: the hyper step's θ-grad kernel "
                         "draws the next window's, lds_theta_grad_sgd_draw)")
    ap.add_argument("--model", default="lds", choices=["lds", "gcn"],
                    help="lds: the LDS bilevel hot path (configs 2-5); gcn: config 1, fixed-graph GCN training")
    ap.add_argument("--dataset", default="cora", help="ldsgnn.data.workloads: cora (config 2, default), "
                    "citeseer (config 3), synthetic20k (config 5), cora-synthetic")
    ap.add_argument("--seed", type=int, default=597905255 % (2 ** 31))
    ap.add_argument("--cpu-steps", type=int, default=11)
    ap.add_argument("--cpu-gcn-epochs", type=int, default=40)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--theta-form", default=None, help="θ-grad assembly form (ldsgnn.ops.THETA_GRAD_FORMS; "
                    "default: bf16x3, the split-bf16 MFMA form picked by shape)")
    ap.add_argument("--two-hop-outer", type=int, default=1, choices=[0, 1], help="engine: the outer step's loss layer "
                    "as one two-hop launch (lds_engine_fwd2_bwd2 over the opt rows; 1, the default) or as "
                    "fwd_layer2 + bwd_layer2 (0)")
    ap.add_argument("--fuse-fill", type=int, default=1, choices=[0, 1], help="engine, prefetched draws: the "
                    "window's CSR fill in the first X-product launch (lds_engine_fill_x_linear; 1, the default) or "
                    "as its own launch (0)")
    ap.add_argument("--sgd-draw-split", type=int, default=1, choices=[0, 1], help="engine, exchange path: the "
                    "SGD + next-window draw (lds_sgd_sample_graphs) with the replica samples split over more "
                    "blocks (1, the default) or one block per tile (0)")
    ap.add_argument("--async-draw", action="store_true", help="engine: draw a window's graphs 1..τ on a side "
                    "stream beside inner step 0 (graph 0 on the main stream; without prefetched draws)")
    ap.add_argument("--xt-pair", type=int, default=0, choices=[0, 1, 2], help="engine: W0 products over pairs of "
                    "replica samples (0 by shape, 1 off, 2 on; LdsEngine.set_xt_pair)")
    ap.add_argument("--samples", type=int, default=1, help="Monte-Carlo replica samples per GPU, batched in "
                    "every launch (BASELINE configs 3/4); value is then sample-steps/s")
    ap.add_argument("--strong-total", type=int, default=None, help="config 4 leg: S_total samples split over "
                    "the ranks, against rank 0 alone (default 64 when N > 1, off at N = 1)")
    ap.add_argument("--strong-steps", type=int, default=50)
    ap.add_argument("--exchange", default="auto", choices=["auto", "split", "noop", "noop-captured", "rccl1",
                                                           "sharded", "allreduce"],
                    help="auto: N > 1 captures the RCCL all-reduce into the window graph when every rank's "
                         "capture probe succeeds (ldsgnn.replicas.collective_capture_probe), else splits; split: "
                         "N > 1 with the round-4 two graphs per window around an eager all-reduce; one GPU: "
                         "noop = the N > 1 per-rank path with a no-op reducer (split graphs), noop-captured = "
                         "the same reducer captured into the window graph, rccl1 = a world-size-1 nccl (RCCL) "
                         "group and its real all-reduce captured into the window graph (DESIGN §5b); the long-row "
                         "engine (config 5): auto = sharded at N > 1 (band-sharded replicas: factor all-gather, "
                         "band update, band draws + all-to-all, eager windows; at N = 1 a world-1 rehearsal), "
                         "allreduce = the dense dθ all-reduce (split graphs)")
    ap.add_argument("--keep-theta-grad", type=int, default=0, choices=[0, 1],
                    help="engine, no exchange: 1 writes dθ to θ.grad beside the fused SGD update (the drop-in "
                         "trainer's state after its backward, what FusedBilevelRunner keeps); 0 (default: the "
                         "bench has no θ.grad consumer) consumes it in the update's registers only — the same θ "
                         "bit for bit.  With an exchange dθ is always written (the all-reduce's input)")
    ap.add_argument("--eager", action="store_true", help="engine: launch windows eagerly (no HIP graph)")
    ap.add_argument("--no-breakdown", action="store_true", help="skip the per-launch window breakdown leg")
    ap.add_argument("--backend", default="nccl", help="process group backend for N>1 (nccl = RCCL; gloo only "
                    "for rehearsing several ranks on one device)")
    ap.add_argument("--graph-model", default="lds", choices=["lds", "embedding", "gae"],
                    help="graph generative model (embedding / gae: P from node embeddings)")
    ap.add_argument("--gae-dropout", type=float, default=0.0, help="--graph-model gae: the proposal GCN's "
                    "dropout (factory default 0; > 0 runs per-draw θ on the engine)")
    ap.add_argument("--path", default="engine", choices=["engine", "autograd"],
                    help="engine: fused HIP engine (HIP-graph replayed tau-windows); autograd: drop-in trainers")
    args = ap.parse_args()

    world, rank, local_rank = world_info()
    dev_index = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(args.backend)
    elif args.exchange == "rccl1":  # a world-size-1 RCCL group on this GPU (the collective's launches, N = 1)
        import socket
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                device_id=device)
    if args.strong_total is None:
        args.strong_total = 64 if world > 1 and args.model == "lds" and args.path == "engine" else 0

    def barrier_sync():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    import ldsgnn  # noqa: F401
    from ldsgnn import ops as ldsops
    if args.theta_form is not None:
        ldsops.theta_grad_form(args.theta_form)
    if args.model == "gcn":
        bench_gcn(args, world, rank, device, barrier_sync)
        if world > 1:
            dist.destroy_process_group()
        return

    data, runner, opt_mask = build(args, rank, device)
    n = data.num_nodes
    use_engine = args.path == "engine"
    # embedding / GAE on the engine: θ = P(model parameters), the outer step
    # (autograd through P + the model's optimizer) runs eagerly between the
    # two replayed graphs of a window, where N>1 runs the all-reduce
    param_theta = args.graph_model != "lds"
    if param_theta and use_engine and (world > 1 or args.samples > 1):
        raise SystemExit("--graph-model embedding/gae on the engine: one GPU, one sample")
    eng = reducer = None
    if use_engine:
        assert args.steps % args.tau == 0 and args.warmup % args.tau == 0, "steps, warmup: multiples of tau"
        eng, reducer = make_engine(runner, args.tau, world, args.samples)
        exchange_label = args.exchange if world == 1 else None
        capture_exchange = False
        sharded = eng.long_rows and (args.exchange == "sharded" or (args.exchange == "auto" and world > 1))
        if args.exchange == "sharded" and not eng.long_rows:
            raise SystemExit("--exchange sharded: the long-row engine (config 5) only")
        if sharded:  # band-sharded replicas: the exchange lives inside the hyper step
            from ldsgnn.replicas import BandShards
            eng.grad_reducer = None
            reducer = None
            eng.set_band_shards(BandShards(eng.n))
            args.eager = True  # (two collectives per window around host-sized buffers: not captured)
            exchange_label = f"band-sharded-{args.backend if world > 1 else 'world1'}"
        elif args.exchange in ("noop", "noop-captured", "rccl1"):
            if world > 1:
                raise SystemExit(f"--exchange {args.exchange} rehearses the N > 1 path on one GPU")
            if args.exchange == "rccl1":
                from ldsgnn.replicas import collective_capture_probe, exchange_capturable

                def reducer(grad, prescaled=False):  # the N > 1 all-reduce mean, on the world-size-1 group
                    dist.all_reduce(grad, op=dist.ReduceOp.SUM)
                    if not prescaled:
                        grad.div_(dist.get_world_size())
                reducer.capturable = exchange_capturable
                # as at N > 1 over a power-of-two world (ldsgnn.fused, replicas.mean_prescale):
                # the assembly scales dθ by 1/world, the exchange is the all-reduce SUM alone
                reducer.prescale = lambda: dist.get_world_size()
                capture_exchange = collective_capture_probe(device)
                exchange_label = "nccl-allreduce-ws1-" + ("captured" if capture_exchange else "split")
            else:
                def reducer(grad):  # the exchange point, without the collective
                    return None
                capture_exchange = args.exchange == "noop-captured"
            eng.grad_reducer = reducer
        elif world > 1 and args.exchange == "auto" and args.backend == "nccl":
            from ldsgnn.replicas import collective_capture_probe
            capture_exchange = collective_capture_probe(device)
        if world > 1 and not sharded:
            exchange_label = f"{args.backend}-allreduce-" + ("captured" if capture_exchange else "split")
        args.capture_exchange = capture_exchange  # (the strong-scaling leg's TN captures the same way)
        eng.async_draw = bool(args.async_draw)
        eng.two_hop_outer = bool(args.two_hop_outer)
        eng.sgd_draw_split = bool(args.sgd_draw_split)
        eng.fuse_fill = bool(args.fuse_fill)
        if not args.keep_theta_grad:  # θ.grad not materialised (the fused update consumes dθ)
            eng.keep_grad = False
            runner.outer_trainer.model.probs.grad = None
        if args.xt_pair:
            eng.set_xt_pair(args.xt_pair)
        # step 0 is its own window (hyper step at step 0, src/trainers/bilevel.py:70-71)
        eng.inner_step()
        eng.hyper_step(grad_reducer=reducer)
        if param_theta:  # the model's outer step runs eagerly between graph A and graph B
            reducer = eng.outer_update
        use_graph = not args.eager and eng.theta_fn is None  # per-draw θ (GAE proposal dropout): eager windows
        # N > 1: the all-reduce captured into the window graph (whole groups of
        # windows per replay, as N = 1), or split at it (graph A, RCCL, graph B)
        whole = reducer is None or capture_exchange
        if use_graph:
            eng.capture_window(args.tau, grad_reducer=reducer,
                               windows=args.graph_windows if whole else 1,
                               prefetch=not args.no_prefetch_draw,
                               capture_exchange=capture_exchange if reducer is not None else None)
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
    if use_engine:
        # the timed windows' device error word (a fill whose degree counts and
        # bits disagree, a CSR the SpMM cannot use, ...): raise, never report
        eng.check_device_error()

    # steady state: the same replays over a longer stretch (>= ~0.2 s), reported beside `value`
    steady = None
    if use_engine and use_graph:
        reps = max(args.steps // args.tau, int(0.2 / max(elapsed / max(1, args.steps // args.tau), 1e-6)))
        barrier_sync()
        t1 = time.perf_counter()
        run_engine_windows(eng, reducer, reps, args.tau, True)
        barrier_sync()
        el = time.perf_counter() - t1
        if world > 1:
            t = torch.tensor([el], device=device, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        steady = {"steps": reps * args.tau, "value": world * args.samples * reps * args.tau / el,
                  "ms_per_step": 1000.0 * el / (reps * args.tau)}

    in_sync = None
    if use_engine and eng.shards is not None:
        eng.sync_theta()  # (band-sharded: every rank's band into every copy, then the same check)
    if world > 1:  # replicas must hold bit-identical θ after every update
        th = eng.theta if use_engine else runner.outer_trainer.model.probs.data
        mine = torch.stack([th.double().sum(), th.double().square().sum()])  # on this rank's device
        if args.backend == "nccl":
            allv = [torch.zeros_like(mine) for _ in range(world)]
            dist.all_gather(allv, mine)
        else:
            mine = mine.cpu()
            allv = [torch.zeros_like(mine) for _ in range(world)]
            dist.all_gather(allv, mine)
        in_sync = all(torch.equal(v.cpu(), allv[0].cpu()) for v in allv)

    nnz = eng.sampled_nnz_mean() if use_engine else None
    roof, window = None, None
    if use_engine and not args.no_breakdown and eng.shards is None:
        rows, ncalls, pre = window_breakdown(eng, reducer, args, device)
        total = sum(r["us_per_window"] for r in rows)
        wall_win = 1000.0 * (steady["ms_per_step"] if steady else 1000.0 * elapsed / args.steps) * args.tau
        window = {"method": "in-window marginal cost: HIP graphs of the window's first j calls (after a restore of "
                            "the window-start state) replayed, call j = T(j) - T(j-1), median of 5 x 10 replays; "
                            "chain_avg_us: the call alone as a dependent chain of 20 copies",
                  "launch_calls_per_window": ncalls,
                  "sum_of_launch_us_per_window": total,
                  "prefix_window_us": pre["window_us"], "restore_us": pre["restore_us"],
                  "replayed_window_us": wall_win,
                  "entries": [{k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()}
                              for r in rows]}
        # the dominant kernel: the largest isolated time per window (the
        # call's chain average × its launches per window: the same per-launch
        # time the roofline entry divides by).  The in-window marginal costs
        # rank the window's entries but are too noisy to pick one: on the same
        # code, runs on different boxes gave the ten xt_adam launches 46.7-55.3
        # µs against the θ-grad's 49.0-53.5, while the chain averages held
        # within 2 % (≈45 against ≈51 µs per window)
        per_win = lambda r: r["chain_avg_us"] * r["launches_per_window"]  # noqa: E731
        top = max(rows, key=per_win)
        roof = roofline_of(top, args)
        roof["share_of_window"] = top["us_per_window"] / total if total else None
        roof["selected_by"] = "largest isolated time per window (chain average x launches per window)"
        theta_rows = [r for r in rows if r["bound"] == "mfma"]
        if theta_rows:
            window["theta_grad"] = roofline_of(theta_rows[0], args)
        agg_rows = [r for r in rows if r["bound"] == "mfma_i8"]
        if agg_rows:  # config 5: the bitmask aggregation, the dense-graph form of the north-star SpMM
            window["bitmask_aggregation"] = roofline_of(agg_rows[0], args)
            window["bitmask_aggregation"]["share_of_window"] = agg_rows[0]["us_per_window"] / total

    prefetched = bool(use_engine and eng.prefetch_draw)  # (the strong leg below frees the engine)
    two_hop_outer = bool(use_engine and eng.two_hop_outer)
    form_name = eng._form_name() if use_engine else ldsops.theta_grad_form()
    long_rows = bool(use_engine and eng.long_rows)
    strong = None
    # (config 5's long-row engine runs one replica sample per engine: no S_total split)
    if use_engine and args.strong_total and not param_theta and not long_rows:
        del eng
        torch.cuda.empty_cache()
        strong = strong_scaling_leg(args, world, rank, device, barrier_sync)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, data, opt_mask)

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": value, "unit": "steps/s" if args.samples == 1 else "sample-steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1000.0 * elapsed / args.steps,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
            "data": data.name + f" (N={n}, F_in={data.num_features}, C={data.num_classes})",
            "config": {"workload": f"{args.dataset}-lds-S{args.samples}-tau{args.tau}", "path": args.path,
                       "nodes": n, "features": data.num_features, "classes": data.num_classes, "hidden": 16,
                       "tau": args.tau, "samples_per_rank": args.samples, "parallelism": f"replicas{world}",
                       "theta_grad_form": form_name, "sampled_nnz": nnz,
                       "replicas_in_sync": in_sync, "graph_model": args.graph_model,
                       "windows_per_graph": (args.graph_windows if whole else 1)
                       if use_engine and use_graph else None,
                       "prefetched_draw": prefetched, "async_draw": bool(args.async_draw),
                       "two_hop_outer": two_hop_outer if use_engine else None,
                       "theta_grad_written": bool(args.keep_theta_grad) or reducer is not None
                       if use_engine else True,
                       "xt_pair": args.xt_pair, "exchange": exchange_label if use_engine else None},
            "steady_state": steady,
            "strong_scaling": strong,
            "window": window,
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out))
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
