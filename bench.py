#!/usr/bin/env python3
"""Benchmark: spectra/s of SIMCA fit + Q/T² score (BASELINE.json metric).

One step = the full SIMCA hot path on the synthetic 1M×2048 fp32 spectra in
HBM, k = 20, type 'alt', t2lim 'Fdist', qlim 'jm' (the driver defaults,
simca_nuts.py:186): outlier-screened int8-digit quantiser + shifted Gram on
integer MFMA (i8×3) → covariance → top-20 eigenpairs + θ1..θ3 → fit-set
scoring (T, T², Q, moments) → limits → predict (fused decision) on the same
rows.  At N = 1 the step is the drop-in itself, ``utils.SIMCA(...).fit(X, y)``
then ``.predict(X)`` on the device tensors; at N > 1 it is
``ocm.dist.ShardedSIMCA`` on each rank's rows with ONE RCCL all-reduce of the
packed moments (and a scalar one for the θ3 trace slices).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--rows R]
                    [--scaling strong|weak] [--dist-backend nccl|gloo]
                    [--no-cpu] [--no-vae] [--no-cv] [--no-weak]

Multi-GPU: ``--gpus N`` with N > 1 and no ``WORLD_SIZE`` in the environment
starts N rank processes itself (a ``torch.distributed.run`` child; this
parent never touches the GPU) and exits with its status; launched under
torch.distributed.run (the driver's form) it runs as one rank.  Scaling is
STRONG by default: R = 1M rows in total, split into contiguous row blocks
(the global matrix does not depend on N: ocm/synth.py), value = R / the
max-over-ranks step time.  At N > 1 the line also carries the weak-scaling
run (R rows per GPU) under ``weak``.  ``cv`` is C3: class-wise 10-fold CV
(the fold engine, ocm/cv.py) of 1M×2048 spectra (10 % other class) sharded
the same way.  ``phases_ms`` is each rank's per-phase time (HIP events on
the launch stream) from extra, untimed steps.

Prints ONE JSON line (rank 0).  The `roofline` object is for the dominant
kernel, k_gram8e: algorithmic FLOP per launch = this rank's rows × p(p+1)
(symmetric Gram) ÷ its mean duration, timed live with HIP events around every
launch in the timed region.  `cpu_baseline` times the oracle's
reference-precision path (float32 full SVD + randomized PCA(k) + NumPy
scoring) on a bounded row sample on this host (N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
# before HIP initialises: the VAE's HIP-graph step needs the runtime's graph
# packet capture off (ocm/__init__.py explains the race)
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
sys.path.insert(0, os.path.join(REPO, "ocm-vae-simca_amd"))
sys.path.insert(0, REPO)

FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: Peak FP32 (matrix)
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: Peak BF16 MFMA, dense
I8_MFMA_PEAK_TOPS = 5000.0      # MI355X_MICROARCH.md: I8 MFMA = 2x BF16 per clock (dense)
GRAM_MODE_DEFAULT = "i8x3"
METRIC = "spectra/sec SIMCA fit+Q/T² score at 1M×2048"
DATA_SEED = 4321


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--rows", type=int, default=1_000_000,
                    help="spectra in total (strong scaling) or per GPU (weak scaling)")
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="nccl = RCCL over xGMI (one GPU per rank); gloo lets several ranks share a GPU (tests)")
    ap.add_argument("--p", type=int, default=2048)
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--cpu-sample", type=int, default=131072, help="rows for the CPU baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-vae", action="store_true", help="skip the secondary VAE train-steps/s measurement")
    ap.add_argument("--vae-steps", type=int, default=200)
    ap.add_argument("--no-cv", action="store_true", help="skip the C3 10-fold CV line")
    ap.add_argument("--no-prep", action="store_true", help="skip the preprocessing + fit + score extra line")
    ap.add_argument("--cv-reps", type=int, default=3)
    ap.add_argument("--no-weak", action="store_true", help="N > 1: skip the weak-scaling extra run")
    ap.add_argument("--phase-steps", type=int, default=3, help="untimed steps with per-phase events (0 = off)")
    ap.add_argument("--gram-mode", default=GRAM_MODE_DEFAULT, choices=["f32", "bf16x3", "i8x3", "i8x3k32"],
                    help="Gram kernel: int8 digit split (default), bf16x3 split or FP32 MFMA")
    return ap.parse_args(argv)


def launch(args) -> int:
    """Start ``args.gpus`` rank processes (torch.distributed.run child) and
    return its exit status.  Nothing here initialises HIP."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=dict(os.environ))


def synth_device(n, p, k, seed, device):
    """Synthetic spectra generated in HBM (ocm/synth.py): rank-40
    Gaussian-band loadings, scores with a gap at k, σ-noise, sloped baseline;
    rows [0, n) of the matrix of ``seed`` (the same matrix the N-rank bench
    shards)."""
    from ocm.synth import spectra_shard

    return spectra_shard(n, p, 0, 1, device, seed=seed, k=k)


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(rows, p, k, repeats=3):
    """Oracle at reference precision (float32 full SVD + randomized PCA(k) +
    NumPy scoring, the reference's solver sequence) on a bounded sample:
    one warm-up on a small sample, then the median of ``repeats`` timed
    fit + predict runs (SURVEY.md §8d protocol)."""
    import numpy as np

    from oracle import simca_oracle as O

    try:
        from threadpoolctl import threadpool_info

        threads = max([i.get("num_threads", 1) for i in threadpool_info() if i.get("user_api") == "blas"] or [1])
    except Exception:
        threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))

    def run(m):
        X = O.synth_spectra(m, p, k, rank=40, seed=1234)
        y = np.zeros(m, dtype=np.int64)
        est = O.OracleSIMCA(n_components=k, model_class=0, precision="reference", predict_loadings="randomized")
        t0 = time.perf_counter()
        est.fit(X, y, rng=np.random.RandomState(0))
        est.predict(X)
        return time.perf_counter() - t0

    run(min(rows, 16384))  # warm-up (BLAS threads, page faults)
    times = sorted(run(rows) for _ in range(repeats))
    dt = times[len(times) // 2]
    return {"value": round(rows / dt, 1), "unit": "spectra/s", "cores": int(threads), "kind": "port",
            "host_cpus": os.cpu_count(), "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "cores_note": ("BLAS threads used = the box's CPU share for one GPU (OMP_NUM_THREADS, set by the pool); "
                           "host_cpus is the whole machine's count"),
            "cpu_model": _cpu_model(), "protocol": f"1 warm-up + median of {repeats}",
            "runs_s": [round(t, 3) for t in times],
            "sample": f"{rows}x{p} fp32, k={k}, alt/Fdist/jm: float32 full SVD + randomized PCA(k) + "
                      f"NumPy scores, fit+predict on the same rows (median {dt:.2f} s)"}


def vae_bench(device, steps, warmup, batch=512, length=2048, dtype=None, latent_rows=1_000_000):
    """Secondary metric (BASELINE.json): VAE-SIMCA train steps/s, C4 network
    (cb=3, nf=3, ks=7, hid=64, d=32) at B=512 × L=2048 in bf16,
    one HIP-graph replay per optimizer step (ocm/vae_train.py).  Every timed
    step takes a distinct batch of a (warmup + steps) × B synthetic set in
    HBM.  Then SIMCA-on-latents, timed on its own (utils/final_vaesimca.py:
    406-442, 500-533) at C4's scale (1M × 2048): encode +
    decode ``latent_rows`` synthetic spectra of the same distribution (eval,
    no grad), latent statistics and the f-distance decision on libocm."""
    import torch

    import vae_model as V
    from ocm import engine
    from ocm.vae import full_distance_decision, latent_stats
    from ocm.vae_train import GraphedVAETrainer

    nb = warmup + steps
    X = synth_device(batch * nb, length, 20, seed=99, device=device)
    mean = X.mean(0).cpu().numpy()
    std = X.std(0).cpu().numpy() + 1e-6
    torch.manual_seed(0)
    m = V.ConvVAE1D(length, 32, mean, std, conv_blocks=3, n_filters=3, kernel_size=7, hidden_fc=64).to(device)
    if dtype is None:
        dtype = torch.float32 if os.environ.get("OCM_VAE_DTYPE") == "f32" else torch.bfloat16
    tr = GraphedVAETrainer(m, batch, lr=1e-3, dtype=dtype)
    for i in range(warmup):
        tr.step(X[i * batch:(i + 1) * batch])
    first = float(tr.out[0].item())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(warmup, nb):
        tr.step(X[i * batch:(i + 1) * batch])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    loss = float(tr.out[0].item())
    finite = all(bool(torch.isfinite(p).all()) for p in m.parameters())

    # SIMCA-on-latents over C4's 1M rows (a fresh synthetic set of the
    # training distribution; the 107k training rows are a tenth of it)
    m.eval()
    if latent_rows:
        del X
        X = synth_device(latent_rows, length, 20, seed=7, device=device)
    n = X.shape[0]
    eb = 8192
    ac = torch.autocast("cuda", dtype=torch.bfloat16, enabled=dtype == torch.bfloat16)

    mus = torch.empty((n, 32), dtype=torch.float32, device=device)
    q = torch.empty(n, dtype=torch.float32, device=device)

    def encode(starts):
        with torch.no_grad(), ac:
            for a in starts:
                xb = X[a:min(n, a + eb)]
                mu, _ = m.encode((xb - m.spec_mean) / m.spec_std)
                xr = m.decode(mu).float() * m.spec_std + m.spec_mean
                mus[a:a + xb.shape[0]] = mu.float()
                q[a:a + xb.shape[0]] = engine.rowsq_residual(xb, xr.contiguous())

    starts = list(range(0, n, eb))
    encode(sorted({starts[0], starts[-1]}))  # kernel selection for both batch shapes (MIOpen find)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    encode(starts)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    lmean, _, t2lim, qlim = latent_stats(mus, q)
    accept, _, fcrit = full_distance_decision(mus, lmean, q)
    acc = float(accept.to(torch.float64).sum().item())
    t3 = time.perf_counter()
    m.train()
    return {"metric": "VAE-SIMCA train steps/sec", "value": round(steps / dt, 2), "unit": "steps/s",
            "ms_per_step": round(dt / steps * 1e3, 4), "steps": steps,
            "dtype": "f32" if dtype == torch.float32 else "bf16",
            "config": {"workload": f"ConvVAE1D cb=3 nf=3 ks=7 hid=64 d=32, B={batch}, L={length}, "
                                   f"BCE-with-logits + KL, Adam, HIP-graph step, {nb} distinct batches",
                       "params": sum(p.numel() for p in m.parameters())},
            "reference_cpu_steps_per_s": 2.5, "loss_after_warmup": round(first, 5), "final_loss": round(loss, 5),
            "params_finite": finite,
            "latents": {"rows": n, "encode_rows_per_s": round(n / (t2 - t1), 1),
                        "encode_s": round(t2 - t1, 4), "stats_decision_s": round(t3 - t2, 4),
                        "t2_limit": float(t2lim), "q_limit": float(qlim), "f_crit": float(fcrit),
                        "accept_rate": round(acc / n, 4)}}


class Ranks:
    """This process's place in the job and the few collectives the bench needs."""

    def __init__(self, args):
        import torch
        import torch.distributed as dist

        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        if self.world != args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={self.world}: launch N ranks with "
                             "torch.distributed.run --nproc-per-node N, or plain `python bench.py --gpus N`")
        self.backend = args.dist_backend
        ndev = torch.cuda.device_count()
        if self.backend == "nccl" and self.world > 1 and self.local >= ndev:
            raise SystemExit(f"bench.py: rank {self.local} has no GPU ({ndev} visible); RCCL needs one GPU per "
                             "rank (use --dist-backend gloo to share one)")
        self.device = torch.device("cuda", self.local % max(ndev, 1))
        torch.cuda.set_device(self.device)
        self.dist = dist
        if self.world > 1:
            if self.backend == "nccl":
                dist.init_process_group("nccl", device_id=self.device)
            else:
                dist.init_process_group("gloo")
            assert dist.get_world_size() == self.world

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def max(self, x: float) -> float:
        import torch

        if self.world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=self.device if self.backend == "nccl" else "cpu")
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def gather(self, obj):
        if self.world == 1:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out


def _timed(rk, step, steps, warmup):
    """W untimed steps, then K steps bracketed by barrier + device sync;
    seconds = max over ranks."""
    import torch

    for _ in range(warmup):
        step()
    rk.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    rk.barrier()
    return rk.max(time.perf_counter() - t0)


def run_simca(args, rk, n_total):
    """The SIMCA fit + score step on this rank's rows of an n_total-row matrix."""
    import torch

    from ocm import _lib, engine
    from ocm.dist import ShardedSIMCA
    from ocm.phases import PhaseTimer
    from ocm.synth import shard_bounds, spectra_shard
    from utils import SIMCA

    p, k = args.p, args.k
    lo, hi = shard_bounds(n_total, rk.rank, rk.world)
    n = hi - lo
    X = spectra_shard(n_total, p, rk.rank, rk.world, rk.device, seed=DATA_SEED, k=k)
    y = torch.zeros(n, dtype=torch.int64, device=rk.device)
    pred = torch.empty(n, dtype=torch.float64, device=rk.device)
    torch.cuda.synchronize()
    result = {}

    def step():
        if rk.world == 1:  # the drop-in estimator on device tensors
            model = SIMCA(n_components=k, model_class=0, type="alt", t2lim="Fdist", qlim="jm", verbose=False)
            model.fit(X, y)
            result["pred"] = model.predict(X)
            info = model._model[0]
            result.update(fit=model._fits[0], T2_limit=info["T2_limit"], Q_limit=info["Q_limit"])
        else:
            model = ShardedSIMCA(n_components=k, type="alt", t2lim="Fdist", qlim="jm").fit(X)
            result["pred"] = model.predict(X, out=pred)
            result.update(fit=model.fit_, T2_limit=model.T2_limit, Q_limit=model.Q_limit)

    for _ in range(args.warmup):
        step()
    ctx = _lib.Context.get(rk.device.index)
    for kid in range(3):
        ctx.read_timing(kid)
    ctx.set_timing(True)
    dt = _timed(rk, step, args.steps, 0)
    ctx.set_timing(False)
    timing = {name: ctx.read_timing(kid) for kid, name in enumerate(("gram", "score", "quant"))}

    phases = None
    if args.phase_steps > 0:
        timer = PhaseTimer(rk.device)
        engine.set_phase_timer(timer)
        try:
            for _ in range(args.phase_steps):
                step()
                timer.mark("predict_score")
            phases = timer.summary(args.phase_steps)
        finally:
            engine.set_phase_timer(None)
    accepted = float(result["pred"].sum().item())
    out = {"n_local": n, "seconds": dt, "timing": timing, "phases": phases, "accepted": accepted,
           "eig_iters": result["fit"].eig_iters, "T2_limit": result["T2_limit"], "Q_limit": result["Q_limit"],
           "marks": engine.last_gram_marks(rk.device.index)}
    del X, y, pred, result
    torch.cuda.empty_cache()
    return out


def run_prep(args, rk, n_total):
    """the drivers' preprocessing before SIMCA, three ways,
    on the same raw rows: the eager pass (``snv_savgol``: X′ written to HBM)
    then fit + predict on X′; the no-copy lazy view (``lazy=True``: the
    transform runs in the Gram quantiser's and the scoring kernel's load paths,
    X′ never exists); and the write-through view (``lazy="write"``: the
    quantiser writes X′ as it forms it, the scoring reads X′).  Settings: simca_nuts.py:47-52 (SNV, w 5, p 2, deriv 1) and
    simca_new_cheese.py:37-39 (w 15, p 2, deriv 1, no SNV)."""
    import torch

    from ocm import _lib, preprocess
    from ocm.prepview import materialised_count
    from ocm.synth import shard_bounds, spectra_shard
    from utils import SIMCA

    p, k = args.p, args.k
    lo, hi = shard_bounds(n_total, rk.rank, rk.world)
    X = spectra_shard(n_total, p, rk.rank, rk.world, rk.device, seed=DATA_SEED, k=k)
    y = torch.zeros(hi - lo, dtype=torch.int64, device=rk.device)
    ctx = _lib.Context.get(rk.device.index)
    out = {"metric": "spectra/s, preprocessing + SIMCA fit + predict", "rows": n_total, "p": p, "k": k}
    for name, (snv, w) in {"nuts_snv_sg5_d1": (True, 5), "cheese_sg15_d1": (False, 15)}.items():
        res = {}
        for mode in ("materialised", "fused", "fused_write"):
            last = {}

            def step():
                lazy = {"materialised": False, "fused": True, "fused_write": "write"}[mode]
                Xp = preprocess.snv_savgol(X, w, 2, 1, 1.0, snv=snv, lazy=lazy)
                model = SIMCA(n_components=k, model_class=0, type="alt", t2lim="Fdist", qlim="jm", verbose=False)
                model.fit(Xp, y)
                last["fit"] = model._fits[0]
                return model.predict(Xp)

            step()
            c0 = materialised_count(rk.device.index)
            for kid in range(3):
                ctx.read_timing(kid)
            ctx.set_timing(True)
            dt = _timed(rk, step, args.steps, 0)
            ctx.set_timing(False)
            t = {nm: ctx.read_timing(kid) for kid, nm in enumerate(("gram", "score", "quant"))}
            res[mode] = {"ms_per_step": round(dt / args.steps * 1e3, 3),
                         "value": round(n_total * args.steps / dt, 1),
                         "quantise_ms": round(t["quant"][0] / max(t["quant"][1], 1), 4),
                         "score_ms": round(t["score"][0] / max(t["score"][1], 1), 4),
                         "gram_ms": round(t["gram"][0] / max(t["gram"][1], 1), 4),
                         "eig_iters": int(last["fit"].eig_iters)}
            if mode != "materialised":
                res[mode]["materialised_views"] = materialised_count(rk.device.index) - c0
        out[name] = res
    del X, y
    torch.cuda.empty_cache()
    return out


def run_cv(args, rk, n_total, folds=10, lv=20):
    """C3: class-wise 10-fold CV (ClasswiseKFoldWithExternalVal(10, cls_label=0),
    utils/CVSIMCA.py:54-80) of n_total spectra, every 10th row another class
    (a shifted band), with the fold engine (ocm/cv.py: one Gram pass with fold
    segments, downdated fold Grams reduced to their owner rank, one eigensolve
    per fold, every rank scoring its own rows).  Seconds per CV run."""
    import numpy as np
    import torch
    from sklearn.model_selection import KFold

    import ocm.cv as fe
    from ocm.synth import shard_bounds, spectra_shard
    from utils import SIMCA

    p = args.p
    lo, hi = shard_bounds(n_total, rk.rank, rk.world)
    y = np.zeros(n_total, dtype=np.int64)
    y[9::10] = 1
    X = spectra_shard(n_total, p, rk.rank, rk.world, rk.device, seed=DATA_SEED + 1, k=lv)
    wl = torch.linspace(0, 1, p, device=rk.device)
    band = (3.0 * torch.exp(-0.5 * ((wl - 0.5) / 0.03) ** 2)).float()
    other = torch.from_numpy(np.flatnonzero(y[lo:hi] == 1)).to(rk.device)
    X[other] += band
    cls_idx = np.flatnonzero(y == 0)
    fold_rows = [cls_idx[te] for _, te in KFold(n_splits=folds).split(cls_idx)]
    base = SIMCA(verbose=False).get_params()
    res = {}

    def once():
        res["recs"], _ = fe.cv_grid(X, y, fold_rows, cls_idx, [lv], [{}], base, [0], False, row_offset=lo)

    dt = _timed(rk, once, max(1, args.cv_reps), 1) / max(1, args.cv_reps)
    r = res["recs"][0]
    del X
    torch.cuda.empty_cache()
    return {"metric": f"CVSIMCA {folds}-fold wall time at {n_total}x{p} (fold engine, LV {lv})",
            "value": round(dt, 5), "unit": "s per CV run", "higher_is_better": False,
            "spectra_per_s": round(n_total / dt, 1), "reps": args.cv_reps, "rows_local": hi - lo,
            "spec": r["spec"], "sens": r["sens"],
            "reference_cpu_s": {"100k": 129.2, "1M_extrapolated": 1440}}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(args))  # this process never initialises HIP
    rk = Ranks(args)
    from ocm import engine

    engine.set_gram_mode(args.gram_mode)
    p, k = args.p, args.k
    n_total = args.rows if args.scaling == "strong" else args.rows * rk.world
    head = run_simca(args, rk, n_total)
    n = head["n_local"]
    dt = head["seconds"]
    ms_per_step = dt / args.steps * 1e3
    value = n_total * args.steps / dt

    gram_ms, gram_n = head["timing"]["gram"]
    score_ms, score_n = head["timing"]["score"]
    quant_ms, quant_n = head["timing"]["quant"]
    gram_avg_s = gram_ms / max(gram_n, 1) / 1e3
    gram_flop = n * p * (p + 1)  # symmetric Gram of this rank's rows, algorithmic
    achieved = gram_flop / gram_avg_s / 1e12 if gram_avg_s > 0 else 0.0
    score_avg_s = score_ms / max(score_n, 1) / 1e3
    score_gbs = n * p * 4 / score_avg_s / 1e9 if score_avg_s > 0 else 0.0

    gram_kernel = {"bf16x3": "k_gram3", "i8x3": "k_gram8e", "i8x3k32": "k_gram8d"}.get(args.gram_mode, "k_gram")
    if args.gram_mode in ("i8x3", "i8x3k32"):
        # fp32-grade product from 6 int8 MFMA digit products (exact int32 sums)
        mfma = "v_mfma_i32_16x16x64_i8" if args.gram_mode == "i8x3" else "v_mfma_i32_32x32x32_i8"
        gram_desc = (f"{gram_kernel} (shifted Gram, 3 int8 digits per value, 6 {mfma} digit products per fp32 "
                     "product, exact int32 sums)")
        gram_peak = round(I8_MFMA_PEAK_TOPS / 6, 1)
        peak_basis = "int8 MFMA dense peak / 6 (fp32-equivalent); achieved counts algorithmic fp32 flops n*p*(p+1)"
    elif args.gram_mode == "bf16x3":
        gram_desc = "k_gram3 (shifted Gram, exact 3-level bf16 split, 6 bf16 MFMA products per fp32 product)"
        gram_peak = round(BF16_MFMA_PEAK_TFLOPS / 6, 1)
        peak_basis = "bf16 MFMA dense peak / 6 (fp32-equivalent); achieved counts algorithmic fp32 flops n*p*(p+1)"
    else:
        gram_desc = "k_gram (FP32 MFMA shifted Gram)"
        gram_peak = FP32_MFMA_PEAK_TFLOPS
        peak_basis = "FP32 MFMA dense peak; achieved counts algorithmic flops n*p*(p+1) (symmetric Gram)"
    # HBM bytes per launch from this round's PMC passes (scripts/pmc_passes.sh →
    # scripts/pmc_latest.py → profiles/pmc_gram_latest.json; FETCH_SIZE doubled)
    traffic, traffic_src, score_traffic, score_src = None, None, None, None
    pmc = os.path.join(REPO, "profiles", "pmc_gram_latest.json")
    if os.path.exists(pmc) and n == 1_000_000:
        try:
            lat = json.load(open(pmc))
            traffic = lat.get(gram_kernel, {}).get("hbm_bytes_per_launch")
            traffic_src = lat.get(gram_kernel, {}).get("source")
            score_traffic = lat.get("k_score_1p", {}).get("hbm_bytes_per_launch")
            score_src = lat.get("k_score_1p", {}).get("source")
        except Exception:
            traffic = None

    par = ("single GPU" if rk.world == 1 else
           f"row shards x{rk.world} ({rk.backend}: one all-reduce of packed moments + θ3 partials)")
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "spectra/s",
        "n_gpus": rk.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (rank-40 band spectra + noise, generated in HBM)",
        "config": {
            "workload": f"SIMCA fit+score, synthetic {n_total}x{p} fp32 in total, k={k}, type=alt t2lim=Fdist qlim=jm",
            "step": ("utils.SIMCA(...).fit(X, y) + .predict(X), device tensors (drop-in)" if rk.world == 1 else
                     "ocm.dist.ShardedSIMCA fit (T kept) + predict per rank"),
            "rows_total": n_total, "rows_per_gpu": n, "p": p, "k": k,
            "parallelism": par, "dist_backend": rk.backend if rk.world > 1 else None,
        },
        "roofline": {
            "kernel": gram_desc,
            "bound": "mfma",
            "achieved": round(achieved, 2),
            "peak": gram_peak,
            "unit": "TFLOP/s",
            "frac": round(achieved / gram_peak, 4),
            "peak_basis": peak_basis,
            "traffic": traffic,
            "traffic_source": traffic_src,
            "flop_per_launch": gram_flop,
            "quantise_ms": round(quant_ms / max(quant_n, 1), 4) if quant_n else None,
            "avg_launch_ms": round(gram_avg_s * 1e3, 4),
            "launches": gram_n,
        },
        "score_kernel": {"kernel": "k_score_1p (fused projection/Q/T2/decision, one HBM pass; row tile kept in registers)", "bound": "hbm",
                         "achieved_GBs": round(score_gbs, 1), "peak_GBs": HBM_PEAK_GBS,
                         "frac": round(score_gbs / HBM_PEAK_GBS, 4), "avg_launch_ms": round(score_avg_s * 1e3, 4),
                         "launches": score_n, "bytes_per_launch": n * p * 4, "traffic": score_traffic,
                         "traffic_source": score_src},
        "checks": {"accept_rate": round(head["accepted"] / max(n, 1), 4),
                   "eig_iters": head["eig_iters"], "T2_limit": head["T2_limit"], "Q_limit": head["Q_limit"],
                   "gram_guard_marks": head["marks"]},
    }
    phases = rk.gather(head["phases"])
    if head["phases"] is not None and rk.rank == 0:
        out["phases_ms"] = {f"rank{r}": ph for r, ph in enumerate(phases)}
    if rk.world > 1 and args.scaling == "strong" and not args.no_weak:
        weak = run_simca(args, rk, args.rows * rk.world)
        out["weak"] = {"scaling": "weak", "rows_per_gpu": weak["n_local"], "rows_total": args.rows * rk.world,
                       "value": round(args.rows * rk.world * args.steps / weak["seconds"], 1), "unit": "spectra/s",
                       "ms_per_step": round(weak["seconds"] / args.steps * 1e3, 3)}
    if rk.world == 1 and not args.no_prep:
        try:
            out["prep_fit_score"] = run_prep(args, rk, args.rows)
        except Exception as e:  # report, never fail the primary number
            out["prep_fit_score"] = {"error": repr(e)}
    if not args.no_cv:
        try:
            out["cv"] = run_cv(args, rk, args.rows if args.scaling == "strong" else args.rows * rk.world)
        except Exception as e:  # report, never fail the primary number
            out["cv"] = {"error": repr(e)}
    if rk.rank == 0 and rk.world == 1 and not args.no_cpu:
        try:
            out["cpu_baseline"] = cpu_baseline(args.cpu_sample, p, k)
        except Exception as e:  # report, never fail the GPU number
            out["cpu_baseline"] = {"error": repr(e)}
    if rk.world == 1 and not args.no_vae:
        try:
            out["vae"] = vae_bench(rk.device, args.vae_steps, 10)
        except Exception as e:  # report, never fail the primary number
            out["vae"] = {"error": repr(e)}
    if rk.rank == 0:
        print(json.dumps(out), flush=True)
    if rk.world > 1:
        rk.dist.destroy_process_group()


if __name__ == "__main__":
    main()
