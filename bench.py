#!/usr/bin/env python3
"""Benchmark: spectra/s of SIMCA fit + Q/T² score (BASELINE.json metric).

One step = the full SIMCA hot path on the synthetic 1M×2048 fp32 batch each
rank holds in HBM, k = 20, type 'alt', t2lim 'Fdist', qlim 'jm' (the driver
defaults, simca_nuts.py:186).  At N = 1 the step is the drop-in itself,
``utils.SIMCA(...).fit(X, y)`` then ``.predict(X)`` on the device tensors; at
N > 1 it is ``ocm.dist.ShardedSIMCA`` on each rank's rows.  Both run:
outlier-screened int8-digit quantiser + shifted Gram on integer MFMA (i8×3)
→ [RCCL all-reduce of Gram/colsum/n when N > 1] → covariance → top-20
eigenpairs + θ1..θ3 → fit-set scoring (T, T², Q, moments) → limits → predict
(fused decision) on the same rows.  value = rows of all ranks / max-over-ranks
step time (weak scaling: rows per GPU fixed).

    python bench.py [--gpus N --steps K --warmup W --rows R --no-cpu]

Prints ONE JSON line (rank 0).  The `roofline` object is for the dominant
kernel, k_gram8d: algorithmic FLOP per launch = rows × p(p+1) (symmetric Gram)
÷ its mean duration, timed live with HIP events around every launch in the
timed region.  `cpu_baseline` times the oracle's reference-precision path
(float32 full SVD + randomized PCA(k) + NumPy scoring) on a bounded row
sample on this host.
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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--rows", type=int, default=1_000_000, help="spectra per GPU")
    ap.add_argument("--p", type=int, default=2048)
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--cpu-sample", type=int, default=131072, help="rows for the CPU baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-vae", action="store_true", help="skip the secondary VAE train-steps/s measurement")
    ap.add_argument("--vae-steps", type=int, default=200)
    ap.add_argument("--gram-mode", default=GRAM_MODE_DEFAULT, choices=["f32", "bf16x3", "i8x3"],
                    help="Gram kernel: int8 digit split (default), bf16x3 split or FP32 MFMA")
    return ap.parse_args()


def synth_device(n, p, k, seed, device, rank_count=40, noise=0.05):
    """Synthetic spectra generated in HBM: rank-40 Gaussian-band
    loadings (shared by all ranks), scores with a gap at k, σ-noise, sloped
    baseline.  Chunked so temporaries stay small."""
    import torch

    g = torch.Generator(device=device).manual_seed(1234)  # loadings: same on every rank
    wl = torch.linspace(0.0, 1.0, p, device=device, dtype=torch.float64)
    centers = torch.rand(rank_count, generator=g, device=device, dtype=torch.float64) * 0.9 + 0.05
    widths = torch.rand(rank_count, generator=g, device=device, dtype=torch.float64) * 0.07 + 0.01
    L = torch.exp(-0.5 * ((wl[None, :] - centers[:, None]) / widths[:, None]) ** 2)
    L = (L / L.norm(dim=1, keepdim=True)).float()
    s = torch.cat([torch.linspace(20, 8, k), torch.linspace(2, 0.5, rank_count - k)]).to(device)
    base = (1.0 + 0.3 * wl).float()
    X = torch.empty((n, p), dtype=torch.float32, device=device)
    gr = torch.Generator(device=device).manual_seed(seed)
    step = 65536
    for a in range(0, n, step):
        b = min(n, a + step)
        S = torch.randn((b - a, rank_count), generator=gr, device=device) * s
        X[a:b] = S @ L + noise * torch.randn((b - a, p), generator=gr, device=device) + base
    return X


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
            "cpu_model": _cpu_model(), "protocol": f"1 warm-up + median of {repeats}",
            "runs_s": [round(t, 3) for t in times],
            "sample": f"{rows}x{p} fp32, k={k}, alt/Fdist/jm: float32 full SVD + randomized PCA(k) + "
                      f"NumPy scores, fit+predict on the same rows (median {dt:.2f} s)"}


def vae_bench(device, steps, warmup, batch=512, length=2048, dtype=None):
    """Secondary metric (BASELINE.json): VAE-SIMCA train steps/s, C4 network
    (cb=3, nf=3, ks=7, hid=64, d=32) at B=512 × L=2048 in bf16,
    one HIP-graph replay per optimizer step (ocm/vae_train.py).  Every timed
    step takes a distinct batch of a (warmup + steps) × B synthetic set in
    HBM.  Then SIMCA-on-latents, timed on its own (utils/final_vaesimca.py:
    406-442, 500-533): encode + decode the training rows (eval, no grad),
    latent statistics and the f-distance decision on libocm."""
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

    # SIMCA-on-latents over every training row
    m.eval()
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


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(device)

    from ocm import _lib, engine
    from ocm.dist import ShardedSIMCA
    from utils import SIMCA

    engine.set_gram_mode(args.gram_mode)
    n, p, k = args.rows, args.p, args.k
    X = synth_device(n, p, k, seed=4321 + rank, device=device)
    y = torch.zeros(n, dtype=torch.int64, device=device)
    pred = torch.empty(n, dtype=torch.float64, device=device)
    torch.cuda.synchronize()
    result = {}

    def step():
        if world == 1:  # the drop-in estimator on device tensors
            model = SIMCA(n_components=k, model_class=0, type="alt", t2lim="Fdist", qlim="jm", verbose=False)
            model.fit(X, y)
            result["pred"] = model.predict(X)
            info = model._model[0]
            result.update(fit=model._fits[0], T2_limit=info["T2_limit"], Q_limit=info["Q_limit"])
        else:
            model = ShardedSIMCA(n_components=k, type="alt", t2lim="Fdist", qlim="jm").fit(X)
            result["pred"] = model.predict(X, out=pred)
            result.update(fit=model.fit_, T2_limit=model.T2_limit, Q_limit=model.Q_limit)
        return model

    for _ in range(args.warmup):
        step()
    ctx = _lib.Context.get(device.index)
    for kid in range(3):
        ctx.read_timing(kid)
    ctx.set_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        model = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    ctx.set_timing(False)
    gram_ms, gram_n = ctx.read_timing(0)
    score_ms, score_n = ctx.read_timing(1)
    quant_ms, quant_n = ctx.read_timing(2)
    dt = t1 - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms_per_step = dt / args.steps * 1e3
    value = world * n * args.steps / dt

    gram_avg_s = gram_ms / max(gram_n, 1) / 1e3
    gram_flop = n * p * (p + 1)  # symmetric Gram, algorithmic
    achieved = gram_flop / gram_avg_s / 1e12 if gram_avg_s > 0 else 0.0
    score_avg_s = score_ms / max(score_n, 1) / 1e3
    score_gbs = n * p * 4 / score_avg_s / 1e9 if score_avg_s > 0 else 0.0

    gram_kernel = {"bf16x3": "k_gram3", "i8x3": "k_gram8d"}.get(args.gram_mode, "k_gram")
    if args.gram_mode == "i8x3":
        # fp32-grade product from 6 int8 MFMA digit products (exact int32 sums)
        gram_desc = (f"{gram_kernel} (shifted Gram, 3 int8 digits per value, 6 i8 MFMA products per fp32 "
                     "product, exact int32 sums)")
        gram_peak = round(I8_MFMA_PEAK_TOPS / 6, 1)
        peak_basis = "int8 MFMA dense peak / 6 (fp32-equivalent); achieved counts algorithmic fp32 flops n*p*(p+1)"
    elif args.gram_mode == "bf16x3":
        # fp32-exact product from 6 bf16 MFMA products: the attainable fp32-equivalent peak is the bf16 peak / 6
        gram_desc = "k_gram3 (shifted Gram, exact 3-level bf16 split, 6 bf16 MFMA products per fp32 product)"
        gram_peak = round(BF16_MFMA_PEAK_TFLOPS / 6, 1)
        peak_basis = "bf16 MFMA dense peak / 6 (fp32-equivalent); achieved counts algorithmic fp32 flops n*p*(p+1)"
    else:
        gram_desc = "k_gram (FP32 MFMA shifted Gram)"
        gram_peak = FP32_MFMA_PEAK_TFLOPS
        peak_basis = "FP32 MFMA dense peak; achieved counts algorithmic flops n*p*(p+1) (symmetric Gram)"
    # HBM bytes per launch from this round's PMC passes (scripts/pmc_passes.sh →
    # scripts/pmc_latest.py → profiles/pmc_gram_latest.json; FETCH_SIZE doubled)
    traffic, traffic_src, score_traffic = None, None, None
    pmc = os.path.join(REPO, "profiles", "pmc_gram_latest.json")
    if os.path.exists(pmc):
        try:
            lat = json.load(open(pmc))
            traffic = lat.get(gram_kernel, {}).get("hbm_bytes_per_launch")
            traffic_src = lat.get(gram_kernel, {}).get("source")
            score_traffic = lat.get("k_score_1p", {}).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    accepted = float(result["pred"].sum().item()) / n
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "spectra/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (rank-40 band spectra + noise, generated in HBM)",
        "config": {
            "workload": f"SIMCA fit+score, synthetic {n}x{p} fp32 per GPU, k={k}, type=alt t2lim=Fdist qlim=jm",
            "step": ("utils.SIMCA(...).fit(X, y) + .predict(X), device tensors (drop-in)" if world == 1 else
                     "ocm.dist.ShardedSIMCA fit (T kept) + predict per rank"),
            "rows_per_gpu": n, "p": p, "k": k,
            "parallelism": f"row shards x{world} (RCCL all-reduce of Gram/colsum/n)",
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
                         "launches": score_n, "bytes_per_launch": n * p * 4, "traffic": score_traffic},
        "checks": {"accept_rate": round(accepted, 4), "eig_iters": result["fit"].eig_iters,
                   "T2_limit": result["T2_limit"], "Q_limit": result["Q_limit"],
                   "gram_guard_marks": engine.last_gram_marks(device.index)},
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        try:
            out["cpu_baseline"] = cpu_baseline(args.cpu_sample, p, k)
        except Exception as e:  # report, never fail the GPU number
            out["cpu_baseline"] = {"error": repr(e)}
    if world == 1 and not args.no_vae:
        try:
            out["vae"] = vae_bench(device, args.vae_steps, 10)
        except Exception as e:  # report, never fail the primary number
            out["vae"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
