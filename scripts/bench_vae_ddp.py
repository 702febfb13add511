#!/usr/bin/env python3
"""C5: VAE-SIMCA data-parallel training plus
SIMCA-on-latents, one process per GPU.

    python scripts/bench_vae_ddp.py --rows 200000                       # one GPU
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \\
        --master-addr 127.0.0.1 --master-port 29511 scripts/bench_vae_ddp.py   # 10M × 4096

Each rank generates its contiguous share of the global synthetic matrix in
HBM (ocm/synth.py: per-chunk Philox seeds, so the matrix does not depend on
the world size; 10M × 4096 fp32 = 164 GB in all, 20.5 GB per rank at 8).  The
standardisation statistics are global (one all-reduce of Σx, Σx², n).  The
C4 network trains through GraphedVAETrainer: one HIP-graph replay per step
with the flat-gradient RCCL all-reduce captured inside it; ``--sweep`` grid
points each build a fresh model and trainer and close it (graph, then its
RCCL communicator) before the next, as the reference's sweep does.  Then every rank
encodes its calibration rows and the latent statistics of
utils/final_vaesimca.py:428-442 (latent Gram, T² / Q percentiles) and the
f-distance moments of :510-523 are all-reduced, so the thresholds are the
whole test set's.  Rank 0 prints one JSON line: train samples/s (all ranks),
ms per step (max over ranks), the latent-statistics time, acceptance rate.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ocm-vae-simca_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000, help="global rows")
    ap.add_argument("--length", type=int, default=4096)
    ap.add_argument("--batch", type=int, default=512, help="per-rank batch")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--latent-rows", type=int, default=262144, help="calibration rows encoded per rank")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--sweep", type=int, default=3,
                    help="grid points: a fresh model + trainer per point, each closed after its steps "
                         "(utils/final_vaesimca.py:312-351); the last point's model scores the latents")
    ap.add_argument("--init-seed", type=int, default=0, help="network init seed of point 0")
    ap.add_argument("--seed-step", type=int, default=0, help="init seed increment per grid point")
    ap.add_argument("--dump", default=None, help="rank 0: save latents, Q and the SIMCA-on-latents outputs (.npz)")
    args = ap.parse_args()

    import ocm  # noqa: F401  (graph-capture runtime flag before the GPU initialises)
    import torch
    import torch.distributed as dist

    import vae_model as V
    from ocm import engine
    from ocm.synth import shard_bounds, spectra_shard
    from ocm.vae import full_distance_decision, latent_stats
    from ocm.vae_train import GraphedVAETrainer

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    group = dist.group.WORLD if world > 1 else None
    L, B = args.length, args.batch

    t0 = time.perf_counter()
    X = spectra_shard(args.rows, L, rank, world, dev, seed=args.seed)
    nloc = X.shape[0]
    assert nloc >= B, "fewer local rows than one batch"
    # global standardisation statistics (chunked fp64 sums; one all-reduce)
    stats = torch.zeros(2 * L + 1, dtype=torch.float64, device=dev)
    for a in range(0, nloc, 65536):
        xb = X[a:a + 65536].double()
        stats[:L] += xb.sum(0)
        stats[L:2 * L] += (xb * xb).sum(0)
    stats[-1] = nloc
    if world > 1:
        dist.all_reduce(stats)
    n = stats[-1]
    mean = stats[:L] / n
    std = ((stats[L:2 * L] - n * mean * mean) / (n - 1)).clamp_min(0).sqrt() + 1e-6
    torch.cuda.synchronize()
    t_data = time.perf_counter() - t0

    nb = max(1, nloc // B)

    def batch(i):
        j = i % nb
        return X[j * B:(j + 1) * B]

    point_s, point_loss = [], []
    for point in range(max(1, args.sweep)):
        torch.manual_seed(args.init_seed + point * args.seed_step)
        m = V.ConvVAE1D(L, 32, mean.float().cpu().numpy(), std.float().cpu().numpy(), conv_blocks=3, n_filters=3,
                        kernel_size=7, hidden_fc=64).to(dev)
        with GraphedVAETrainer(m, B, lr=1e-3, dtype=torch.bfloat16, group=group) as tr:
            for i in range(args.warmup):
                tr.step(batch(i))
            loss0 = float(tr.out[0].item()) if args.warmup else float("nan")
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for i in range(args.steps):
                tr.step(batch(args.warmup + i))
            torch.cuda.synchronize()
            dt = torch.tensor([time.perf_counter() - t1], dtype=torch.float64, device=dev)
            if world > 1:
                dist.all_reduce(dt, op=dist.ReduceOp.MAX)
            dt = float(dt.item())
            loss = float(tr.out[0].item())
            tr.sync_buffers()
        point_s.append(dt)
        point_loss.append((round(loss0, 5), round(loss, 5)))
    dt = sum(point_s) / len(point_s)  # mean over the grid points

    # SIMCA-on-latents: calibration latents and reconstruction residuals of
    # this rank's rows, global statistics
    m.eval()
    nl = min(args.latent_rows, nloc)
    mus = torch.empty((nl, 32), dtype=torch.float32, device=dev)
    q = torch.empty(nl, dtype=torch.float32, device=dev)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):  # kernel selection for both batch shapes
        for a in sorted({0, (nl - 1) // 8192 * 8192}):
            m.decode(m.encode((X[a:min(nl, a + 8192)] - m.spec_mean) / m.spec_std)[0])
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        for a in range(0, nl, 8192):
            xb = X[a:min(nl, a + 8192)]
            mu, _ = m.encode((xb - m.spec_mean) / m.spec_std)
            xr = m.decode(mu).float() * m.spec_std + m.spec_mean
            mus[a:a + xb.shape[0]] = mu.float()
            q[a:a + xb.shape[0]] = engine.rowsq_residual(xb, xr.contiguous())
    torch.cuda.synchronize()
    t_enc = time.perf_counter() - t2
    t3 = time.perf_counter()
    lmean, inv, t2lim, qlim = latent_stats(mus, q, group=group)
    accept, f, fcrit = full_distance_decision(mus, lmean, q, group=group)
    acc = accept.to(torch.float64).sum()
    if world > 1:
        dist.all_reduce(acc)
    torch.cuda.synchronize()
    t_stats = time.perf_counter() - t3

    lo, hi = shard_bounds(args.rows, rank, world)
    if rank == 0 and args.dump:
        import numpy as np

        np.savez(args.dump, mus=mus.cpu().numpy(), q=q.cpu().numpy(), lmean=lmean.cpu().numpy(),
                 inv=inv.cpu().numpy(), t2lim=t2lim, qlim=qlim, accept=accept.cpu().numpy(), f=f.cpu().numpy(),
                 fcrit=fcrit, world=world)
    if rank == 0:
        print(json.dumps({
            "metric": "VAE-SIMCA DDP train samples/s", "value": round(args.steps * B * world / dt, 1),
            "unit": "samples/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4), "dtype": "bf16", "data": "synthetic (ocm/synth.py)",
            "config": {"workload": f"ConvVAE1D cb=3 nf=3 ks=7 hid=64 d=32, B={B}/rank, L={L}, "
                                   f"{args.rows} rows global ({hi - lo} on rank 0), grad all-reduce in the step graph",
                       "params": sum(p.numel() for p in m.parameters())},
            "sweep_points": len(point_s), "point_ms_per_step": [round(t / args.steps * 1e3, 4) for t in point_s],
            "point_loss": point_loss,
            "loss_after_warmup": round(loss0, 5), "final_loss": round(loss, 5), "data_gen_s": round(t_data, 2),
            "params_finite": all(bool(torch.isfinite(p_).all()) for p_ in m.parameters()),
            "latents": {"rows_per_rank": nl, "encode_s": round(t_enc, 3), "stats_s": round(t_stats, 4),
                        "t2_limit": float(t2lim), "q_limit": float(qlim), "f_crit": float(fcrit),
                        "accept_rate": float(acc.item()) / (nl * world)},
        }), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
