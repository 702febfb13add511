#!/usr/bin/env python3
"""Kernel trace of the graphed C4 VAE train step alone (the bench's VAE line:
cb=3, nf=3, ks=7, hid=64, d=32, B=512, L=2048, bf16).  The timed replays are
bracketed by two libocm k_cast_f64_f32 launches (sentinels), so the window can
be cut out of a rocprofv3 kernel trace that also holds MIOpen's kernel search
and the graph capture:

    rocprofv3 --kernel-trace -d OUT -o run --output-format csv -- python3 scripts/vae_step_trace.py 50
    python3 scripts/vae_step_trace.py --summarize OUT/run_kernel_trace.csv 50 > profiles/<name>.md
"""
import collections
import csv
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
sys.path.insert(0, os.path.join(REPO, "ocm-vae-simca_amd"))

SENTINEL = "k_cast_f64_f32"


def run(steps: int):
    import torch

    import vae_model as V
    from bench import synth_device
    from ocm import engine
    from ocm.vae_train import GraphedVAETrainer

    dev = torch.device("cuda", 0)
    batch, length, warmup = 512, 2048, 10
    X = synth_device(batch * (warmup + steps), length, 20, seed=99, device=dev)
    mean = X.mean(0).cpu().numpy()
    std = X.std(0).cpu().numpy() + 1e-6
    torch.manual_seed(0)
    m = V.ConvVAE1D(length, 32, mean, std, conv_blocks=3, n_filters=3, kernel_size=7, hidden_fc=64).to(dev)
    tr = GraphedVAETrainer(m, batch, lr=1e-3, dtype=torch.bfloat16)
    for i in range(warmup):
        tr.step(X[i * batch:(i + 1) * batch])
    probe = torch.zeros(7, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    engine.cast_f32(probe)  # sentinel: window start
    for i in range(warmup, warmup + steps):
        tr.step(X[i * batch:(i + 1) * batch])
    engine.cast_f32(probe)  # sentinel: window end
    torch.cuda.synchronize()
    print(f"vae_step_trace: {steps} graphed steps, loss {float(tr.out[0].item()):.5f}")


def summarize(path: str, steps: int, by_grid: bool = False):
    rows = list(csv.DictReader(open(path)))
    for r in rows:
        r["_s"], r["_e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    rows.sort(key=lambda r: r["_s"])
    marks = [i for i, r in enumerate(rows) if SENTINEL in r["Kernel_Name"]]
    a, b = marks[-2], marks[-1]
    win = rows[a + 1:b]
    span_ns = rows[b]["_s"] - rows[a]["_e"]
    agg = collections.defaultdict(lambda: [0, 0])
    busy = 0
    grid_cols = [c for c in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z", "Grid_Size") if c in win[0]] if win else []
    for r in win:
        d = r["_e"] - r["_s"]
        busy += d
        grid = "×".join(r[c] for c in grid_cols)
        key = r["Kernel_Name"] if not by_grid else f"{r['Kernel_Name'][:70]} [{grid}]"
        agg[key][0] += 1
        agg[key][1] += d
    print(f"# C4 VAE train step (graphed, bf16, B=512, L=2048): kernel trace of {steps} replays\n")
    print(f"* kernels per step: {len(win) / steps:.1f}; wall per step (sentinel to sentinel): "
          f"{span_ns / steps / 1e3:.1f} µs; summed kernel time per step: {busy / steps / 1e3:.1f} µs\n")
    print("| kernel | per step | avg µs | µs per step | % of kernel time |")
    print("|---|---|---|---|---|")
    for name, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"| `{name[:90]}` | {n / steps:.1f} | {t / n / 1e3:.2f} | {t / steps / 1e3:.1f} | {100 * t / busy:.1f} |")


if __name__ == "__main__":
    if sys.argv[1] == "--summarize":
        summarize(sys.argv[2], int(sys.argv[3]), "--by-grid" in sys.argv[4:])
    else:
        run(int(sys.argv[1]))
