#!/usr/bin/env python3
"""Which torch ops launch the graphed VAE step's non-libocm kernels (fills,
copies, elementwise): one eager fused bf16 step of the bench's C4 net under
torch.profiler, listing every aten op that launched device work with the
innermost repository frames of its Python stack.

    python3 scripts/vae_torch_ops.py > gpurun_out/vae_torch_ops.txt
"""
import collections
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
sys.path.insert(0, os.path.join(REPO, "ocm-vae-simca_amd"))


def main():
    import torch
    from torch.profiler import ProfilerActivity, profile

    import vae_model as V
    from bench import synth_device
    from ocm.vae_train import GraphedVAETrainer

    dev = torch.device("cuda", 0)
    batch, length = 512, 2048
    X = synth_device(batch * 4, length, 20, seed=99, device=dev)
    mean = X.mean(0).cpu().numpy()
    std = X.std(0).cpu().numpy() + 1e-6
    torch.manual_seed(0)
    m = V.ConvVAE1D(length, 32, mean, std, conv_blocks=3, n_filters=3, kernel_size=7, hidden_fc=64).to(dev)
    tr = GraphedVAETrainer(m, batch, lr=1e-3, dtype=torch.bfloat16, graph=False)
    for i in range(3):
        tr.step(X[i * batch:(i + 1) * batch])
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        tr.step(X[3 * batch:4 * batch])
        torch.cuda.synchronize()
    counts = collections.Counter()
    for ev in prof.events():
        if ev.device_type != torch.autograd.DeviceType.CPU or not ev.name.startswith("aten::"):
            continue
        kern = [k.name for k in ev.kernels] if hasattr(ev, "kernels") else []
        if not kern and ev.cuda_time_total == 0:
            continue
        stack = [s for s in (ev.stack or []) if "ocm-vae-simca_amd" in s or "vae_model" in s]
        key = (ev.name, tuple(stack[:3]))
        counts[key] += 1
    for (name, stack), n in sorted(counts.items(), key=lambda kv: kv[0][0]):
        print(f"{n}x {name}")
        for s in stack:
            print(f"      {s}")
    print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=40))


if __name__ == "__main__":
    main()
