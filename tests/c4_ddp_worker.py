"""Child process of tests/test_vae_train.py::test_c4_graph_step_with_grad_allreduce
(GPU): a world-1 RCCL process group, the C4 network trained by the graphed
step with and without the captured gradient all-reduce; prints one JSON line
and leaves without tearing the communicator down under a live graph."""
import copy
import json
import os
import socket
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ocm-vae-simca_amd"))
import ocm  # noqa: E402,F401  (sets the HIP graph runtime flag before the GPU initialises)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import vae_model as V  # noqa: E402
from ocm.vae_train import GraphedVAETrainer  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    L, d, B = 2048, 32, 512
    g = torch.Generator(device="cpu").manual_seed(3)
    X = (1.0 + 0.3 * torch.randn(B * 4, L, generator=g)).to(dev)
    mean, std = X.mean(0).cpu().numpy(), X.std(0).cpu().numpy()
    torch.manual_seed(0)
    m1 = V.ConvVAE1D(L, d, mean, std, conv_blocks=3, n_filters=3, kernel_size=7, hidden_fc=64).to(dev)
    m2 = copy.deepcopy(m1)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    # the round-4 abort: an eager ProcessGroupNCCL collective still tracked by
    # its watchdog when the step is captured.  Issue one right before the
    # trainer, so its capture has to wait it out (ocm/rccl.py)
    from ocm.rccl import pending_pg_collectives

    dist.all_reduce(torch.ones(4, device=dev))
    pending_before = pending_pg_collectives()
    tr = GraphedVAETrainer(m1, B, lr=1e-3, dtype=torch.bfloat16, graph=True, grad_allreduce=True)
    lo, hi = tr.flat_grad.data_ptr(), tr.flat_grad.data_ptr() + tr.flat_grad.numel() * 4
    views = all(lo <= p.grad.data_ptr() < hi for p in m1.parameters())
    ref = GraphedVAETrainer(m2, B, lr=1e-3, dtype=torch.bfloat16, graph=True, grad_allreduce=False)
    la, lb = torch.zeros(40, device=dev), torch.zeros(40, device=dev)
    for i in range(40):
        xb = X[(i % 4) * B:(i % 4 + 1) * B]
        la[i].copy_(tr.step(xb)[0])
        lb[i].copy_(ref.step(xb)[0])
    torch.cuda.synchronize()
    tr.sync_buffers()
    torch.cuda.synchronize()
    print(json.dumps({"allreduce": tr.allreduce, "graphed": tr.graphed, "grads_are_views": views,
                      "own_comm": tr._comm is not None, "pending_before": pending_before,
                      "pending_at_capture": tr.pending_at_capture, "pending_after": pending_pg_collectives(),
                      "loss_ddp": la.cpu().tolist(), "loss_single": lb.cpu().tolist(),
                      "params_finite": all(bool(torch.isfinite(p).all()) for p in m1.parameters())}), flush=True)
    sys.stdout.flush()
    os._exit(0)


if __name__ == "__main__":
    main()
