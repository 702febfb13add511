"""Child process of tests/test_vae_train.py::test_c4_graph_step_with_grad_allreduce
(GPU): a world-1 RCCL process group and a sweep of three graphed C4 trainers
with the captured gradient all-reduce, built and closed one after another as
the reference's grid builds a model per point (utils/final_vaesimca.py:312-351).

Before each trainer the caller issues an eager ``dist.all_reduce`` that is
held behind a GPU spin (``torch.cuda._sleep``), so the ProcessGroupNCCL
watchdog still tracks it when the trainer reaches its capture: the capture
guard (``ocm.rccl.wait_pg_collectives_retired``) must find it and wait it out
(``pending_at_capture >= 1``), or the watchdog's poll during the capture would
abort the process.  Each trainer is closed (graph, then its communicator),
then the process group is destroyed and the process returns normally.
Prints one JSON line."""
import copy
import json
import os
import socket
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ocm-vae-simca_amd"))
os.environ["TORCH_FR_BUFFER_SIZE"] = "2000"  # the flight recorder the capture guard reads
import ocm  # noqa: E402,F401  (sets the HIP graph runtime flag before the GPU initialises)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import vae_model as V  # noqa: E402
from ocm.rccl import pending_pg_collectives  # noqa: E402
from ocm.vae_train import GraphedVAETrainer  # noqa: E402

HOLD_S = 2.0  # GPU spin that holds the eager collective (the trainer's host-side build is far shorter)


def hold_cycles(dev) -> int:
    """torch.cuda._sleep's cycle count for HOLD_S seconds (its clock is measured)."""
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(1000)
    a.record()
    torch.cuda._sleep(20_000_000)
    b.record()
    b.synchronize()
    per_s = 20_000_000 / max(a.elapsed_time(b) * 1e-3, 1e-6)
    return int(min(per_s * HOLD_S, 2**62))


def main():
    dev = torch.device("cuda", 0)
    L, d, B = 2048, 32, 512
    g = torch.Generator(device="cpu").manual_seed(3)
    X = (1.0 + 0.3 * torch.randn(B * 4, L, generator=g)).to(dev)
    mean, std = X.mean(0).cpu().numpy(), X.std(0).cpu().numpy()
    torch.manual_seed(0)
    base = V.ConvVAE1D(L, d, mean, std, conv_blocks=3, n_filters=3, kernel_size=7, hidden_fc=64).to(dev)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    cycles = hold_cycles(dev)
    out = {"points": [], "hold_cycles": cycles}
    for point in range(3):
        m1, m2 = copy.deepcopy(base), copy.deepcopy(base)
        # the round-4 abort: an eager collective still tracked by its watchdog
        # when the step is captured — held here behind a GPU spin
        torch.cuda._sleep(cycles)
        dist.all_reduce(torch.ones(4, device=dev))
        pending_before = pending_pg_collectives()
        t0 = time.perf_counter()
        tr = GraphedVAETrainer(m1, B, lr=1e-3, dtype=torch.bfloat16, graph=True, grad_allreduce=True)
        build_s = time.perf_counter() - t0
        lo, hi = tr.flat_grad.data_ptr(), tr.flat_grad.data_ptr() + tr.flat_grad.numel() * 4
        views = all(lo <= p.grad.data_ptr() < hi for p in m1.parameters())
        with GraphedVAETrainer(m2, B, lr=1e-3, dtype=torch.bfloat16, graph=True, grad_allreduce=False) as ref:
            la, lb = torch.zeros(40, device=dev), torch.zeros(40, device=dev)
            for i in range(40):
                xb = X[(i % 4) * B:(i % 4 + 1) * B]
                la[i].copy_(tr.step(xb)[0])
                lb[i].copy_(ref.step(xb)[0])
            torch.cuda.synchronize()
        tr.sync_buffers()
        torch.cuda.synchronize()
        rec = {"allreduce": tr.allreduce, "graphed": tr.graphed, "grads_are_views": views,
               "own_comm": tr._comm is not None, "pending_before": pending_before,
               "pending_at_capture": tr.pending_at_capture, "build_s": build_s,
               "loss_ddp": la.cpu().tolist(), "loss_single": lb.cpu().tolist(),
               "params_finite": all(bool(torch.isfinite(p).all()) for p in m1.parameters())}
        tr.close()
        rec["closed"] = tr._comm is None and tr.graph is None
        try:
            tr.step(X[:B])
            rec["step_after_close_raises"] = False
        except RuntimeError:
            rec["step_after_close_raises"] = True
        rec["pending_after"] = pending_pg_collectives()
        out["points"].append(rec)
        del tr, m1, m2
    dist.destroy_process_group()
    out["exit"] = "normal"
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
