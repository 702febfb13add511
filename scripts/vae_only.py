"""VAE secondary metric alone: bench.vae_bench (C4 network, B=512, bf16, HIP graph)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ocm-vae-simca_amd"))
import bench  # noqa: E402  (sets the graph-capture flag before HIP init)
import torch  # noqa: E402

print(json.dumps(bench.vae_bench(torch.device("cuda", 0), int(sys.argv[1]) if len(sys.argv) > 1 else 200, 10)))
