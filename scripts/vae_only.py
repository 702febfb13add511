#!/usr/bin/env python3
"""The bench's VAE line alone (C4 network, B = 512, L = 2048, bf16, HIP-graph
step), for kernel traces:  python scripts/vae_only.py [steps]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
sys.path.insert(0, os.path.join(REPO, "ocm-vae-simca_amd"))

if __name__ == "__main__":
    import torch

    from bench import vae_bench

    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    if "benchmark" in sys.argv[2:]:
        torch.backends.cudnn.benchmark = True  # MIOpen find with timing for every conv shape
    print(json.dumps(vae_bench(torch.device("cuda", 0), steps, 10)), flush=True)
