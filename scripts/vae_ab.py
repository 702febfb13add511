#!/usr/bin/env python3
"""A/B of module-level switches of the bf16 VAE step: the bench's VAE line
(C4, B = 512, L = 2048, HIP graph) in alternating child processes, one per
variant, each variant a set of ``module.ATTR=value`` assignments made before
the trainer is built, or ``env.NAME=value`` environment settings of the child.

    python scripts/vae_ab.py --steps 300 --rounds 2 \\
        --variant new: --variant old:ocm.conv.QSUM_FUSED=False,ocm.vae_train.PERSISTENT_ONE=False
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = """
import importlib, json, os, sys
sys.path.insert(0, {repo!r}); sys.path.insert(0, os.path.join({repo!r}, "ocm-vae-simca_amd"))
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
for k, v in {sets!r}:
    mod, attr = k.rsplit(".", 1)
    setattr(importlib.import_module(mod), attr, eval(v))
import torch
from bench import vae_bench
r = vae_bench(torch.device("cuda", 0), {steps}, 10, latent_rows=0)
print(json.dumps({{"variant": {name!r}, "steps_per_s": r["value"] if "value" in r else r}}))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--variant", action="append", required=True, help="name:mod.ATTR=value,...")
    a = ap.parse_args()
    variants = []
    for v in a.variant:
        name, _, spec = v.partition(":")
        sets = [tuple(kv.split("=", 1)) for kv in spec.split(",") if kv]
        variants.append((name, sets))
    for _ in range(a.rounds):
        for name, sets in variants:
            env = dict(os.environ)
            env.update({k[4:]: v for k, v in sets if k.startswith("env.")})
            mods = [(k, v) for k, v in sets if not k.startswith("env.")]
            code = CHILD.format(repo=REPO, sets=mods, steps=a.steps, name=name)
            r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env)
            if r.returncode != 0:
                sys.exit(r.stderr[-3000:])
            print(r.stdout.strip().splitlines()[-1], flush=True)


if __name__ == "__main__":
    main()
