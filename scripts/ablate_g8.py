"""Timing ablations of an i8x3 Gram variant (OCM_GRAM8_NOLOAD bits; the Gram
is wrong under any nonzero bit) on the bench workload: ms per launch."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ocm-vae-simca_amd"))
sys.path.insert(0, REPO)

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=1_000_000)
ap.add_argument("--p", type=int, default=2048)
ap.add_argument("--variant", default="shared")
ap.add_argument("--flags", default="0,1,2,4,8,9,12,3,6")
ap.add_argument("--chunk", default="4096")
args = ap.parse_args()
import torch  # noqa: E402

from bench import synth_device  # noqa: E402
from ocm import engine  # noqa: E402
from ocm._lib import Context  # noqa: E402

os.environ["OCM_GRAM_MODE"] = "i8x3"
os.environ["OCM_GRAM_CHUNK"] = args.chunk
X = synth_device(args.rows, args.p, 20, seed=7, device=torch.device("cuda", 0))
shift = engine.cast_f32(engine.colmean(X, None, 4096))
ctx = Context.get(0)
for var in args.variant.split(","):
    os.environ["OCM_GRAM8_VARIANT"] = var
    for f in args.flags.split(","):
        os.environ["OCM_GRAM8_NOLOAD"] = f
        engine.gram(X, None, [0, args.rows], shift)
        torch.cuda.synchronize()
        ctx.read_timing(0)
        ctx.set_timing(True)
        for _ in range(3):
            engine.gram(X, None, [0, args.rows], shift)
        ctx.set_timing(False)
        ms, cnt = ctx.read_timing(0)
        print(f"{var:7s} flags {int(f):2d}: {ms / max(cnt, 1):7.3f} ms/launch", flush=True)
