"""Child process of tests/test_gpu_dist.py::test_cv_engine_over_rccl_world1 (GPU):
the distributed CV fold engine (ocm/cv.py: reduce-to-owner train Grams, model
broadcasts, all-reduced counts and moments, radix-select percentile
histograms, the device all-gather of the pooled predictions) over a REAL RCCL
process group of one rank, against the same engine without a group.  One
process per GPU is all a one-GPU box allows, so the collectives are RCCL's
one-rank forms — but every nccl branch of the engine runs.  Prints one JSON
line, destroys the process group and returns normally."""
import json
import os
import socket
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ocm-vae-simca_amd"))
sys.path.insert(0, REPO)
import ocm  # noqa: E402,F401
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    from sklearn.model_selection import KFold

    import ocm.cv as fe
    from oracle import simca_oracle as O

    dev = torch.device("cuda", 0)
    X0 = O.synth_spectra(2400, 256, 8, rank=24, seed=21)
    X1 = O.synth_spectra(600, 256, 8, rank=24, seed=22, outlier_frac=1.0)
    X = torch.from_numpy(np.concatenate([X0, X1]).astype(np.float32)).to(dev)
    y = np.concatenate([np.zeros(2400, np.int64), np.ones(600, np.int64)])
    cls_idx = np.flatnonzero(y == 0)
    folds = [cls_idx[te] for _, te in KFold(n_splits=5).split(cls_idx)]
    combos = [{"type": "alt", "t2lim": "Fdist", "qlim": "jm"}, {"type": "ci", "t2lim": "perc", "qlim": "perc"},
              {"type": "dd"}]
    base = dict(n_components=2, model_class=None, type="alt", t2lim="Fdist", t2cl=0.95, qlim="jm", qcl=0.95,
                dcl=0.95, maxPC=20, criteria="compl", verbose=False)
    ref, rby = fe.cv_grid(X, y, folds, cls_idx, [6, 7, 8], combos, base, [0], True)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    got, gby = fe.cv_grid(X, y, folds, cls_idx, [6, 7, 8], combos, base, [0], True, group=dist.group.WORLD)
    torch.cuda.synchronize()
    print(json.dumps({"backend": dist.get_backend(), "spec": [r["spec"] for r in got], "spec_ref": [r["spec"] for r in ref],
                      "sens": [r["sens"] for r in got], "sens_ref": [r["sens"] for r in ref],
                      "pred_diff": int(sum(int((np.asarray(a["prediction"]) != np.asarray(b["prediction"])).sum())
                                           for a, b in zip(gby, rby)))}), flush=True)
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
