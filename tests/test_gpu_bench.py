"""bench.py as the driver runs it, on the box's one GPU.

``python bench.py --gpus 2`` (no WORLD_SIZE) must start two ranks itself; with
``--dist-backend gloo`` both share cuda:0, so the launcher, the strong / weak
scaling runs, the per-rank phase breakdown and the C3 CV line all execute
the same code the driver's 8-GPU RCCL run takes (only the backend differs).
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-4000:]
    return json.loads(lines[0])


def test_bench_two_ranks_gloo_one_gpu():
    out = _run(["--gpus", "2", "--dist-backend", "gloo", "--rows", "65536", "--steps", "2", "--warmup", "1",
                "--no-cpu", "--no-vae", "--cv-reps", "1", "--phase-steps", "1"])
    assert out["n_gpus"] == 2
    assert out["scaling"] == "strong"
    assert out["value"] > 0 and out["ms_per_step"] > 0
    assert out["config"]["rows_total"] == 65536 and out["config"]["rows_per_gpu"] == 32768
    assert set(out["phases_ms"]) == {"rank0", "rank1"}
    for ph in out["phases_ms"].values():
        assert {"gram", "allreduce", "eig", "fit_score", "limits", "predict_score"} <= set(ph)
    assert out["weak"]["rows_total"] == 131072 and out["weak"]["value"] > 0
    cv = out["cv"]
    assert "error" not in cv, cv
    assert cv["value"] > 0 and 0 <= cv["spec"] <= 100 and 0 <= cv["sens"] <= 100
    assert 0.8 < out["checks"]["accept_rate"] <= 1.0


def test_bench_single_gpu_small():
    out = _run(["--rows", "65536", "--steps", "2", "--warmup", "1", "--no-cpu", "--no-vae", "--cv-reps", "1",
                "--phase-steps", "1"])
    assert out["n_gpus"] == 1 and out["value"] > 0
    assert {"gram", "eig", "fit_score", "limits", "predict_score"} <= set(out["phases_ms"]["rank0"])
    assert out["roofline"]["launches"] == 2 and out["roofline"]["frac"] > 0
    assert "error" not in out["cv"], out["cv"]
