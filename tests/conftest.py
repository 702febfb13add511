import os
import sys

import pytest

# before any HIP initialisation: see ocm/__init__.py (graph packet-capture race)
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "ocm-vae-simca_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: large-size property checks")


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
