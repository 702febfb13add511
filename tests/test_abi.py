"""CPU-side checks of the C ABI: the library exists, loads next to torch's
HIP runtime and exports every symbol include/ocm.h declares."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "ocm.h")
LIB = os.path.join(REPO, "ocm-vae-simca_amd", "ocm", "libocm.so")


def header_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|size_t|const char\*)\s+(ocm_\w+)\s*\(", txt, re.M)))


def test_header_parses():
    syms = header_symbols()
    assert "ocm_gram_f32" in syms and "ocm_score_f32" in syms and "ocm_eig_topk" in syms
    assert len(syms) >= 15


@pytest.mark.skipif(not os.path.exists(LIB), reason="libocm.so not built")
def test_library_exports_every_header_symbol():
    import torch  # noqa: F401  (HIP runtime first, as the product loads it)

    lib = ctypes.CDLL(LIB)
    for s in header_symbols():
        assert hasattr(lib, s), f"missing export {s}"


@pytest.mark.skipif(not os.path.exists(LIB), reason="libocm.so not built")
def test_binding_signatures_cover_header():
    from ocm import _lib

    assert set(_lib.SIGNATURES) == set(header_symbols())
    lib = _lib.load()
    assert lib.ocm_abi_version() == _lib.ABI_VERSION == 12


@pytest.mark.skipif(not os.path.exists(LIB), reason="libocm.so not built")
def test_ctx_create_fails_loudly_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from ocm import _lib

    with pytest.raises(Exception):
        _lib.Context(0)


@pytest.mark.skipif(not os.path.exists(LIB), reason="libocm.so not built")
def test_build_id_matches_sources():
    """the library carries the hash of its build inputs; the
    binding recomputes it from the sources beside the package."""
    from ocm import _lib

    want = _lib.source_build_id()
    assert want is not None and len(want) == 16
    assert _lib.file_build_id(LIB) == want
    assert _lib.load().ocm_build_id().decode() == want


def test_stale_library_is_refused(tmp_path):
    """A library whose build id differs from the sources is refused at load
    (a fresh interpreter: the binding loads once per process)."""
    import shutil
    import subprocess
    import sys

    if not os.path.exists(LIB):
        pytest.skip("libocm.so not built")
    from ocm import _lib

    stale = tmp_path / "libocm.so"
    data = open(LIB, "rb").read()
    want = _lib.source_build_id().encode()
    other = b"f" * 16 if want != b"f" * 16 else b"0" * 16
    stale.write_bytes(data.replace(b"ocm-build-id:" + want, b"ocm-build-id:" + other))
    code = ("import sys; sys.path.insert(0, %r); import ocm; from ocm import _lib\n"
            "try:\n    _lib.load()\nexcept _lib.OcmError as e:\n    print('refused', e)\n") % \
        os.path.join(REPO, "ocm-vae-simca_amd")
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, OCM_LIB=str(stale)), capture_output=True,
                       text=True, timeout=120)
    assert "refused" in r.stdout and "stale" in r.stdout, (r.stdout, r.stderr[-2000:])
    shutil.rmtree(tmp_path, ignore_errors=True)
