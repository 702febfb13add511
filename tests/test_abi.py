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
    assert lib.ocm_abi_version() == _lib.ABI_VERSION == 9


@pytest.mark.skipif(not os.path.exists(LIB), reason="libocm.so not built")
def test_ctx_create_fails_loudly_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from ocm import _lib

    with pytest.raises(Exception):
        _lib.Context(0)
