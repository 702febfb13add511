"""ctypes binding of libocm.so (include/ocm.h).

torch is imported first so that libocm.so binds to the HIP runtime torch
already loaded (both carry SONAME libamdhip64.so.7): device pointers and
streams then belong to one runtime.  There is no fallback: if the library or
a gfx950 device is missing, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("OCM_LIB", os.path.join(_HERE, "libocm.so"))
# `make exp` builds (csrc/build/exp/) carry diagnostic variants, some of which
# give wrong results on purpose (load-path ablations): they are loaded only
# when the A/B scripts ask for it explicitly
if os.sep + os.path.join("build", "exp") + os.sep in os.path.abspath(LIB_PATH) and \
        os.environ.get("OCM_ALLOW_EXP_LIB") != "1":
    raise ImportError(f"OCM_LIB={LIB_PATH} is a `make exp` diagnostic build; set OCM_ALLOW_EXP_LIB=1 to load it "
                      "(A/B scripts only, never the product path)")

OCM_OK = 0
OCM_ERR_ARG = -1
OCM_ERR_HIP = -2
OCM_ERR_NOMEM = -3
OCM_ERR_NOCONV = -4
OCM_ERR_UNSUPPORTED = -5

TYPE_CODES = {"sim": 0, "alt": 1, "ci": 2, "dd": 3}

c_void_p = ctypes.c_void_p
c_i32 = ctypes.c_int32
c_i64 = ctypes.c_int64
c_f64 = ctypes.c_double


class OcmDecision(ctypes.Structure):
    _fields_ = [("type", c_i32), ("pad_", c_i32), ("t2_scale", c_f64), ("q_scale", c_f64), ("dlim", c_f64)]


class OcmCvConfig(ctypes.Structure):
    _fields_ = [("lv", c_i32), ("type", c_i32), ("t2_scale", c_f64), ("q_scale", c_f64), ("dlim", c_f64)]


OCM_CV_MAXCFG = 1024


class OcmError(RuntimeError):
    pass


class OcmNotConverged(OcmError):
    pass


# name -> (restype, argtypes); every symbol include/ocm.h declares
SIGNATURES = {
    "ocm_abi_version": (c_i32, []),
    "ocm_build_id": (ctypes.c_char_p, []),
    "ocm_last_error": (ctypes.c_char_p, []),
    "ocm_ctx_create": (c_i32, [c_i32, ctypes.POINTER(c_void_p)]),
    "ocm_ctx_destroy": (c_i32, [c_void_p]),
    "ocm_ctx_reserve": (c_i32, [c_void_p, ctypes.c_size_t]),
    "ocm_ctx_set_timing": (c_i32, [c_void_p, c_i32]),
    "ocm_ctx_read_timing": (c_i32, [c_void_p, c_i32, ctypes.POINTER(c_f64), ctypes.POINTER(c_i64)]),
    "ocm_colmean_f32": (c_i32, [c_void_p, c_void_p, c_i64, c_void_p, c_i64, c_i32, c_void_p, c_void_p]),
    "ocm_gram_f32": (c_i32, [c_void_p, c_void_p, c_i64, c_void_p, c_i64, c_i32, c_void_p,
                             ctypes.POINTER(c_i64), c_i32, c_void_p, c_void_p, c_void_p]),
    "ocm_gram_f32_ex": (c_i32, [c_void_p, c_void_p, c_i64, c_void_p, c_i64, c_i32, c_void_p,
                                ctypes.POINTER(c_i64), c_i32, c_i32, c_i64, c_void_p, c_void_p, c_void_p]),
    "ocm_gram_last_marks": (c_i32, [c_void_p, ctypes.POINTER(c_i64)]),
    "ocm_cov_from_gram": (c_i32, [c_void_p, ctypes.POINTER(c_void_p), ctypes.POINTER(c_void_p),
                                  ctypes.POINTER(c_f64), c_i32, c_void_p, c_i64, c_i32, c_void_p, c_void_p,
                                  c_void_p]),
    "ocm_eig_topk": (c_i32, [c_void_p, c_void_p, c_i32, c_i32, c_f64, c_i32, c_i32, c_void_p, c_void_p, c_void_p,
                             ctypes.POINTER(c_i32), c_void_p]),
    "ocm_eig_topk_ex": (c_i32, [c_void_p, c_void_p, c_i32, c_i32, c_f64, c_i32, c_i32, c_i32, c_i32, c_void_p,
                                c_void_p, c_void_p, ctypes.POINTER(c_i32), c_void_p]),
    "ocm_eig_topk_ex2": (c_i32, [c_void_p, c_void_p, c_i32, c_i32, c_f64, c_i32, c_i32, c_i32, c_i32, c_void_p,
                                 c_void_p, c_void_p, ctypes.POINTER(c_i32), c_f64, c_void_p, c_void_p]),
    "ocm_gram_pack": (c_i32, [c_void_p, c_void_p, c_void_p, c_void_p, c_i64, c_i32, c_void_p, c_void_p]),
    "ocm_cov_from_packed": (c_i32, [c_void_p, c_void_p, c_i32, c_void_p, c_void_p, c_void_p]),
    "ocm_sym_pinv_f64": (c_i32, [c_void_p, c_void_p, c_i32, c_f64, c_void_p, c_void_p]),
    "ocm_inv_evals_f64": (c_i32, [c_void_p, c_void_p, c_i32, c_f64, c_void_p, c_void_p]),
    "ocm_score_f32": (c_i32, [c_void_p, c_void_p, c_i64, c_void_p, c_i64, c_i32, c_void_p, c_void_p, c_void_p,
                              c_i32, c_void_p, c_void_p, c_void_p, ctypes.POINTER(OcmDecision), c_void_p, c_i64,
                              c_void_p, c_void_p]),
    "ocm_score_f32_diag": (c_i32, [c_void_p, c_void_p, c_i64, c_void_p, c_i64, c_i32, c_void_p, c_void_p,
                                   c_void_p, c_i32, c_void_p, c_void_p, c_void_p, ctypes.POINTER(OcmDecision),
                                   c_void_p, c_i64, c_void_p, c_void_p]),
    "ocm_decide": (c_i32, [c_void_p, c_void_p, c_void_p, c_i64, ctypes.POINTER(OcmDecision), c_void_p, c_void_p,
                           c_void_p, c_void_p, c_i64, c_void_p]),
    "ocm_rowsq_residual_f32": (c_i32, [c_void_p, c_void_p, c_i64, c_void_p, c_i64, c_i64, c_i32, c_void_p,
                                       c_void_p]),
    "ocm_rowsq_minmax_f32": (c_i32, [c_void_p, c_void_p, c_i64, c_void_p, c_i64, c_i64, c_i32, ctypes.c_float,
                                     c_void_p, c_void_p]),
    "ocm_cast_f64_f32": (c_i32, [c_void_p, c_void_p, c_i64, c_void_p, c_void_p]),
    "ocm_percentile": (c_i32, [c_void_p, c_void_p, c_i32, c_i64, c_f64, ctypes.POINTER(c_f64), c_void_p]),
    "ocm_radix_hist": (c_i32, [c_void_p, c_void_p, c_i32, c_i64, ctypes.c_uint64, c_i32, c_void_p, c_void_p]),
    "ocm_gram_combine": (c_i32, [c_void_p, ctypes.POINTER(c_void_p), ctypes.POINTER(c_void_p),
                                 ctypes.POINTER(c_f64), c_i32, c_i32, c_void_p, c_void_p, c_void_p]),
    "ocm_cv_prefix": (c_i32, [c_void_p, c_void_p, c_i64, c_i32, c_void_p, c_void_p, ctypes.POINTER(c_i32), c_i32,
                              c_void_p, c_void_p, c_void_p, c_void_p]),
    "ocm_confusion_counts": (c_i32, [c_void_p, c_void_p, c_i64, c_i64, c_void_p, c_void_p, c_void_p]),
    "ocm_snv_savgol_f32": (c_i32, [c_void_p, c_void_p, c_i64, c_i64, c_i32, c_i32, c_i32,
                                   ctypes.POINTER(c_f64), c_void_p, c_i64, c_void_p]),
    "ocm_cv_counts": (c_i32, [c_void_p, c_void_p, c_i64, c_i32, c_void_p, c_void_p, c_void_p, c_i64,
                              ctypes.POINTER(OcmCvConfig), c_i32, c_void_p, c_void_p, c_void_p]),
    "ocm_colmean_f64": (c_i32, [c_void_p, c_void_p, c_i64, c_void_p, c_i64, c_i32, c_void_p, c_void_p]),
    "ocm_gram_f64": (c_i32, [c_void_p, c_void_p, c_i64, c_void_p, c_i64, c_i32, c_void_p,
                             ctypes.POINTER(c_i64), c_i32, c_void_p, c_void_p, c_void_p]),
    "ocm_score_f64_diag": (c_i32, [c_void_p, c_void_p, c_i64, c_void_p, c_i64, c_i32, c_void_p, c_void_p,
                                   c_void_p, c_i32, c_void_p, c_void_p, c_void_p, ctypes.POINTER(OcmDecision),
                                   c_void_p, c_i64, c_void_p, c_void_p]),
    "ocm_decide_f64": (c_i32, [c_void_p, c_void_p, c_void_p, c_i64, ctypes.POINTER(OcmDecision), c_void_p,
                               c_void_p, c_void_p, c_void_p, c_i64, c_void_p]),
    "ocm_bn_scratch_bytes": (ctypes.c_size_t, [c_i32]),
    "ocm_bn_fwd_train": (c_i32, [c_void_p, c_i32, c_void_p, c_i32, c_i32, c_i32, c_void_p, c_void_p, ctypes.c_float,
                                 ctypes.c_float, c_void_p, c_void_p, c_void_p, c_i32, c_void_p, c_void_p, c_void_p,
                                 c_void_p, c_void_p]),
    "ocm_bn_fwd_eval": (c_i32, [c_void_p, c_i32, c_void_p, c_i32, c_i32, c_i32, c_void_p, c_void_p, ctypes.c_float,
                                c_void_p, c_void_p, c_i32, c_void_p, c_void_p]),
    "ocm_bn_bwd": (c_i32, [c_void_p, c_i32, c_void_p, c_void_p, c_i32, c_i32, c_i32, c_void_p, c_void_p, c_void_p,
                           c_i32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "ocm_conv1d_scratch_bytes": (ctypes.c_size_t, [c_i32, c_i32, c_i32]),
    "ocm_conv1d": (c_i32, [c_void_p, c_i32, c_i32, c_void_p, c_i32, c_i32, c_i32, c_void_p, c_void_p, c_i32, c_i32,
                           c_i32, c_i32, c_i32, c_i32, c_void_p, c_void_p]),
    "ocm_conv1d_wgrad": (c_i32, [c_void_p, c_i32, c_void_p, c_i32, c_i32, c_i32, c_void_p, c_i32, c_i32, c_i32,
                                 c_i32, c_i32, c_i32, c_void_p, c_void_p, c_void_p, c_void_p]),
    "ocm_conv1d_wgrad_qsum": (c_i32, [c_void_p, c_i32, c_void_p, c_i32, c_i32, c_i32, c_void_p, c_i32, c_i32, c_i32,
                                 c_i32, c_i32, c_i32, c_void_p, c_void_p, c_void_p, c_void_p]),
    "ocm_chan_sum": (c_i32, [c_void_p, c_i32, c_void_p, c_i32, c_i32, c_i32, c_void_p, c_void_p, c_void_p]),
    "ocm_vae_scratch_bytes": (ctypes.c_size_t, [c_i32]),
    "ocm_vae_bottleneck_scratch_bytes": (ctypes.c_size_t, []),
    "ocm_vae_bottleneck_fwd": (c_i32, [c_void_p, c_i32, c_void_p, c_void_p, c_void_p, c_i32, c_i32, c_void_p,
                                       c_void_p, c_void_p, c_void_p]),
    "ocm_vae_bottleneck_bwd": (c_i32, [c_void_p, c_i32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_i32,
                                       c_i32, c_void_p, c_void_p, c_void_p]),
    "ocm_vae_bottleneck_fwd_ld": (c_i32, [c_void_p, c_i32, c_void_p, c_void_p, c_i32, c_void_p, c_i32, c_i32,
                                          c_void_p, c_void_p, c_void_p, c_void_p]),
    "ocm_vae_bottleneck_bwd_ld": (c_i32, [c_void_p, c_i32, c_void_p, c_void_p, c_void_p, c_void_p, c_i32, c_void_p,
                                          c_i32, c_i32, c_void_p, c_void_p, c_void_p]),
    "ocm_vae_linear_act": (c_i32, [c_void_p, c_void_p, c_void_p, c_void_p, c_i32, c_i32, c_i32, c_void_p, c_void_p,
                                   c_void_p]),
    "ocm_bn_fused_timeouts": (c_i32, [ctypes.POINTER(c_i64)]),
    "ocm_vae_recon_fwd": (c_i32, [c_void_p, c_i32, c_void_p, c_i32, c_void_p, c_i32, c_i32, c_void_p, c_void_p,
                                  ctypes.c_float, c_void_p, ctypes.c_float, c_void_p, c_void_p, c_void_p, c_void_p]),
    "ocm_vae_recon_bwd": (c_i32, [c_void_p, c_void_p, c_void_p, c_i64, c_i32, c_void_p, ctypes.c_float, c_void_p,
                                  c_void_p]),
    "ocm_adam_step": (c_i32, [c_void_p, c_void_p, c_i32, c_i64, c_void_p, ctypes.c_float, ctypes.c_float,
                              ctypes.c_float, ctypes.c_float, ctypes.c_float, c_void_p, c_void_p]),
    "ocm_cast_multi": (c_i32, [c_void_p, c_i32, c_void_p, c_i32, c_void_p, c_i32, c_void_p, c_void_p]),
    "ocm_vae_standardise": (c_i32, [c_void_p, c_void_p, c_i32, c_i32, c_void_p, c_void_p, c_i32, c_void_p, c_void_p]),
    "ocm_eigh_f64": (c_i32, [c_void_p, c_void_p, c_i32, c_void_p, c_i32, c_void_p, c_void_p]),
    "ocm_prep_materialised": (c_i32, [c_void_p, ctypes.POINTER(c_i64)]),
    "ocm_eig_test_reruns": (c_i32, [c_void_p, ctypes.POINTER(c_i64)]),
    "ocm_vae_act_bias_bwd": (c_i32, [c_void_p, c_i32, c_void_p, c_void_p, c_i32, c_i32, c_void_p, c_void_p,
                                     c_void_p]),
    "ocm_gemm_bf16_sk_scratch_bytes": (ctypes.c_size_t, [c_i32, c_i32, c_i32]),
    "ocm_gemm_bf16_sk": (c_i32, [c_void_p, c_i32, c_void_p, c_void_p, c_void_p, c_i32, c_i32, c_i32, c_void_p,
                                 c_void_p, c_void_p]),
    "ocm_prep_rowstats_f32": (c_i32, [c_void_p, c_void_p, c_i64, c_i64, c_i32, c_void_p, c_void_p]),
    "ocm_prep_apply_f32": (c_i32, [c_void_p, c_void_p, c_i64, c_void_p, c_i64, c_i32, c_void_p, c_void_p, c_i64,
                                   c_void_p]),
    "ocm_colmean_f32_prep": (c_i32, [c_void_p, c_void_p, c_i64, c_void_p, c_i64, c_i32, c_void_p, c_void_p,
                                     c_void_p]),
    "ocm_gram_f32_prep": (c_i32, [c_void_p, c_void_p, c_i64, c_void_p, c_i64, c_i32, c_void_p,
                                  ctypes.POINTER(c_i64), c_i32, c_i32, c_i64, c_void_p, c_void_p, c_void_p,
                                  c_void_p]),
    "ocm_gram_f32_prep_write": (c_i32, [c_void_p, c_void_p, c_i64, c_i64, c_i32, c_void_p, ctypes.POINTER(c_i64),
                                        c_i32, c_i64, c_void_p, c_void_p, c_void_p, c_void_p, c_i64, c_void_p]),
    "ocm_score_f32_diag_prep": (c_i32, [c_void_p, c_void_p, c_i64, c_void_p, c_i64, c_i32, c_void_p, c_void_p,
                                        c_void_p, c_void_p, c_i32, c_void_p, c_void_p, c_void_p,
                                        ctypes.POINTER(OcmDecision), c_void_p, c_i64, c_void_p, c_void_p]),
}

ABI_VERSION = 12  # include/ocm.h OCM_ABI_VERSION
CSRC = os.path.join(os.path.dirname(_HERE), "csrc")


def source_build_id(csrc: str = CSRC) -> str | None:
    """The build id the Makefile derives from the library's inputs (the first
    16 hex digits of the SHA-256 of ID_INPUTS, concatenated in order), or None
    when the sources are not beside the package."""
    import hashlib
    import re

    mk = os.path.join(csrc, "Makefile")
    if not os.path.exists(mk):
        return None
    text = open(mk).read()
    srcs = re.search(r"^SRCS\s*:=\s*(.+)$", text, re.M).group(1).split()
    extra = re.search(r"^ID_INPUTS\s*:=\s*\$\(SRCS\)\s*(.+)$", text, re.M).group(1).split()
    h = hashlib.sha256()
    for f in srcs + extra:
        with open(os.path.join(csrc, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def file_build_id(path: str = LIB_PATH) -> str | None:
    """The build id compiled into a libocm.so, read from the file (no load)."""
    import re

    if not os.path.exists(path):
        return None
    with open(path, "rb") as fh:
        m = re.search(rb"ocm-build-id:([0-9a-f]{16})", fh.read())
    return m.group(1).decode() if m else None

_lib = None
_lib_lock = threading.Lock()


def load() -> ctypes.CDLL:
    """Load libocm.so (raises if it is missing: the product path has no fallback)."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise OcmError(f"libocm.so not found at {LIB_PATH}: build it with `make -C ocm-vae-simca_amd/csrc` "
                           "(or __graft_entry__.build()); there is no CPU fallback")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.ocm_abi_version() != ABI_VERSION:
            raise OcmError(f"libocm ABI version mismatch: {LIB_PATH} has {lib.ocm_abi_version()}, the binding "
                           f"expects {ABI_VERSION}; rebuild it (`make -C ocm-vae-simca_amd/csrc`)")
        want, have = source_build_id(), lib.ocm_build_id().decode()
        if want is not None and have != want:
            raise OcmError(f"{LIB_PATH} is stale: built from sources with id {have}, the sources beside it hash to "
                           f"{want}; rebuild it (`make -C ocm-vae-simca_amd/csrc -B`, or __graft_entry__.build())")
        _lib = lib
        return lib


def check(rc: int, what: str = ""):
    if rc == OCM_OK:
        return
    msg = load().ocm_last_error().decode(errors="replace")
    if rc == OCM_ERR_ARG:
        raise ValueError(f"{what}: {msg}")
    if rc == OCM_ERR_NOCONV:
        raise OcmNotConverged(f"{what}: {msg}")
    raise OcmError(f"{what}: rc={rc}: {msg}")


def ptr(t) -> int | None:
    """Device pointer of a torch tensor (None passes NULL)."""
    if t is None:
        return None
    return t.data_ptr()


class Context:
    """One libocm context per device (its workspace is stream-ordered)."""

    _ctxs: dict[int, "Context"] = {}

    def __init__(self, device: int):
        lib = load()
        h = c_void_p()
        check(lib.ocm_ctx_create(device, ctypes.byref(h)), "ocm_ctx_create")
        self.handle = h
        self.device = device

    @classmethod
    def get(cls, device: int | None = None) -> "Context":
        if device is None:
            device = torch.cuda.current_device()
        ctx = cls._ctxs.get(device)
        if ctx is None:
            ctx = cls._ctxs[device] = Context(device)
        return ctx

    KERNEL_GRAM = 0
    KERNEL_SCORE = 1

    def set_timing(self, enable: bool):
        check(load().ocm_ctx_set_timing(self.handle, 1 if enable else 0), "ocm_ctx_set_timing")

    def read_timing(self, kernel_id: int):
        """(total_ms, launches) of a timed kernel since the last read."""
        ms = c_f64(0.0)
        cnt = c_i64(0)
        check(load().ocm_ctx_read_timing(self.handle, kernel_id, ctypes.byref(ms), ctypes.byref(cnt)),
              "ocm_ctx_read_timing")
        return ms.value, cnt.value

    def __del__(self):
        try:
            if _lib is not None and getattr(self, "handle", None):
                _lib.ocm_ctx_destroy(self.handle)
        except Exception:
            pass


def stream_handle(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream
