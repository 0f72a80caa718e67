"""ctypes binding of libraft_hip.so (the C-ABI declared in include/raft_hip.h).

The library is built in-tree by `python __graft_entry__.py build` (or
`make -C raft_optical_flow_amd/csrc`).  There is no fallback: if the library
is missing or fails to load, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RAFT_HIP_LIB") or os.path.join(_HERE, "libraft_hip.so")

c_int = ctypes.c_int
c_float = ctypes.c_float
c_size_t = ctypes.c_size_t
c_void_p = ctypes.c_void_p
c_char_p = ctypes.c_char_p
P = c_void_p  # device pointers are passed as integers / void*

RAFT_CONV_VEC = 0
RAFT_CONV_GATHER = 1

PREC_FP32 = 0    # v_mfma_f32_32x32x2_f32
PREC_F16X3 = 1   # fp32-accurate hi/lo f16 split on v_mfma_f32_32x32x16_f16
PREC_F16 = 2     # single f16 product (mixed precision)
PREC_BF16 = 3    # single bf16 product on v_mfma_f32_32x32x16_bf16 (bf16 mixed precision)
PRECISIONS = {"fp32": PREC_FP32, "f16x3": PREC_F16X3, "f16": PREC_F16, "bf16": PREC_BF16}

ABI_VERSION = 18
RANGE_LIMIT = 32768.0  # RAFT_RANGE_LIMIT: |x| above it raises the f16x3 range guard

EPI_LINEAR = 0
EPI_RELU = 1
EPI_RESID_RELU = 2
EPI_GRU_ZR = 3
EPI_GRU_Q = 4
EPI_TANH_RELU = 5
EPI_ADD_TO_OUT = 6


class ConvParams(ctypes.Structure):
    """Mirror of `raft_conv2d_params` (include/raft_hip.h)."""

    _fields_ = [
        ("in0", P), ("in0_ld", c_int), ("in0_c", c_int),
        ("in1", P), ("in1_ld", c_int), ("in1_c", c_int),
        ("batch", c_int), ("in_h", c_int), ("in_w", c_int),
        ("out_h", c_int), ("out_w", c_int),
        ("kh", c_int), ("kw", c_int), ("stride_h", c_int), ("stride_w", c_int), ("pad_h", c_int), ("pad_w", c_int),
        ("mode", c_int),
        ("weight", P), ("bias", P),
        ("n", c_int),
        ("out", P), ("out_ld", c_int),
        ("epilogue", c_int), ("alpha", c_float), ("split", c_int),
        ("aux0", P), ("aux0_ld", c_int),
        ("aux1", P), ("aux1_ld", c_int),
        ("out1", P), ("out1_ld", c_int),
        ("add0", P), ("add0_ld", c_int),
        ("precision", c_int),
        ("range_flag", P),
        ("stats_part", P), ("stats_ld", c_int),
        ("in_norm", P), ("in_norm_relu", c_int),
        ("weight_s", P),
    ]


# name -> (restype, argtypes)
_PROTOS = {
    "raft_hip_abi_version": (c_int, []),
    "raft_hip_arch": (c_char_p, []),
    "raft_hip_last_error": (c_char_p, []),
    "raft_hip_source_hash": (c_char_p, []),
    "raft_debug_fill_lds_nan": (c_int, [P]),
    "raft_corr_pyramid_floats": (c_size_t, [c_int, c_int, c_int, c_int]),
    "raft_corr_build": (c_int, [P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_float, P, P]),
    "raft_corr_build_prec": (c_int, [P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_int, P, P]),
    "raft_corr_build_ws_bytes": (c_size_t, [c_int, c_int, c_int, c_int]),
    "raft_corr_build_ws_bytes_prec": (c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    "raft_corr_build_ws": (c_int, [P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_int, P, P, c_size_t, P]),
    "raft_corr_pyramid_level": (c_int, [P, c_int, c_int, c_int, c_int, c_int, P, P]),
    "raft_corr_lookup": (c_int, [P, c_int, c_int, c_int, c_int, c_int, P, c_int, P, c_int, c_int, P, c_int, P, P]),
    "raft_corr_lookup_convf1": (c_int, [P, c_int, c_int, c_int, c_int, c_int, P, c_int, P, c_int, c_int, P, c_int, P,
                                        P, P, c_int, c_int, c_int, P, c_int, P, P]),
    "raft_convf1_flow": (c_int, [P, c_int, c_int, c_int, c_int, P, P, c_int, c_int, c_int, P, c_int, P, P]),
    "raft_corr_lookup_conv": (c_int, [P, c_int, c_int, c_int, c_int, c_int, P, P, c_int, P, c_int, P, P, c_int, P,
                                      c_int, P, P, P, c_int, c_int, P, c_int, P, P]),
    "raft_lookup_conv_weight_floats": (c_size_t, [c_int, c_int]),
    "raft_lookup_conv_pack_weight": (c_int, [P, c_int, c_int, c_int, P, P]),
    "raft_alt_corr_forward": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_float, P]),
    "raft_alt_corr_forward_prec": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_float,
                                           c_int, P]),
    "raft_alt_corr_lookup_levels_prec": (c_int, [P, P, P, P, c_int, P, c_int, P, c_int, c_int, c_int, c_int, c_int,
                                                 c_int, ctypes.c_float, P, c_int, P, c_int, P]),
    "raft_alt_corr_lookup_nhwc_prec": (c_int, [P, P, P, c_int, c_float, P, c_int, c_int, c_int, c_int, c_int, c_int,
                                               c_int, c_int, c_float, P, c_int, P, c_int, P]),
    "raft_alt_corr_lookup_levels": (c_int, [P, P, P, P, c_int, P, c_int, P, c_int, c_int, c_int, c_int, c_int, c_int,
                                            ctypes.c_float, P, c_int, P, P]),
    "raft_alt_corr_lookup_nhwc": (c_int, [P, P, P, c_int, c_float, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                          c_int, c_float, P, c_int, P, P]),
    "raft_alt_corr_backward": (c_int, [P, P, P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                       P, c_size_t, P]),
    "raft_alt_corr_backward_workspace_floats": (c_size_t, [c_int] * 8),
    "raft_avgpool2_nhwc": (c_int, [P, P, c_int, c_int, c_int, c_int, P]),
    "raft_conv2d_packed_shape": (c_int, [c_int, c_int, c_int, c_int, c_int, ctypes.POINTER(c_int),
                                         ctypes.POINTER(c_int)]),
    "raft_conv2d": (c_int, [ctypes.POINTER(ConvParams), P]),
    "raft_conv2d_pair": (c_int, [ctypes.POINTER(ConvParams), ctypes.POINTER(ConvParams), P]),
    "raft_conv2d_stats_slots": (c_int, [ctypes.POINTER(ConvParams)]),
    "raft_conv2d_halo_tile_rows": (c_int, [ctypes.POINTER(ConvParams)]),
    "raft_conv2d_halo_tiles_per_wg": (c_int, [ctypes.POINTER(ConvParams)]),
    "raft_debug_launch_span": (c_int, [c_int]),
    "raft_debug_launch_span_read": (c_int, [P, c_int]),
    "raft_conv2d_in_norm_ok": (c_int, [ctypes.POINTER(ConvParams)]),
    "raft_instnorm_merge": (c_int, [P, c_int, c_int, c_int, c_int, c_float, P, P]),
    "raft_instnorm_merge_ws_floats": (c_size_t, [c_int, c_int, c_int]),
    "raft_instnorm_merge_ws": (c_int, [P, c_int, c_int, c_int, c_int, c_float, P, P, P]),
    "raft_instnorm_merge_counters": (c_size_t, [c_int, c_int]),
    "raft_conv2d_set_halo_loaders": (c_int, [c_int]),
    "raft_conv2d_set_halo_ks": (c_int, [c_int]),
    "raft_instnorm_merge_fused": (c_int, [P, c_int, c_int, c_int, c_int, c_float, P, P, P, P]),
    "raft_conv2d_split_weight": (c_int, [P, P, c_int, c_int, P]),
    "raft_conv2d_split_weight_prec": (c_int, [P, P, c_int, c_int, c_int, P]),
    "raft_conv2d_split_scaled_bytes": (c_size_t, [c_int, c_int]),
    "raft_conv2d_split_weight_scaled": (c_int, [P, P, c_int, c_int, P]),
    "raft_instnorm_workspace_floats": (c_size_t, [c_int, c_int, c_int]),
    "raft_instnorm_stats": (c_int, [P, c_int, c_int, c_int, c_int, c_float, P, P, P]),
    "raft_groupnorm_stats": (c_int, [P, c_int, c_int, c_int, c_int, c_int, c_float, P, P]),
    "raft_norm_apply_affine": (c_int, [P, c_int, P, P, P, P, c_int, P, P, P, c_int, P, c_int, c_int, c_int, c_int, P]),
    "raft_instnorm_apply": (c_int, [P, c_int, P, P, c_int, P, c_int, P, c_int, c_int, c_int, c_int, P]),
    "raft_prep_images": (c_int, [P, P, P, c_int, c_int, c_int, P]),
    "raft_init_coords": (c_int, [P, P, c_int, c_int, c_int, P]),
    "raft_flow_from_coords": (c_int, [P, P, c_int, c_int, c_int, P]),
    "raft_convex_upsample": (c_int, [P, P, c_int, P, c_int, c_int, c_int, P]),
    "raft_upflow8": (c_int, [P, P, c_int, c_int, c_int, P]),
    "raft_nchw_to_nhwc": (c_int, [P, P, c_int, c_int, c_int, c_int, c_int, P]),
    "raft_nhwc_to_nchw": (c_int, [P, c_int, P, c_int, c_int, c_int, c_int, P]),
    "raft_pad_replicate": (c_int, [P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, P]),
    "raft_bilinear_sample": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, P]),
    "raft_forward_interpolate": (c_int, [P, P, c_int, c_int, c_int, P]),
}

EXPORTED = tuple(_PROTOS)

_lib = None
_lock = threading.Lock()


class RaftHipError(RuntimeError):
    pass


def load():
    """Load libraft_hip.so (once).  Raises RaftHipError if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RaftHipError(
                f"libraft_hip.so not found at {LIB_PATH}: build it with `python __graft_entry__.py build` "
                "(there is no CPU fallback)")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _PROTOS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.raft_hip_abi_version() != ABI_VERSION:
            raise RaftHipError("libraft_hip.so ABI version mismatch")
        want = source_hash()
        got = lib.raft_hip_source_hash().decode()
        if want is not None and got != want and os.environ.get("RAFT_SKIP_SRC_CHECK", "0") != "1":
            raise RaftHipError(f"{LIB_PATH} was built from other sources (hash {got}, the sources here hash "
                               f"{want}; the hash covers csrc/*.hip, csrc/*.hpp and include/raft_hip.h): rebuild it "
                               f"with `python __graft_entry__.py build`, or set RAFT_SKIP_SRC_CHECK=1 to load it anyway")
        _lib = lib
        return lib


def source_hash() -> str | None:
    """sha256[:16] of the HIP sources beside this package, as csrc/Makefile bakes into the library
    (raft_hip_source_hash); None when the sources are not present."""
    import glob
    import hashlib
    csrc = os.path.join(_HERE, "csrc")
    mk = os.path.join(csrc, "Makefile")
    hdr = os.path.join(os.path.dirname(_HERE), "include", "raft_hip.h")
    if not (os.path.exists(mk) and os.path.exists(hdr)):
        return None
    with open(mk) as fh:
        srcs = next((ln.split(":=", 1)[1].split() for ln in fh if ln.startswith("SRCS :=")), None)
    if not srcs:
        raise RaftHipError(f"{mk} has no one-line 'SRCS := ...' list: cannot hash the HIP sources to check "
                           f"{LIB_PATH} against them (RAFT_SKIP_SRC_CHECK=1 skips the check)")
    files = [os.path.join(csrc, f) for f in srcs] + sorted(glob.glob(os.path.join(csrc, "*.hpp"))) + [hdr]
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def check(rc: int, what: str):
    if rc != 0:
        msg = _lib.raft_hip_last_error().decode(errors="replace") if _lib is not None else ""
        raise RaftHipError(f"{what} failed (rc={rc}): {msg}")


def call(name: str, *args):
    lib = load()
    rc = getattr(lib, name)(*args)
    check(rc, name)
    return rc
