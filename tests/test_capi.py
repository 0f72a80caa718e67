"""The C-ABI library loads and exports every entry point include/raft_hip.h declares
(no compute calls: runs without a GPU)."""
import ctypes
import os
import re

import pytest

from conftest import REPO
from raft_optical_flow_amd import _lib

HEADER = os.path.join(REPO, "include", "raft_hip.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\**\s+\**(raft_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("raft_alt_corr_forward", "raft_alt_corr_backward", "raft_corr_build", "raft_corr_lookup",
                 "raft_conv2d", "raft_convex_upsample", "raft_hip_abi_version"):
        assert must in names


def test_library_exports_every_declared_symbol():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail(f"{_lib.LIB_PATH} not built (run python __graft_entry__.py build)")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    # the ctypes prototype table covers the same set
    assert sorted(_lib.EXPORTED) == declared_functions()


def test_abi_queries_without_gpu():
    lib = _lib.load()
    assert lib.raft_hip_abi_version() == _lib.ABI_VERSION == 18
    # the library was built from the sources beside it (csrc/Makefile SRC_HASH)
    assert lib.raft_hip_source_hash().decode() == _lib.source_hash()
    assert lib.raft_hip_arch() == b"gfx950"
    # size queries are pure host arithmetic
    assert lib.raft_corr_pyramid_floats(1, 55, 128, 4) == 7040 * 16 * (14 * 32 + 7 * 16 + 4 * 8 + 2 * 4)
    n, k = ctypes.c_int(), ctypes.c_int()
    assert lib.raft_conv2d_packed_shape(0, 126, 3, 3, 256, ctypes.byref(n), ctypes.byref(k)) == 0
    assert (n.value, k.value) == (128, 9 * 256)
    assert lib.raft_conv2d_packed_shape(1, 128, 7, 7, 2, ctypes.byref(n), ctypes.byref(k)) == 0
    assert (n.value, k.value) == (128, 128)


def test_argument_errors_are_reported_without_launch():
    lib = _lib.load()
    rc = lib.raft_corr_lookup(None, 1, 8, 8, 4, 4, None, 0, None, 0, 0, None, 0, None, None)
    assert rc == -1
    assert b"null" in lib.raft_hip_last_error()
    rc = lib.raft_corr_build(16, 16, 256, 1, 8, 8, 102, 4, 10.0, 16, None)  # C % 4 != 0
    assert rc == -1 and b"multiple of 4" in lib.raft_hip_last_error()
    rc = lib.raft_instnorm_merge_fused(None, 4, 1, 64, 64, 1e-5, None, None, None, None)
    assert rc == -1 and b"bad arguments" in lib.raft_hip_last_error()
    assert lib.raft_instnorm_merge_counters(2, 96) == 4 and lib.raft_instnorm_merge_counters(0, 64) == 0
    rc = lib.raft_conv2d_pair(None, None, None)
    assert rc == -1 and b"null params" in lib.raft_hip_last_error()
    # the fused lookup + convf1 checks its convf1 arguments before any launch
    rc = lib.raft_corr_lookup_convf1(16, 1, 8, 8, 4, 4, 16, 0, 16, 324, 0, None, 0, None, 16, None, 128, 5, 0, 16,
                                     128, None, None)
    assert rc == -1 and b"kernel size must be 7" in lib.raft_hip_last_error()
    rc = lib.raft_corr_lookup_convf1(16, 1, 8, 8, 4, 4, 16, 0, 16, 324, 0, None, 0, None, 16, None, 80, 7, 0, 16,
                                     128, None, None)
    assert rc == -1 and b"multiple of 32" in lib.raft_hip_last_error()
    rc = lib.raft_convf1_flow(16, 0, 1, 8, 8, 16, None, 128, 5, 0, 16, 128, None, None)
    assert rc == -1 and b"kernel size must be 7" in lib.raft_hip_last_error()


def test_halo_tile_rule_host_side():
    """The halo kernel's tile choice (raft_conv2d_halo_tile_rows: host logic only, no launch): the
    rounds rule takes the 256-pixel tiles only where ceil(T_big / CUs) * 1.8 < ceil(T_128 / CUs)
    (256 CUs without a device): a frame pair's update convs and config 5's 1/8-res convs keep the
    128-pixel tiles, fnet layer2 at config 2 and convc2 at B = 8 take the big ones."""
    import ctypes
    import torch
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    lib = _lib.load()
    fake = 1 << 20  # 16-byte aligned stand-in pointers: the query never dereferences them

    def rows(cin, cout, kh, kw, B, H, W, prec="f16x3", scaled=True):
        pc = K.pack_conv(torch.zeros(cout, cin, kh, kw), None, 1, ((kh - 1) // 2, (kw - 1) // 2))
        p = _lib.ConvParams()
        p.in0, p.in0_ld, p.in0_c = fake, cin, cin
        p.batch, p.in_h, p.in_w, p.out_h, p.out_w = B, H, W, H, W
        p.kh, p.kw, p.stride_h, p.stride_w, p.pad_h, p.pad_w = kh, kw, 1, 1, (kh - 1) // 2, (kw - 1) // 2
        p.mode, p.weight, p.n, p.out, p.out_ld = pc.mode, fake, cout, fake, cout
        p.precision = _lib.PRECISIONS[prec]
        p.weight_s = fake if (scaled and prec == "f16x3") else None
        return lib.raft_conv2d_halo_tile_rows(ctypes.byref(p))

    assert rows(256, 192, 3, 3, 1, 55, 128) == 8          # config 2 convc2 (B = 1)
    assert rows(96, 96, 3, 3, 2, 110, 256) == 16          # fnet layer2 at config 2
    assert rows(256, 192, 3, 3, 8, 55, 128) == 16         # convc2 at B = 8
    assert rows(256, 192, 3, 3, 8, 55, 128, scaled=False) == 8   # f16x3 without the scaled weight
    assert rows(128, 256, 3, 3, 8, 68, 120) == 8          # config 4's fh1: 5 vs 9 rounds
    assert rows(256, 128, 3, 3, 1, 135, 240, "bf16") == 8  # config 5's conv (bf16): 2 vs 2 rounds
    assert rows(256, 128, 1, 5, 8, 55, 128) == 16         # q (1x5) at B = 8
    assert rows(64, 64, 3, 3, 1, 16, 16) == 8


def test_halo_tiles_per_work_group_host_side():
    """Spatial tiles per work-group of the halo launch (raft_conv2d_halo_tiles_per_wg: host logic
    only): the m of least rounds x (1 + 0.8 (m - 1)) tile times over 256 CUs, where padding each
    tile's K loop to lcm(U, T) K-steps costs at most 1/8."""
    import ctypes
    import torch
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    lib = _lib.load()
    fake = 1 << 20

    def mt(cin, cout, kh, kw, B, H, W, prec="f16x3"):
        pc = K.pack_conv(torch.zeros(cout, cin, kh, kw), None, 1, ((kh - 1) // 2, (kw - 1) // 2))
        p = _lib.ConvParams()
        p.in0, p.in0_ld, p.in0_c = fake, cin, cin
        p.batch, p.in_h, p.in_w, p.out_h, p.out_w = B, H, W, H, W
        p.kh, p.kw, p.stride_h, p.stride_w, p.pad_h, p.pad_w = kh, kw, 1, 1, (kh - 1) // 2, (kw - 1) // 2
        p.mode, p.weight, p.n, p.out, p.out_ld = pc.mode, fake, cout, fake, cout
        p.precision = _lib.PRECISIONS[prec]
        p.weight_s = fake if prec == "f16x3" else None
        return lib.raft_conv2d_halo_tiles_per_wg(ctypes.byref(p))

    assert mt(256, 192, 3, 3, 1, 55, 128) == 1        # a frame pair's convc2: one round
    assert mt(64, 64, 3, 3, 2, 220, 512) == 7         # fnet layer1 at config 2: 1792 tiles
    assert mt(96, 96, 3, 3, 2, 110, 256) == 1         # 3 chunks of 9 taps: 27 -> 36 K-steps, too much padding
    assert mt(128, 128, 3, 3, 2, 55, 128) == 1        # fnet layer3 at config 2: 224 tiles, one round
    assert mt(256, 192, 3, 3, 8, 55, 128) == 1        # convc2 at B = 8: 3 rounds of big tiles beat 4 per work-group
    assert mt(256, 192, 3, 3, 1, 135, 240) == 3       # config 5's convc2: 255 spatial tiles x 3 N-tiles
    assert mt(128, 256, 3, 3, 8, 68, 120) == 9        # config 4's fh1: 576 spatial tiles x 4 N-tiles


def test_stats_slots_host_side():
    """InstanceNorm statistics slots per image (raft_conv2d_stats_slots: host logic only): 4 per
    spatial tile on the halo kernel; on the 64x64-tile GEMM (the strided encoder convs, round 5) two
    per 64-row tile of one image's output rows; none for a non-linear epilogue."""
    import ctypes
    import torch
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    lib = _lib.load()
    fake = 1 << 20

    def slots(cin, cout, k, stride, B, H, W, epilogue=None):
        pad = (k - 1) // 2
        pc = K.pack_conv(torch.zeros(cout, cin, k, k), None, stride, pad)
        p = _lib.ConvParams()
        p.in0, p.in0_ld, p.in0_c = fake, cin, cin
        ho, wo = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
        p.batch, p.in_h, p.in_w, p.out_h, p.out_w = B, H, W, ho, wo
        p.kh, p.kw, p.stride_h, p.stride_w, p.pad_h, p.pad_w = k, k, stride, stride, pad, pad
        p.mode, p.weight, p.n, p.out, p.out_ld = pc.mode, fake, cout, fake, cout
        p.precision = _lib.PRECISIONS["f16x3"]
        p.alpha = 1.0
        if epilogue is not None:
            p.epilogue = epilogue
        return lib.raft_conv2d_stats_slots(ctypes.byref(p)), ho * wo

    s, hw = slots(64, 96, 3, 2, 2, 220, 512)           # fnet layer2's strided conv at config 2
    assert s == 2 * ((hw + 63) // 64)
    s, hw = slots(64, 96, 1, 2, 2, 220, 512)           # its 1x1 downsample
    assert s == 2 * ((hw + 63) // 64)
    s, hw = slots(96, 128, 3, 2, 3, 9, 11)             # 30 output rows per image: one tile each
    assert s == 2
    assert slots(64, 96, 3, 2, 2, 220, 512, epilogue=_lib.EPI_RELU)[0] == 0


def test_corr_build_ws_bytes_prec_host_side():
    """raft_corr_build_ws_bytes_prec (host logic only): the 256 x 256 correlation build's workspace where
    raft_corr_build_ws takes that kernel (f16x3, C % 16 == 0, 64 <= C <= 1024), 0 where it falls back."""
    from raft_optical_flow_amd import _lib
    lib = _lib.load()
    full = lib.raft_corr_build_ws_bytes(1, 55, 128, 256)
    assert full > 0
    assert lib.raft_corr_build_ws_bytes_prec(1, 55, 128, 256, _lib.PREC_F16X3) == full
    for prec in (_lib.PREC_FP32, _lib.PREC_F16, _lib.PREC_BF16):
        assert lib.raft_corr_build_ws_bytes_prec(1, 55, 128, 256, prec) == 0
    assert lib.raft_corr_build_ws_bytes_prec(1, 55, 128, 72, _lib.PREC_F16X3) == 0
    assert lib.raft_corr_build_ws_bytes_prec(1, 55, 128, 48, _lib.PREC_F16X3) == 0
