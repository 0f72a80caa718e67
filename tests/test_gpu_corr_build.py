"""GPU parity of the workspace correlation build (raft_corr_build_ws: the f16 split of both maps once,
then corr_build3_kernel's LDS-DMA GEMM; CorrBlock.__init__ / CorrBlock.corr, core/corr.py:25-54,96-127).

It runs the products, summation order and epilogue of raft_corr_build_prec's f16x3 kernel, so every
level of the pyramid must be bit-identical to it (which test_gpu_parity.py pins to the oracle), over
ragged maps (partial M tiles and 8 x 16 blocks), channel counts that are not a multiple of the
32-channel K-step, a row stride past C, separate (non-adjacent) fmap tensors and 1-4 levels.
(The kernel is opt-in, RAFT_CORR_BUILD3=1; the forward's build otherwise runs corr_build2.)"""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _build(f1, f2, ld, B, H, W, C, L, ws):
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    pyr = torch.full((K.pyramid_floats(B, H, W, L),), float("nan"), device=DEV)
    if ws is None:
        _lib.call("raft_corr_build_prec", f1.data_ptr(), f2.data_ptr(), ld, B, H, W, C, L, K.sqrt_c(C),
                  _lib.PREC_F16X3, pyr.data_ptr(), K.stream_handle())
    else:
        _lib.call("raft_corr_build_ws", f1.data_ptr(), f2.data_ptr(), ld, B, H, W, C, L, K.sqrt_c(C),
                  _lib.PREC_F16X3, ws.data_ptr(), ws.numel() * 4, pyr.data_ptr(), K.stream_handle())
    torch.cuda.synchronize()
    return pyr


@pytest.mark.parametrize("B,H,W,C,ld,L,adjacent", [
    (1, 55, 128, 256, 256, 4, True),    # config 2's map
    (2, 13, 21, 256, 256, 4, True),     # ragged tiles, B = 2
    (1, 20, 37, 100, 100, 2, True),     # C not a multiple of 32
    (3, 9, 17, 64, 72, 3, False),       # row stride past C, separate tensors
    (1, 8, 16, 256, 256, 1, False),     # one 8 x 16 block, level 0 only
    (2, 47, 61, 128, 128, 4, True),
])
def test_corr_build_ws_bit_identical(monkeypatch, B, H, W, C, ld, L, adjacent):
    from raft_optical_flow_amd import _lib
    monkeypatch.setenv("RAFT_CORR_BUILD3", "1")
    g = torch.Generator(device=DEV).manual_seed(B * 1000 + H * 10 + C)
    P = B * H * W
    if adjacent:
        f = torch.randn(2 * P, ld, device=DEV, generator=g) * 2.0
        f1, f2 = f[:P], f[P:]
    else:
        f1 = torch.randn(P, ld, device=DEV, generator=g)
        f2 = torch.randn(P, ld, device=DEV, generator=g) * 3.0
    nbytes = int(_lib.load().raft_corr_build_ws_bytes(B, H, W, C))
    assert nbytes == 2 * P * ((C + 31) // 32) * 128
    ws = torch.full(((nbytes + 3) // 4,), float("nan"), device=DEV)
    ref = _build(f1, f2, ld, B, H, W, C, L, None)
    got = _build(f1, f2, ld, B, H, W, C, L, ws)
    assert not torch.isnan(got).any()
    assert torch.equal(got, ref)


def test_corr_build_ws_too_small_is_an_error():
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    B, H, W, C = 1, 8, 16, 64
    f = torch.randn(2 * B * H * W, C, device=DEV)
    pyr = torch.empty(K.pyramid_floats(B, H, W, 2), device=DEV)
    need = int(_lib.load().raft_corr_build_ws_bytes(B, H, W, C))
    ws = torch.empty(need // 4, device=DEV)
    rc = _lib.load().raft_corr_build_ws(ctypes.c_void_p(f.data_ptr()), ctypes.c_void_p(f[B * H * W:].data_ptr()), C,
                                        B, H, W, C, 2, K.sqrt_c(C), _lib.PREC_F16X3, ctypes.c_void_p(ws.data_ptr()),
                                        need - 16, ctypes.c_void_p(pyr.data_ptr()), ctypes.c_void_p(K.stream_handle()))
    assert rc != 0


def test_forward_corr_build3_bit_exact(monkeypatch):
    """RAFT-full at config 2's size: the forward with the pre-split LDS-DMA correlation build
    (RAFT_CORR_BUILD3=1) gives the flow of the default build bit for bit."""
    import argparse
    from raft_optical_flow_amd import RAFT
    from raft_optical_flow_amd.init import seeded_images, seeded_state_dict
    m = RAFT(argparse.Namespace(small=False, mixed_precision=False, alternate_corr=False))
    m.conv_precision = "f16x3"
    m.load_state_dict(seeded_state_dict(m, 0))
    m = m.to(DEV).eval()
    i1, i2 = seeded_images(1, 440, 1024, seed=4)
    i1, i2 = i1.to(DEV), i2.to(DEV)
    outs = []
    for v in ("0", "1"):
        monkeypatch.setenv("RAFT_CORR_BUILD3", v)
        with torch.no_grad():
            outs.append(m(i1, i2, iters=4, test_mode=True))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("order", ["8,0,1", "1,1,0", "4,1,1", "3,0,0"])
def test_corr_build_tile_order_bit_identical(monkeypatch, order):
    """RAFT_CB_ORDER only permutes which work-group builds which tile: every order gives the same
    pyramid bit for bit (ragged tiles, B = 2, so the XCD runs straddle images)."""
    B, H, W, C, L = 2, 29, 70, 256, 4
    g = torch.Generator(device=DEV).manual_seed(7)
    f = torch.randn(2 * B * H * W, C, device=DEV, generator=g)
    f1, f2 = f[: B * H * W], f[B * H * W:]
    monkeypatch.delenv("RAFT_CB_ORDER", raising=False)
    ref = _build(f1, f2, C, B, H, W, C, L, None)
    monkeypatch.setenv("RAFT_CB_ORDER", order)
    got = _build(f1, f2, C, B, H, W, C, L, None)
    assert torch.equal(got, ref)
