"""GPU checks of the f16x3 correlation build (raft_corr_build_prec: corr_build2_kernel; CorrBlock.__init__ /
CorrBlock.corr, core/corr.py:25-54,96-127) beyond the oracle parity of test_gpu_parity.py: the work-group
-> tile order is a pure permutation, so every order gives the same pyramid bit for bit."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _build(f1, f2, ld, B, H, W, C, L):
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    pyr = torch.full((K.pyramid_floats(B, H, W, L),), float("nan"), device=DEV)
    _lib.call("raft_corr_build_prec", f1.data_ptr(), f2.data_ptr(), ld, B, H, W, C, L, K.sqrt_c(C),
              _lib.PREC_F16X3, pyr.data_ptr(), K.stream_handle())
    torch.cuda.synchronize()
    return pyr


@pytest.mark.parametrize("order", ["8,0,1", "1,1,0", "4,1,1", "3,0,0"])
def test_corr_build_tile_order_bit_identical(monkeypatch, order):
    """RAFT_CB_ORDER only permutes which work-group builds which tile: every order gives the same
    pyramid bit for bit (ragged tiles, B = 2, so the XCD runs straddle images)."""
    B, H, W, C, L = 2, 29, 70, 256, 4
    g = torch.Generator(device=DEV).manual_seed(7)
    f = torch.randn(2 * B * H * W, C, device=DEV, generator=g)
    f1, f2 = f[: B * H * W], f[B * H * W:]
    monkeypatch.delenv("RAFT_CB_ORDER", raising=False)
    ref = _build(f1, f2, C, B, H, W, C, L)
    monkeypatch.setenv("RAFT_CB_ORDER", order)
    got = _build(f1, f2, C, B, H, W, C, L)
    assert torch.equal(got, ref)
