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


def _build_ws(f1, f2, ld, B, H, W, C, L, pad=None):
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    pyr = torch.full((K.pyramid_floats(B, H, W, L),), float("nan") if pad is None else pad, device=DEV)
    wsb = int(_lib.load().raft_corr_build_ws_bytes(B, H, W, C))
    ws = torch.full(((wsb + 3) // 4,), float("nan"), device=DEV)
    _lib.call("raft_corr_build_ws", f1.data_ptr(), f2.data_ptr(), ld, B, H, W, C, L, K.sqrt_c(C), _lib.PREC_F16X3,
              pyr.data_ptr(), ws.data_ptr(), wsb, K.stream_handle())
    torch.cuda.synchronize()
    return pyr


@pytest.mark.parametrize("B,H,W,C,L,ld", [
    (1, 55, 128, 256, 4, 256),   # config 2's map: 28 query tiles x 32 target tiles
    (2, 37, 53, 256, 4, 256),    # ragged target blocks, odd sizes (level-1 padding rows / columns)
    (1, 20, 36, 96, 2, 100),     # C = 96 (6 half-steps), ld > C, H = 20 (level-1 tile rows past H / 2)
    (3, 9, 70, 64, 1, 64),       # one level only (no level-1 stores), 4 half-steps
])
def test_corr_build_ws_vs_fp64(B, H, W, C, L, ld):
    """raft_corr_build_ws (split maps + corr_build4_kernel: 256 x 256 tiles, one accumulator chain,
    stores from registers): every level within 1e-5 of its scale of fp64 (the oracle's algorithm,
    core/corr.py:25-54, 96-127), padding zeros written (the buffer starts as NaN), level 1 the
    exact avg_pool2d of the kernel's own level 0."""
    import numpy as np
    from oracle import raft_oracle as O
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    g = torch.Generator().manual_seed(B * H + W)
    x1 = torch.randn(B, C, H, W, generator=g)
    x2 = torch.randn(B, C, H, W, generator=g)
    r1 = torch.zeros(B * H * W, ld)
    r2 = torch.zeros(B * H * W, ld)
    r1[:, :C] = x1.permute(0, 2, 3, 1).reshape(-1, C)
    r2[:, :C] = x2.permute(0, 2, 3, 1).reshape(-1, C)
    r1, r2 = r1.to(DEV), r2.to(DEV)
    pyr = _build_ws(r1, r2, ld, B, H, W, C, L)
    assert not bool(torch.isnan(pyr).any()), "a pyramid element was not written"
    ref = O.corr_pyramid(x1.double().numpy(), x2.double().numpy(), L)
    dims = K.pyramid_dims(H, W, L)
    levels = []
    for i, (lh, lw) in enumerate(dims):
        out = torch.empty(B * H * W, lh, lw, device=DEV)
        _lib.call("raft_corr_pyramid_level", pyr.data_ptr(), B, H, W, L, i, out.data_ptr(), K.stream_handle())
        levels.append(out.cpu())
        scale = max(1.0, float(np.abs(ref[i]).max()))
        assert float(np.abs(out.cpu().double().numpy().reshape(ref[i].shape) - ref[i]).max()) < 1e-5 * scale, i
    if L > 1:
        l0 = levels[0]
        h1, w1 = dims[1]
        a = l0[:, 0:2 * h1:2, 0:2 * w1:2] + l0[:, 0:2 * h1:2, 1:2 * w1:2]
        a = (a + l0[:, 1:2 * h1:2, 0:2 * w1:2]) + l0[:, 1:2 * h1:2, 1:2 * w1:2]
        assert torch.equal(levels[1], a / 4.0)
    if L > 2:
        # level 2 (pooled in the build's registers since round 5): the exact avg_pool2d of level 1
        l1 = levels[1]
        h2, w2 = dims[2]
        a = l1[:, 0:2 * h2:2, 0:2 * w2:2] + l1[:, 0:2 * h2:2, 1:2 * w2:2]
        a = (a + l1[:, 1:2 * h2:2, 0:2 * w2:2]) + l1[:, 1:2 * h2:2, 1:2 * w2:2]
        assert torch.equal(levels[2], a / 4.0)


def test_corr_build_ws_matches_the_plain_build():
    """The workspace build and raft_corr_build_prec(F16X3) agree to the split's accuracy (different
    accumulation orders of the same products), and the workspace build is run to run bit-identical."""
    from raft_optical_flow_amd import _lib
    B, H, W, C, L = 1, 55, 128, 256, 4
    g = torch.Generator(device=DEV).manual_seed(3)
    f = torch.randn(2 * B * H * W, C, device=DEV, generator=g)
    f1, f2 = f[: B * H * W], f[B * H * W:]
    a = _build_ws(f1, f2, C, B, H, W, C, L)
    b = _build(f1, f2, C, B, H, W, C, L)
    assert float((a - b).abs().max()) < 1e-5 * max(1.0, float(b.abs().max()))
    assert torch.equal(_build_ws(f1, f2, C, B, H, W, C, L, pad=0.0), a)
    assert _lib.load().raft_corr_build_ws_bytes(B, H, W, C) == 2 * B * H * W * C * 4 + 4096


def test_corr_build_ws_without_workspace_falls_back():
    """raft_corr_build_ws with ws == NULL (ws_bytes 0), or with an operand off 16-B alignment, takes
    raft_corr_build_prec: the same pyramid bit for bit (argument order: ..., pyramid, ws, ws_bytes,
    stream)."""
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    B, H, W, C, L = 1, 24, 40, 128, 4
    g = torch.Generator(device=DEV).manual_seed(4)
    f = torch.randn(2 * B * H * W, C, device=DEV, generator=g)
    f1, f2 = f[: B * H * W], f[B * H * W:]
    n = int(_lib.load().raft_corr_pyramid_floats(B, H, W, L))
    ref = torch.zeros(n, device=DEV)  # (tile padding the builds may leave unwritten: zeros in all three)
    _lib.call("raft_corr_build_prec", f1.data_ptr(), f2.data_ptr(), C, B, H, W, C, L, K.sqrt_c(C), _lib.PREC_F16X3,
              ref.data_ptr(), K.stream_handle())
    out = torch.zeros(n, device=DEV)
    _lib.call("raft_corr_build_ws", f1.data_ptr(), f2.data_ptr(), C, B, H, W, C, L, K.sqrt_c(C), _lib.PREC_F16X3,
              out.data_ptr(), None, 0, K.stream_handle())
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    # a workspace off 16-B alignment: the same fallback
    wsb = int(_lib.load().raft_corr_build_ws_bytes(B, H, W, C))
    ws = torch.empty(wsb // 4 + 8, device=DEV)
    out2 = torch.zeros(n, device=DEV)
    _lib.call("raft_corr_build_ws", f1.data_ptr(), f2.data_ptr(), C, B, H, W, C, L, K.sqrt_c(C), _lib.PREC_F16X3,
              out2.data_ptr(), ws.data_ptr() + 4, wsb, K.stream_handle())
    torch.cuda.synchronize()
    assert torch.equal(out2, ref)


@pytest.mark.parametrize("B,H,W,C,L", [(1, 55, 128, 256, 4), (2, 37, 53, 256, 2), (3, 9, 70, 64, 1)])
def test_corr_build_w4_equals_default(monkeypatch, B, H, W, C, L):
    """The opt-in 4-wave correlation build (RAFT_CB4_W4=1: two work-groups per CU, 256 targets x 128 queries
    per unit, level 2 pooled in registers where L > 2) writes the same pyramid as the default 8-wave build
    bit for bit (each query's sums run the same K walk), for L = 1, 2 and 4."""
    g = torch.Generator(device=DEV).manual_seed(B * 100 + L)
    f = torch.randn(2 * B * H * W, C, device=DEV, generator=g)
    f1, f2 = f[: B * H * W], f[B * H * W:]
    monkeypatch.delenv("RAFT_CB4_W4", raising=False)
    ref = _build_ws(f1, f2, C, B, H, W, C, L, pad=0.0)
    monkeypatch.setenv("RAFT_CB4_W4", "1")
    got = _build_ws(f1, f2, C, B, H, W, C, L, pad=0.0)
    assert torch.equal(got, ref)


def test_corr_build_ws_bytes_prec_is_the_librarys_rule(monkeypatch):
    """raft_corr_build_ws_bytes_prec: the workspace where raft_corr_build_ws takes the 256 x 256 kernel, 0 where
    it falls back (so callers do not restate the rule)."""
    from raft_optical_flow_amd import _lib
    lib = _lib.load()
    assert lib.raft_corr_build_ws_bytes_prec(1, 55, 128, 256, _lib.PREC_F16X3) == lib.raft_corr_build_ws_bytes(1, 55, 128, 256)
    assert lib.raft_corr_build_ws_bytes_prec(1, 55, 128, 256, _lib.PREC_FP32) == 0
    assert lib.raft_corr_build_ws_bytes_prec(1, 55, 128, 72, _lib.PREC_F16X3) == 0     # C % 16
    assert lib.raft_corr_build_ws_bytes_prec(1, 55, 128, 48, _lib.PREC_F16X3) == 0     # C < 64
    monkeypatch.setenv("RAFT_CORR_BUILD4", "0")
    assert lib.raft_corr_build_ws_bytes_prec(1, 55, 128, 256, _lib.PREC_F16X3) == 0
