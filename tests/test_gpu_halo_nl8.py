"""The halo kernel's 8-loader form (raft_conv2d_set_halo_loaders(8): 768-thread work-groups for the
one-tile f16x3 update convs) gives the 4-loader results bit for bit: every update-block conv shape at
one and two frame pairs (ragged tiles too), a raft_conv2d_pair, and a whole RAFT forward."""
import argparse

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.fixture
def loaders():
    from raft_optical_flow_amd import _lib
    lib = _lib.load()
    prev = lib.raft_conv2d_set_halo_loaders(0)
    prev_ks = lib.raft_conv2d_set_halo_ks(1)  # (the one-compute-wave form, whose loader count this varies)
    yield lib
    lib.raft_conv2d_set_halo_loaders(prev)
    lib.raft_conv2d_set_halo_ks(prev_ks)


def _run(lib, nl, pc, x, B, H, W, cout):
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    lib.raft_conv2d_set_halo_loaders(nl)
    out = K.Rows(torch.full((B * H * W, cout), 7.0, device=DEV))
    K.conv_launch(K.conv_params(pc, x, B, H, W, out, epilogue=_lib.EPI_RELU))(K.stream_handle())
    torch.cuda.synchronize()
    return out.t


@pytest.mark.parametrize("cin,cout,kh,kw", [(256, 192, 3, 3), (128, 64, 3, 3), (256, 126, 3, 3), (256, 256, 1, 5),
                                             (256, 128, 1, 5), (256, 256, 5, 1), (256, 128, 5, 1), (128, 256, 3, 3)])
@pytest.mark.parametrize("B,H,W", [(1, 55, 128), (2, 37, 61)])
def test_eight_loaders_equal_four(loaders, cin, cout, kh, kw, B, H, W):
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    g = torch.Generator().manual_seed(cin + cout + kh * 7 + H)
    x = K.Rows(K.nchw_to_rows(torch.randn(B, cin, H, W, generator=g).to(DEV)))
    w = torch.randn(cout, cin, kh, kw, generator=g) / np.sqrt(cin * kh * kw)
    pc = K.pack_conv(w, torch.randn(cout, generator=g), 1, ((kh - 1) // 2, (kw - 1) // 2), device=DEV)
    pc.precision = _lib.PREC_F16X3
    a = _run(loaders, 4, pc, x, B, H, W, cout)
    b = _run(loaders, 8, pc, x, B, H, W, cout)
    assert torch.equal(a, b)


def test_eight_loaders_forward(loaders):
    from raft_optical_flow_amd import RAFT
    from raft_optical_flow_amd.init import seeded_images, seeded_state_dict
    i1, i2 = seeded_images(1, 128, 192, seed=3)
    i1, i2 = i1.to(DEV), i2.to(DEV)
    outs = []
    for nl in (4, 8):
        loaders.raft_conv2d_set_halo_loaders(nl)
        m = RAFT(argparse.Namespace(small=False, mixed_precision=False, alternate_corr=False))
        m.load_state_dict(seeded_state_dict(m, 0))
        m.to(DEV).eval()
        with torch.no_grad():
            outs.append(m(i1, i2, iters=12, test_mode=True)[1])
        torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("cin,cout,B,H,W,in_norm", [(64, 64, 2, 61, 131, True), (64, 64, 2, 61, 131, False),
                                                    (96, 96, 2, 30, 70, True), (64, 64, 1, 9, 20, True)])
def test_encoder_eight_loaders_equal_four(monkeypatch, cin, cout, B, H, W, in_norm):
    """The encoders' 3x3 convs with 8 loader waves (default) and 4 (RAFT_HALO_NL8_ENC=0) -- with the loaders'
    input InstanceNorm and the epilogue's statistics partials, on multi-tile (several rounds) and one-tile grids
    -- give the same outputs and the same statistics bit for bit."""
    import ctypes
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    lib = _lib.load()
    g = torch.Generator().manual_seed(cin + H + W)
    x = torch.randn(B, cin, H, W, generator=g) * 2.0 + 0.5
    w = torch.randn(cout, cin, 3, 3, generator=g) / np.sqrt(cin * 9)
    b = torch.randn(cout, generator=g) * 0.1
    pc = K.pack_conv(w, b, 1, 1, device=DEV)
    pc.precision = _lib.PREC_F16X3
    src = K.Rows(K.nchw_to_rows(x.to(DEV)))
    mean = x.double().mean((2, 3))
    rstd = 1.0 / torch.sqrt(x.double().var((2, 3), unbiased=False) + 1e-5)
    st = torch.stack([mean, rstd], -1).float().contiguous().to(DEV)

    def run():
        out = K.Rows(torch.full((B * H * W, cout), 7.0, device=DEV))
        p = K.conv_params(pc, src, B, H, W, out)
        if in_norm:
            p.in_norm, p.in_norm_relu = st.data_ptr(), 1
            assert lib.raft_conv2d_in_norm_ok(ctypes.byref(p)) == 1
        slots = int(lib.raft_conv2d_stats_slots(ctypes.byref(p)))
        assert slots > 0
        part = torch.full((B * slots * cout * 4,), float("nan"), device=DEV)
        p.stats_part, p.stats_ld = part.data_ptr(), cout
        K.conv_launch(p)(K.stream_handle())
        torch.cuda.synchronize()
        return out.t.clone(), part.clone()

    monkeypatch.delenv("RAFT_HALO_NL8_ENC", raising=False)
    a_out, a_st = run()
    monkeypatch.setenv("RAFT_HALO_NL8_ENC", "0")
    b_out, b_st = run()
    assert torch.equal(a_out, b_out)
    assert torch.equal(a_st, b_st)
