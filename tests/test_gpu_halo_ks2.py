"""The halo kernel's K-split form (raft_conv2d_set_halo_ks(2), the default for the one-tile f16x3 update convs
with 64-column tiles): two compute waves per SIMD take the even / odd K-steps of one 32 x 64 block and meet in
LDS.  Against torch fp64 at the conv tolerance, against the one-compute-wave form within fp32 rounding (the
K-steps are summed in another order), run to run bit for bit, through every GRU epilogue (a whole forward), and
for ragged / multi-image shapes."""
import argparse

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.fixture
def ks():
    from raft_optical_flow_amd import _lib
    lib = _lib.load()
    prev = lib.raft_conv2d_set_halo_ks(0)  # (query)
    yield lib
    lib.raft_conv2d_set_halo_ks(prev)


def _run(lib, k, pc, x, B, H, W, cout, epi):
    from raft_optical_flow_amd import kernels as K
    lib.raft_conv2d_set_halo_ks(k)
    out = K.Rows(torch.full((B * H * W, cout), 7.0, device=DEV))
    K.conv_launch(K.conv_params(pc, x, B, H, W, out, epilogue=epi))(K.stream_handle())
    torch.cuda.synchronize()
    return out


def test_default_is_the_k_split_form(ks):
    assert ks.raft_conv2d_set_halo_ks(0) == 2


@pytest.mark.parametrize("cin,cout,kh,kw", [(256, 192, 3, 3), (256, 256, 1, 5), (256, 256, 5, 1), (128, 256, 3, 3),
                                             (96, 64, 3, 3), (384, 128, 1, 5)])
@pytest.mark.parametrize("B,H,W", [(1, 55, 128), (2, 37, 61), (1, 9, 19)])
def test_k_split_vs_fp64_and_one_wave(ks, cin, cout, kh, kw, B, H, W):
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    g = torch.Generator().manual_seed(cin + cout + kh * 7 + H)
    xn = torch.randn(B, cin, H, W, generator=g)
    x = K.Rows(K.nchw_to_rows(xn.to(DEV)))
    w = torch.randn(cout, cin, kh, kw, generator=g) / np.sqrt(cin * kh * kw)
    b = torch.randn(cout, generator=g)
    pad = ((kh - 1) // 2, (kw - 1) // 2)
    pc = K.pack_conv(w, b, 1, pad, device=DEV)
    pc.precision = _lib.PREC_F16X3
    ref = F.conv2d(xn.double(), w.double(), b.double(), 1, pad)
    a2 = _run(ks, 2, pc, x, B, H, W, cout, _lib.EPI_LINEAR)
    a2b = _run(ks, 2, pc, x, B, H, W, cout, _lib.EPI_LINEAR)
    a1 = _run(ks, 1, pc, x, B, H, W, cout, _lib.EPI_LINEAR)
    y2 = K.rows_to_nchw(a2, B, H, W).double().cpu()
    y1 = K.rows_to_nchw(a1, B, H, W).double().cpu()
    scale = max(1.0, float(ref.abs().max()))
    assert float((y2 - ref).abs().max()) < 1e-4 * scale
    assert float((y2 - y1).abs().max()) < 1e-5 * scale
    assert torch.equal(a2.t, a2b.t)  # deterministic


def test_k_split_forward_matches_one_wave(ks):
    """A whole RAFT-full forward (every update-block epilogue: relu, GRU z|r, GRU q, the flow head) in both
    forms: the flows agree within 1e-4 and each form is reproducible bit for bit (graph replay included)."""
    from raft_optical_flow_amd import RAFT
    from raft_optical_flow_amd.init import seeded_images, seeded_state_dict
    i1, i2 = seeded_images(1, 128, 192, seed=3)
    i1, i2 = i1.to(DEV), i2.to(DEV)
    outs = {}
    for k in (1, 2):
        ks.raft_conv2d_set_halo_ks(k)
        m = RAFT(argparse.Namespace(small=False, mixed_precision=False, alternate_corr=False))
        m.load_state_dict(seeded_state_dict(m, 0))
        m.to(DEV).eval()
        with torch.no_grad():
            runs = [m(i1, i2, iters=12, test_mode=True)[1] for _ in range(3)]  # eager, capture, replay
        torch.cuda.synchronize()
        assert torch.equal(runs[0], runs[1]) and torch.equal(runs[1], runs[2])
        outs[k] = runs[0]
    assert float((outs[1] - outs[2]).abs().max()) < 1e-4
