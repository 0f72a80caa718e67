"""GPU parity of the weight-resident persistent 3x3 conv (csrc/conv_resident.hip): the encoders'
stride-1 convs over <= 96 channels when the grid has more than two rounds of tiles
(core/extractor.py:6-56 ResidualBlock convs at 1/2 and 1/4 resolution).

The kernel runs the same f16x3 products in the same K order as the one-tile halo kernel, so its
outputs (every epilogue, the InstanceNorm partials, the input InstanceNorm in the loaders) must be
bit-identical to RAFT_RESIDENT=0's; and within the conv tolerance of a torch fp64 conv.  (The kernel is
opt-in, RAFT_RESIDENT=1: on one box it measured as fast as the halo kernel, not faster.)"""
import ctypes

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
    from raft_optical_flow_amd import _lib
    _lib.load()


def _run(monkeypatch, resident, pc, src, B, H, W, cout, epi, aux, norm, stats):
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    monkeypatch.setenv("RAFT_RESIDENT", "1" if resident else "0")
    out = K.Rows(torch.full((B * H * W, cout + 4), -7.0, device=DEV), 0, cout)
    p = K.conv_params(pc, src, B, H, W, out, epilogue=epi, aux0=aux)
    if norm is not None:
        p.in_norm, p.in_norm_relu = norm.data_ptr(), 1
    part = None
    if stats:
        slots = _lib.load().raft_conv2d_stats_slots(ctypes.byref(p))
        assert slots > 0
        part = torch.full((B * slots * cout * 4,), float("nan"), device=DEV)
        p.stats_part, p.stats_ld = part.data_ptr(), cout
    K.conv_launch(p)(K.stream_handle())
    torch.cuda.synchronize()
    return out.t.clone(), (part.clone() if part is not None else None)


@pytest.mark.parametrize("cin,cout,H,W,B", [(64, 64, 220, 512, 2), (96, 96, 110, 256, 2), (64, 64, 100, 150, 2),
                                            (64, 96, 61, 300, 3), (80, 64, 96, 200, 2)])
@pytest.mark.parametrize("kind", ["relu", "resid", "stats", "norm_stats"])
def test_resident_matches_halo_and_fp64(monkeypatch, cin, cout, H, W, B, kind):
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    g = torch.Generator().manual_seed(cin * 7 + H)
    x = torch.randn(B, cin, H, W, generator=g) * 1.5 + 0.3
    w = torch.randn(cout, cin, 3, 3, generator=g) / np.sqrt(cin * 9)
    b = torch.randn(cout, generator=g) * 0.2
    pc = K.pack_conv(w, b, 1, 1, device=DEV)
    pc.precision = _lib.PRECISIONS["f16x3"]
    src = K.Rows(K.nchw_to_rows(x.to(DEV)))
    xin = x.double()
    norm = None
    if kind == "norm_stats":
        mean = xin.mean((2, 3))
        rstd = 1.0 / torch.sqrt(xin.var((2, 3), unbiased=False) + 1e-5)
        norm = torch.stack([mean, rstd], -1).float().contiguous().to(DEV)
        xin = torch.relu((xin - mean[:, :, None, None]) * rstd[:, :, None, None])
    aux = None
    epi = _lib.EPI_LINEAR if kind in ("stats", "norm_stats") else (_lib.EPI_RELU if kind == "relu" else _lib.EPI_RESID_RELU)
    if kind == "resid":
        r = torch.randn(B, cout, H, W, generator=g)
        aux = K.Rows(K.nchw_to_rows(r.to(DEV)))
    stats = kind in ("stats", "norm_stats")
    y1, s1 = _run(monkeypatch, True, pc, src, B, H, W, cout, epi, aux, norm, stats)
    y0, s0 = _run(monkeypatch, False, pc, src, B, H, W, cout, epi, aux, norm, stats)
    assert torch.equal(y1, y0)
    if stats:
        assert torch.equal(s1, s0)
    ref = F.conv2d(xin, w.double(), b.double(), 1, 1)
    if kind == "relu":
        ref = torch.relu(ref)
    elif kind == "resid":
        ref = torch.relu(r.double() + torch.relu(ref))
    got = y1[:, :cout].view(B, H, W, cout).permute(0, 3, 1, 2).cpu().double()
    assert float((got - ref).abs().max()) < 1e-4 * max(1.0, float(ref.abs().max()))
    assert bool((y1[:, cout:] == -7.0).all())


def test_resident_forward_bit_exact(monkeypatch):
    """RAFT-full at config 2's size: the encoders on the resident kernel vs the halo kernel give the
    same flow bit for bit."""
    import argparse
    from raft_optical_flow_amd import RAFT
    from raft_optical_flow_amd.init import seeded_images, seeded_state_dict
    m = RAFT(argparse.Namespace(small=False, mixed_precision=False, alternate_corr=False))
    m.conv_precision = "f16x3"
    m.load_state_dict(seeded_state_dict(m, 0))
    m = m.to(DEV).eval()
    i1, i2 = seeded_images(1, 440, 1024, seed=3)
    i1, i2 = i1.to(DEV), i2.to(DEV)
    outs = []
    for res in ("0", "1"):
        monkeypatch.setenv("RAFT_RESIDENT", res)
        with torch.no_grad():
            outs.append(m(i1, i2, iters=4, test_mode=True))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
