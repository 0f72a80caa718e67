"""GPU parity of the halo conv's K-split form (RAFT_HALO_KS=2: two MFMA waves per SIMD share each
32-pixel block and take alternate K-steps, their partial sums added before the epilogue): the same
products in a different summation order, so within fp32 rounding of the one-wave form; the
config-2 forward against the reference golden (1e-3) and against RAFT_HALO_KS=1 (1e-4)."""
import argparse

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import load_golden

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from raft_optical_flow_amd import _lib
    _lib.load()


@pytest.mark.parametrize("kh,kw,cin,cout,B,H,W", [(3, 3, 256, 192, 1, 55, 128), (3, 3, 256, 126, 1, 55, 128),
                                                  (1, 5, 256, 256, 1, 55, 128), (5, 1, 256, 128, 2, 37, 61),
                                                  (3, 3, 128, 256, 3, 20, 30)])
def test_halo_ks2_conv(monkeypatch, kh, kw, cin, cout, B, H, W):
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    g = torch.Generator().manual_seed(kh * 100 + cout)
    x = torch.randn(B, cin, H, W, generator=g)
    w = torch.randn(cout, cin, kh, kw, generator=g) / np.sqrt(cin * kh * kw)
    b = torch.randn(cout, generator=g) * 0.1
    pc = K.pack_conv(w, b, 1, ((kh - 1) // 2, (kw - 1) // 2), device=DEV)
    pc.precision = _lib.PREC_F16X3
    src = K.Rows(K.nchw_to_rows(x.to(DEV)))
    outs = []
    for ks in ("1", "2"):
        monkeypatch.setenv("RAFT_HALO_KS", ks)
        out = K.Rows(torch.full((B * H * W, cout + 2), -7.0, device=DEV), 0, cout)
        K.conv_launch(K.conv_params(pc, src, B, H, W, out, epilogue=_lib.EPI_RELU))(K.stream_handle())
        torch.cuda.synchronize()
        outs.append(out.t.clone())
    ref = torch.relu(F.conv2d(x.double(), w.double(), b.double(), padding=((kh - 1) // 2, (kw - 1) // 2)))
    got = outs[1][:, :cout].view(B, H, W, cout).permute(0, 3, 1, 2).cpu().double()
    assert float((got - ref).abs().max()) < 1e-4 * max(1.0, float(ref.abs().max()))
    assert float((outs[1] - outs[0]).abs().max()) < 1e-5 * max(1.0, float(ref.abs().max()))
    assert bool((outs[1][:, cout:] == -7.0).all())


def test_halo_ks2_forward(monkeypatch):
    from raft_optical_flow_amd import RAFT
    from raft_optical_flow_amd.init import seeded_state_dict
    g = load_golden("raft_full_smooth_b2_128x192_i12.npz")
    res = []
    for ks in ("1", "2"):
        monkeypatch.setenv("RAFT_HALO_KS", ks)
        m = RAFT(argparse.Namespace(small=False, mixed_precision=False, alternate_corr=False))
        m.conv_precision = "f16x3"
        m.load_state_dict(seeded_state_dict(m, int(g["seed"])))
        m = m.to(DEV).eval()
        i1 = torch.from_numpy(g["image1"]).float().to(DEV)
        i2 = torch.from_numpy(g["image2"]).float().to(DEV)
        with torch.no_grad():
            res.append(m(i1, i2, iters=12, test_mode=True))
    for lo, up in res:
        assert float((lo.cpu() - torch.from_numpy(g["flow_low"])).abs().max()) < 1e-3
        assert float((up.cpu() - torch.from_numpy(g["flow_up"])).abs().max()) < 1e-3
    assert float((res[1][1] - res[0][1]).abs().max()) < 1e-4
