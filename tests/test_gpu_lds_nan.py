"""Uninitialised-LDS guard: every launch of a forward runs right behind raft_debug_fill_lds_nan
(include/raft_hip.h), which leaves NaN in every CU's whole LDS.  A kernel that reads LDS it did not
write (round 3's conv_stem read past its patch at the K padding: NaN x zero weight = NaN) then turns
the flow non-finite or different; the test requires the flow bit-identical to the plain run's and
finite, for each precision mode and model variant (RAFT.forward, core/raft.py:145-251)."""
import argparse

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _plan(small, alternate, precision, B, H, W, iters):
    from raft_optical_flow_amd import RAFT
    from raft_optical_flow_amd.init import seeded_images, seeded_state_dict
    m = RAFT(argparse.Namespace(small=small, mixed_precision=False, alternate_corr=alternate))
    m.conv_precision = precision
    m.load_state_dict(seeded_state_dict(m, 0))
    m = m.to(DEV).eval()
    i1, i2 = seeded_images(B, H, W, seed=11)
    pl = m.plan(B, H, W, iters, test_mode=True, device=torch.device(DEV))
    pl.set_inputs(i1.to(DEV), i2.to(DEV))
    return m, pl


def _run_with_lds_nan(pl):
    """The plan's launches in order on the current stream, each behind an LDS fill with NaN."""
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    s = K.stream_handle()
    n = 0
    for launch in pl.launches:
        if launch is K.FORK or launch is K.JOIN:
            continue
        _lib.call("raft_debug_fill_lds_nan", s)
        launch(s)
        n += 1
    return n


@pytest.mark.timeout(300)
@pytest.mark.parametrize("small,alternate,precision,B,H,W", [
    (False, False, "f16x3", 1, 128, 192),   # the default path: stem, halo, fused lookup + convc1/convf1
    (False, False, "f16x3", 2, 96, 136),    # ragged tiles, B = 2
    (False, False, "bf16", 1, 128, 192),    # one-product modes (wide 128-column tiles where they apply)
    (False, False, "fp32", 1, 64, 96),      # exact f32 MFMA GEMM path
    (False, True, "f16x3", 1, 128, 192),    # alternate corr (MFMA box GEMM lookup)
    (True, False, "f16x3", 1, 128, 192),    # RAFT-small
])
def test_forward_ignores_uninitialised_lds(small, alternate, precision, B, H, W):
    _, pl = _plan(small, alternate, precision, B, H, W, iters=4)
    with torch.no_grad():
        pl.run()
        torch.cuda.synchronize()
        ref = [t.clone() for t in pl.outputs(clone=True)]
        n = _run_with_lds_nan(pl)
        torch.cuda.synchronize()
        got = pl.outputs(clone=True)
    assert n > 10
    for r, g in zip(ref, got):
        assert bool(torch.isfinite(g).all()), "non-finite flow after LDS filled with NaN"
        assert torch.equal(r, g), f"flow differs after LDS filled with NaN: max {float((r - g).abs().max())}"


def test_fill_lds_nan_leaves_memory_alone():
    """The fill kernel touches LDS only: a device buffer is unchanged around it."""
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    x = torch.arange(1 << 20, device=DEV, dtype=torch.float32)
    y = x.clone()
    _lib.call("raft_debug_fill_lds_nan", K.stream_handle())
    torch.cuda.synchronize()
    assert torch.equal(x, y)
