"""GPU parity of raft_conv2d_chain: the update block's convc2|convf2 -> conv -> z|r1 -> q1 -> z|r2 ->
q2 -> flow-head conv1 sequence of one refinement iteration (core/update.py:74-121,169-216,297-325)
as ONE persistent launch whose tiles wait on completion counters of their neighbourhood in the
previous stage.

The chained launch runs the same tile bodies with the same arithmetic as one launch per conv, so
the whole forward must be bit-identical with RAFT_CHAIN=1 and RAFT_CHAIN=0; any stale read of a
neighbour's output (a hand-off ordering bug) shows up as a mismatch.  Checked eager and under
hipGraph replay, at one frame pair (one tile per work-group), at 1080x1920 and at B=4 (several
tiles per work-group), and that no wait timed out (the timeout flag stays 0)."""
import argparse
import ctypes

import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from raft_optical_flow_amd import _lib
    _lib.load()


def t(x):
    return torch.from_numpy(np.ascontiguousarray(x)).float().to(DEV)


def make_model(seed=0, precision="f16x3"):
    from raft_optical_flow_amd import RAFT
    from raft_optical_flow_amd.init import seeded_state_dict
    m = RAFT(argparse.Namespace(small=False, mixed_precision=False, alternate_corr=False))
    m.conv_precision = precision
    m.load_state_dict(seeded_state_dict(m, seed))
    return m.to(DEV).eval()


def chain_launches(pl):
    return [l for l in pl.launches if getattr(l, "name", "") == "raft_conv2d_chain"]


def run(m, monkeypatch, chain, i1, i2, iters, graph):
    monkeypatch.setenv("RAFT_CHAIN", "1" if chain else "0")
    B, _, H, W = i1.shape
    m.hip_graph = graph
    with torch.no_grad():
        low, up = m(i1, i2, iters=iters, test_mode=True)
        if graph:  # the second forward of a plan is captured and replayed
            low, up = m(i1, i2, iters=iters, test_mode=True)
    torch.cuda.synchronize()
    pl = m.plan(B, H, W, iters, True)
    return low, up, pl


@pytest.mark.parametrize("B,H,W,iters", [(1, 440, 1024, 32), (1, 1080, 1920, 3), (4, 256, 384, 4), (3, 64, 96, 6)])
@pytest.mark.parametrize("graph", [False, True])
def test_chain_forward_bit_exact(monkeypatch, B, H, W, iters, graph):
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd.init import seeded_images
    m = make_model(0)
    i1, i2 = seeded_images(B, H, W, seed=7)
    i1, i2 = i1.to(DEV), i2.to(DEV)
    low0, up0, pl0 = run(m, monkeypatch, False, i1, i2, iters, graph)
    assert not chain_launches(pl0)
    low1, up1, pl1 = run(m, monkeypatch, True, i1, i2, iters, graph)
    ch = chain_launches(pl1)
    assert len(ch) == iters
    lib = _lib.load()
    assert all(lib.raft_conv2d_chain_covered(l.args[0], l.args[1]) == 1 for l in ch)
    assert int(pl1.ub.chain_err.item()) == 0 and int(pl1.range_flag.item()) == 0
    assert int(pl1.ub.chain_sync.abs().sum().item()) == 0  # every launch leaves its counters zeroed
    assert torch.equal(low1, low0) and torch.equal(up1, up0)


def test_chain_golden_and_repeat(monkeypatch):
    """The chained forward against the reference golden (1e-3, as the unchained one), and ten
    back-to-back graph replays bit-identical (the counters are reset by each launch)."""
    g = load_golden("raft_full_smooth_b2_128x192_i12.npz")
    from raft_optical_flow_amd.init import seeded_state_dict  # noqa: F401
    m = make_model(int(g["seed"]))
    i1, i2 = t(g["image1"]), t(g["image2"])
    monkeypatch.setenv("RAFT_CHAIN", "1")
    with torch.no_grad():
        low, up = m(i1, i2, iters=12, test_mode=True)
        assert float((low.cpu() - torch.from_numpy(g["flow_low"])).abs().max()) < 1e-3
        assert float((up.cpu() - torch.from_numpy(g["flow_up"])).abs().max()) < 1e-3
        outs = [m(i1, i2, iters=12, test_mode=True) for _ in range(10)]
    for lo, u in outs:
        assert torch.equal(lo, low) and torch.equal(u, up)
    pl = m.plan(2, 128, 192, 12, True)
    assert pl.graph is not None and chain_launches(pl)
    assert int(pl.ub.chain_err.item()) == 0


def test_chain_capi_fallbacks():
    """raft_conv2d_chain runs uncovered stages (exact fp32 convs, or no sync buffer) in order:
    identical to raft_conv2d per stage."""
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    rng = np.random.default_rng(3)
    B, h, w = 1, 20, 36
    P = B * h * w
    lib = _lib.load()
    for prec in ("fp32", "f16x3"):
        x = K.Rows(t(rng.standard_normal((P, 64))))
        mid = K.Rows(torch.zeros(P, 64, device=DEV))
        outs = [K.Rows(torch.zeros(P, 32, device=DEV)) for _ in range(2)]
        pcs = []
        for kh, kw, cin, cout in ((3, 3, 64, 64), (1, 5, 64, 32)):
            wt = torch.from_numpy((rng.standard_normal((cout, cin, kh, kw)) * 0.05).astype(np.float32))
            pc = K.pack_conv(wt, torch.zeros(cout), 1, ((kh - 1) // 2, (kw - 1) // 2), device=DEV)
            pc.precision = _lib.PRECISIONS[prec]
            pcs.append(pc)
        for k, sync in enumerate((True, False)):
            p0 = K.conv_params(pcs[0], x, B, h, w, mid, epilogue=_lib.EPI_RELU)
            p1 = K.conv_params(pcs[1], mid, B, h, w, outs[k], epilogue=_lib.EPI_RELU)
            arr = (ctypes.POINTER(_lib.ConvParams) * 4)(ctypes.pointer(p0), None, ctypes.pointer(p1), None)
            assert lib.raft_conv2d_chain_covered(arr, 2) == (1 if prec == "f16x3" else 0)
            sbuf = torch.zeros(int(lib.raft_conv2d_chain_sync_ints(2, B, h, w)), dtype=torch.int32, device=DEV)
            _lib.call("raft_conv2d_chain", arr, 2, sbuf.data_ptr() if sync else None, None, K.stream_handle())
        ref = torch.zeros(P, 32, device=DEV)
        p0 = K.conv_params(pcs[0], x, B, h, w, mid, epilogue=_lib.EPI_RELU)
        p1 = K.conv_params(pcs[1], mid, B, h, w, K.Rows(ref), epilogue=_lib.EPI_RELU)
        _lib.call("raft_conv2d", ctypes.byref(p0), K.stream_handle())
        _lib.call("raft_conv2d", ctypes.byref(p1), K.stream_handle())
        torch.cuda.synchronize()
        assert torch.equal(outs[0].t, ref) and torch.equal(outs[1].t, ref)
