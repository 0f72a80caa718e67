"""The halo conv kernel's multi-tile work-groups (conv_halo.hip halo_body): a launch with more tiles
than CUs runs ceil(tiles / CUs) tiles per work-group back to back, the loaders running on into the
next tile while the compute waves store the last one.  Every image of each conv is checked against
torch fp64 (a wrong tile hand-over shows up in whichever tile follows it), with the encoder
features (InstanceNorm partials, the loaders' input norm over work-groups that straddle images), the
1x1 path (fp32 patches by LDS-DMA), the 1x5 big tiles (D = 2) and pair launches.  Tolerances as
test_gpu_parity.py's CONV_TOL."""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"
CONV_TOL = {"fp32": 1e-4, "f16x3": 1e-4, "f16": 5e-3, "bf16": 3e-2}


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _err(y, ref):
    return float((y.double().cpu() - ref).abs().max()) / max(1.0, float(ref.abs().max()))


@pytest.mark.parametrize("prec", ["f16x3", "bf16"])
@pytest.mark.parametrize("cin,cout,kh,kw,H,W,B", [
    (64, 64, 3, 3, 110, 256, 4),     # fnet layer1 shape, 128-pixel tiles: 3584 tiles, 14 per work-group
    (128, 128, 3, 3, 55, 128, 6),    # fnet layer3 shape (4 chunks)
    (256, 192, 3, 3, 61, 70, 8),     # ragged tiles in both axes
    (96, 256, 1, 1, 60, 70, 8),      # 1x1: fp32 patches by LDS-DMA, a patch per K-step
    (256, 128, 1, 5, 55, 128, 8),    # q (1x5): big tiles, D = 2 in f16x3
    (256, 128, 5, 1, 50, 120, 8),
])
def test_multi_tile_work_groups_vs_fp64(cin, cout, kh, kw, H, W, B, prec):
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    g = torch.Generator().manual_seed(cin + cout + kh + H)
    x = torch.randn(B, cin, H, W, generator=g)
    w = torch.randn(cout, cin, kh, kw, generator=g) / np.sqrt(cin * kh * kw)
    b = torch.randn(cout, generator=g)
    pad = ((kh - 1) // 2, (kw - 1) // 2)
    pc = K.pack_conv(w, b, 1, pad, device=DEV)
    pc.precision = _lib.PRECISIONS[prec]
    src = K.Rows(K.nchw_to_rows(x.to(DEV)))
    out = K.Rows(torch.full((B * H * W, cout + 4), -7.0, device=DEV), 0, cout)
    p = K.conv_params(pc, src, B, H, W, out, epilogue=_lib.EPI_RELU)
    m = _lib.load().raft_conv2d_halo_tiles_per_wg(ctypes.byref(p))
    # (the one-product modes keep one tile per work-group on 3x3 convs with several N-tiles: conv_halo.hip)
    assert (m == 1) if (prec != "f16x3" and kh * kw == 9 and cout > 64) else (m > 1), m
    K.conv_launch(p)(K.stream_handle())
    y = K.rows_to_nchw(out, B, H, W)
    ref = torch.relu(F.conv2d(x.double(), w.double(), b.double(), 1, pad))
    assert _err(y, ref) < CONV_TOL[prec]
    assert bool((out.t[:, cout:] == -7.0).all())


@pytest.mark.parametrize("prec", ["f16x3", "bf16"])
@pytest.mark.parametrize("H,W,B", [(110, 256, 4), (37, 301, 7)])
def test_multi_tile_encoder_features(H, W, B, prec):
    """The fnet residual blocks' 3x3 conv with both encoder features on multi-tile work-groups: the
    input InstanceNorm applied by the loaders (tables of every image a work-group's tiles cover) and
    the output's InstanceNorm partials (merged by raft_instnorm_merge_ws) against fp64."""
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    cin = cout = 64
    g = torch.Generator().manual_seed(H + W + B)
    x = torch.randn(B, cin, H, W, generator=g) * 2.0 + 1.5
    w = torch.randn(cout, cin, 3, 3, generator=g) / np.sqrt(cin * 9)
    b = torch.randn(cout, generator=g) * 0.5
    mean = x.double().mean((2, 3))
    rstd = 1.0 / torch.sqrt(x.double().var((2, 3), unbiased=False) + 1e-5)
    xn = torch.relu((x.double() - mean[:, :, None, None]) * rstd[:, :, None, None])
    ref = F.conv2d(xn, w.double(), b.double(), 1, 1)
    pc = K.pack_conv(w, b, 1, 1, device=DEV)
    pc.precision = _lib.PRECISIONS[prec]
    src = K.Rows(K.nchw_to_rows(x.to(DEV)))
    out = K.Rows(torch.empty(B * H * W, cout, device=DEV))
    st = torch.stack([mean, rstd], -1).float().contiguous().to(DEV)
    p = K.conv_params(pc, src, B, H, W, out)
    p.in_norm, p.in_norm_relu = st.data_ptr(), 1
    lib = _lib.load()
    slots = lib.raft_conv2d_stats_slots(ctypes.byref(p))
    assert slots > 0
    part = torch.full((B * slots * cout * 4,), float("nan"), device=DEV)
    p.stats_part, p.stats_ld = part.data_ptr(), cout
    assert lib.raft_conv2d_halo_tiles_per_wg(ctypes.byref(p)) > 1
    K.conv_launch(p)(K.stream_handle())
    y = K.rows_to_nchw(out, B, H, W)
    assert _err(y, ref) < CONV_TOL[prec]
    nws = int(lib.raft_instnorm_merge_ws_floats(slots, B, cout))
    ws = torch.empty(nws, device=DEV)
    stats = torch.empty(2 * B * cout, device=DEV)
    _lib.call("raft_instnorm_merge_ws", part.data_ptr(), slots, B, cout, cout, 1e-5, ws.data_ptr(), stats.data_ptr(),
              K.stream_handle())
    # the one-launch merge: the same statistics bit for bit, counters left zero (twice: a replay)
    cnt = torch.zeros(int(lib.raft_instnorm_merge_counters(B, cout)), dtype=torch.int32, device=DEV)
    for _ in range(2):
        stats1 = torch.full_like(stats, float("nan"))
        _lib.call("raft_instnorm_merge_fused", part.data_ptr(), slots, B, cout, cout, 1e-5, ws.data_ptr(),
                  cnt.data_ptr(), stats1.data_ptr(), K.stream_handle())
        torch.cuda.synchronize()
        assert torch.equal(stats1, stats)
        assert int(cnt.abs().sum()) == 0
    got = stats.view(B, cout, 2).cpu().double()
    yd = out.t.view(B, H * W, cout).cpu().double()
    assert float((got[..., 0] - yd.mean(1)).abs().max()) < 1e-5 * max(1.0, float(yd.mean(1).abs().max()))
    r = 1.0 / torch.sqrt(yd.var(1, unbiased=False) + 1e-5)
    assert float(((got[..., 1] - r) / r).abs().max()) < 1e-5


@pytest.mark.parametrize("prec,k,shapes,scaled", [
    ("f16x3", 3, [(256, 192, 8), (128, 64, 8)], False),
    ("f16x3", 3, [(256, 192, 8), (128, 64, 8)], True),    # both convs pick the 16x16 tiles: one launch
    ("f16x3", 3, [(256, 192, 8), (128, 64, 2)], True),    # 16x16 vs 128-pixel tiles: run in order
    ("bf16", 1, [(256, 256, 8), (128, 128, 8)], False)])  # (1x1: no big tiles)
def test_multi_tile_pair_launch_equals_two_convs(prec, k, shapes, scaled):
    """A multi-round raft_conv2d_pair (each conv's tiles on their own work-groups, several per
    work-group) == the two convs launched alone (other tile counts per work-group), bit for bit,
    also with the column-scaled split weight set (raft_hip.h: the pair's contract; a pair whose convs
    pick different tile rows runs them in order)."""
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    H, W = 55, 128
    g = torch.Generator().manual_seed(5)
    xs, pcs, pair, seq = [], [], [], []
    for cin, cout, B in shapes:
        x = torch.randn(B, cin, H, W, generator=g)
        w = torch.randn(cout, cin, k, k, generator=g) / np.sqrt(cin * k * k)
        pc = K.pack_conv(w, torch.randn(cout, generator=g), 1, (k // 2, k // 2), device=DEV)
        pc.precision = _lib.PRECISIONS[prec]
        xs.append(K.Rows(K.nchw_to_rows(x.to(DEV))))
        pcs.append(pc)
        pair.append(K.Rows(torch.full((B * H * W, cout), 7.0, device=DEV)))
        seq.append(K.Rows(torch.full((B * H * W, cout), 7.0, device=DEV)))
    bs = [sh[2] for sh in shapes]
    prm = [K.conv_params(pcs[i], xs[i], bs[i], H, W, pair[i], epilogue=_lib.EPI_RELU) for i in range(2)]
    one = [K.conv_params(pcs[i], xs[i], bs[i], H, W, seq[i], epilogue=_lib.EPI_RELU) for i in range(2)]
    if not scaled:  # (f16x3: every launch on the 128-pixel tiles)
        for q in prm + one:
            q.weight_s = None
    lib = _lib.load()
    if not scaled:  # (on the 16x16 tiles the cost rule keeps one tile per work-group here)
        assert lib.raft_conv2d_halo_tiles_per_wg(ctypes.byref(one[0])) > 1
    else:
        rows = [lib.raft_conv2d_halo_tile_rows(ctypes.byref(q)) for q in one]
        assert rows == ([16, 16] if bs[1] == 8 else [16, 8]), rows
    K.conv_pair_launch(prm[0], prm[1])(K.stream_handle())
    for q in one:
        K.conv_launch(q)(K.stream_handle())
    torch.cuda.synchronize()
    for i in range(2):
        assert torch.equal(pair[i].t, seq[i].t), i
