"""GPU parity: the HIP path (through the C-ABI) against the golden vectors of the
reference and against the numpy oracle.  Tolerances (max-abs, fp32):
  lookup / pyramid   1e-5   (values O(1..10))
  conv GEMM          1e-4 x max|ref| scale (fp32, f16x3); 5e-3 (f16, one half-precision product)
  update block       1e-4
  end-to-end flow    1e-3   (north_star bound on the final flow field)
"""
import argparse
import io

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import load_golden
from oracle import raft_oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda"


def maxabs(a, b):
    a = a.detach().cpu().numpy() if torch.is_tensor(a) else np.asarray(a)
    b = b.detach().cpu().numpy() if torch.is_tensor(b) else np.asarray(b)
    return float(np.max(np.abs(a.astype(np.float64) - b.astype(np.float64))))


def t(x):
    return torch.from_numpy(np.ascontiguousarray(x)).float().to(DEV)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from raft_optical_flow_amd import _lib
    _lib.load()


def make_model(small, seed=0, alternate=False, precision=None):
    from raft_optical_flow_amd import RAFT
    from raft_optical_flow_amd.init import seeded_state_dict
    m = RAFT(argparse.Namespace(small=small, mixed_precision=False, alternate_corr=alternate))
    m.conv_precision = precision
    sd = seeded_state_dict(m, seed)
    m.load_state_dict(sd)
    return m.to(DEV).eval(), {k: v.numpy() for k, v in sd.items()}


# ----------------------------------------------------------------------------- instance norm


@pytest.mark.parametrize("case", [
    dict(cin=64, cout=64, k=3, stride=1, pad=1, H=37, W=53, B=2, mode=None),   # halo 3x3, ragged tiles
    dict(cin=96, cout=96, k=1, stride=1, pad=0, H=20, W=33, B=2, mode=None),   # halo 1x1
    dict(cin=3, cout=64, k=7, stride=2, pad=3, H=90, W=150, B=2, mode="gather"),  # the stem
    dict(cin=96, cout=96, k=3, stride=1, pad=1, H=110, W=256, B=2, mode=None),  # big tiles (fnet layer2)
    # the 64x64-tile GEMM (round 5): strided convs, M tiled per image (513 rows: a ragged last tile)
    dict(cin=64, cout=96, k=3, stride=2, pad=1, H=37, W=53, B=3, mode=None),
    dict(cin=64, cout=96, k=1, stride=2, pad=0, H=37, W=53, B=3, mode=None),    # the downsample 1x1
    dict(cin=96, cout=128, k=3, stride=2, pad=1, H=9, W=11, B=3, mode=None),    # 30 rows per image
])
@pytest.mark.parametrize("prec", ["f16x3", "bf16"])
def test_conv_epilogue_instnorm_stats(case, prec):
    """InstanceNorm statistics from the conv epilogue (raft_conv2d_stats_slots + raft_instnorm_merge):
    per-(image, channel) mean and 1/sqrt(var + eps) of the conv output against fp64 over the
    output the same launch wrote; run twice, bit-identical (fixed merge order)."""
    import ctypes
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    g = torch.Generator().manual_seed(case["cin"] + case["k"])
    B, H, W = case["B"], case["H"], case["W"]
    x = torch.randn(B, case["cin"], H, W, generator=g) + 0.5
    w = torch.randn(case["cout"], case["cin"], case["k"], case["k"], generator=g) / np.sqrt(case["cin"] * case["k"] ** 2)
    b = torch.randn(case["cout"], generator=g) * 3.0   # an offset the M2 form must not lose precision to
    mode = _lib.RAFT_CONV_GATHER if case["mode"] == "gather" else None
    pc = K.pack_conv(w, b, case["stride"], case["pad"], mode=mode, device=DEV)
    pc.precision = _lib.PRECISIONS[prec]
    src = K.Rows(K.nchw_to_rows(x.to(DEV)))
    ho, wo = K.conv_out_hw(pc, H, W)
    out = K.Rows(torch.empty(B * ho * wo, case["cout"], device=DEV))
    p = K.conv_params(pc, src, B, H, W, out)
    slots = _lib.load().raft_conv2d_stats_slots(ctypes.byref(p))
    assert slots > 0
    part = torch.full((B * slots * case["cout"] * 4,), float("nan"), device=DEV)
    p.stats_part, p.stats_ld = part.data_ptr(), case["cout"]
    got = []
    for _ in range(2):
        K.conv_launch(p)(K.stream_handle())
        st = torch.empty(2 * B * case["cout"], device=DEV)
        _lib.call("raft_instnorm_merge", part.data_ptr(), slots, B, case["cout"], case["cout"], 1e-5, st.data_ptr(),
                  K.stream_handle())
        got.append(st.view(B, case["cout"], 2).cpu())
    assert torch.equal(got[0], got[1])
    # the two-level merge the forward runs (raft_instnorm_merge_ws): run to run bit-identical too
    nws = int(_lib.load().raft_instnorm_merge_ws_floats(slots, B, case["cout"]))
    ws = torch.full((nws,), float("nan"), device=DEV)
    for _ in range(2):
        st = torch.empty(2 * B * case["cout"], device=DEV)
        _lib.call("raft_instnorm_merge_ws", part.data_ptr(), slots, B, case["cout"], case["cout"], 1e-5, ws.data_ptr(),
                  st.data_ptr(), K.stream_handle())
        got.append(st.view(B, case["cout"], 2).cpu())
    assert torch.equal(got[2], got[3])
    y = out.t.view(B, ho * wo, case["cout"]).cpu().double()
    mean = y.mean(1)
    rstd = 1.0 / torch.sqrt(y.var(1, unbiased=False) + 1e-5)
    for gg in (got[0], got[2]):
        assert float((gg[..., 0].double() - mean).abs().max()) < 1e-5 * max(1.0, float(mean.abs().max()))
        assert float(((gg[..., 1].double() - rstd) / rstd).abs().max()) < 1e-5


@pytest.mark.parametrize("cin,cout,H,W,B,relu", [(64, 64, 37, 53, 2, 1), (128, 96, 23, 30, 1, 0), (96, 96, 16, 16, 1, 1),
                                                (96, 96, 110, 256, 2, 1)])   # (the last: big tiles)
@pytest.mark.parametrize("prec", ["f16x3", "bf16"])
def test_conv_in_norm_loader(cin, cout, H, W, B, relu, prec):
    """raft_conv2d_params.in_norm: the 3x3 halo conv reads act((x - mean) * rstd) of its raw input
    (the residual blocks' conv2 over conv1's un-normalised output), zero padding staying zero;
    against torch fp64 of conv(act(instance_norm(x)))."""
    import ctypes
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    g = torch.Generator().manual_seed(cin + H)
    x = torch.randn(B, cin, H, W, generator=g) * 2.0 + 1.5
    w = torch.randn(cout, cin, 3, 3, generator=g) / np.sqrt(cin * 9)
    b = torch.randn(cout, generator=g) * 0.1
    mean = x.double().mean((2, 3))
    rstd = 1.0 / torch.sqrt(x.double().var((2, 3), unbiased=False) + 1e-5)
    xn = (x.double() - mean[:, :, None, None]) * rstd[:, :, None, None]
    if relu:
        xn = torch.relu(xn)
    ref = F.conv2d(xn, w.double(), b.double(), 1, 1)
    pc = K.pack_conv(w, b, 1, 1, device=DEV)
    pc.precision = _lib.PRECISIONS[prec]
    src = K.Rows(K.nchw_to_rows(x.to(DEV)))
    out = K.Rows(torch.full((B * H * W, cout + 4), -7.0, device=DEV), 0, cout)
    st = torch.stack([mean, rstd], -1).float().contiguous().to(DEV)   # [B][cin][2]
    p = K.conv_params(pc, src, B, H, W, out)
    p.in_norm, p.in_norm_relu = st.data_ptr(), relu
    assert _lib.load().raft_conv2d_in_norm_ok(ctypes.byref(p)) == 1
    K.conv_launch(p)(K.stream_handle())
    y = K.rows_to_nchw(out, B, H, W)
    assert maxabs(y, ref) < CONV_TOL[prec] * max(1.0, float(ref.abs().max()))
    assert bool((out.t[:, cout:] == -7.0).all())


def test_encoders_in_norm_matches_apply_pass(monkeypatch):
    """The encoders with the loaders' InstanceNorm (default) vs the separate normalised copy
    (RAFT_IN_NORM=0): the same features to 1e-4 of their scale."""
    m, _ = make_model(False)
    g = torch.Generator().manual_seed(11)
    img = (torch.rand(2, 3, 96, 128, generator=g) * 255).to(DEV)
    with torch.no_grad():
        a = m.fnet(img)
        monkeypatch.setenv("RAFT_IN_NORM", "0")
        b = m.fnet(img)
    assert maxabs(a, b) < 1e-4 * max(1.0, float(b.abs().max()))


@pytest.mark.parametrize("B,HW,C,ld", [(2, 220 * 512, 64, 64), (3, 1000, 96, 100), (1, 77, 6, 6), (2, 513, 300, 300)])
def test_instnorm_stats_vs_fp64(B, HW, C, ld):
    """raft_instnorm_stats (one launch: chunk partials, the last block of each image finalizes):
    mean and 1/sqrt(var + eps) against fp64, per (image, channel); the vectorised and scalar
    partial kernels, > 256 channels; three calls on one workspace (its arrival counters re-arm)
    give bit-identical stats."""
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    g = torch.Generator().manual_seed(B * 7 + C)
    x = (torch.randn(B * HW, ld, generator=g) * 3 + torch.linspace(-5, 5, ld)).float()
    xd = x.to(DEV)
    ws = K.instnorm_workspace(B, HW, C, DEV)
    outs = []
    for _ in range(3):
        st = torch.full((B * C * 2,), -1.0, device=DEV)
        _lib.call("raft_instnorm_stats", xd.data_ptr(), ld, B, HW, C, 1e-5, st.data_ptr(), ws.data_ptr(),
                  K.stream_handle())
        torch.cuda.synchronize()
        outs.append(st.cpu())
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    xv = x[:, :C].double().reshape(B, HW, C)
    mean = xv.mean(1)
    rstd = 1.0 / torch.sqrt(xv.var(1, unbiased=False) + 1e-5)
    got = outs[0].double().reshape(B, C, 2)
    assert float((got[..., 0] - mean).abs().max()) < 1e-5 * max(1.0, float(mean.abs().max()))
    assert float(((got[..., 1] - rstd) / rstd).abs().max()) < 1e-5


# ----------------------------------------------------------------------------- correlation


def test_pyramid_golden():
    from raft_optical_flow_amd import CorrBlock
    g = load_golden("pyramid_b1c32_8x12.npz")
    cb = CorrBlock(t(g["fmap1"]), t(g["fmap2"]), num_levels=4, radius=4)
    for i in range(4):
        assert maxabs(cb.corr_pyramid[i], g[f"level{i}"]) < 1e-5


def test_pyramid_vs_oracle_ragged():
    """C=256, odd sizes (floor pooling, partial GEMM tiles), B=2."""
    from raft_optical_flow_amd import CorrBlock
    rng = np.random.default_rng(0)
    f1 = rng.standard_normal((2, 256, 23, 37)).astype(np.float32)
    f2 = rng.standard_normal((2, 256, 23, 37)).astype(np.float32)
    cb = CorrBlock(t(f1), t(f2), num_levels=4, radius=4)
    ref = O.corr_pyramid(f1, f2, 4)
    for i in range(4):
        scale = np.abs(ref[i]).max()
        assert maxabs(cb.corr_pyramid[i], ref[i]) < 1e-5 * max(1.0, scale)


def test_pyramid_f16x3_vs_oracle():
    """raft_corr_build_prec(RAFT_PREC_F16X3): the split-f16 correlation GEMM of the RAFT
    forward, every level within 1e-5 (relative to the level's max) of the fp64 oracle."""
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    rng = np.random.default_rng(5)
    B, C, H, W, L = 2, 256, 23, 37, 4
    f1 = rng.standard_normal((B, C, H, W)).astype(np.float32)
    f2 = rng.standard_normal((B, C, H, W)).astype(np.float32)
    r1, r2 = K.nchw_to_rows(t(f1)), K.nchw_to_rows(t(f2))
    pyr = torch.empty(K.pyramid_floats(B, H, W, L), device=DEV)
    _lib.call("raft_corr_build_prec", r1.data_ptr(), r2.data_ptr(), C, B, H, W, C, L, K.sqrt_c(C), _lib.PREC_F16X3,
              pyr.data_ptr(), K.stream_handle())
    ref = O.corr_pyramid(f1.astype(np.float64), f2.astype(np.float64), L)
    dims = K.pyramid_dims(H, W, L)
    for i, (lh, lw) in enumerate(dims):
        out = torch.empty(B * H * W, lh, lw, device=DEV)
        _lib.call("raft_corr_pyramid_level", pyr.data_ptr(), B, H, W, L, i, out.data_ptr(), K.stream_handle())
        scale = np.abs(ref[i]).max()
        assert maxabs(out.view(ref[i].shape), ref[i]) < 1e-5 * max(1.0, scale), i


@pytest.mark.parametrize("r", [4, 3])
def test_lookup_golden(r):
    from raft_optical_flow_amd import CorrBlock
    g = load_golden("lookup_b2c64_16x20.npz")
    cb = CorrBlock(t(g["fmap1"]), t(g["fmap2"]), num_levels=4, radius=r)
    out = cb(t(g["coords"]))
    assert maxabs(out, g[f"corr_r{r}"]) < 1e-5


@pytest.mark.parametrize("r", [5, 6])
def test_lookup_any_radius_golden(r):
    """Radius > 4 (the reference takes any r): the generic lookup kernels against the reference's
    CorrBlock at r = 5, 6 (all-pairs and alternate paths)."""
    from raft_optical_flow_amd import AlternateCorrBlock, CorrBlock
    g = load_golden("lookup_b2c64_16x20.npz")
    big = load_golden("lookup_b2c64_16x20_r56.npz")
    cb = CorrBlock(t(g["fmap1"]), t(g["fmap2"]), num_levels=4, radius=r)
    assert maxabs(cb(t(g["coords"])), big[f"corr_r{r}"]) < 1e-5
    ab = AlternateCorrBlock(t(g["fmap1"]), t(g["fmap2"]), num_levels=4, radius=r)
    assert maxabs(ab(t(g["coords"])), big[f"corr_r{r}"]) < 5e-5


def test_lookup_radius_zero_and_alt_radius_seven_vs_oracle():
    from raft_optical_flow_amd import CorrBlock, alt_cuda_corr
    rng = np.random.default_rng(4)
    f1 = rng.standard_normal((1, 32, 12, 15)).astype(np.float32)
    f2 = rng.standard_normal((1, 32, 12, 15)).astype(np.float32)
    coords = rng.uniform(-3, 17, (1, 2, 12, 15)).astype(np.float32)
    ref = O.corr_lookup(O.corr_pyramid(f1, f2, 3), coords, 0)
    assert maxabs(CorrBlock(t(f1), t(f2), num_levels=3, radius=0)(t(coords)), ref) < 1e-5
    a1 = np.ascontiguousarray(f1.transpose(0, 2, 3, 1))
    a2 = np.ascontiguousarray(f2.transpose(0, 2, 3, 1))
    c5 = np.ascontiguousarray(coords.transpose(0, 2, 3, 1)[:, None])
    corr, = alt_cuda_corr.forward(t(a1), t(a2), t(c5), 7)
    assert maxabs(corr, O.alt_corr_forward(a1, a2, c5, 7)) < 1e-4


def test_lookup_degenerate_level_nan():
    from raft_optical_flow_amd import CorrBlock
    g = load_golden("lookup_degenerate_6x8.npz")
    cb = CorrBlock(t(g["fmap1"]), t(g["fmap2"]), num_levels=3, radius=2)
    out = cb(t(g["coords"])).cpu().numpy()
    ref = g["corr"]
    np.testing.assert_array_equal(np.isnan(out), np.isnan(ref))
    ok = ~np.isnan(ref)
    assert maxabs(out[ok], ref[ok]) < 1e-5


def test_lookup_far_out_of_bounds_and_large_coords():
    from raft_optical_flow_amd import CorrBlock
    rng = np.random.default_rng(1)
    f1 = rng.standard_normal((1, 64, 20, 30)).astype(np.float32)
    f2 = rng.standard_normal((1, 64, 20, 30)).astype(np.float32)
    coords = (rng.uniform(-60, 90, (1, 2, 20, 30))).astype(np.float32)
    coords[0, :, 0, :5] = np.round(coords[0, :, 0, :5])  # exact integers
    cb = CorrBlock(t(f1), t(f2), num_levels=4, radius=4)
    ref = O.corr_lookup(O.corr_pyramid(f1, f2, 4), coords, 4)
    assert maxabs(cb(t(coords)), ref) < 2e-5


@pytest.mark.parametrize("B,h,w", [(32, 16, 20), (33, 17, 21), (50, 17, 21)])
def test_lookup_pipelined_grid_vs_oracle(B, h, w):
    """Batches past one resident grid of the lookup (> 8 blocks per CU), a ragged pixel
    count, coords spread over and beyond the maps.  Up to 16384 query pixels the launch runs
    the scalar-interval window form, beyond it the VALU form (B=50: 17850 pixels)."""
    from raft_optical_flow_amd import CorrBlock
    rng = np.random.default_rng(7)
    f1 = rng.standard_normal((B, 32, h, w)).astype(np.float32)
    f2 = rng.standard_normal((B, 32, h, w)).astype(np.float32)
    ys, xs = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    grid = np.stack([xs, ys])[None].astype(np.float32)
    coords = (grid + rng.normal(0, 3.0, (B, 2, h, w))).astype(np.float32)
    coords[B - 1] = rng.uniform(-40, 60, (2, h, w)).astype(np.float32)
    cb = CorrBlock(t(f1), t(f2), num_levels=4, radius=4)
    ref = O.corr_lookup(O.corr_pyramid(f1, f2, 4), coords, 4)
    assert maxabs(cb(t(coords)), ref) < 2e-5


def test_lookup_window_forms_bit_equal():
    """The two window-test forms of the lookup kernel (scalar intervals for <= 16384 query
    pixels, per-lane VALU tests beyond) fetch the same tiles and share the tap arithmetic:
    a B=80 launch (VALU form) equals B=40 launches of its halves (scalar form) bit for bit,
    with windows hanging off every map edge, far outside, and on exact integers."""
    from raft_optical_flow_amd import CorrBlock
    rng = np.random.default_rng(12)
    B, h, w = 80, 17, 21
    f1 = rng.standard_normal((B, 32, h, w)).astype(np.float32)
    f2 = rng.standard_normal((B, 32, h, w)).astype(np.float32)
    ys, xs = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    grid = np.stack([xs, ys])[None].astype(np.float32)
    coords = (grid + rng.normal(0, 4.0, (B, 2, h, w))).astype(np.float32)
    coords[::7] = rng.uniform(-30, 50, (len(coords[::7]), 2, h, w)).astype(np.float32)
    coords[3] = np.round(coords[3])
    full = CorrBlock(t(f1), t(f2), num_levels=4, radius=4)(t(coords))
    for s in (slice(0, 40), slice(40, 80)):
        half = CorrBlock(t(f1[s]), t(f2[s]), num_levels=4, radius=4)(t(coords[s]))
        assert torch.equal(full[s], half)


def _lookup_convf1_case(B, h, w, r, prec, coord_scale=1.0, seed=11):
    """raft_corr_lookup_convf1 vs raft_corr_lookup + an fp64 torch conv of the flow."""
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    rng = np.random.default_rng(seed)
    C, L = 64, 4
    f1 = rng.standard_normal((B, C, h, w)).astype(np.float32)
    f2 = rng.standard_normal((B, C, h, w)).astype(np.float32)
    r1, r2 = K.nchw_to_rows(t(f1)), K.nchw_to_rows(t(f2))
    pyr = torch.empty(K.pyramid_floats(B, h, w, L), device=DEV)
    _lib.call("raft_corr_build", r1.data_ptr(), r2.data_ptr(), C, B, h, w, C, L, K.sqrt_c(C), pyr.data_ptr(),
              K.stream_handle())
    ys, xs = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    grid = np.stack([xs, ys], -1)[None].astype(np.float32)
    coords = (grid + coord_scale * rng.normal(0, 3.0, (B, h, w, 2))).astype(np.float32)
    cr = t(coords.reshape(-1, 2))
    ntap = L * (2 * r + 1) ** 2
    P = B * h * w
    out_a = torch.full((P, ntap), -7.0, device=DEV)
    out_b = torch.full((P, ntap), -7.0, device=DEV)
    flow_a = torch.zeros(P, 4, device=DEV)
    flow_b = torch.zeros(P, 4, device=DEV)
    n = 128
    wt = rng.standard_normal((n, 2, 7, 7)).astype(np.float32) * 0.1
    bias = rng.standard_normal(n).astype(np.float32) * 0.1
    rnd = {_lib.PREC_F16: torch.float16, _lib.PREC_BF16: torch.bfloat16}.get(prec)
    wq = torch.from_numpy(wt)
    if rnd is not None:
        wq = wq.to(rnd).float()
    wv = wq.reshape(n // 32, 32, 2, 49).permute(0, 3, 2, 1).contiguous().to(DEV)  # [n/32][k*k][2][32]
    f1o = torch.full((P, n + 4), -7.0, device=DEV)
    flag = torch.zeros(1, dtype=torch.int32, device=DEV)
    _lib.call("raft_corr_lookup", pyr.data_ptr(), B, h, w, L, r, cr.data_ptr(), 0, out_a.data_ptr(), ntap, 0,
              flow_a.data_ptr(), 4, None, K.stream_handle())
    _lib.call("raft_corr_lookup_convf1", pyr.data_ptr(), B, h, w, L, r, cr.data_ptr(), 0, out_b.data_ptr(), ntap, 0,
              flow_b.data_ptr(), 4, None, wv.data_ptr(), t(bias).data_ptr(), n, 7, prec, f1o.data_ptr(), n + 4,
              flag.data_ptr(), K.stream_handle())
    f1s = torch.full((P, n + 4), -7.0, device=DEV)  # convf1 alone (raft_convf1_flow, the alternate loop's)
    _lib.call("raft_convf1_flow", cr.data_ptr(), 0, B, h, w, wv.data_ptr(), t(bias).data_ptr(), n, 7, prec,
              f1s.data_ptr(), n + 4, None, K.stream_handle())
    torch.cuda.synchronize()
    assert torch.equal(f1s, f1o)
    # the lookup's outputs are the plain lookup's, bit for bit
    def same(x, y):  # bitwise, NaN where NaN
        return bool(((x == y) | (torch.isnan(x) & torch.isnan(y))).all())

    assert same(out_a, out_b) and same(flow_a, flow_b)
    # convf1 = relu(conv7x7(flow) + b) (core/update.py:205), fp64 reference on the same operands
    flow = torch.from_numpy(coords - grid).permute(0, 3, 1, 2)
    if rnd is not None:
        flow = flow.to(rnd).float()
    ref = torch.relu(F.conv2d(flow.double(), wq.double(), torch.from_numpy(bias).double(), padding=3))
    ref = ref.permute(0, 2, 3, 1).reshape(P, n)
    got = f1o[:, :n].cpu().double()
    scale = float(ref.abs().max())
    err = float((got - ref).abs().max())
    assert err < 2e-6 * max(1.0, scale) * 10, (err, scale)
    assert bool((f1o[:, n:] == -7.0).all())  # nothing past n channels of a row
    return int(flag.item()), scale


@pytest.mark.parametrize("B,h,w,r", [(1, 55, 128, 4), (2, 17, 21, 3), (1, 19, 27, 6)])
@pytest.mark.parametrize("prec", ["f16x3", "f16", "bf16"])
def test_lookup_convf1_equals_lookup_and_conv(B, h, w, r, prec):
    """The fused lookup + motion-encoder convf1 (raft_corr_lookup_convf1): lookup outputs
    bit-identical to raft_corr_lookup's (RAFT's r = 4, r = 3, and r = 6 through the generic
    lookup then the convf1 blocks alone), convf1 within fp32 rounding of an fp64 conv of the
    same operands (flow and weights rounded to f16 / bf16 in those modes); ragged tiles."""
    from raft_optical_flow_amd import _lib
    p = {"f16x3": _lib.PREC_F16X3, "f16": _lib.PREC_F16, "bf16": _lib.PREC_BF16}[prec]
    flag, _ = _lookup_convf1_case(B, h, w, r, p)
    assert flag == 0


def test_lookup_convf1_range_guard():
    """A flow so large that convf1's output leaves the f16x3 split range raises the flag."""
    from raft_optical_flow_amd import _lib
    flag, scale = _lookup_convf1_case(1, 12, 20, 4, _lib.PREC_F16X3, coord_scale=3e5, seed=3)
    assert scale > 32768 and flag == 1


@pytest.mark.parametrize("n", [1, 2])
@pytest.mark.parametrize("C", [96, 260])
def test_alt_cuda_corr_forward_vs_oracle(n, C):
    """C = 96: a partial 256-channel slab; C = 260: two slabs (NV = 2), the second a single quad."""
    from raft_optical_flow_amd import alt_cuda_corr
    rng = np.random.default_rng(2)
    B, H1, W1, H2, W2, r = 2, 9, 13, 5, 7, 4
    f1 = rng.standard_normal((B, H1, W1, C)).astype(np.float32)
    f2 = rng.standard_normal((B, H2, W2, C)).astype(np.float32)
    coords = rng.uniform(-4, 12, (B, n, H1, W1, 2)).astype(np.float32)
    corr, = alt_cuda_corr.forward(t(f1), t(f2), t(coords), r)
    ref = O.alt_corr_forward(f1, f2, coords, r)
    assert corr.shape == ref.shape
    assert maxabs(corr, ref) < 1e-4


@pytest.mark.parametrize("layout", [0, 1])
def test_alt_corr_tiled_vs_oracle(layout):
    """The tiled alt kernel (8x8 query tiles, window box staged in LDS): tiles whose box fits,
    one tile forced onto the per-pixel path by a far coordinate, ragged edge tiles; the
    reference's [B,N,81,H,W] output and the NHWC-row variant."""
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    rng = np.random.default_rng(5)
    B, H1, W1, C, r = 2, 19, 29, 64, 4
    H2, W2 = 19, 29
    f1 = rng.standard_normal((B, H1, W1, C)).astype(np.float32)
    f2 = rng.standard_normal((B, H2, W2, C)).astype(np.float32)
    ys, xs = np.meshgrid(np.arange(H1), np.arange(W1), indexing="ij")
    coords = np.stack([xs, ys], -1)[None, None].astype(np.float32).repeat(B, 0)
    coords = (coords + rng.normal(0, 1.0, coords.shape)).astype(np.float32)
    coords[1, 0, 9, 12] = (40.5, -7.25)  # that tile's box does not fit
    ref = O.alt_corr_forward(f1, f2, coords, r)  # [B, 1, 81, H1, W1], unscaled
    if layout == 0:
        from raft_optical_flow_amd import alt_cuda_corr
        corr, = alt_cuda_corr.forward(t(f1), t(f2), t(coords), r)
        assert maxabs(corr, ref) < 1e-4
    else:
        out = torch.empty(B * H1 * W1, 81, device=DEV)
        f1t, f2t, ct = t(f1), t(f2), t(coords)
        _lib.call("raft_alt_corr_lookup_nhwc", f1t.data_ptr(), f2t.data_ptr(), ct.data_ptr(), 0, 1.0, out.data_ptr(),
                  81, B, H1, W1, H2, W2, C, r, 8.0, None, 0, None, K.stream_handle())
        torch.cuda.synchronize()
        got = out.reshape(B, H1, W1, 81).permute(0, 3, 1, 2).cpu().numpy()
        assert maxabs(got, ref[:, 0] / 8.0) < 2e-5


@pytest.mark.parametrize("C,size", [(64, 95), (64, 96), (64, 97), (40, 27), (40, 28), (40, 29)])
@pytest.mark.parametrize("edge", [False, True])
def test_alt_corr_box_size_limits_vs_oracle(C, size, edge):
    """Exact window-box sizes at the alternate lookup's path limits: the 8x8 query
    tile at (0, 0) gets a box of exactly size x size fmap2 pixels — C = 64 runs the MFMA box
    GEMM (box <= 96, per-pixel path at 97), C = 40 the VALU tile kernel (box <= 28, per-pixel
    at 29); edge=True puts that box over the map's right and bottom edges (zeros there)."""
    from raft_optical_flow_amd import _lib
    from raft_optical_flow_amd import kernels as K
    rng = np.random.default_rng(size + C)
    B, H1, W1, r = 1, 16, 16, 4
    H2 = W2 = 112
    f1 = rng.standard_normal((B, H1, W1, C)).astype(np.float32)
    f2 = rng.standard_normal((B, H2, W2, C)).astype(np.float32)
    ys, xs = np.meshgrid(np.arange(H1), np.arange(W1), indexing="ij")
    coords = np.stack([xs, ys], -1)[None, None].astype(np.float32)
    coords = (coords + rng.normal(0, 0.7, coords.shape)).astype(np.float32)
    # tile (0, 0): floor(x) spans exactly size - (2r + 2) columns (and rows): box = size x size
    span = size - (2 * r + 2)
    x0 = (W2 - span + 2.3) if edge else 6.3
    y0 = (H2 - span + 1.6) if edge else 5.6
    jj, ii = np.meshgrid(np.arange(8), np.arange(8))
    coords[0, 0, :8, :8, 0] = x0 + np.round(span * jj / 7.0)
    coords[0, 0, :8, :8, 1] = y0 + np.round(span * ii / 7.0)
    ref = O.alt_corr_forward(f1, f2, coords, r)  # [B, 1, 81, H1, W1], unscaled
    out = torch.empty(B * H1 * W1, 81, device=DEV)
    f1t, f2t, ct = t(f1), t(f2), t(coords)
    _lib.call("raft_alt_corr_lookup_nhwc", f1t.data_ptr(), f2t.data_ptr(), ct.data_ptr(), 0, 1.0, out.data_ptr(), 81,
              B, H1, W1, H2, W2, C, r, 8.0, None, 0, None, K.stream_handle())
    torch.cuda.synchronize()
    got = out.reshape(B, H1, W1, 81).permute(0, 3, 1, 2).cpu().numpy()
    assert maxabs(got, ref[:, 0] / 8.0) < 2e-5


@pytest.mark.parametrize("r,spread", [(4, 0.7), (4, 6.0), (3, 0.7)])
def test_alt_corr_levels_equals_per_level_calls(r, spread):
    """raft_alt_corr_lookup_levels (one launch at r = 4) == the L raft_alt_corr_lookup_nhwc calls, bit for bit,
    with small and large window boxes (spread 6 px: boxes beyond the VALU kernel's 28 x 28)."""
    from raft_optical_flow_amd import kernels as K
    from raft_optical_flow_amd import _lib
    g = torch.Generator().manual_seed(21)
    B, h, w, C, L = 2, 24, 40, 256, 4
    f1 = torch.randn(B * h * w, C, generator=g).to(DEV)
    lv = [(torch.randn(B * (h >> l) * (w >> l), C, generator=g).to(DEV), h >> l, w >> l) for l in range(L)]
    ys, xs = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
    grid = torch.stack([xs, ys], -1).float().reshape(1, h * w, 2).repeat(B, 1, 1)
    coords = (grid + spread * torch.randn(grid.shape, generator=g)).reshape(-1, 2).contiguous().to(DEV)
    nb = (2 * r + 1) ** 2
    one = torch.full((B * h * w, L * nb), 7.0, device=DEV)
    per = torch.full((B * h * w, L * nb), 7.0, device=DEV)
    f1o, f1p = (torch.zeros(B * h * w, 2, device=DEV) for _ in range(2))
    s = K.stream_handle()
    arrs = K.alt_levels_args(lv)
    _lib.call("raft_alt_corr_lookup_levels", f1.data_ptr(), *arrs, L, coords.data_ptr(), 0, one.data_ptr(), L * nb,
              B, h, w, C, r, 16.0, f1o.data_ptr(), 2, None, s)
    for l, (f2, hh, ww) in enumerate(lv):
        _lib.call("raft_alt_corr_lookup_nhwc", f1.data_ptr(), f2.data_ptr(), coords.data_ptr(), 0, float(2 ** l),
                  per.data_ptr() + 4 * l * nb, L * nb, B, h, w, hh, ww, C, r, 16.0,
                  f1p.data_ptr() if l == 0 else None, 2, None, s)
    torch.cuda.synchronize()
    assert torch.equal(one, per) and torch.equal(f1o, f1p)
    # and the oracle, per level
    from oracle import raft_oracle as O
    co = coords.cpu().numpy().reshape(B, 1, h, w, 2)
    for l, (f2, hh, ww) in enumerate(lv):
        ref = O.alt_corr_forward(f1.cpu().numpy().reshape(B, h, w, C), f2.cpu().numpy().reshape(B, hh, ww, C),
                                 co / 2 ** l, r)[:, 0] / 16.0
        got = one[:, l * nb:(l + 1) * nb].cpu().numpy().reshape(B, h, w, nb).transpose(0, 3, 1, 2)
        assert np.abs(got - ref).max() < 2e-5, (l, np.abs(got - ref).max())


@pytest.mark.parametrize("r", [4, 3])
def test_alternate_corr_block_golden(r):
    from raft_optical_flow_amd import AlternateCorrBlock
    g = load_golden("lookup_b2c64_16x20.npz")
    ab = AlternateCorrBlock(t(g["fmap1"]), t(g["fmap2"]), num_levels=4, radius=r)
    out = ab(t(g["coords"]))
    assert maxabs(out, g[f"iter_r{r}"]) < 5e-5
    assert maxabs(out, g[f"corr_r{r}"]) < 5e-5


def _alt_bwd_case(seed, B, H1, W1, H2, W2, C, N, r, spread):
    rng = np.random.default_rng(seed)
    f1 = rng.standard_normal((B, H1, W1, C)).astype(np.float32)
    f2 = rng.standard_normal((B, H2, W2, C)).astype(np.float32)
    ys, xs = np.meshgrid(np.arange(H1), np.arange(W1), indexing="ij")
    base = np.stack([xs * (W2 / W1), ys * (H2 / H1)], -1)[None, None]
    coords = (base + rng.normal(0, spread, (B, N, H1, W1, 2))).astype(np.float32)
    gout = rng.standard_normal((B, N, (2 * r + 1) ** 2, H1, W1)).astype(np.float32)
    return f1, f2, coords, gout


@pytest.mark.parametrize("case", [
    dict(seed=3, B=1, H1=6, W1=7, H2=6, W2=7, C=32, N=1, r=2, spread=2.0),
    dict(seed=4, B=2, H1=9, W1=13, H2=5, W2=7, C=96, N=2, r=4, spread=3.0),    # pooled level, N = 2
    dict(seed=5, B=1, H1=8, W1=8, H2=8, W2=8, C=260, N=1, r=3, spread=9.0),    # far out of bounds, C > 256
    dict(seed=6, B=1, H1=10, W1=12, H2=10, W2=12, C=64, N=1, r=6, spread=3.0),  # r = 6: 196 taps (4-wave blocks)
    dict(seed=7, B=1, H1=5, W1=6, H2=9, W2=11, C=32, N=1, r=23, spread=2.0),   # r = 23: 2304 taps (1-wave blocks)
])
def test_alt_cuda_corr_backward_vs_autograd(case):
    """alt_cuda_corr.backward against autograd (fp64) through the differentiable restatement
    oracle/torch_cpu.alt_corr_forward (correlation_kernel.cu:18-119): fmap1, fmap2 and the
    coordinate gradient (the reference leaves coords_grad zero)."""
    from oracle import torch_cpu as T
    from raft_optical_flow_amd import alt_cuda_corr
    r = case["r"]
    f1, f2, coords, gout = _alt_bwd_case(**case)
    f1g, f2g, cg = alt_cuda_corr.backward(t(f1), t(f2), t(coords), t(gout), r)
    a, b, c = (torch.tensor(x, dtype=torch.float64, requires_grad=True) for x in (f1, f2, coords))
    (T.alt_corr_forward(a, b, c, r) * torch.tensor(gout, dtype=torch.float64)).sum().backward()
    for got, ref in ((f1g, a.grad), (f2g, b.grad), (cg, c.grad)):
        scale = max(1.0, float(ref.abs().max()))
        assert maxabs(got, ref) < 2e-5 * scale * np.sqrt(case["C"])


def test_alt_cuda_corr_backward_is_deterministic():
    """Bit-identical gradients run to run (the reference's fmap2 scatter uses float atomics),
    on a field where every fmap2 pixel collects many (query, tap) contributions."""
    from raft_optical_flow_amd import alt_cuda_corr
    f1, f2, coords, gout = _alt_bwd_case(seed=8, B=2, H1=24, W1=40, H2=24, W2=40, C=128, N=1, r=4, spread=1.5)
    args = (t(f1), t(f2), t(coords), t(gout), 4)
    first = alt_cuda_corr.backward(*args)
    for _ in range(3):
        again = alt_cuda_corr.backward(*args)
        for x, y in zip(first, again):
            assert torch.equal(x, y)


def test_alt_corr_autograd_function():
    """alt_cuda_corr.alt_corr (torch.autograd.Function): forward equals forward(); gradients reach
    fmap1, fmap2 and coords and equal backward()."""
    from raft_optical_flow_amd import alt_cuda_corr
    f1, f2, coords, gout = _alt_bwd_case(seed=9, B=1, H1=7, W1=9, H2=7, W2=9, C=64, N=1, r=4, spread=1.0)
    a, b, c = (t(x).requires_grad_(True) for x in (f1, f2, coords))
    out = alt_cuda_corr.alt_corr(a, b, c, 4)
    ref, = alt_cuda_corr.forward(t(f1), t(f2), t(coords), 4)
    assert torch.equal(out.detach(), ref)
    (out * t(gout)).sum().backward()
    f1g, f2g, cg = alt_cuda_corr.backward(t(f1), t(f2), t(coords), t(gout), 4)
    assert torch.equal(a.grad, f1g) and torch.equal(b.grad, f2g) and torch.equal(c.grad, cg)


# ----------------------------------------------------------------------------- convolution


CONV_CASES = [
    # cin, cout, kh, kw, stride, pad, H, W, B
    (324, 256, 1, 1, 1, (0, 0), 11, 13, 2),
    (256, 192, 3, 3, 1, (1, 1), 9, 17, 1),
    (2, 128, 7, 7, 1, (3, 3), 10, 12, 1),
    (384, 256, 1, 5, 1, (0, 2), 8, 19, 1),
    (384, 128, 5, 1, 1, (2, 0), 21, 6, 1),
    (3, 64, 7, 7, 2, (3, 3), 37, 45, 2),
    (64, 96, 3, 3, 2, (1, 1), 19, 24, 1),
    (96, 96, 1, 1, 2, (0, 0), 19, 24, 1),
    (256, 2, 3, 3, 1, (1, 1), 7, 9, 1),
    (256, 2, 3, 3, 1, (1, 1), 13, 35, 2),
    (96, 3, 3, 3, 1, (1, 1), 9, 21, 1),
    (128, 2, 1, 1, 1, (0, 0), 6, 10, 1),
    (128, 576, 1, 1, 1, (0, 0), 5, 6, 1),
    (256, 126, 3, 3, 1, (1, 1), 12, 12, 1),
]


CONV_TOL = {"fp32": 1e-4, "f16x3": 1e-4, "f16": 5e-3, "bf16": 3e-2}


@pytest.mark.parametrize("prec", ["fp32", "f16x3", "f16", "bf16"])
@pytest.mark.parametrize("cin,cout,kh,kw,stride,pad,H,W,B", CONV_CASES)
def test_conv2d_vs_torch_fp64(cin, cout, kh, kw, stride, pad, H, W, B, prec):
    from raft_optical_flow_amd import kernels as K
    from raft_optical_flow_amd import _lib
    g = torch.Generator().manual_seed(cin * 1000 + cout)
    x = torch.randn(B, cin, H, W, generator=g)
    w = torch.randn(cout, cin, kh, kw, generator=g) / np.sqrt(cin * kh * kw)
    b = torch.randn(cout, generator=g)
    ref = F.conv2d(x.double(), w.double(), b.double(), stride, pad)
    pc = K.pack_conv(w, b, stride, pad, device=DEV)
    pc.precision = _lib.PRECISIONS[prec]
    src = K.Rows(K.nchw_to_rows(x.to(DEV)))
    ho, wo = ref.shape[-2:]
    out = K.Rows(torch.empty(B * ho * wo, cout, device=DEV))
    K.conv2d_rows(pc, src, B, H, W, out, epilogue=_lib.EPI_LINEAR)
    y = K.rows_to_nchw(out, B, ho, wo)
    err = maxabs(y, ref)
    assert err < CONV_TOL[prec] * max(1.0, float(ref.abs().max())), err


@pytest.mark.parametrize("prec", ["bf16", "f16"])
@pytest.mark.parametrize("cin,cout,kh,kw,H,W", [
    (96, 256, 3, 3, 60, 70),    # ragged tiles in both axes, 640 128-column tiles
    (128, 128, 1, 5, 60, 130),  # N = 128: one column tile per spatial tile, 576 tiles
    (64, 256, 5, 1, 61, 64),
    (64, 256, 1, 1, 60, 70),
])
def test_conv_halo_wide_tiles_multi_round(cin, cout, kh, kw, H, W, prec):
    """The one-product modes' 128-column halo tiles (2 x 2 waves of 64 pixels x 64 columns, chosen
    for convs with >= 2 rounds of work-groups: configs 3 - 5) vs torch fp64 on the first and last
    image; the output row padding stays untouched."""
    from raft_optical_flow_amd import kernels as K
    from raft_optical_flow_amd import _lib
    B = 8
    g = torch.Generator().manual_seed(cin + cout + kh)
    x = torch.randn(B, cin, H, W, generator=g)
    w = torch.randn(cout, cin, kh, kw, generator=g) / np.sqrt(cin * kh * kw)
    b = torch.randn(cout, generator=g)
    pad = ((kh - 1) // 2, (kw - 1) // 2)
    pc = K.pack_conv(w, b, 1, pad, device=DEV)
    pc.precision = _lib.PRECISIONS[prec]
    src = K.Rows(K.nchw_to_rows(x.to(DEV)))
    out = K.Rows(torch.full((B * H * W, cout + 4), -7.0, device=DEV), 0, cout)
    K.conv2d_rows(pc, src, B, H, W, out, epilogue=_lib.EPI_RELU)
    y = K.rows_to_nchw(out, B, H, W)
    for i in (0, B - 1):
        ref = torch.relu(F.conv2d(x[i:i + 1].double(), w.double(), b.double(), 1, pad))
        assert maxabs(y[i:i + 1], ref) < CONV_TOL[prec] * max(1.0, float(ref.abs().max())), i
    assert bool((out.t[:, cout:] == -7.0).all())


@pytest.mark.parametrize("prec", ["f16x3", "bf16", "f16"])
@pytest.mark.parametrize("cin,cout,H,W,B", [
    (96, 96, 110, 256, 2),    # fnet layer2 at config 2 (448 big tiles, N padded to 128)
    (256, 192, 61, 70, 8),    # ragged tiles in both axes (480 big tiles)
    (256, 192, 55, 128, 8),   # convc2 at B = 8
])
def test_conv_halo_big_tiles_multi_round(cin, cout, H, W, B, prec):
    import ctypes
    """The multi-round 3x3 halo tiles (16 x 16 pixels x 64 columns, each compute wave 2 x 2 MFMA blocks;
    f16x3 on the column-scaled weight with one accumulator) vs torch fp64 on the first and last image,
    and vs the 128-pixel tiles of the same conv (RAFT_HALO_BIG_MIN is read once per process, so the
    small-tile reference is the same conv without weight_s in f16x3, or at fp64 in the other modes);
    the output row padding stays untouched."""
    from raft_optical_flow_amd import kernels as K
    from raft_optical_flow_amd import _lib
    g = torch.Generator().manual_seed(cin + cout + H)
    x = torch.randn(B, cin, H, W, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) / np.sqrt(cin * 9)
    w[:, :, 1, 1] *= 1e-4  # small weights beside large ones in every column (the scaled lo's range)
    b = torch.randn(cout, generator=g)
    pc = K.pack_conv(w, b, 1, 1, device=DEV)
    pc.precision = _lib.PRECISIONS[prec]
    src = K.Rows(K.nchw_to_rows(x.to(DEV)))
    out = K.Rows(torch.full((B * H * W, cout + 4), -7.0, device=DEV), 0, cout)
    p = K.conv_params(pc, src, B, H, W, out, epilogue=_lib.EPI_RELU)
    assert (p.weight_s is not None) == (prec == "f16x3")
    assert _lib.load().raft_conv2d_halo_tile_rows(ctypes.byref(p)) == 16  # the rounds rule picks big tiles
    K.conv_launch(p)(K.stream_handle())
    y = K.rows_to_nchw(out, B, H, W)
    for i in (0, B - 1):
        ref = torch.relu(F.conv2d(x[i:i + 1].double(), w.double(), b.double(), 1, 1))
        assert maxabs(y[i:i + 1], ref) < CONV_TOL[prec] * max(1.0, float(ref.abs().max())), i
    assert bool((out.t[:, cout:] == -7.0).all())
    if prec == "f16x3":
        out2 = K.Rows(torch.full((B * H * W, cout + 4), -7.0, device=DEV), 0, cout)
        p2 = K.conv_params(pc, src, B, H, W, out2, epilogue=_lib.EPI_RELU)
        p2.weight_s = None  # the 128-pixel tiles, unscaled two-chain form
        K.conv_launch(p2)(K.stream_handle())
        ref2 = out2.t[:, :cout]
        assert maxabs(out.t[:, :cout], ref2) < 2e-5 * max(1.0, float(ref2.abs().max()))


@pytest.mark.parametrize("prec", ["f16x3", "bf16", "f16"])
@pytest.mark.parametrize("cin,cout,kh,kw,H,W,B", [
    (256, 128, 1, 5, 55, 128, 8),   # q (1x5) at B = 8: 512 big tiles, 16 x 20 patch
    (256, 128, 5, 1, 50, 120, 8),   # q (5x1), ragged rows: 512 big tiles, 20 x 16 patch
])
def test_conv_halo_big_tiles_1x5_5x1(cin, cout, kh, kw, H, W, B, prec):
    """1x5 / 5x1 convs on the multi-round 16 x 16 tiles vs torch fp64 (f16x3: the scaled split, D = 2 with
    fp32 patches; one-product modes: pre-split patches, D = 3)."""
    from raft_optical_flow_amd import kernels as K
    from raft_optical_flow_amd import _lib
    g = torch.Generator().manual_seed(cin + cout + kh * 7)
    x = torch.randn(B, cin, H, W, generator=g)
    w = torch.randn(cout, cin, kh, kw, generator=g) / np.sqrt(cin * kh * kw)
    b = torch.randn(cout, generator=g)
    pad = ((kh - 1) // 2, (kw - 1) // 2)
    pc = K.pack_conv(w, b, 1, pad, device=DEV)
    pc.precision = _lib.PRECISIONS[prec]
    src = K.Rows(K.nchw_to_rows(x.to(DEV)))
    out = K.Rows(torch.full((B * H * W, cout + 4), -7.0, device=DEV), 0, cout)
    import ctypes
    p = K.conv_params(pc, src, B, H, W, out, epilogue=_lib.EPI_LINEAR)
    assert _lib.load().raft_conv2d_halo_tile_rows(ctypes.byref(p)) == 16
    K.conv_launch(p)(K.stream_handle())
    y = K.rows_to_nchw(out, B, H, W)
    for i in (0, B - 1):
        ref = F.conv2d(x[i:i + 1].double(), w.double(), b.double(), 1, pad)
        assert maxabs(y[i:i + 1], ref) < CONV_TOL[prec] * max(1.0, float(ref.abs().max())), i
    assert bool((out.t[:, cout:] == -7.0).all())


def test_conv2d_split_weight_scaled_layout():
    """raft_conv2d_split_weight_scaled: per row a power of two S_n with max |w S_n| in [2^13, 2^14), per
    K-step 32 f16 hi = f16(w S_n) then 32 f16 lo = f16(w S_n - hi), then the n_pad floats 1 / S_n; a zero
    row gets S_n = 1."""
    from raft_optical_flow_amd import _lib
    g = torch.Generator().manual_seed(13)
    w = (torch.randn(64, 96, generator=g) * 0.05)
    w[5] *= 1e-6
    w[7] = 0.0
    w = w.to(DEV)
    nbytes = int(_lib.load().raft_conv2d_split_scaled_bytes(64, 96))
    assert nbytes == 64 * 96 * 4 + 64 * 4
    out = torch.empty(nbytes // 4, device=DEV)
    _lib.call("raft_conv2d_split_weight_scaled", w.data_ptr(), out.data_ptr(), 64, 96, 0)
    torch.cuda.synchronize()
    inv = out[64 * 96:].cpu().double()
    h = out[: 64 * 96].view(torch.float16).view(64, 3, 2, 32).cpu()
    wc = w.cpu().double()
    mx = wc.abs().max(1).values
    sc = 1.0 / inv
    assert bool((torch.log2(sc) == torch.round(torch.log2(sc))).all())
    nz = mx > 0
    assert bool(((mx * sc)[nz] < 2 ** 14).all()) and bool(((mx * sc)[nz] >= 2 ** 13).all()) and float(sc[7]) == 1.0
    ws = (wc * sc[:, None]).view(64, 3, 32)
    hi = ws.float().half()
    lo = (ws - hi.double()).float().half()
    assert torch.equal(h[:, :, 0], hi) and torch.equal(h[:, :, 1], lo)
    rec = (h[:, :, 0].double() + h[:, :, 1].double()) * inv[:, None, None]
    assert float(((rec - wc.view(64, 3, 32)).abs() / mx[:, None, None].clamp_min(1e-30)).max()) < 2.0 ** -21


@pytest.mark.parametrize("prec", ["f16x3", "bf16"])
def test_conv_stem_full_size_relu(prec):
    """The encoders' 7x7 / stride-2 stem (conv_stem.hip) at config 2's size (440x1024 -> 220x512:
    896 tiles per image, more than one per work-group) with the relu epilogue and the range guard,
    against torch fp64."""
    from raft_optical_flow_amd import kernels as K
    from raft_optical_flow_amd import _lib
    g = torch.Generator().manual_seed(7)
    B, H, W = 2, 440, 1024
    x = torch.rand(B, 3, H, W, generator=g) * 2 - 1
    w = torch.randn(64, 3, 7, 7, generator=g) / np.sqrt(147)
    b = torch.randn(64, generator=g) * 0.1
    ref = torch.relu(F.conv2d(x.double(), w.double(), b.double(), 2, 3))
    pc = K.pack_conv(w, b, 2, 3, device=DEV)
    pc.precision = _lib.PRECISIONS[prec]
    src = K.Rows(K.nchw_to_rows(x.to(DEV)))
    out = K.Rows(torch.full((B * 220 * 512, 68), -7.0, device=DEV), 0, 64)
    flag = torch.zeros(1, dtype=torch.int32, device=DEV)
    K.conv2d_rows(pc, src, B, H, W, out, epilogue=_lib.EPI_RELU, range_flag=flag)
    y = K.rows_to_nchw(out, B, 220, 512)
    assert maxabs(y, ref) < CONV_TOL[prec] * max(1.0, float(ref.abs().max()))
    assert bool((out.t[:, 64:] == -7.0).all())
    assert int(flag.item()) == 0


def test_conv2d_split_weight_layout():
    """raft_conv2d_split_weight: per 32-wide K-step, 32 f16 hi then 32 f16 lo (x2048)."""
    from raft_optical_flow_amd import _lib
    g = torch.Generator().manual_seed(11)
    w = (torch.randn(64, 96, generator=g) * 0.05).to(DEV)
    out = torch.empty_like(w)
    _lib.call("raft_conv2d_split_weight", w.data_ptr(), out.data_ptr(), 64, 96, 0)
    torch.cuda.synchronize()
    h = out.view(torch.float16).view(64, 3, 2, 32)
    hi = w.view(64, 3, 32).half()
    lo = ((w.view(64, 3, 32) - hi.float()) * 2048).half()
    assert torch.equal(h[:, :, 0], hi) and torch.equal(h[:, :, 1], lo)
    rec = h[:, :, 0].double() + h[:, :, 1].double() / 2048
    assert float((rec - w.view(64, 3, 32).double()).abs().max()) < 2.0 ** -22 * 0.25


def test_conv2d_split_weight_bf16_layout():
    """raft_conv2d_split_weight_prec(RAFT_PREC_BF16): per K-step 32 bf16 hi (RNE) then 32 bf16 lo = bf16(x - hi)."""
    from raft_optical_flow_amd import _lib
    g = torch.Generator().manual_seed(12)
    w = (torch.randn(64, 96, generator=g) * 0.05).to(DEV)
    out = torch.empty_like(w)
    _lib.call("raft_conv2d_split_weight_prec", w.data_ptr(), out.data_ptr(), 64, 96, _lib.PREC_BF16, 0)
    torch.cuda.synchronize()
    h = out.view(torch.bfloat16).view(64, 3, 2, 32)
    hi = w.view(64, 3, 32).bfloat16()
    lo = (w.view(64, 3, 32) - hi.float()).bfloat16()
    assert torch.equal(h[:, :, 0], hi) and torch.equal(h[:, :, 1], lo)


@pytest.mark.parametrize("prec", ["fp32", "f16x3"])
def test_conv2d_two_segments_and_gru_epilogues(prec):
    """Virtual concat [RH | x] + the GRU z/r and q epilogues vs a torch restatement."""
    from raft_optical_flow_amd import kernels as K
    from raft_optical_flow_amd import _lib
    g = torch.Generator().manual_seed(7)
    B, H, W, hd, xd = 1, 9, 14, 128, 256
    h = torch.tanh(torch.randn(B, hd, H, W, generator=g))
    x = torch.randn(B, xd, H, W, generator=g)
    wz = torch.randn(hd, hd + xd, 1, 5, generator=g) * 0.02
    wr = torch.randn(hd, hd + xd, 1, 5, generator=g) * 0.02
    wq = torch.randn(hd, hd + xd, 1, 5, generator=g) * 0.02
    bz, br, bq = (torch.randn(hd, generator=g) * 0.1 for _ in range(3))
    hx = torch.cat([h, x], 1).double()
    z = torch.sigmoid(F.conv2d(hx, wz.double(), bz.double(), 1, (0, 2)))
    r = torch.sigmoid(F.conv2d(hx, wr.double(), br.double(), 1, (0, 2)))
    q = torch.tanh(F.conv2d(torch.cat([r * h.double(), x.double()], 1), wq.double(), bq.double(), 1, (0, 2)))
    ref = (1 - z) * h.double() + z * q
    HX = K.nchw_to_rows(torch.cat([h, x], 1).to(DEV))
    Z = torch.empty(B * H * W, hd, device=DEV)
    RH = torch.empty(B * H * W, hd, device=DEV)
    pzr = K.pack_conv(torch.cat([wz, wr]), torch.cat([bz, br]), 1, (0, 2), device=DEV)
    pq = K.pack_conv(wq, bq, 1, (0, 2), seg_real=[hd, xd], device=DEV)
    pzr.precision = pq.precision = _lib.PRECISIONS[prec]
    hrows = K.Rows(HX, 0, hd)
    K.conv2d_rows(pzr, K.Rows(HX), B, H, W, K.Rows(Z), epilogue=_lib.EPI_GRU_ZR, split=hd, aux0=hrows,
                  out1=K.Rows(RH))
    K.conv2d_rows(pq, K.Rows(RH), B, H, W, hrows, src1=K.Rows(HX, hd, xd), epilogue=_lib.EPI_GRU_Q, aux0=hrows,
                  aux1=K.Rows(Z))
    hn = K.rows_to_nchw(hrows, B, H, W)
    assert maxabs(hn, ref) < 1e-5


@pytest.mark.parametrize("prec", ["f16x3", "bf16", "fp32"])
@pytest.mark.parametrize("kh,kw,c0,n0,c1,n1,B,H,W", [
    (3, 3, 256, 192, 128, 64, 1, 55, 128),   # convc2 | convf2 of RAFT-full at config 2 (one launch)
    (3, 3, 64, 96, 32, 40, 2, 13, 21),       # ragged tiles, N padded, two images
    (1, 5, 96, 128, 64, 64, 1, 9, 19),       # another shape class
    (3, 3, 64, 64, 64, 64, 1, 8, 16),        # 3x3 beside 1x1 below: shapes differ -> two launches
])
@pytest.mark.parametrize("ks", [1, 2])
def test_conv2d_pair_equals_two_convs(kh, kw, c0, n0, c1, n1, B, H, W, prec, ks):
    """raft_conv2d_pair == raft_conv2d twice, bit for bit (each tile runs the same K-walk), with one compute
    wave per SIMD (raft_conv2d_set_halo_ks(1)).  With two (the K-split form, the default) a conv that runs
    64-column tiles in the pair but 32-column ones alone sums its K-steps in another order: there the two
    agree within 1e-5 of the output's magnitude, and bit for bit wherever both take the same form."""
    from raft_optical_flow_amd import kernels as K
    from raft_optical_flow_amd import _lib
    lib = _lib.load()
    prev_ks = lib.raft_conv2d_set_halo_ks(ks)
    try:
        g = torch.Generator().manual_seed(c0 + n1)
        shapes = [(c0, n0, kh, kw), (c1, n1, kh, kw) if (c1, n1) != (64, 64) or kh == 1 else (c1, n1, 1, 1)]
        xs, pcs, outs_pair, outs_seq = [], [], [], []
        for cin, cout, a, b in shapes:
            x = torch.randn(B, cin, H, W, generator=g)
            w = torch.randn(cout, cin, a, b, generator=g) / np.sqrt(cin * a * b)
            pc = K.pack_conv(w, torch.randn(cout, generator=g), 1, ((a - 1) // 2, (b - 1) // 2), device=DEV)
            pc.precision = _lib.PRECISIONS[prec]
            xs.append(K.Rows(K.nchw_to_rows(x.to(DEV))))
            pcs.append(pc)
            outs_pair.append(K.Rows(torch.full((B * H * W, cout), 7.0, device=DEV)))
            outs_seq.append(K.Rows(torch.full((B * H * W, cout), 7.0, device=DEV)))
        prm = [K.conv_params(pcs[i], xs[i], B, H, W, outs_pair[i], epilogue=_lib.EPI_RELU) for i in range(2)]
        K.conv_pair_launch(prm[0], prm[1])(K.stream_handle())
        for i in range(2):
            K.conv2d_rows(pcs[i], xs[i], B, H, W, outs_seq[i], epilogue=_lib.EPI_RELU)
        torch.cuda.synchronize()
        for i in range(2):
            err = maxabs(outs_pair[i].t, outs_seq[i].t)
            if ks == 1:
                assert torch.equal(outs_pair[i].t, outs_seq[i].t), (i, err)
            else:
                assert err <= 1e-5 * float(outs_seq[i].t.abs().max()), (i, err)
    finally:
        lib.raft_conv2d_set_halo_ks(prev_ks)


def test_conv2d_pair_with_a_dependence_runs_in_order():
    """The second conv reads the first one's output: the pair must not share a launch."""
    from raft_optical_flow_amd import kernels as K
    from raft_optical_flow_amd import _lib
    g = torch.Generator().manual_seed(5)
    B, H, W = 1, 16, 32
    x = K.Rows(K.nchw_to_rows(torch.randn(B, 64, H, W, generator=g).to(DEV)))
    pa = K.pack_conv(torch.randn(64, 64, 3, 3, generator=g) * 0.05, torch.zeros(64), 1, (1, 1), device=DEV)
    pb = K.pack_conv(torch.randn(64, 64, 3, 3, generator=g) * 0.05, torch.zeros(64), 1, (1, 1), device=DEV)
    mid, out, mid2, out2 = (K.Rows(torch.zeros(B * H * W, 64, device=DEV)) for _ in range(4))
    K.conv_pair_launch(K.conv_params(pa, x, B, H, W, mid, epilogue=_lib.EPI_RELU),
                       K.conv_params(pb, mid, B, H, W, out, epilogue=_lib.EPI_RELU))(K.stream_handle())
    K.conv2d_rows(pa, x, B, H, W, mid2, epilogue=_lib.EPI_RELU)
    K.conv2d_rows(pb, mid2, B, H, W, out2, epilogue=_lib.EPI_RELU)
    torch.cuda.synchronize()
    assert torch.equal(out.t, out2.t) and float(out.t.abs().max()) > 0


# ----------------------------------------------------------------------------- blocks


@pytest.mark.parametrize("small", [False, True])
def test_update_block_golden(small):
    tag = "small" if small else "full"
    g = load_golden(f"update_{tag}_16x24.npz")
    m, _ = make_model(small)
    net, mask, delta = m.update_block(t(g["net"]), t(g["inp"]), t(g["corr"]), t(g["flow"]))
    assert maxabs(net, g["net_out"]) < 1e-4
    assert maxabs(delta, g["delta_out"]) < 1e-4
    if not small:
        assert maxabs(mask, g["mask_out"]) < 1e-4


def test_upsample_golden():
    g = load_golden("upsample_16x24.npz")
    m, _ = make_model(False)
    assert maxabs(m.upsample_flow(t(g["flow"]), t(g["mask"])), g["flow_up"]) < 1e-4
    from raft_optical_flow_amd.utils.utils import upflow8
    g = load_golden("upflow8_5x7.npz")
    # the kernel works on coords = grid + flow (RAFT's state), so the API round trip adds one rounding
    assert maxabs(upflow8(t(g["flow"])), g["flow_up"]) < 2e-6 * float(np.abs(g["flow_up"]).max())


def test_encoders_golden():
    g = load_golden("encoders_64x96.npz")
    m, _ = make_model(False)
    ms, _ = make_model(True)
    img = t(g["image"])
    assert maxabs(m.fnet(img), g["fnet"]) < 1e-4
    assert maxabs(m.cnet(img[:1]), g["cnet"]) < 1e-4
    assert maxabs(ms.fnet(img), g["fnet_small"]) < 1e-4
    assert maxabs(ms.cnet(img[:1]), g["cnet_small"]) < 1e-4
    f1, f2 = m.fnet([img[:1], img[1:]])
    assert maxabs(torch.cat([f1, f2]), g["fnet"]) < 1e-4


# ----------------------------------------------------------------------------- end to end


E2E = [("raft_full_smooth_b2_128x192_i12", False, False),
       ("raft_full_rand_b1_128x192_i32", False, False),
       ("raft_full_smooth_b2_128x192_i12", False, True),   # alternate_corr path, same reference flow
       ("raft_small_smooth_b1_128x192_i12", True, False)]


@pytest.mark.parametrize("prec", ["fp32", "f16x3"])
@pytest.mark.parametrize("name,small,alt", E2E)
def test_raft_e2e_golden(name, small, alt, prec):
    g = load_golden(name + ".npz")
    m, _ = make_model(small, int(g["seed"]), alternate=alt, precision=prec)
    with torch.no_grad():
        low, up = m(t(g["image1"]), t(g["image2"]), iters=int(g["iters"]), test_mode=True)
    assert maxabs(low, g["flow_low"]) < 1e-3
    assert maxabs(up, g["flow_up"]) < 1e-3


def test_raft_train_mode_output_list_and_graph_replay():
    g = load_golden("raft_full_smooth_b2_128x192_i12.npz")
    m, _ = make_model(False, 0)
    i1, i2 = t(g["image1"]), t(g["image2"])
    with torch.no_grad():
        preds = m(i1, i2, iters=12, test_mode=False)
        assert isinstance(preds, list) and len(preds) == 12
        assert maxabs(preds[-1], g["flow_up"]) < 1e-3
        assert m.hip_graph  # the default: graph replay from a plan's second forward on
        low0, up0 = m(i1, i2, iters=12, test_mode=True)   # first forward of the plan: eager
        pl = m.plan(2, 128, 192, 12, True)
        assert pl.graph is None and pl.runs == 1
        low1, up1 = m(i1, i2, iters=12, test_mode=True)   # captured, replayed
        assert pl.graph is not None
        low2, up2 = m(i1, i2, iters=12, test_mode=True)   # replayed
    assert maxabs(low1, low0) == 0.0 and maxabs(up1, up0) == 0.0
    assert maxabs(up2, up0) == 0.0


def test_plan_cache_is_a_bounded_lru():
    """RAFT_MAX_PLANS (default 2) plans per model; the evicted plan's buffers and graph are freed."""
    m, _ = make_model(False, 0)
    x = torch.zeros(1, 3, 64, 96, device=DEV)
    with torch.no_grad():
        for _ in range(2):
            m(x, x, iters=2, test_mode=True)
        first = m.plan(1, 64, 96, 2, True)
        assert first.graph is not None
        m(x, x, iters=3, test_mode=True)
        m(x, x, iters=4, test_mode=True)
    assert len(m._plans) == 2 and first.graph is None and first.pyramid is None
    m.release_plans()
    assert len(m._plans) == 0


def test_raft_flow_init_warm_start():
    g = load_golden("raft_full_smooth_b2_128x192_i12.npz")
    m, p = make_model(False, 0)
    rng = np.random.default_rng(5)
    finit = rng.uniform(-2, 2, (2, 2, 16, 24)).astype(np.float32)
    with torch.no_grad():
        low, up = m(t(g["image1"]), t(g["image2"]), iters=3, flow_init=t(finit), test_mode=True)
    rlow, rup = O.raft_forward(p, g["image1"], g["image2"], iters=3, flow_init=finit)
    assert maxabs(low, rlow) < 1e-3 and maxabs(up, rup) < 1e-3


@pytest.mark.parametrize("prec", ["fp32", "f16x3"])
def test_raft_full_size_golden(prec):
    """Config 2 shape: B=1, 436x1024 padded to 440x1024, iters=32."""
    from raft_optical_flow_amd.init import seeded_images
    g = load_golden("raft_full_rand_b1_440x1024_i32.npz")
    m, _ = make_model(False, int(g["seed"]), precision=prec)
    i1, i2 = seeded_images(1, 440, 1024, seed=int(g["img_seed"]))
    with torch.no_grad():
        low, up = m(i1.to(DEV), i2.to(DEV), iters=32, test_mode=True)
    err = (maxabs(low, g["flow_low"]), maxabs(up[:, :, ::8], g["flow_up_rows8"]))
    print(f"full-size {prec}: flow_low {err[0]:.3g} flow_up {err[1]:.3g}")
    assert err[0] < 1e-3 and err[1] < 1e-3


def test_raft_mixed_precision_band():
    """args.mixed_precision -> one f16 product per MAC (the reference autocasts to fp16,
    core/raft.py:156): its own band against the fp32 reference flow."""
    from raft_optical_flow_amd import RAFT
    from raft_optical_flow_amd.init import seeded_state_dict
    g = load_golden("raft_full_rand_b1_128x192_i32.npz")
    m = RAFT(argparse.Namespace(small=False, mixed_precision=True, alternate_corr=False))
    m.load_state_dict(seeded_state_dict(m, int(g["seed"])))
    m.to(DEV).eval()
    assert m.resolved_precision() == "f16"
    with torch.no_grad():
        low, up = m(t(g["image1"]), t(g["image2"]), iters=int(g["iters"]), test_mode=True)
    d = (up.cpu().double() - torch.from_numpy(g["flow_up"]).double()).abs()
    print(f"f16 band: max {float(d.max()):.3g} mean {float(d.mean()):.3g}")
    assert float(d.max()) < 0.5 and float(d.mean()) < 0.05


def test_raft_small_demo_frames_golden():
    """Config 1: raft-small.pth on demo-frames 0016 -> 0017 (InputPadder, iters=12)."""
    from PIL import Image
    from raft_optical_flow_amd import RAFT, InputPadder
    g = load_golden("raft_small_demo_0016_0017_i12.npz")
    wts = load_golden("raft_small_weights.npz")
    m = RAFT(argparse.Namespace(small=True, mixed_precision=False, alternate_corr=False))
    m.load_state_dict({k: torch.from_numpy(v) for k, v in wts.items()})
    m.to(DEV).eval()

    def load(key):
        a = np.array(Image.open(io.BytesIO(g[key].tobytes()))).astype(np.uint8)
        return torch.from_numpy(a).permute(2, 0, 1).float()[None].to(DEV)

    i1, i2 = load("png1"), load("png2")
    padder = InputPadder(i1.shape)
    assert list(padder._pad) == list(g["pad"])
    i1, i2 = padder.pad(i1, i2)
    with torch.no_grad():
        low, up = m(i1, i2, iters=12, test_mode=True)
    assert maxabs(low, g["flow_low"]) < 1e-3
    assert maxabs(up[:, :, ::4], g["flow_up_rows4"]) < 1e-3


def test_f16x3_range_guard_falls_back_to_fp32():
    """Activations beyond f16's range (fnet head scaled so |fmap| ~ 1e5 > 65504): the split-f16
    arithmetic alone would turn them into inf; the range guard (raft_hip.h, RAFT_RANGE_LIMIT) is
    raised by the fnet head's epilogue and the lookups, and RAFT.forward (the default "fallback"
    mode) returns the re-run on exact f32 MFMA (same result as conv_precision="fp32"); "deferred"
    corrects the returned tensors at check_range_guard(); "raise" raises; with the guard off the
    hole it closes shows."""
    import warnings
    g = load_golden("raft_full_rand_b1_128x192_i32.npz")
    m, _ = make_model(False, 0)
    with torch.no_grad():
        m.fnet.conv2.weight.mul_(20000.0)
        m.fnet.conv2.bias.mul_(20000.0)
    i1, i2 = t(g["image1"]), t(g["image2"])
    ref_m, _ = make_model(False, 0, precision="fp32")
    ref_m.load_state_dict(m.state_dict())
    with torch.no_grad():
        fm = ref_m.fnet(i1)
        assert float(fm.abs().max()) > 65504.0
        rlow, rup = ref_m(i1, i2, iters=4, test_mode=True)
        # "fallback" (default): forward() itself waits for the flag and returns the re-run's result
        assert m.range_guard == "fallback"
        with pytest.warns(RuntimeWarning, match="range guard"):
            low, up = m(i1, i2, iters=4, test_mode=True)
        assert maxabs(low, rlow) == 0.0 and maxabs(up, rup) == 0.0
        # "deferred": the check waits; check_range_guard() resolves it and the returned tensors
        # then hold the exact-f32 re-run's result
        m.range_guard = "deferred"
        low, up = m(i1, i2, iters=4, test_mode=True)
        with pytest.warns(RuntimeWarning, match="inexact"):
            m.check_range_guard()
        assert maxabs(low, rlow) == 0.0 and maxabs(up, rup) == 0.0
        m.range_guard = "raise"
        with pytest.raises(FloatingPointError):
            m(i1, i2, iters=4, test_mode=True)
        m.range_guard = "off"
        with warnings.catch_warnings():
            warnings.simplefilter("error")
            low_off, up_off = m(i1, i2, iters=4, test_mode=True)
    assert not bool(torch.isfinite(up_off).all()) or maxabs(up_off, rup) > 1e-3


def test_forward_repacks_weights_changed_between_calls():
    """The steady-state forward() enqueues its cached plan before it checks the weights key (raft.py):
    weights edited in place or reloaded by load_state_dict after earlier forwards must still give the
    result of a model built from the new weights, bit for bit, and the original weights the original
    result."""
    from raft_optical_flow_amd.init import seeded_state_dict
    g = load_golden("raft_full_rand_b1_128x192_i32.npz")
    m, _ = make_model(False, 0)
    i1, i2 = t(g["image1"]), t(g["image2"])
    with torch.no_grad():
        for _ in range(3):  # eager run, graph capture, replay: the plan is cached
            a_low, a_up = m(i1, i2, iters=4, test_mode=True)
        m.update_block.flow_head.conv2.weight.mul_(1.5)  # in place, after the plan was packed
        b_low, b_up = m(i1, i2, iters=4, test_mode=True)
        ref, _ = make_model(False, 0)
        ref.load_state_dict(m.state_dict())
        r_low, r_up = ref(i1, i2, iters=4, test_mode=True)
        assert maxabs(b_up, r_up) == 0.0 and maxabs(b_low, r_low) == 0.0
        assert maxabs(a_up, b_up) > 1e-3
        m.load_state_dict(seeded_state_dict(m, 0))  # back to the first weights (an in-place copy_)
        c_low, c_up = m(i1, i2, iters=4, test_mode=True)
        assert maxabs(c_up, a_up) == 0.0 and maxabs(c_low, a_low) == 0.0


def test_range_guard_deferred_forwards_queue_without_host_sync():
    """"deferred" mode: back-to-back forwards enqueue without waiting for the GPU (the flag is read
    once its copy has landed): behind a ~50 ms spin kernel, two forward() calls return while the
    stream is still busy; the deferred checks resolve quietly in range, and a forward whose inputs
    were modified in place before a raised flag is read warns that it cannot be corrected."""
    import warnings
    g = load_golden("raft_full_rand_b1_128x192_i32.npz")
    m, _ = make_model(False, 0)
    m.range_guard = "deferred"
    i1, i2 = t(g["image1"]), t(g["image2"])
    with torch.no_grad(), warnings.catch_warnings():
        warnings.simplefilter("error")
        for _ in range(2):  # eager run, then the graph capture (which synchronises)
            m(i1, i2, iters=4, test_mode=True)
        m.check_range_guard()
        s = torch.cuda.current_stream()
        torch.cuda._sleep(int(1e8))
        a = m(i1, i2, iters=4, test_mode=True)
        b = m(i1, i2, iters=4, test_mode=True)
        busy = not s.query()
        m.check_range_guard()
    assert busy, "forward() synchronised with the device"
    assert not m._pending
    assert maxabs(a[1], b[1]) == 0.0
    # a raised flag with modified inputs: warned, not corrected
    with torch.no_grad():
        m.fnet.conv2.weight.mul_(20000.0)
        m.fnet.conv2.bias.mul_(20000.0)
        j1 = i1.clone()
        m(j1, i2, iters=4, test_mode=True)
        j1.add_(1.0)
        with pytest.warns(RuntimeWarning, match="cannot be recomputed"):
            m.check_range_guard()


def test_range_guard_quiet_in_range():
    """In range (the random-init model, |x| < 2^15 everywhere) the flag stays clear: no warning."""
    import warnings
    g = load_golden("raft_full_rand_b1_128x192_i32.npz")
    m, _ = make_model(False, 0)
    with torch.no_grad(), warnings.catch_warnings():
        warnings.simplefilter("error")
        m(t(g["image1"]), t(g["image2"]), iters=4, test_mode=True)
    pl = m.plan(1, 128, 192, 4, True)
    assert pl.guarded and int(pl.range_flag.item()) == 0
