"""Block-level forwards of the reference's sub-modules on the HIP path, against a plain PyTorch
fp64 restatement of the same op with the module's own weights (tolerance 1e-4 x max|ref|, the
block-level default arithmetic being exact f32 MFMA):

  FlowHead (core/update.py:6-28), ConvGRU (:30-72), SepConvGRU (:74-121),
  SmallMotionEncoder (:123-167), BasicMotionEncoder (:169-216),
  ResidualBlock (core/extractor.py:6-56), BottleneckBlock (:60-116);
plus the weight-pack cache (reused until a parameter changes).
"""
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


def close(got, ref, tol=1e-4):
    err = float((got.double().cpu() - ref.cpu()).abs().max())
    scale = max(1.0, float(ref.abs().max()))
    assert err < tol * scale, (err, scale)


def conv64(x, c):
    return F.conv2d(x, c.weight.double(), c.bias.double() if c.bias is not None else None, c.stride, c.padding)


def rnd(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(DEV)


def test_flow_head():
    from raft_optical_flow_amd.update import FlowHead
    torch.manual_seed(1)
    m = FlowHead(128, 256).to(DEV)
    x = rnd(2, 128, 9, 13)
    ref = conv64(F.relu(conv64(x.double(), m.conv1)), m.conv2)
    with torch.no_grad():
        close(m(x), ref)


@pytest.mark.parametrize("sep", [False, True])
def test_conv_gru(sep):
    from raft_optical_flow_amd.update import ConvGRU, SepConvGRU
    torch.manual_seed(2)
    hd, xd = (128, 256) if sep else (96, 146)
    m = (SepConvGRU(hd, xd) if sep else ConvGRU(hd, xd)).to(DEV)
    h = torch.tanh(rnd(1, hd, 11, 17, seed=3))
    x = rnd(1, xd, 11, 17, seed=4)

    def half(h, cz, cr, cq):
        hx = torch.cat([h, x.double()], 1)
        z, r = torch.sigmoid(conv64(hx, cz)), torch.sigmoid(conv64(hx, cr))
        q = torch.tanh(conv64(torch.cat([r * h, x.double()], 1), cq))
        return (1 - z) * h + z * q

    if sep:
        ref = half(half(h.double(), m.convz1, m.convr1, m.convq1), m.convz2, m.convr2, m.convq2)
    else:
        ref = half(h.double(), m.convz, m.convr, m.convq)
    with torch.no_grad():
        close(m(h, x), ref, 1e-5)


@pytest.mark.parametrize("small", [False, True])
def test_motion_encoder(small):
    from raft_optical_flow_amd.update import BasicMotionEncoder, SmallMotionEncoder
    torch.manual_seed(5)
    r = 3 if small else 4
    args = argparse.Namespace(corr_levels=4, corr_radius=r)
    m = (SmallMotionEncoder(args) if small else BasicMotionEncoder(args)).to(DEV)
    flow = rnd(2, 2, 10, 14, seed=6, scale=3.0)
    corr = rnd(2, 4 * (2 * r + 1) ** 2, 10, 14, seed=7, scale=2.0)
    cor = F.relu(conv64(corr.double(), m.convc1))
    if not small:
        cor = F.relu(conv64(cor, m.convc2))
    flo = F.relu(conv64(F.relu(conv64(flow.double(), m.convf1)), m.convf2))
    ref = torch.cat([F.relu(conv64(torch.cat([cor, flo], 1), m.conv)), flow.double()], 1)
    with torch.no_grad():
        out = m(flow, corr)
    assert out.shape == ref.shape
    close(out, ref)


def _norm64(x, norm, mod):
    if isinstance(mod, torch.nn.BatchNorm2d):
        return F.batch_norm(x, mod.running_mean.double(), mod.running_var.double(), mod.weight.double(),
                            mod.bias.double(), False, 0.0, mod.eps)
    if isinstance(mod, torch.nn.InstanceNorm2d):
        return F.instance_norm(x, eps=mod.eps)
    if isinstance(mod, torch.nn.GroupNorm):
        return F.group_norm(x, mod.num_groups, mod.weight.double(), mod.bias.double(), mod.eps)
    return x


def _randomise_bn(m, seed):
    g = torch.Generator().manual_seed(seed)
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            n = mod.num_features
            mod.running_mean.copy_(torch.randn(n, generator=g) * 0.1)
            mod.running_var.copy_(torch.rand(n, generator=g) * 0.4 + 0.8)
            mod.weight.data.copy_(torch.rand(n, generator=g) * 0.4 + 0.8)
            mod.bias.data.copy_(torch.randn(n, generator=g) * 0.1)
        if isinstance(mod, torch.nn.GroupNorm):  # a non-trivial affine (its init is 1 / 0)
            n = mod.num_channels
            mod.weight.data.copy_(torch.rand(n, generator=g) * 0.8 + 0.6)
            mod.bias.data.copy_(torch.randn(n, generator=g) * 0.2)


@pytest.mark.parametrize("norm", ["instance", "batch", "none", "group"])
@pytest.mark.parametrize("stride", [1, 2])
@pytest.mark.parametrize("bottleneck", [False, True])
def test_encoder_blocks(norm, stride, bottleneck):
    from raft_optical_flow_amd.extractor import BottleneckBlock, ResidualBlock
    torch.manual_seed(8)
    cin, planes = (64, 96) if stride == 2 else (96, 96)
    m = (BottleneckBlock if bottleneck else ResidualBlock)(cin, planes, norm, stride)
    with torch.no_grad():
        _randomise_bn(m, 9)
    m = m.to(DEV).eval()
    x = F.relu(rnd(2, cin, 19, 24, seed=10))
    xd = x.double()
    if bottleneck:
        y = F.relu(_norm64(conv64(xd, m.conv1), norm, m.norm1))
        y = F.relu(_norm64(conv64(y, m.conv2), norm, m.norm2))
        y = F.relu(_norm64(conv64(y, m.conv3), norm, m.norm3))
        dsn = getattr(m, "norm4", None)
    else:
        y = F.relu(_norm64(conv64(xd, m.conv1), norm, m.norm1))
        y = F.relu(_norm64(conv64(y, m.conv2), norm, m.norm2))
        dsn = getattr(m, "norm3", None)
    if m.downsample is not None:
        xd = _norm64(conv64(xd, m.downsample[0]), norm, dsn)
    ref = F.relu(xd + y)
    with torch.no_grad():
        close(m(x), ref)


def test_block_pack_cache_reused_until_weights_change():
    from raft_optical_flow_amd.update import FlowHead
    torch.manual_seed(11)
    m = FlowHead(128, 256).to(DEV)
    x = rnd(1, 128, 6, 8, seed=12)
    with torch.no_grad():
        a = m(x)
        pk = m.__dict__["_hip_pack"][1]
        b = m(x)
        assert m.__dict__["_hip_pack"][1] is pk and torch.equal(a, b)
        m.conv2.weight.mul_(2.0)
        m.conv2.bias.mul_(2.0)
        c = m(x)
    assert m.__dict__["_hip_pack"][1] is not pk
    np.testing.assert_allclose(c.cpu().numpy(), 2 * a.cpu().numpy(), rtol=1e-5, atol=1e-5)


def test_block_plans_cached_per_shape():
    """BasicUpdateBlock, SepConvGRU and ResidualBlock keep their buffers and launch lists per input
    shape (kernels.cached_plan): a repeated call reuses them (same plan object, results of an
    input identical whatever ran in between), a new shape or new weights rebuild them."""
    from raft_optical_flow_amd.extractor import ResidualBlock
    from raft_optical_flow_amd.update import BasicUpdateBlock, SepConvGRU
    args = argparse.Namespace(corr_levels=4, corr_radius=4)
    torch.manual_seed(5)
    ub = BasicUpdateBlock(args, 128).to(DEV).eval()
    gru = SepConvGRU(128, 256).to(DEV).eval()
    blk = ResidualBlock(64, 64, "instance", 1).to(DEV).eval()
    cases = [
        (ub, lambda s: (rnd(1, 128, 6, 10, seed=s), rnd(1, 128, 6, 10, seed=s + 1), rnd(1, 324, 6, 10, seed=s + 2),
                        rnd(1, 2, 6, 10, seed=s + 3))),
        (gru, lambda s: (rnd(2, 128, 5, 7, seed=s), rnd(2, 256, 5, 7, seed=s + 1))),
        (blk, lambda s: (rnd(2, 64, 9, 12, seed=s),)),
    ]
    with torch.no_grad():
        for m, mk in cases:
            a = m(*mk(1))
            plan = cur_plan(m)
            m(*mk(7))
            a2 = m(*mk(1))
            assert cur_plan(m) is plan
            for x, y in zip(a if isinstance(a, tuple) else (a,), a2 if isinstance(a2, tuple) else (a2,)):
                assert (x is None and y is None) or torch.equal(x, y)
            # a new shape rebuilds the plan
            big = tuple(t.repeat(1, 1, 2, 1) if t.dim() == 4 else t for t in mk(3))
            m(*big)
            assert cur_plan(m) is not plan
            # another stream gets buffers of its own; back on the first stream, its plan is reused
            s2 = torch.cuda.Stream()
            s2.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s2):
                b2 = m(*mk(1))
            s2.synchronize()
            assert cur_plan(m, s2) is not cur_plan(m)
            for x, y in zip(a if isinstance(a, tuple) else (a,), b2 if isinstance(b2, tuple) else (b2,)):
                assert (x is None and y is None) or torch.equal(x, y)


def cur_plan(m, stream=None):
    """The block's cached plan for `stream` (default: the current stream), kernels.cached_plan."""
    sid = (stream or torch.cuda.current_stream()).cuda_stream
    return m.__dict__["_hip_plan"][sid][2]
