"""PyTorch-CPU restatement of the reference RAFT inference path: the CPU BASELINE.

TEST / MEASUREMENT INFRASTRUCTURE ONLY: `bench.py`'s cpu_baseline leg times it on the
GPU box's host cores (the reference itself cannot travel there), and `tests/` pin it
to the reference's golden vectors.  The product path never imports it.

It is the same computation as the reference's `core/` forward on CPU, expressed with
the same torch CPU operators the reference dispatches to (oneDNN conv2d, bmm,
avg_pool2d, grid_sample, instance/batch norm, softmax/unfold), so its speed stands for
the reference's CPU path: in the build container it measured within a few percent of
the reference's own `core/` at the same thread count.  Functions
take the reference's state_dict keys; each cites the reference lines it restates.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _conv(x, p, key, stride=1, padding=0):
    return F.conv2d(x, p[key + ".weight"], p.get(key + ".bias"), stride, padding)


def _norm(x, p, key, norm_fn):
    """core/extractor.py:15-33 norm selection (eval mode)."""
    if norm_fn == "instance":
        return F.instance_norm(x)
    if norm_fn == "batch":
        return F.batch_norm(x, p[key + ".running_mean"], p[key + ".running_var"], p[key + ".weight"],
                            p[key + ".bias"], False)
    return x


def _residual(x, p, pre, norm_fn, stride):
    """core/extractor.py:6-56."""
    y = F.relu(_norm(_conv(x, p, pre + ".conv1", stride, 1), p, pre + ".norm1", norm_fn))
    y = F.relu(_norm(_conv(y, p, pre + ".conv2", 1, 1), p, pre + ".norm2", norm_fn))
    if stride != 1:
        x = _norm(_conv(x, p, pre + ".downsample.0", stride, 0), p, pre + ".downsample.1", norm_fn)
    return F.relu(x + y)


def _bottleneck(x, p, pre, norm_fn, stride):
    """core/extractor.py:60-116."""
    y = F.relu(_norm(_conv(x, p, pre + ".conv1", 1, 0), p, pre + ".norm1", norm_fn))
    y = F.relu(_norm(_conv(y, p, pre + ".conv2", stride, 1), p, pre + ".norm2", norm_fn))
    y = F.relu(_norm(_conv(y, p, pre + ".conv3", 1, 0), p, pre + ".norm3", norm_fn))
    if stride != 1:
        x = _norm(_conv(x, p, pre + ".downsample.0", stride, 0), p, pre + ".downsample.1", norm_fn)
    return F.relu(x + y)


def encoder(x, p, pre, norm_fn, small=False):
    """core/extractor.py:118-192 (BasicEncoder) / :195-267 (SmallEncoder), eval mode."""
    x = F.relu(_norm(_conv(x, p, pre + ".conv1", 2, 3), p, pre + ".norm1", norm_fn))
    blk = _bottleneck if small else _residual
    for li, stride in ((1, 1), (2, 2), (3, 2)):
        x = blk(x, p, f"{pre}.layer{li}.0", norm_fn, stride)
        x = blk(x, p, f"{pre}.layer{li}.1", norm_fn, 1)
    return _conv(x, p, pre + ".conv2")


def corr_pyramid(f1, f2, levels=4):
    """core/corr.py:25-54 + :96-127: bmm / sqrt(C), then 2x2 average pools."""
    b, c, h, w = f1.shape
    corr = torch.bmm(f1.view(b, c, h * w).transpose(1, 2), f2.view(b, c, h * w))
    corr = (corr / torch.sqrt(torch.tensor(c).float())).reshape(b * h * w, 1, h, w)
    pyr = [corr]
    for _ in range(levels - 1):
        corr = F.avg_pool2d(corr, 2, stride=2)
        pyr.append(corr)
    return pyr


def _sample(img, xy):
    """core/utils/utils.py:57-71: pixel coords -> [-1, 1], grid_sample(align_corners=True)."""
    hh, ww = img.shape[-2:]
    gx = 2 * xy[..., :1] / (ww - 1) - 1
    gy = 2 * xy[..., 1:] / (hh - 1) - 1
    return F.grid_sample(img, torch.cat([gx, gy], -1), align_corners=True)


def corr_lookup(pyr, coords, r):
    """core/corr.py:56-94: window offset (i, j) samples (x + d_i, y + d_j) at channel
    lvl*(2r+1)^2 + i*(2r+1) + j (the first window index moves x)."""
    b, _, h, w = coords.shape
    c = coords.permute(0, 2, 3, 1).reshape(b * h * w, 1, 1, 2)
    d = torch.linspace(-r, r, 2 * r + 1)
    off = torch.stack([d.view(-1, 1).expand(-1, 2 * r + 1), d.view(1, -1).expand(2 * r + 1, -1)], -1)
    outs = []
    for i, lvl in enumerate(pyr):
        xy = c / 2 ** i + off.view(1, 2 * r + 1, 2 * r + 1, 2)
        outs.append(_sample(lvl, xy).view(b, h, w, -1))
    return torch.cat(outs, -1).permute(0, 3, 1, 2).contiguous().float()


def _gru_half(h, x, p, zk, rk, qk, pad):
    """core/update.py:99-121 (one SepConvGRU half-step) / :52-72 (ConvGRU)."""
    hx = torch.cat([h, x], 1)
    z = torch.sigmoid(_conv(hx, p, zk, 1, pad))
    r = torch.sigmoid(_conv(hx, p, rk, 1, pad))
    q = torch.tanh(_conv(torch.cat([r * h, x], 1), p, qk, 1, pad))
    return (1 - z) * h + z * q


def update_block(net, inp, corr, flow, p, small=False, pre="update_block"):
    """core/update.py:297-325 (BasicUpdateBlock) / :250-263 (SmallUpdateBlock)."""
    e = pre + ".encoder"
    cor = F.relu(_conv(corr, p, e + ".convc1"))
    if not small:
        cor = F.relu(_conv(cor, p, e + ".convc2", 1, 1))
    flo = F.relu(_conv(flow, p, e + ".convf1", 1, 3))
    flo = F.relu(_conv(flo, p, e + ".convf2", 1, 1))
    motion = torch.cat([F.relu(_conv(torch.cat([cor, flo], 1), p, e + ".conv", 1, 1)), flow], 1)
    x = torch.cat([inp, motion], 1)
    g = pre + ".gru"
    if small:
        net = _gru_half(net, x, p, g + ".convz", g + ".convr", g + ".convq", 1)
    else:
        net = _gru_half(net, x, p, g + ".convz1", g + ".convr1", g + ".convq1", (0, 2))
        net = _gru_half(net, x, p, g + ".convz2", g + ".convr2", g + ".convq2", (2, 0))
    fh = pre + ".flow_head"
    delta = _conv(F.relu(_conv(net, p, fh + ".conv1", 1, 1)), p, fh + ".conv2", 1, 1)
    if small:
        return net, None, delta
    mask = 0.25 * _conv(F.relu(_conv(net, p, pre + ".mask.0", 1, 1)), p, pre + ".mask.2")
    return net, mask, delta


def upsample(flow, mask):
    """core/raft.py:112-142 (convex upsampling)."""
    n, _, h, w = flow.shape
    m = torch.softmax(mask.view(n, 1, 9, 8, 8, h, w), dim=2)
    u = F.unfold(8 * flow, [3, 3], padding=1).view(n, 2, 9, 1, 1, h, w)
    return (m * u).sum(2).permute(0, 1, 4, 2, 5, 3).reshape(n, 2, 8 * h, 8 * w)


def upflow8(flow):
    """core/utils/utils.py:80-82."""
    return 8 * F.interpolate(flow, size=(8 * flow.shape[2], 8 * flow.shape[3]), mode="bilinear", align_corners=True)


@torch.no_grad()
def raft_forward(p, image1, image2, iters=12, small=False):
    """core/raft.py:145-251 (eval, test_mode, all-pairs correlation) -> (flow_low, flow_up)."""
    hdim, cdim, r = (96, 64, 3) if small else (128, 128, 4)
    image1 = 2 * (image1 / 255.0) - 1.0
    image2 = 2 * (image2 / 255.0) - 1.0
    b, _, hh, ww = image1.shape
    fm = encoder(torch.cat([image1, image2], 0), p, "fnet", "instance", small)
    pyr = corr_pyramid(fm[:b].float(), fm[b:].float(), 4)
    cn = encoder(image1, p, "cnet", "none" if small else "batch", small)
    net, inp = torch.tanh(cn[:, :hdim]), torch.relu(cn[:, hdim:hdim + cdim])
    ys, xs = torch.meshgrid(torch.arange(hh // 8), torch.arange(ww // 8), indexing="ij")
    coords0 = torch.stack([xs, ys], 0).float()[None].repeat(b, 1, 1, 1)
    coords1 = coords0.clone()
    flow_up = None
    for _ in range(iters):
        corr = corr_lookup(pyr, coords1, r)
        net, mask, delta = update_block(net, inp, corr, coords1 - coords0, p, small)
        coords1 = coords1 + delta
        flow_up = upflow8(coords1 - coords0) if mask is None else upsample(coords1 - coords0, mask)
    return coords1 - coords0, flow_up


def alt_corr_forward(f1, f2, coords, r):
    """alt_cuda_corr/correlation_kernel.cu:18-119 (corr_forward_kernel) as differentiable torch
    ops, for the gradient checks of the plugin's backward: f1 [B,H1,W1,C], f2 [B,H2,W2,C],
    coords [B,N,H1,W1,2] -> [B,N,(2r+1)^2,H1,W1], unscaled, channel oy + (2r+1)*ox.  The taps sit
    at floor(coords) - r + (0..2r+1) (piecewise constant: no gradient through the floor); the
    bilinear weights carry the coordinate gradient."""
    B, H1, W1, C = f1.shape
    _, H2, W2, _ = f2.shape
    N = coords.shape[1]
    rd, wd = 2 * r + 1, 2 * r + 2
    x, y = coords[..., 0], coords[..., 1]
    fx, fy = torch.floor(x).detach(), torch.floor(y).detach()
    dx, dy = x - fx, y - fy
    ar = torch.arange(wd)
    h2 = (fy.long() - r)[..., None, None] + ar.view(wd, 1)
    w2 = (fx.long() - r)[..., None, None] + ar.view(1, wd)
    ok = ((h2 >= 0) & (h2 < H2) & (w2 >= 0) & (w2 < W2)).to(f1.dtype)
    idx = (h2.clamp(0, H2 - 1) * W2 + w2.clamp(0, W2 - 1)).reshape(B, -1)        # [B, N*H1*W1*wd*wd]
    taps = torch.gather(f2.reshape(B, H2 * W2, C), 1, idx[..., None].expand(-1, -1, C))
    taps = taps.reshape(B, N, H1, W1, wd, wd, C)
    s = (f1[:, None, :, :, None, None, :] * taps).sum(-1) * ok                   # s[..., iy, ix]
    ex, ey = dx[..., None, None], dy[..., None, None]
    o = (s[..., :rd, :rd] * ((1 - ey) * (1 - ex)) + s[..., :rd, 1:] * ((1 - ey) * ex)
         + s[..., 1:, :rd] * (ey * (1 - ex)) + s[..., 1:, 1:] * (ey * ex))        # o[..., oy, ox]
    return o.permute(0, 1, 5, 4, 2, 3).reshape(B, N, rd * rd, H1, W1)
