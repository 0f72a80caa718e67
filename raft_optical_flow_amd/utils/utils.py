"""Tensor utilities — drop-in for core/utils/utils.py.

InputPadder (`core/utils/utils.py:7-24`), coords_grid (`:74-77`),
bilinear_sampler (`:57-71`) and forward_interpolate (`:26-54`) keep the
reference's torch/scipy semantics (they are caller-side helpers, not kernels of
the accelerated path).  upflow8 (`:80-82`) runs the HIP kernel on GPU tensors.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F


class InputPadder:
    """Pads images such that dimensions are divisible by 8."""

    def __init__(self, dims, mode="sintel"):
        self.ht, self.wd = dims[-2:]
        pad_ht = (((self.ht // 8) + 1) * 8 - self.ht) % 8
        pad_wd = (((self.wd // 8) + 1) * 8 - self.wd) % 8
        if mode == "sintel":
            self._pad = [pad_wd // 2, pad_wd - pad_wd // 2, pad_ht // 2, pad_ht - pad_ht // 2]
        else:
            self._pad = [pad_wd // 2, pad_wd - pad_wd // 2, 0, pad_ht]

    def pad(self, *inputs):
        return [F.pad(x, self._pad, mode="replicate") for x in inputs]

    def unpad(self, x):
        ht, wd = x.shape[-2:]
        c = [self._pad[2], ht - self._pad[3], self._pad[0], wd - self._pad[1]]
        return x[..., c[0]:c[1], c[2]:c[3]]


def forward_interpolate(flow):
    """Warm-start flow for the next frame (scipy nearest-neighbour griddata on the host)."""
    from scipy import interpolate
    flow = flow.detach().cpu().numpy()
    dx, dy = flow[0], flow[1]
    ht, wd = dx.shape
    x0, y0 = np.meshgrid(np.arange(wd), np.arange(ht))
    x1 = (x0 + dx).reshape(-1)
    y1 = (y0 + dy).reshape(-1)
    dx = dx.reshape(-1)
    dy = dy.reshape(-1)
    valid = (x1 > 0) & (x1 < wd) & (y1 > 0) & (y1 < ht)
    x1, y1, dx, dy = x1[valid], y1[valid], dx[valid], dy[valid]
    flow_x = interpolate.griddata((x1, y1), dx, (x0, y0), method="nearest", fill_value=0)
    flow_y = interpolate.griddata((x1, y1), dy, (x0, y0), method="nearest", fill_value=0)
    return torch.from_numpy(np.stack([flow_x, flow_y], axis=0)).float()


def bilinear_sampler(img, coords, mode="bilinear", mask=False):
    """Wrapper for grid_sample, uses pixel coordinates."""
    H, W = img.shape[-2:]
    xgrid, ygrid = coords.split([1, 1], dim=-1)
    xgrid = 2 * xgrid / (W - 1) - 1
    ygrid = 2 * ygrid / (H - 1) - 1
    grid = torch.cat([xgrid, ygrid], dim=-1)
    img = F.grid_sample(img, grid, align_corners=True)
    if mask:
        m = (xgrid > -1) & (ygrid > -1) & (xgrid < 1) & (ygrid < 1)
        return img, m.float()
    return img


def coords_grid(batch, ht, wd, device):
    ys, xs = torch.meshgrid(torch.arange(ht, device=device), torch.arange(wd, device=device), indexing="ij")
    coords = torch.stack([xs, ys], dim=0).float()
    return coords[None].repeat(batch, 1, 1, 1)


def upflow8(flow, mode="bilinear"):
    """8 * bilinear(align_corners=True) x8 upsampling; HIP kernel for GPU tensors."""
    from .. import _lib
    from .. import kernels as K
    if mode != "bilinear" or not flow.is_cuda:
        new_size = (8 * flow.shape[2], 8 * flow.shape[3])
        return 8 * F.interpolate(flow, size=new_size, mode=mode, align_corners=True)
    n, _, h, w = flow.shape
    coords = (coords_grid(n, h, w, flow.device) + flow).contiguous()
    crow = K.nchw_to_rows(coords)
    out = torch.empty(n, 2, 8 * h, 8 * w, device=flow.device)
    _lib.call("raft_upflow8", crow.data_ptr(), out.data_ptr(), n, h, w, K.stream_handle())
    return out
