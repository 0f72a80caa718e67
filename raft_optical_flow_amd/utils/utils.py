"""Caller-side tensor helpers — drop-in for core/utils/utils.py, on the GPU.

  InputPadder          core/utils/utils.py:7-24   replicate padding to multiples of 8
                                                   (raft_pad_replicate for GPU tensors)
  forward_interpolate  :26-54                      Sintel warm start: nearest forward-splatted
                                                   flow (raft_forward_interpolate, fp64 search)
  bilinear_sampler     :57-71                      grid_sample(align_corners=True) in pixel
                                                   coordinates (raft_bilinear_sample)
  coords_grid          :74-77                      (x, y) pixel grid
  upflow8              :80-82                      8 * bilinear x8 upsampling (raft_upflow8)

Every helper computes on the GPU through the HIP kernels of libraft_hip.so; a CPU tensor is
copied to the current GPU and the result copied back (there is no host computation path).
Kernels run on the tensor's own device (its current stream), whatever device is current.
"""
from __future__ import annotations

import torch


def _lib():
    from .. import _lib as L
    return L


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _on_device(fn):
    """Run fn(x, ...) with x's GPU current (so launches take that device's current stream);
    CPU inputs go to the current GPU first (inside fn)."""
    import functools

    @functools.wraps(fn)
    def wrapped(x, *args, **kw):
        if torch.is_tensor(x) and x.is_cuda:
            with torch.cuda.device(x.device):
                return fn(x, *args, **kw)
        return fn(x, *args, **kw)
    return wrapped


def _on_gpu(x: torch.Tensor) -> torch.Tensor:
    if x.is_cuda:
        return x
    if not torch.cuda.is_available():
        raise RuntimeError("raft_optical_flow_amd helpers run on a ROCm GPU only (no CPU path)")
    return x.cuda()


class InputPadder:
    """Replicate-pad NCHW images so H and W become multiples of 8: centred ('sintel', the
    default) or all rows at the bottom (any other mode, e.g. 'kitti'); `unpad` crops back.
    `_pad` = [left, right, top, bottom] (F.pad order), as the reference keeps it."""

    def __init__(self, dims, mode="sintel"):
        self.ht, self.wd = int(dims[-2]), int(dims[-1])
        ph, pw = -self.ht % 8, -self.wd % 8
        top = ph // 2 if mode == "sintel" else 0
        self._pad = [pw // 2, pw - pw // 2, top, ph - top]

    def _pad_one(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda:
            with torch.cuda.device(x.device):
                return self._pad_dev(x)
        return self._pad_dev(x)

    def _pad_dev(self, x: torch.Tensor) -> torch.Tensor:
        left, right, top, bottom = self._pad
        src = x
        x = _on_gpu(x).float().contiguous()
        h, w = x.shape[-2:]
        out = torch.empty(*x.shape[:-2], h + top + bottom, w + left + right, device=x.device)
        nc = x.numel() // (h * w)
        _lib().call("raft_pad_replicate", x.data_ptr(), out.data_ptr(), nc, h, w, top, bottom, left, right, _stream())
        return out.to(device=src.device, dtype=src.dtype)

    def pad(self, *inputs):
        return [self._pad_one(x) for x in inputs]

    def unpad(self, x):
        left, right, top, bottom = self._pad
        h, w = x.shape[-2:]
        return x[..., top:h - bottom, left:w - right]


@_on_device
def forward_interpolate(flow):
    """Warm-start flow for the next frame pair (evaluate.py:37-41): each pixel takes the flow of
    the nearest point the flow moves a pixel to, over the points that land strictly inside the
    frame (scipy griddata 'nearest' in the reference; 0 where none lands).  flow [2, H, W] (or
    [B, 2, H, W]) -> float32, same shape, same device."""
    f = _on_gpu(flow.detach()).float().contiguous()
    batched = f.dim() == 4
    if not batched:
        f = f[None]
    b, c, h, w = f.shape
    if c != 2:
        raise ValueError(f"flow must be [2, H, W] or [B, 2, H, W], got {tuple(flow.shape)}")
    out = torch.empty_like(f)
    _lib().call("raft_forward_interpolate", f.data_ptr(), out.data_ptr(), b, h, w, _stream())
    out = out if batched else out[0]
    return out.to(flow.device)


@_on_device
def bilinear_sampler(img, coords, mode="bilinear", mask=False):
    """Sample img [N, C, H, W] at pixel coordinates coords [N, Ho, Wo, 2] (x, y): bilinear,
    corners outside the image read 0 (grid_sample align_corners=True).  With mask=True also
    returns the in-range mask [N, Ho, Wo, 1] as float."""
    if mode != "bilinear":
        raise NotImplementedError("bilinear_sampler: only mode='bilinear' is on the RAFT path")
    from .. import kernels as K
    K.require_device(img, coords)
    img = img.contiguous()
    coords = coords.contiguous()
    n, c, h, w = img.shape
    ho, wo = coords.shape[1:3]
    out = torch.empty(n, c, ho, wo, device=img.device)
    m = torch.empty(n, ho, wo, 1, device=img.device) if mask else None
    _lib().call("raft_bilinear_sample", img.data_ptr(), coords.data_ptr(), out.data_ptr(),
                m.data_ptr() if mask else None, n, c, h, w, ho, wo, _stream())
    return (out, m) if mask else out


def coords_grid(batch, ht, wd, device):
    """[batch, 2, ht, wd] float grid: channel 0 = x (column index), channel 1 = y (row index)."""
    x = torch.arange(wd, device=device, dtype=torch.float32).view(1, wd).expand(ht, wd)
    y = torch.arange(ht, device=device, dtype=torch.float32).view(ht, 1).expand(ht, wd)
    return torch.stack([x, y], 0)[None].repeat(batch, 1, 1, 1)


@_on_device
def upflow8(flow, mode="bilinear"):
    """8 * bilinear(align_corners=True) x8 upsampling (raft_upflow8)."""
    from .. import kernels as K
    if mode != "bilinear":
        raise NotImplementedError("upflow8: only mode='bilinear' is on the RAFT path")
    src = flow
    flow = _on_gpu(flow).float()
    n, _, h, w = flow.shape
    coords = (coords_grid(n, h, w, flow.device) + flow).contiguous()
    crow = K.nchw_to_rows(coords)
    out = torch.empty(n, 2, 8 * h, 8 * w, device=flow.device)
    _lib().call("raft_upflow8", crow.data_ptr(), out.data_ptr(), n, h, w, K.stream_handle())
    return out.to(src.device)
