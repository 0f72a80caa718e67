"""`alt_cuda_corr` plugin shim — same module API as the reference's pybind
extension (alt_cuda_corr/correlation.cpp:23-54), backed by libraft_hip.so.

    corr, = forward(fmap1, fmap2, coords, radius)
    fmap1_grad, fmap2_grad, coords_grad = backward(fmap1, fmap2, coords, corr_grad, radius)
    corr = alt_corr(fmap1, fmap2, coords, radius)       # the same, as an autograd Function

fmap1 [B,H1,W1,C], fmap2 [B,H2,W2,C], coords [B,N,H1,W1,2], corr [B,N,(2r+1)^2,H1,W1]
(unscaled), float32, contiguous, on the GPU.  Launches go to the *current*
stream (the reference uses the legacy default stream), so hipGraph capture
works.  Validation errors raise RuntimeError like TORCH_CHECK.
"""
from __future__ import annotations

import torch

from . import _lib
from . import kernels as K


def _check(x, name):
    if not (torch.is_tensor(x) and x.is_cuda):
        raise RuntimeError(f"{name} must be a CUDA tensor")
    if not x.is_contiguous():
        raise RuntimeError(f"{name} must be contiguous")
    if x.dtype != torch.float32:
        raise RuntimeError(f"{name} must be float32")


def forward(fmap1, fmap2, coords, radius):
    for t, n in ((fmap1, "fmap1"), (fmap2, "fmap2"), (coords, "coords")):
        _check(t, n)
    B, H1, W1, C = fmap1.shape
    _, H2, W2, _ = fmap2.shape
    _, N, _, _, _ = coords.shape
    rd = 2 * radius + 1
    corr = torch.empty(B, N, rd * rd, H1, W1, device=fmap1.device, dtype=torch.float32)
    _lib.call("raft_alt_corr_forward", fmap1.data_ptr(), fmap2.data_ptr(), coords.data_ptr(), corr.data_ptr(),
              B, H1, W1, H2, W2, C, N, int(radius), 1.0, K.stream_handle())
    return [corr]


def backward(fmap1, fmap2, coords, corr_grad, radius):
    for t, n in ((fmap1, "fmap1"), (fmap2, "fmap2"), (coords, "coords"), (corr_grad, "corr_grad")):
        _check(t, n)
    B, H1, W1, C = fmap1.shape
    _, H2, W2, _ = fmap2.shape
    _, N, _, _, _ = coords.shape
    f1g = torch.empty_like(fmap1)
    f2g = torch.empty_like(fmap2)
    cg = torch.empty_like(coords)
    nws = int(_lib.load().raft_alt_corr_backward_workspace_floats(B, H1, W1, H2, W2, C, N, int(radius)))
    ws = torch.empty(max(nws, 1), device=fmap1.device, dtype=torch.float32)
    _lib.call("raft_alt_corr_backward", fmap1.data_ptr(), fmap2.data_ptr(), coords.data_ptr(), corr_grad.data_ptr(),
              f1g.data_ptr(), f2g.data_ptr(), cg.data_ptr(), B, H1, W1, H2, W2, C, N, int(radius), ws.data_ptr(), nws,
              K.stream_handle())
    return [f1g, f2g, cg]


class AltCorrFunction(torch.autograd.Function):
    """forward / backward above as an autograd Function (the wiring the reference lacks: its
    AlternateCorrBlock calls the plugin outside autograd, core/corr.py:190): gradients reach
    fmap1, fmap2 and coords."""

    @staticmethod
    def forward(ctx, fmap1, fmap2, coords, radius):
        fmap1, fmap2, coords = fmap1.contiguous(), fmap2.contiguous(), coords.contiguous()
        ctx.save_for_backward(fmap1, fmap2, coords)
        ctx.radius = int(radius)
        corr, = forward(fmap1, fmap2, coords, radius)
        return corr

    @staticmethod
    def backward(ctx, grad):
        fmap1, fmap2, coords = ctx.saved_tensors
        f1g, f2g, cg = backward(fmap1, fmap2, coords, grad.contiguous(), ctx.radius)
        return f1g, f2g, cg, None


def alt_corr(fmap1, fmap2, coords, radius):
    """Differentiable alternate correlation: corr [B,N,(2r+1)^2,H1,W1] (unscaled)."""
    return AltCorrFunction.apply(fmap1, fmap2, coords, radius)
