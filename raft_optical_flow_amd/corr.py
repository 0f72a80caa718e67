"""Correlation blocks — drop-in for core/corr.py.

CorrBlock (`core/corr.py:12-127`): the all-pairs volume and its average-pool
pyramid are built by one fp32-MFMA GEMM kernel (levels 0 and 1 from its
epilogue, deeper levels by a pooling kernel); __call__ is the radius-r window
lookup kernel (one wave per query pixel, LDS-staged windows).

AlternateCorrBlock (`core/corr.py:130-198`): the memory-light path, on-the-fly
dot products against pooled fmap2 levels (the alt_cuda_corr plugin's kernel).

Both take and return NCHW float32 tensors on the GPU, with the reference's
channel order (lvl*(2r+1)^2 + ix*(2r+1) + iy).
"""
from __future__ import annotations

import torch

from . import _lib
from . import kernels as K


class CorrBlock:
    def __init__(self, fmap1, fmap2, num_levels=4, radius=4):
        K.require_device(fmap1, fmap2)
        self.num_levels = num_levels
        self.radius = radius
        b, c, h, w = fmap1.shape
        if fmap2.shape != fmap1.shape:
            raise ValueError(f"fmap shapes differ: {tuple(fmap1.shape)} vs {tuple(fmap2.shape)}")
        self.shape = (b, c, h, w)
        dims = K.pyramid_dims(h, w, num_levels)
        for lh, lw in dims[1:]:
            if lh < 1 or lw < 1:
                # F.avg_pool2d raises on an empty output (core/corr.py:53)
                raise RuntimeError(f"CorrBlock: {h}x{w} feature map too small for {num_levels} pyramid levels")
        if c % 4:
            raise ValueError(f"CorrBlock HIP path needs C % 4 == 0 (got C={c})")
        f1 = K.nchw_to_rows(fmap1)
        f2 = K.nchw_to_rows(fmap2)
        self.pyramid_flat = torch.empty(K.pyramid_floats(b, h, w, num_levels), device=fmap1.device)
        _lib.call("raft_corr_build", f1.data_ptr(), f2.data_ptr(), c, b, h, w, c, num_levels, K.sqrt_c(c),
                  self.pyramid_flat.data_ptr(), K.stream_handle())
        self._dims = dims

    @property
    def corr_pyramid(self):
        """Reference-shaped copies of the levels, [B*H*W, 1, H_i, W_i] (the device
        pyramid itself is stored in 4x4 tiles, include/raft_hip.h)."""
        b, c, h, w = self.shape
        out = []
        for i, (lh, lw) in enumerate(self._dims):
            t = torch.empty(b * h * w, 1, lh, lw, device=self.pyramid_flat.device)
            _lib.call("raft_corr_pyramid_level", self.pyramid_flat.data_ptr(), b, h, w, self.num_levels, i,
                      t.data_ptr(), K.stream_handle())
            out.append(t)
        return out

    def __call__(self, coords):
        K.require_device(coords)
        b, c, h, w = self.shape
        if tuple(coords.shape) != (b, 2, h, w):
            raise ValueError(f"coords must be [{b}, 2, {h}, {w}], got {tuple(coords.shape)}")
        coords = coords.contiguous()
        r = self.radius
        out = torch.empty(b, self.num_levels * (2 * r + 1) ** 2, h, w, device=coords.device)
        _lib.call("raft_corr_lookup", self.pyramid_flat.data_ptr(), b, h, w, self.num_levels, r, coords.data_ptr(), 1,
                  out.data_ptr(), 0, 1, None, 0, None, K.stream_handle())
        return out

    @staticmethod
    def corr(fmap1, fmap2):
        """Level 0 of the volume, [B, H, W, 1, H, W] (core/corr.py:96-127)."""
        b, c, h, w = fmap1.shape
        cb = CorrBlock(fmap1, fmap2, num_levels=1, radius=1)
        return cb.corr_pyramid[0].view(b, h, w, 1, h, w)


class AlternateCorrBlock:
    def __init__(self, fmap1, fmap2, num_levels=4, radius=4):
        K.require_device(fmap1, fmap2)
        self.num_levels = num_levels
        self.radius = radius
        b, c, h, w = fmap1.shape
        self.dim = c
        # NHWC copies once per pair (the reference re-permutes on every call, core/corr.py:183-184)
        f1 = K.nchw_to_rows(fmap1)
        f2 = K.nchw_to_rows(fmap2)
        self._f1 = (f1, h, w)
        self._f2 = [(f2, h, w)]
        # the reference pools num_levels times (one unused level); keep its size check
        hh, ww = h, w
        for i in range(num_levels):
            if hh // 2 < 1 or ww // 2 < 1:
                raise RuntimeError(f"AlternateCorrBlock: {h}x{w} feature map too small for {num_levels} levels")
            hh, ww = hh // 2, ww // 2
        s = K.stream_handle()
        for i in range(num_levels - 1):
            src, hh, ww = self._f2[-1]
            dst = torch.empty(b * (hh // 2) * (ww // 2), c, device=fmap1.device)
            _lib.call("raft_avgpool2_nhwc", src.data_ptr(), dst.data_ptr(), b, hh, ww, c, s)
            self._f2.append((dst, hh // 2, ww // 2))
        # reference-shaped pyramid of (fmap1, fmap2) NCHW views (fmap1 levels > 0 are unused)
        self.pyramid = [(fmap1, fmap2)] + [
            (None, t.view(b, lh, lw, c).permute(0, 3, 1, 2)) for (t, lh, lw) in self._f2[1:]]

    def __call__(self, coords):
        K.require_device(coords)
        f1, h, w = self._f1
        b = coords.shape[0]
        if tuple(coords.shape) != (b, 2, h, w):
            raise ValueError(f"coords must be [{b}, 2, {h}, {w}], got {tuple(coords.shape)}")
        coords = coords.contiguous()
        r = self.radius
        nb = (2 * r + 1) ** 2
        out = torch.empty(b * h * w, self.num_levels * nb, device=coords.device)
        s = K.stream_handle()
        div = K.sqrt_c(self.dim)
        levels = list(self._f2[: self.num_levels])
        ptrs, hs, ws = K.alt_levels_args(levels)
        # exact fp32 products, as the reference's kernel (set .precision = "f16x3" for the
        # fp32-accurate split-f16 box GEMM on MFMA)
        prec = _lib.PRECISIONS[getattr(self, "precision", "fp32")]
        _lib.call("raft_alt_corr_lookup_levels_prec", f1.data_ptr(), ptrs, hs, ws, len(levels), coords.data_ptr(), 1,
                  out.data_ptr(), out.shape[1], b, h, w, self.dim, r, div, None, 0, None, prec, s)
        return K.rows_to_nchw(K.Rows(out), b, h, w)
