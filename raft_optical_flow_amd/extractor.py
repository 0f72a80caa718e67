"""Feature / context encoders — drop-in for core/extractor.py.

Same module tree and parameter names as the reference (ResidualBlock
`core/extractor.py:6-56`, BottleneckBlock `:60-116`, BasicEncoder `:118-192`,
SmallEncoder `:195-267`), so reference state_dicts load unchanged.  forward()
runs the HIP path (implicit-GEMM convs on fp32 MFMA with BatchNorm folded and
ReLU / residual fused, InstanceNorm as stats + apply kernels) on NHWC rows.
Inference only (eval semantics for BatchNorm, no dropout).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib
from . import kernels as K
from .kernels import Rows


def _norm(norm_fn, planes, groups=None):
    if norm_fn == "group":
        return nn.GroupNorm(num_groups=groups, num_channels=planes)
    if norm_fn == "batch":
        return nn.BatchNorm2d(planes)
    if norm_fn == "instance":
        return nn.InstanceNorm2d(planes)
    if norm_fn == "none":
        return nn.Sequential()
    raise ValueError(norm_fn)


class _BlockBase(nn.Module):
    """Shared forward of ResidualBlock / BottleneckBlock on the HIP path (engine._plan_residual /
    _plan_bottleneck: the encoders' own launch sequence, BatchNorm folded, InstanceNorm as
    stats + apply kernels)."""
    _small = False

    def forward(self, x):
        from types import SimpleNamespace

        from .engine import Arena, _plan_bottleneck, _plan_residual, check_norm, pack_block
        if self.training and isinstance(self.norm1, nn.BatchNorm2d):
            raise NotImplementedError("raft_optical_flow_amd blocks are inference-only: call .eval()")
        check_norm(self.norm_fn, block=True)
        K.require_device(x)
        n, c, h, w = x.shape
        d = K.cached_pack(self, x.device, lambda: pack_block(self, self.norm_fn, self._small, x.device))
        pe = SimpleNamespace(norm=self.norm_fn, small=self._small)

        def build():  # input rows, buffers and launches, cached per input shape (K.cached_plan)
            L, A = [], Arena(x.device)
            xr = Rows(A.rows(n * h * w, c))
            plan = _plan_bottleneck if self._small else _plan_residual
            y, ho, wo = plan(L, A, pe, d, xr, n, h, w)
            return A, xr, L, y, ho, wo

        _, xr, L, y, ho, wo = K.cached_plan(self, d, (n, c, h, w, str(x.device)), build)
        xc = x.contiguous()
        _lib.call("raft_nchw_to_nhwc", xc.data_ptr(), xr.ptr, xr.ld, n, c, h, w, K.stream_handle())
        K.run(L)
        return K.rows_to_nchw(y, n, ho, wo)


class ResidualBlock(_BlockBase):
    def __init__(self, in_planes, planes, norm_fn="group", stride=1):
        super().__init__()
        self.norm_fn = norm_fn
        self.conv1 = nn.Conv2d(in_planes, planes, kernel_size=3, padding=1, stride=stride)
        self.conv2 = nn.Conv2d(planes, planes, kernel_size=3, padding=1)
        self.relu = nn.ReLU(inplace=True)
        g = planes // 8
        self.norm1 = _norm(norm_fn, planes, g)
        self.norm2 = _norm(norm_fn, planes, g)
        if stride != 1:
            self.norm3 = _norm(norm_fn, planes, g)
        self.downsample = None if stride == 1 else nn.Sequential(
            nn.Conv2d(in_planes, planes, kernel_size=1, stride=stride), self.norm3)


class BottleneckBlock(_BlockBase):
    _small = True

    def __init__(self, in_planes, planes, norm_fn="group", stride=1):
        super().__init__()
        self.norm_fn = norm_fn
        self.conv1 = nn.Conv2d(in_planes, planes // 4, kernel_size=1, padding=0)
        self.conv2 = nn.Conv2d(planes // 4, planes // 4, kernel_size=3, padding=1, stride=stride)
        self.conv3 = nn.Conv2d(planes // 4, planes, kernel_size=1, padding=0)
        self.relu = nn.ReLU(inplace=True)
        g = planes // 8
        self.norm1 = _norm(norm_fn, planes // 4, g)
        self.norm2 = _norm(norm_fn, planes // 4, g)
        self.norm3 = _norm(norm_fn, planes, g)
        if stride != 1:
            self.norm4 = _norm(norm_fn, planes, g)
        self.downsample = None if stride == 1 else nn.Sequential(
            nn.Conv2d(in_planes, planes, kernel_size=1, stride=stride), self.norm4)


class _EncoderBase(nn.Module):
    """Shared forward: NCHW (or [img1, img2] list) -> HIP trunk + head -> NCHW."""

    def forward(self, x):
        from .engine import Arena, PackedEncoder, plan_encoder_trunk
        if self.training and any(isinstance(m, (nn.BatchNorm2d, nn.Dropout2d)) for m in self.modules()):
            raise NotImplementedError("raft_optical_flow_amd encoders are inference-only: call .eval()")
        is_list = isinstance(x, (tuple, list))
        if is_list:
            batch_dim = x[0].shape[0]
            x = torch.cat(x, dim=0)
        K.require_device(x)
        n, c, h, w = x.shape
        pe = K.cached_pack(self, x.device, lambda: PackedEncoder(self, x.device))
        A = Arena(x.device)
        L = []
        src = Rows(K.nchw_to_rows(x))
        t, ho, wo = plan_encoder_trunk(L, A, pe, src, n, h, w)
        out = Rows(A.rows(n * ho * wo, pe.head.n))
        L.append(K.conv_launch(K.conv_params(pe.head, t, n, ho, wo, out)))
        K.run(L)
        y = K.rows_to_nchw(out, n, ho, wo)
        if is_list:
            return torch.split(y, [batch_dim, batch_dim], dim=0)
        return y


class BasicEncoder(_EncoderBase):
    def __init__(self, output_dim=128, norm_fn="batch", dropout=0.0):
        super().__init__()
        self.norm_fn = norm_fn
        self.norm1 = _norm(norm_fn, 64, 8)
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3)
        self.relu1 = nn.ReLU(inplace=True)
        self.in_planes = 64
        self.layer1 = self._make_layer(64, stride=1)
        self.layer2 = self._make_layer(96, stride=2)
        self.layer3 = self._make_layer(128, stride=2)
        self.conv2 = nn.Conv2d(128, output_dim, kernel_size=1)
        self.dropout = nn.Dropout2d(p=dropout) if dropout > 0 else None
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.InstanceNorm2d, nn.GroupNorm)):
                if m.weight is not None:
                    nn.init.constant_(m.weight, 1)
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)

    def _make_layer(self, dim, stride=1):
        layers = (ResidualBlock(self.in_planes, dim, self.norm_fn, stride=stride),
                  ResidualBlock(dim, dim, self.norm_fn, stride=1))
        self.in_planes = dim
        return nn.Sequential(*layers)


class SmallEncoder(_EncoderBase):
    def __init__(self, output_dim=128, norm_fn="batch", dropout=0.0):
        super().__init__()
        self.norm_fn = norm_fn
        self.norm1 = _norm(norm_fn, 32, 8)
        self.conv1 = nn.Conv2d(3, 32, kernel_size=7, stride=2, padding=3)
        self.relu1 = nn.ReLU(inplace=True)
        self.in_planes = 32
        self.layer1 = self._make_layer(32, stride=1)
        self.layer2 = self._make_layer(64, stride=2)
        self.layer3 = self._make_layer(96, stride=2)
        self.dropout = nn.Dropout2d(p=dropout) if dropout > 0 else None
        self.conv2 = nn.Conv2d(96, output_dim, kernel_size=1)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.InstanceNorm2d, nn.GroupNorm)):
                if m.weight is not None:
                    nn.init.constant_(m.weight, 1)
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)

    def _make_layer(self, dim, stride=1):
        layers = (BottleneckBlock(self.in_planes, dim, self.norm_fn, stride=stride),
                  BottleneckBlock(dim, dim, self.norm_fn, stride=1))
        self.in_planes = dim
        return nn.Sequential(*layers)
