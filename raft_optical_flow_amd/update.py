"""Update blocks — drop-in for core/update.py.

Same module tree and parameter names as the reference: FlowHead
(`core/update.py:6-28`), ConvGRU (`:30-72`), SepConvGRU (`:74-121`),
SmallMotionEncoder (`:123-167`), BasicMotionEncoder (`:169-216`),
SmallUpdateBlock (`:218-263`), BasicUpdateBlock (`:265-325`).

`BasicUpdateBlock(args, hidden_dim)(net, inp, corr, flow) -> (net, mask, delta)`
runs one update step on the HIP path (engine.plan_update): NHWC implicit-GEMM
convs on fp32 MFMA with the concatenations elided (virtual-concat inputs and
channel-offset outputs), the z/r gates of each GRU half-step as one GEMM with a
sigmoid / r*h epilogue, and the candidate conv's epilogue doing tanh and the
GRU blend in place.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib
from . import kernels as K


class FlowHead(nn.Module):
    def __init__(self, input_dim=128, hidden_dim=256):
        super().__init__()
        self.conv1 = nn.Conv2d(input_dim, hidden_dim, 3, padding=1)
        self.conv2 = nn.Conv2d(hidden_dim, 2, 3, padding=1)
        self.relu = nn.ReLU(inplace=True)


class ConvGRU(nn.Module):
    def __init__(self, hidden_dim=128, input_dim=192 + 128):
        super().__init__()
        self.convz = nn.Conv2d(hidden_dim + input_dim, hidden_dim, 3, padding=1)
        self.convr = nn.Conv2d(hidden_dim + input_dim, hidden_dim, 3, padding=1)
        self.convq = nn.Conv2d(hidden_dim + input_dim, hidden_dim, 3, padding=1)


class SepConvGRU(nn.Module):
    def __init__(self, hidden_dim=128, input_dim=192 + 128):
        super().__init__()
        self.convz1 = nn.Conv2d(hidden_dim + input_dim, hidden_dim, (1, 5), padding=(0, 2))
        self.convr1 = nn.Conv2d(hidden_dim + input_dim, hidden_dim, (1, 5), padding=(0, 2))
        self.convq1 = nn.Conv2d(hidden_dim + input_dim, hidden_dim, (1, 5), padding=(0, 2))
        self.convz2 = nn.Conv2d(hidden_dim + input_dim, hidden_dim, (5, 1), padding=(2, 0))
        self.convr2 = nn.Conv2d(hidden_dim + input_dim, hidden_dim, (5, 1), padding=(2, 0))
        self.convq2 = nn.Conv2d(hidden_dim + input_dim, hidden_dim, (5, 1), padding=(2, 0))


class SmallMotionEncoder(nn.Module):
    def __init__(self, args):
        super().__init__()
        cor_planes = args.corr_levels * (2 * args.corr_radius + 1) ** 2
        self.convc1 = nn.Conv2d(cor_planes, 96, 1, padding=0)
        self.convf1 = nn.Conv2d(2, 64, 7, padding=3)
        self.convf2 = nn.Conv2d(64, 32, 3, padding=1)
        self.conv = nn.Conv2d(128, 80, 3, padding=1)


class BasicMotionEncoder(nn.Module):
    def __init__(self, args):
        super().__init__()
        cor_planes = args.corr_levels * (2 * args.corr_radius + 1) ** 2
        self.convc1 = nn.Conv2d(cor_planes, 256, 1, padding=0)
        self.convc2 = nn.Conv2d(256, 192, 3, padding=1)
        self.convf1 = nn.Conv2d(2, 128, 7, padding=3)
        self.convf2 = nn.Conv2d(128, 64, 3, padding=1)
        self.conv = nn.Conv2d(64 + 192, 128 - 2, 3, padding=1)


class _UpdateBase(nn.Module):
    _small = False

    def forward(self, net, inp, corr, flow, upsample=True):
        from .engine import Arena, PackedUpdate, UpdateBuffers, plan_gru_context, plan_update
        K.require_device(net, inp, corr, flow)
        b, _, h, w = net.shape
        P = b * h * w
        pu = PackedUpdate(self, self._small, net.device)
        if corr.shape[1] != pu.cor_planes:
            raise ValueError(f"corr has {corr.shape[1]} channels, expected {pu.cor_planes}")
        A = Arena(net.device)
        ub = UpdateBuffers(A, pu, P, pu.cor_planes)
        s = K.stream_handle()
        lib = _lib.load()
        for t, rows in ((net, ub.h(pu)), (inp, ub.inp(pu)), (flow, K.Rows(ub.hx, ub.flow_off(pu), 2)),
                        (corr, K.Rows(ub.corr))):
            t = t.contiguous()
            _lib.check(lib.raft_nchw_to_nhwc(t.data_ptr(), rows.ptr, rows.ld, b, t.shape[1], h, w, s), "nchw_to_nhwc")
        ub.coords.zero_()  # coords1 += delta  ->  delta
        L = []
        plan_gru_context(L, pu, ub, b, h, w)
        plan_update(L, pu, ub, b, h, w, with_mask=not self._small)
        K.run(L)
        net_out = K.rows_to_nchw(ub.h(pu), b, h, w)
        delta = K.rows_to_nchw(K.Rows(ub.coords), b, h, w)
        mask = None if self._small else K.rows_to_nchw(K.Rows(ub.mask), b, h, w)
        return net_out, mask, delta


class SmallUpdateBlock(_UpdateBase):
    _small = True

    def __init__(self, args, hidden_dim=96):
        super().__init__()
        self.encoder = SmallMotionEncoder(args)
        self.gru = ConvGRU(hidden_dim=hidden_dim, input_dim=82 + 64)
        self.flow_head = FlowHead(hidden_dim, hidden_dim=128)


class BasicUpdateBlock(_UpdateBase):
    _small = False

    def __init__(self, args, hidden_dim=128, input_dim=128):
        super().__init__()
        self.args = args
        self.encoder = BasicMotionEncoder(args)
        self.gru = SepConvGRU(hidden_dim=hidden_dim, input_dim=128 + hidden_dim)
        self.flow_head = FlowHead(hidden_dim, hidden_dim=256)
        self.mask = nn.Sequential(
            nn.Conv2d(128, 256, 3, padding=1),
            nn.ReLU(inplace=True),
            nn.Conv2d(256, 64 * 9, 1, padding=0))
