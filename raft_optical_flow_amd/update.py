"""Update blocks — drop-in for core/update.py.

Same module tree and parameter names as the reference: FlowHead
(`core/update.py:6-28`), ConvGRU (`:30-72`), SepConvGRU (`:74-121`),
SmallMotionEncoder (`:123-167`), BasicMotionEncoder (`:169-216`),
SmallUpdateBlock (`:218-263`), BasicUpdateBlock (`:265-325`).

`BasicUpdateBlock(args, hidden_dim)(net, inp, corr, flow) -> (net, mask, delta)`
runs one update step on the HIP path (engine.plan_update): NHWC implicit-GEMM
convs on MFMA with the concatenations elided (virtual-concat inputs and
channel-offset outputs), the z/r gates of each GRU half-step as one GEMM with a
sigmoid / r*h epilogue, and the candidate conv's epilogue doing tanh and the
GRU blend in place.  Every sub-module keeps the reference's forward as well
(FlowHead(x), ConvGRU / SepConvGRU(h, x), the motion encoders (flow, corr)), on
the same kernels.  Block-level calls compute in exact fp32 MFMA unless the
module's `conv_precision` says otherwise; their packed weights are cached on
the module until a parameter changes.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib
from . import kernels as K
from .kernels import Rows


def _pk(conv, **kw):
    """pack_conv of an nn.Conv2d (its own stride / padding)."""
    return K.pack_conv(conv.weight, conv.bias, conv.stride, conv.padding, device=conv.weight.device, **kw)


def _rows(x: torch.Tensor, ld=None) -> torch.Tensor:
    K.require_device(x)
    return K.nchw_to_rows(x.contiguous(), ld)


def _pad4(c):
    return -(-c // 4) * 4


class FlowHead(nn.Module):
    def __init__(self, input_dim=128, hidden_dim=256):
        super().__init__()
        self.conv1 = nn.Conv2d(input_dim, hidden_dim, 3, padding=1)
        self.conv2 = nn.Conv2d(hidden_dim, 2, 3, padding=1)
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        """conv2(relu(conv1(x))) (core/update.py:6-28)."""
        c1, c2 = K.cached_pack(self, x.device, lambda: (_pk(self.conv1), _pk(self.conv2)))
        b, _, h, w = x.shape
        hid = Rows(torch.empty(b * h * w, c1.n, device=x.device))
        out = Rows(torch.empty(b * h * w, 4, device=x.device), 0, 2)
        K.conv2d_rows(c1, Rows(_rows(x)), b, h, w, hid, epilogue=_lib.EPI_RELU)
        K.conv2d_rows(c2, hid, b, h, w, out)
        return K.rows_to_nchw(out, b, h, w)


class _GRUHalf:
    """One GRU half-step as two GEMMs: z|r (sigmoid, r*h epilogue) over [h | x], then q over
    [r*h | x] with the tanh + (1-z)h + zq blend in its epilogue, h updated in place."""

    def __init__(self, cz, cr, cq, hd, xd):
        xp = _pad4(xd)
        w = torch.cat([cz.weight, cr.weight], 0)
        self.zr = K.pack_conv(w, torch.cat([cz.bias, cr.bias]), 1, cz.padding, seg_real=[hd + xd],
                              seg_decl=[hd + xp], device=w.device)
        self.q = K.pack_conv(cq.weight, cq.bias, 1, cq.padding, seg_real=[hd, xd], seg_decl=[hd, xp],
                             device=w.device)

    def launches(self, hx: torch.Tensor, hd, xp, z, rh, b, h, w):
        hrows = Rows(hx, 0, hd)
        return [K.conv_launch(K.conv_params(self.zr, Rows(hx), b, h, w, Rows(z), epilogue=_lib.EPI_GRU_ZR, split=hd,
                                            aux0=hrows, out1=Rows(rh))),
                K.conv_launch(K.conv_params(self.q, Rows(rh), b, h, w, hrows, src1=Rows(hx, hd, xp),
                                            epilogue=_lib.EPI_GRU_Q, aux0=hrows, aux1=Rows(z)))]


def _gru_forward(mod, steps, h, x):
    """Shared ConvGRU / SepConvGRU forward on NHWC rows [h | x | zero pad] (buffers and launches
    cached per input shape: K.cached_plan)."""
    K.require_device(h, x)
    b, hd, hh, ww = h.shape
    xd = x.shape[1]
    xp = _pad4(xd)
    halves = K.cached_pack(mod, h.device, lambda: [_GRUHalf(*s, hd, xd) for s in steps])

    def build():
        hx = torch.zeros(b * hh * ww, hd + xp, device=h.device)
        z = torch.empty(b * hh * ww, hd, device=h.device)
        rh = torch.empty_like(z)
        # (z and rh stay referenced by the plan: the launches hold raw pointers only)
        return hx, z, rh, [l for half in halves for l in half.launches(hx, hd, xp, z, rh, b, hh, ww)]

    hx, _, _, L = K.cached_plan(mod, halves, (b, hd, xd, hh, ww, str(h.device)), build)
    s = K.stream_handle()
    for t, off in ((h, 0), (x, hd)):
        t = t.contiguous()
        _lib.call("raft_nchw_to_nhwc", t.data_ptr(), hx.data_ptr() + 4 * off, hx.shape[1], b, t.shape[1], hh, ww, s)
    K.run(L)
    return K.rows_to_nchw(Rows(hx, 0, hd), b, hh, ww)


class ConvGRU(nn.Module):
    def __init__(self, hidden_dim=128, input_dim=192 + 128):
        super().__init__()
        self.convz = nn.Conv2d(hidden_dim + input_dim, hidden_dim, 3, padding=1)
        self.convr = nn.Conv2d(hidden_dim + input_dim, hidden_dim, 3, padding=1)
        self.convq = nn.Conv2d(hidden_dim + input_dim, hidden_dim, 3, padding=1)

    def forward(self, h, x):
        """h <- (1-z) h + z tanh(convq([r h, x])), z, r = sigmoid(convz / convr([h, x])) (core/update.py:52-72)."""
        return _gru_forward(self, [(self.convz, self.convr, self.convq)], h, x)


class SepConvGRU(nn.Module):
    def __init__(self, hidden_dim=128, input_dim=192 + 128):
        super().__init__()
        self.convz1 = nn.Conv2d(hidden_dim + input_dim, hidden_dim, (1, 5), padding=(0, 2))
        self.convr1 = nn.Conv2d(hidden_dim + input_dim, hidden_dim, (1, 5), padding=(0, 2))
        self.convq1 = nn.Conv2d(hidden_dim + input_dim, hidden_dim, (1, 5), padding=(0, 2))
        self.convz2 = nn.Conv2d(hidden_dim + input_dim, hidden_dim, (5, 1), padding=(2, 0))
        self.convr2 = nn.Conv2d(hidden_dim + input_dim, hidden_dim, (5, 1), padding=(2, 0))
        self.convq2 = nn.Conv2d(hidden_dim + input_dim, hidden_dim, (5, 1), padding=(2, 0))

    def forward(self, h, x):
        """The 1x5 half-step, then the 5x1 half-step (core/update.py:99-121)."""
        return _gru_forward(self, [(self.convz1, self.convr1, self.convq1), (self.convz2, self.convr2, self.convq2)],
                            h, x)


def _motion_forward(mod, flow, corr, small):
    """BasicMotionEncoder / SmallMotionEncoder forward (core/update.py:145-167, :193-216):
    cor = relu(convc1(corr)) [-> relu(convc2)], flo = relu(convf2(relu(convf1(flow)))),
    out = relu(conv([cor, flo])); returns [out, flow]."""
    K.require_device(flow, corr)
    b, _, h, w = flow.shape
    dev = flow.device

    def build():
        return {n: _pk(getattr(mod, n), **({"mode": _lib.RAFT_CONV_GATHER} if n == "convf1" else {}))
                for n in ("convc1", "convc2", "convf1", "convf2", "conv") if hasattr(mod, n)}

    pc = K.cached_pack(mod, dev, build)
    P = b * h * w
    cor_c, flo_c = (96, 32) if small else (192, 64)
    out_c = pc["conv"].n
    fl = Rows(_rows(flow))
    cr = Rows(_rows(corr, _pad4(corr.shape[1])), 0, corr.shape[1])
    cf = Rows(torch.empty(P, cor_c + flo_c, device=dev))
    if small:
        K.conv2d_rows(pc["convc1"], cr, b, h, w, cf.sub(0, cor_c), epilogue=_lib.EPI_RELU)
    else:
        cor1 = Rows(torch.empty(P, pc["convc1"].n, device=dev))
        K.conv2d_rows(pc["convc1"], cr, b, h, w, cor1, epilogue=_lib.EPI_RELU)
        K.conv2d_rows(pc["convc2"], cor1, b, h, w, cf.sub(0, cor_c), epilogue=_lib.EPI_RELU)
    flo1 = Rows(torch.empty(P, pc["convf1"].n, device=dev))
    K.conv2d_rows(pc["convf1"], fl, b, h, w, flo1, epilogue=_lib.EPI_RELU)
    K.conv2d_rows(pc["convf2"], flo1, b, h, w, cf.sub(cor_c, flo_c), epilogue=_lib.EPI_RELU)
    out = torch.empty(P, _pad4(out_c + 2), device=dev)
    K.conv2d_rows(pc["conv"], cf, b, h, w, Rows(out, 0, out_c), epilogue=_lib.EPI_RELU)
    # cat([out, flow]): the flow lands in the last two channels of the output rows
    _lib.call("raft_nchw_to_nhwc", flow.contiguous().data_ptr(), out.data_ptr() + 4 * out_c, out.shape[1], b, 2, h, w,
              K.stream_handle())
    return K.rows_to_nchw(Rows(out, 0, out_c + 2), b, h, w)


class SmallMotionEncoder(nn.Module):
    def __init__(self, args):
        super().__init__()
        cor_planes = args.corr_levels * (2 * args.corr_radius + 1) ** 2
        self.convc1 = nn.Conv2d(cor_planes, 96, 1, padding=0)
        self.convf1 = nn.Conv2d(2, 64, 7, padding=3)
        self.convf2 = nn.Conv2d(64, 32, 3, padding=1)
        self.conv = nn.Conv2d(128, 80, 3, padding=1)

    def forward(self, flow, corr):
        return _motion_forward(self, flow, corr, small=True)


class BasicMotionEncoder(nn.Module):
    def __init__(self, args):
        super().__init__()
        cor_planes = args.corr_levels * (2 * args.corr_radius + 1) ** 2
        self.convc1 = nn.Conv2d(cor_planes, 256, 1, padding=0)
        self.convc2 = nn.Conv2d(256, 192, 3, padding=1)
        self.convf1 = nn.Conv2d(2, 128, 7, padding=3)
        self.convf2 = nn.Conv2d(128, 64, 3, padding=1)
        self.conv = nn.Conv2d(64 + 192, 128 - 2, 3, padding=1)

    def forward(self, flow, corr):
        return _motion_forward(self, flow, corr, small=False)


class _UpdateBase(nn.Module):
    _small = False

    def forward(self, net, inp, corr, flow, upsample=True):
        from .engine import Arena, PackedUpdate, UpdateBuffers, plan_gru_context, plan_update
        K.require_device(net, inp, corr, flow)
        b, _, h, w = net.shape
        P = b * h * w
        pu = K.cached_pack(self, net.device, lambda: PackedUpdate(self, self._small, net.device))
        if corr.shape[1] != pu.cor_planes:
            raise ValueError(f"corr has {corr.shape[1]} channels, expected {pu.cor_planes}")
        def build():  # buffers and launches, cached per input shape (K.cached_plan)
            A = Arena(net.device)
            ub = UpdateBuffers(A, pu, P, pu.cor_planes)
            L = []
            plan_gru_context(L, pu, ub, b, h, w)
            plan_update(L, pu, ub, b, h, w, with_mask=not self._small)
            return A, ub, L

        _, ub, L = K.cached_plan(self, pu, (b, h, w, str(net.device)), build)
        s = K.stream_handle()
        lib = _lib.load()
        for t, rows in ((net, ub.h(pu)), (inp, ub.inp(pu)), (flow, K.Rows(ub.hx, ub.flow_off(pu), 2)),
                        (corr, K.Rows(ub.corr))):
            t = t.contiguous()
            _lib.check(lib.raft_nchw_to_nhwc(t.data_ptr(), rows.ptr, rows.ld, b, t.shape[1], h, w, s), "nchw_to_nhwc")
        ub.coords.zero_()  # coords1 += delta  ->  delta
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
