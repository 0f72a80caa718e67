"""Execution plans for the RAFT inference path on MI355X.

A plan is built once per (model weights, batch, image size, iters, mode): it
allocates every device buffer up front (NHWC row buffers, correlation
pyramid, recurrent state) and records the exact sequence of C-ABI kernel
launches with their fixed pointers.  `RaftPlan.run()` replays the launch list
on the current stream; `RaftPlan.capture()` records it into a hipGraph
(torch.cuda.CUDAGraph on ROCm) so the 32-iteration refinement loop replays
with no host work per kernel.

Buffer layout of the recurrent state (P = B * H/8 * W/8 rows), RAFT-full:
  HX   [P, 384]  = h (128) | motion conv (126) | flow (2) | inp (128)
                 -> hx = cat[h, x] of core/update.py:106 without a copy
                    (x = cat[inp, motion, flow], core/update.py:318, with its
                    channels permuted; the packed GRU weights follow)
  CTX1, CTX2 [P, 384]  iteration-invariant GRU term W_inp * inp + b of each
                 half-step's z | r | q convs, computed once per pair: inp never
                 changes inside the loop, so the per-iteration GRU GEMMs only
                 contract over h | motion | flow (K = 5*256 instead of 5*384)
  CORR [P, 324]  lookup output, channel lvl*81 + ix*9 + iy
  COR1 [P, 256], CF [P, 256] = cor (192) | flo (64), FLO1 [P, 128]
  Z, RH [P, 128] GRU gate z and r*h
  FH   [P, 512]  flow-head conv1 (256) | mask conv1 (256), one fused GEMM
  MASK [P, 576], coords1 [P, 2]
RAFT-small uses the same scheme with hdim 96 / cdim 64: HX [P, 244] =
h (96) | motion (80) | flow (2) | 2 zero pad channels | inp (64) (rows and the
inp slot stay 16-byte aligned).
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _lib
from . import kernels as K
from .kernels import Launch, PackedConv, Rows, conv_launch, conv_params, pack_conv, fold_bn, set_precision

# ----------------------------------------------------------------------------
# Weight packing
# ----------------------------------------------------------------------------


def _conv_bn(conv, bn, device, **kw):
    if bn is None:
        return pack_conv(conv.weight, conv.bias, conv.stride, conv.padding, device=device, **kw)
    w, b = fold_bn(conv.weight, conv.bias, bn)
    return pack_conv(w, b, conv.stride, conv.padding, device=device, **kw)


def check_norm(norm, block=False):
    """The norms the HIP path plans: the encoders' instance / batch / none; block-level calls
    (ResidualBlock / BottleneckBlock, core/extractor.py:6-116) also take their default, group."""
    if norm not in ("instance", "batch", "none") and not (block and norm == "group"):
        raise NotImplementedError(f"norm_fn={norm!r} is not on the RAFT inference path")


def _gn(mod):
    """(num_groups, gamma, beta, eps) of an nn.GroupNorm, fp32 on its device."""
    g = mod.weight.detach().float().contiguous() if mod.weight is not None else None
    b = mod.bias.detach().float().contiguous() if mod.bias is not None else None
    return (mod.num_groups, g, b, float(mod.eps))


def pack_block(blk, norm, small, device) -> dict:
    """One ResidualBlock (core/extractor.py:6-56) / BottleneckBlock (:60-116), eval BatchNorm folded."""
    bn = (lambda m: m) if norm == "batch" else (lambda m: None)
    d = {"stride": blk.conv1.stride[0] if not small else blk.conv2.stride[0]}
    d["conv1"] = _conv_bn(blk.conv1, bn(blk.norm1), device)
    d["conv2"] = _conv_bn(blk.conv2, bn(blk.norm2), device)
    if small:
        d["conv3"] = _conv_bn(blk.conv3, bn(blk.norm3), device)
        dsn = getattr(blk, "norm4", None)
    else:
        dsn = getattr(blk, "norm3", None)
    d["ds"] = None if blk.downsample is None else _conv_bn(blk.downsample[0], bn(dsn), device)
    d["planes"] = d["conv3" if small else "conv2"].n
    if norm == "group":
        d["n1"], d["n2"] = _gn(blk.norm1), _gn(blk.norm2)
        if small:
            d["n3"] = _gn(blk.norm3)
        d["nds"] = None if blk.downsample is None else _gn(dsn)
    return d


class PackedEncoder:
    """BasicEncoder (core/extractor.py:118-192) / SmallEncoder (:195-267) weights, packed."""

    def __init__(self, enc, device):
        self.norm = enc.norm_fn
        check_norm(self.norm)
        self.small = enc.__class__.__name__ == "SmallEncoder"
        bn = (lambda m: m) if self.norm == "batch" else (lambda m: None)
        self.stem = _conv_bn(enc.conv1, bn(enc.norm1), device, mode=_lib.RAFT_CONV_GATHER)
        self.blocks = [pack_block(blk, self.norm, self.small, device)
                       for layer in (enc.layer1, enc.layer2, enc.layer3) for blk in layer]
        self.head = pack_conv(enc.conv2.weight, enc.conv2.bias, 1, 0, device=device)


class PackedUpdate:
    """BasicUpdateBlock (core/update.py:265-325) / SmallUpdateBlock (:218-263) weights, packed.

    * each GRU half-step's z and r convs are one GEMM (N = 2*hdim, sigmoid / r*h epilogue);
    * the GRU convs are split by input channel: the columns acting on `inp`
      (constant over the iterations) form the once-per-pair context GEMM `ctx`
      (N = 3*hdim: z | r | q, bias folded in), the rest the per-iteration GEMMs
      over HX's h | motion | flow prefix (reference column order
      h | inp | motion | flow, core/update.py:106 + :318, permuted to match);
    * the basic block's flow-head and mask-head first convs are one GEMM (N = 512).
    """

    def __init__(self, ub, small, device):
        e, g, fh = ub.encoder, ub.gru, ub.flow_head
        self.small = small
        if small:
            hd, cd, mc, pad = 96, 64, 80, 2
            steps = [(g.convz, g.convr, g.convq)]
        else:
            hd, cd, mc, pad = 128, 128, 126, 0
            steps = [(g.convz1, g.convr1, g.convq1), (g.convz2, g.convr2, g.convq2)]
        self.hdim, self.cdim, self.mc, self.pad = hd, cd, mc, pad
        self.inp_off = hd + mc + 2 + pad          # HX: h | motion | flow | pad | inp
        self.ld = self.inp_off + cd
        self.convc1 = pack_conv(e.convc1.weight, e.convc1.bias, 1, 0, device=device)
        self.convc2 = None if small else pack_conv(e.convc2.weight, e.convc2.bias, 1, 1, device=device)
        self.convf1 = pack_conv(e.convf1.weight, e.convf1.bias, 1, 3, device=device, mode=_lib.RAFT_CONV_GATHER)
        self.convf2 = pack_conv(e.convf2.weight, e.convf2.bias, 1, 1, device=device)
        self.conv = pack_conv(e.conv.weight, e.conv.bias, 1, 1, device=device)
        # reference input columns of a GRU conv: h [0,hd) | inp [hd,hd+cd) | motion | flow
        hcols = slice(0, hd)
        icols = slice(hd, hd + cd)
        mcols = slice(hd + cd, hd + cd + mc + 2)   # motion + flow, contiguous
        self.gru = []
        for cz, cr, cq in steps:
            wzr = torch.cat([cz.weight, cr.weight], 0).detach()
            wq = cq.weight.detach()
            # per iteration: [h | motion | flow (| pad)] for z,r ; [r*h | motion | flow (| pad)] for q
            zr = pack_conv(torch.cat([wzr[:, hcols], wzr[:, mcols]], 1), None, 1, cz.padding,
                           seg_real=[hd + mc + 2], seg_decl=[hd + mc + 2 + pad], device=device)
            q = pack_conv(torch.cat([wq[:, hcols], wq[:, mcols]], 1), None, 1, cq.padding,
                          seg_real=[hd, mc + 2], seg_decl=[hd, mc + 2 + pad], device=device)
            # once per pair: inp -> z | r | q pre-activations (+ biases)
            wctx = torch.cat([wzr[:, icols], wq[:, icols]], 0)
            bctx = torch.cat([cz.bias, cr.bias, cq.bias], 0)
            ctx = pack_conv(wctx, bctx, 1, cz.padding, device=device)
            self.gru.append((zr, q, ctx))
        self.fh1 = pack_conv(fh.conv1.weight, fh.conv1.bias, 1, 1, device=device)
        self.fh2 = pack_conv(fh.conv2.weight, fh.conv2.bias, 1, 1, device=device)
        if not small:
            m0, m2 = ub.mask[0], ub.mask[2]
            self.fh1_mask = pack_conv(torch.cat([fh.conv1.weight, m0.weight], 0), torch.cat([fh.conv1.bias, m0.bias], 0),
                                      1, 1, device=device)
            self.mask2 = pack_conv(m2.weight, m2.bias, 1, 0, device=device)
        else:
            self.fh1_mask = None
            self.mask2 = None
        self.cor_planes = e.convc1.weight.shape[1]


class PackedRaft:
    def __init__(self, model, device, precision=_lib.PREC_FP32):
        self.small = bool(model.args.small)
        self.hdim, self.cdim = model.hidden_dim, model.context_dim
        self.radius = model.args.corr_radius
        self.levels = model.args.corr_levels
        self.fnet = PackedEncoder(model.fnet, device)
        self.cnet = PackedEncoder(model.cnet, device)
        self.update = PackedUpdate(model.update_block, self.small, device)
        self.fdim = self.fnet.head.n
        self.precision = precision
        set_precision(self, precision)


# ----------------------------------------------------------------------------
# Plan building blocks
# ----------------------------------------------------------------------------


class Arena:
    def __init__(self, device):
        self.device = device
        self.bufs = []

    def rows(self, npix, ld, zero=False) -> torch.Tensor:
        t = (torch.zeros if zero else torch.empty)(npix, ld, device=self.device, dtype=torch.float32)
        self.bufs.append(t)
        return t

    def flat(self, n, zero=False) -> torch.Tensor:
        t = (torch.zeros if zero else torch.empty)(max(int(n), 1), device=self.device, dtype=torch.float32)
        self.bufs.append(t)
        return t


def _in_stats(L, A: Arena, x: Rows, n_img, hw):
    c = x.c
    st = A.flat(2 * n_img * c)
    ws = A.flat(_lib.load().raft_instnorm_workspace_floats(n_img, hw, c))
    L.append(Launch("raft_instnorm_stats", x.ptr, x.ld, n_img, hw, c, 1e-5, st.data_ptr(), ws.data_ptr()))
    return st


def _conv_in(L, A: Arena, pc: PackedConv, src: Rows, n_img, h, w, out: Rows, src_norm=None):
    """A conv whose raw output feeds an InstanceNorm; returns that norm's statistics.  On the halo /
    stem kernel the conv's epilogue writes per-wave (count, mean, M2) partials and one merge launch
    replaces raft_instnorm_stats' pass over the output (raft_conv2d_stats_slots; RAFT_EPI_STATS=0:
    always the separate pass).  src_norm: src is a raw conv output whose relu(InstanceNorm) the conv
    applies in its loaders (the statistics; the caller checked _norm_in_loader).  (The raw conv
    outputs of an InstanceNorm encoder feed the fp32 statistics and normalisation only: no range
    guard, raft_hip.h.)"""

    p = conv_params(pc, src, n_img, h, w, out)
    if src_norm is not None:
        p.in_norm, p.in_norm_relu = src_norm.data_ptr(), 1
    slots = int(_lib.load().raft_conv2d_stats_slots(ctypes.byref(p)))
    ho, wo = K.conv_out_hw(pc, h, w)
    if slots > 0 and os.environ.get("RAFT_EPI_STATS", "1") != "0":
        part = A.flat(n_img * slots * out.c * 4)
        p.stats_part, p.stats_ld = part.data_ptr(), out.c
        L.append(conv_launch(p))
        st = A.flat(2 * n_img * out.c)
        ws = A.flat(_lib.load().raft_instnorm_merge_ws_floats(slots, n_img, out.c))
        if os.environ.get("RAFT_MERGE_FUSED", "1") != "0":
            # one launch (the last level-1 block per channel group and image runs level 2); its
            # counters start at zero and every launch leaves them zero
            cnt = torch.zeros(int(_lib.load().raft_instnorm_merge_counters(n_img, out.c)), dtype=torch.int32,
                              device=A.device)
            A.bufs.append(cnt)
            L.append(Launch("raft_instnorm_merge_fused", part.data_ptr(), slots, n_img, out.c, out.c, 1e-5,
                            ws.data_ptr(), cnt.data_ptr(), st.data_ptr()))
        else:
            L.append(Launch("raft_instnorm_merge_ws", part.data_ptr(), slots, n_img, out.c, out.c, 1e-5,
                            ws.data_ptr(), st.data_ptr()))
        return st
    L.append(conv_launch(p))
    return _in_stats(L, A, out, n_img, ho * wo)


def _norm_in_loader(pc: PackedConv, src: Rows, n_img, h, w) -> bool:
    """Whether the conv of pc over src can apply src's relu(InstanceNorm) in its loaders
    (raft_conv2d_in_norm_ok; RAFT_IN_NORM=0: never), which saves the normalised copy's pass."""

    if os.environ.get("RAFT_IN_NORM", "1") == "0":
        return False
    p = conv_params(pc, src, n_img, h, w, src)   # (only checked, never launched)
    p.in_norm, p.in_norm_relu = src.ptr, 1
    return bool(_lib.load().raft_conv2d_in_norm_ok(ctypes.byref(p)))


def _in_apply(L, A: Arena, x: Rows, st, n_img, hw, mode, resid: Rows | None = None, rst=None) -> Rows:
    out = Rows(A.rows(n_img * hw, x.c))
    L.append(Launch("raft_instnorm_apply", x.ptr, x.ld, st.data_ptr(), resid.ptr if resid else None,
                    resid.ld if resid else 0, rst.data_ptr() if rst is not None else None, mode,
                    out.ptr, out.ld, n_img, hw, x.c))
    return out


# the f16x3 range guard's device flag of the plan being built (RaftPlan.__init__ sets it):
# every conv whose output feeds a split-precision conv raises it on |x| > 2^15 (raft_hip.h)
_GUARD = {"flag": None}


def _conv(L, pc: PackedConv, src: Rows, n_img, h, w, out: Rows, side=False, **kw):
    kw.setdefault("range_flag", _GUARD["flag"])
    L.append(conv_launch(conv_params(pc, src, n_img, h, w, out, **kw), side=side))


def plan_encoder_trunk(L, A: Arena, pe: PackedEncoder, x: Rows, n_img, h, w):
    """Everything of the encoder but its final 1x1 conv.  Returns (rows, h, w)."""
    ho, wo = K.conv_out_hw(pe.stem, h, w)
    if pe.norm == "instance":
        # (the raw conv outputs of an InstanceNorm encoder feed the fp32 statistics and the
        # normalisation, whose outputs are bounded by sqrt(H*W): no range guard, raft_hip.h)
        t = Rows(A.rows(n_img * ho * wo, pe.stem.n))
        st = _conv_in(L, A, pe.stem, x, n_img, h, w, t)
        x = _in_apply(L, A, t, st, n_img, ho * wo, 1)
    else:
        t = Rows(A.rows(n_img * ho * wo, pe.stem.n))
        _conv(L, pe.stem, x, n_img, h, w, t, epilogue=_lib.EPI_RELU)
        x = t
    h, w = ho, wo
    for d in pe.blocks:
        if pe.small:
            x, h, w = _plan_bottleneck(L, A, pe, d, x, n_img, h, w)
        else:
            x, h, w = _plan_residual(L, A, pe, d, x, n_img, h, w)
    return x, h, w


def _gn_stats(L, A: Arena, x: Rows, n_img, hw, gn):
    st = A.flat(2 * n_img * x.c)
    L.append(Launch("raft_groupnorm_stats", x.ptr, x.ld, n_img, hw, x.c, gn[0], gn[3], st.data_ptr()))
    return st


def _gn_apply(L, A: Arena, x: Rows, st, gn, n_img, hw, mode, resid: Rows | None = None, rst=None, rgn=None) -> Rows:
    """relu / residual tail of a GroupNorm (raft_norm_apply_affine: the normalisation, its affine, the
    residual's own normalisation + affine where given)."""
    out = Rows(A.rows(n_img * hw, x.c))
    p = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    L.append(Launch("raft_norm_apply_affine", x.ptr, x.ld, st.data_ptr(), p(gn[1]), p(gn[2]),
                    resid.ptr if resid else None, resid.ld if resid else 0, p(rst),
                    p(rgn[1]) if rgn else None, p(rgn[2]) if rgn else None, mode, out.ptr, out.ld, n_img, hw, x.c,
                    keep=(gn, rgn)))
    return out


def _plan_residual_group(L, A, d, x: Rows, n, h, w):
    """ResidualBlock with norm_fn='group' (core/extractor.py:6-56, the block's default norm):
    relu(gn1(conv1 x)) -> relu(gn2(conv2 .)) -> relu(x or gn3(downsample x) + .)."""
    c1, c2, ds = d["conv1"], d["conv2"], d["ds"]
    ho, wo = K.conv_out_hw(c1, h, w)
    npx, hw = n * ho * wo, ho * wo
    t1 = Rows(A.rows(npx, c1.n))
    _conv(L, c1, x, n, h, w, t1)
    y1 = _gn_apply(L, A, t1, _gn_stats(L, A, t1, n, hw, d["n1"]), d["n1"], n, hw, 1)
    t2 = Rows(A.rows(npx, c2.n))
    _conv(L, c2, y1, n, ho, wo, t2)
    st2 = _gn_stats(L, A, t2, n, hw, d["n2"])
    if ds is not None:
        t3 = Rows(A.rows(npx, ds.n))
        _conv(L, ds, x, n, h, w, t3)
        out = _gn_apply(L, A, t2, st2, d["n2"], n, hw, 2, resid=t3, rst=_gn_stats(L, A, t3, n, hw, d["nds"]),
                        rgn=d["nds"])
    else:
        out = _gn_apply(L, A, t2, st2, d["n2"], n, hw, 2, resid=x)
    return out, ho, wo


def _plan_bottleneck_group(L, A, d, x: Rows, n, h, w):
    """BottleneckBlock with norm_fn='group' (core/extractor.py:60-116)."""
    c1, c2, c3, ds = d["conv1"], d["conv2"], d["conv3"], d["ds"]
    ho, wo = K.conv_out_hw(c2, h, w)
    t1 = Rows(A.rows(n * h * w, c1.n))
    _conv(L, c1, x, n, h, w, t1)
    y1 = _gn_apply(L, A, t1, _gn_stats(L, A, t1, n, h * w, d["n1"]), d["n1"], n, h * w, 1)
    hw = ho * wo
    t2 = Rows(A.rows(n * hw, c2.n))
    _conv(L, c2, y1, n, h, w, t2)
    y2 = _gn_apply(L, A, t2, _gn_stats(L, A, t2, n, hw, d["n2"]), d["n2"], n, hw, 1)
    t3 = Rows(A.rows(n * hw, c3.n))
    _conv(L, c3, y2, n, ho, wo, t3)
    st3 = _gn_stats(L, A, t3, n, hw, d["n3"])
    if ds is not None:
        t4 = Rows(A.rows(n * hw, ds.n))
        _conv(L, ds, x, n, h, w, t4)
        out = _gn_apply(L, A, t3, st3, d["n3"], n, hw, 2, resid=t4, rst=_gn_stats(L, A, t4, n, hw, d["nds"]),
                        rgn=d["nds"])
    else:
        out = _gn_apply(L, A, t3, st3, d["n3"], n, hw, 2, resid=x)
    return out, ho, wo


def _plan_residual(L, A, pe, d, x: Rows, n, h, w):
    """ResidualBlock (core/extractor.py:6-56)."""
    if pe.norm == "group":
        return _plan_residual_group(L, A, d, x, n, h, w)
    c1, c2, ds = d["conv1"], d["conv2"], d["ds"]
    ho, wo = K.conv_out_hw(c1, h, w)
    npx = n * ho * wo
    if pe.norm == "instance":
        t1 = Rows(A.rows(npx, c1.n))
        st1 = _conv_in(L, A, c1, x, n, h, w, t1)
        t2 = Rows(A.rows(npx, c2.n))
        if _norm_in_loader(c2, t1, n, ho, wo):
            st2 = _conv_in(L, A, c2, t1, n, ho, wo, t2, src_norm=st1)
        else:
            y1 = _in_apply(L, A, t1, st1, n, ho * wo, 1)
            st2 = _conv_in(L, A, c2, y1, n, ho, wo, t2)
        if ds is not None:
            t3 = Rows(A.rows(npx, ds.n))
            out = _in_apply(L, A, t2, st2, n, ho * wo, 2, resid=t3, rst=_conv_in(L, A, ds, x, n, h, w, t3))
        else:
            out = _in_apply(L, A, t2, st2, n, ho * wo, 2, resid=x)
        return out, ho, wo
    y1 = Rows(A.rows(npx, c1.n))
    _conv(L, c1, x, n, h, w, y1, epilogue=_lib.EPI_RELU)
    if ds is not None:
        xs = Rows(A.rows(npx, ds.n))
        _conv(L, ds, x, n, h, w, xs)
    else:
        xs = x
    out = Rows(A.rows(npx, c2.n))
    _conv(L, c2, y1, n, ho, wo, out, epilogue=_lib.EPI_RESID_RELU, aux0=xs)
    return out, ho, wo


def _plan_bottleneck(L, A, pe, d, x: Rows, n, h, w):
    """BottleneckBlock (core/extractor.py:60-116)."""
    if pe.norm == "group":
        return _plan_bottleneck_group(L, A, d, x, n, h, w)
    c1, c2, c3, ds = d["conv1"], d["conv2"], d["conv3"], d["ds"]
    ho, wo = K.conv_out_hw(c2, h, w)
    if pe.norm == "instance":
        t1 = Rows(A.rows(n * h * w, c1.n))
        st1 = _conv_in(L, A, c1, x, n, h, w, t1)
        t2 = Rows(A.rows(n * ho * wo, c2.n))
        if _norm_in_loader(c2, t1, n, h, w):
            st2 = _conv_in(L, A, c2, t1, n, h, w, t2, src_norm=st1)
        else:
            st2 = _conv_in(L, A, c2, _in_apply(L, A, t1, st1, n, h * w, 1), n, h, w, t2)
        y2 = _in_apply(L, A, t2, st2, n, ho * wo, 1)
        t3 = Rows(A.rows(n * ho * wo, c3.n))
        st3 = _conv_in(L, A, c3, y2, n, ho, wo, t3)
        if ds is not None:
            t4 = Rows(A.rows(n * ho * wo, ds.n))
            out = _in_apply(L, A, t3, st3, n, ho * wo, 2, resid=t4, rst=_conv_in(L, A, ds, x, n, h, w, t4))
        else:
            out = _in_apply(L, A, t3, st3, n, ho * wo, 2, resid=x)
        return out, ho, wo
    y1 = Rows(A.rows(n * h * w, c1.n))
    _conv(L, c1, x, n, h, w, y1, epilogue=_lib.EPI_RELU)
    y2 = Rows(A.rows(n * ho * wo, c2.n))
    _conv(L, c2, y1, n, h, w, y2, epilogue=_lib.EPI_RELU)
    if ds is not None:
        xs = Rows(A.rows(n * ho * wo, ds.n))
        _conv(L, ds, x, n, h, w, xs)
    else:
        xs = x
    out = Rows(A.rows(n * ho * wo, c3.n))
    _conv(L, c3, y2, n, ho, wo, out, epilogue=_lib.EPI_RESID_RELU, aux0=xs)
    return out, ho, wo


class UpdateBuffers:
    """Recurrent-state buffers of the update block for P rows (module docstring)."""

    def __init__(self, A: Arena, pu: PackedUpdate, P, corr_ld):
        self.P = P
        self.hx = A.rows(P, pu.ld, zero=True)
        self.corr = A.rows(P, corr_ld)
        hd = pu.hdim
        if pu.small:
            self.cor1 = None
            self.cf = A.rows(P, 128)       # cor (96) | flo (32)
            self.flo1 = A.rows(P, 64)
            self.fh = A.rows(P, 128)
            self.mask = None
        else:
            self.cor1 = A.rows(P, 256)
            self.cf = A.rows(P, 256)       # cor (192) | flo (64)
            self.flo1 = A.rows(P, 128)
            self.fh = A.rows(P, 512)
            self.mask = A.rows(P, 576)
        self.z = A.rows(P, hd)
        self.rh = A.rows(P, hd)
        self.ctx = [A.rows(P, 3 * hd) for _ in pu.gru]   # z | r | q context terms per half-step
        self.coords = A.rows(P, 2)

    # channel slots of HX
    def h(self, pu):
        return Rows(self.hx, 0, pu.hdim)

    def motion(self, pu):
        return Rows(self.hx, pu.hdim, pu.mc)

    def flow_off(self, pu):
        return pu.hdim + pu.mc

    def inp(self, pu):
        return Rows(self.hx, pu.inp_off, pu.cdim)

    def gru_in(self, pu):
        """h | motion | flow (| pad): the per-iteration input of the z/r GEMM."""
        return Rows(self.hx, 0, pu.inp_off)

    def x_dyn(self, pu):
        """motion | flow (| pad): the second segment of the q GEMM's input."""
        return Rows(self.hx, pu.hdim, pu.inp_off - pu.hdim)


def plan_gru_context(L, pu: PackedUpdate, ub: UpdateBuffers, B, h, w):
    """Once per pair: W_inp * inp + b for the z | r | q convs of every GRU half-step."""
    for (zr, q, ctx), buf in zip(pu.gru, ub.ctx):
        _conv(L, ctx, ub.inp(pu), B, h, w, Rows(buf), epilogue=_lib.EPI_LINEAR)


def convf1_fused(pu: PackedUpdate) -> bool:
    """Whether the all-pairs loop computes convf1 inside the lookup launch
    (raft_corr_lookup_convf1; RAFT_FUSE_CONVF1=0 keeps it a conv launch of its own)."""
    return (not pu.small and pu.convf1.kh == 7 and pu.convf1.n % 32 == 0
            and os.environ.get("RAFT_FUSE_CONVF1", "1") != "0")


def convf1_vec_weight(pu: PackedUpdate) -> torch.Tensor:
    """convf1's weight in raft_corr_lookup_convf1's layout [n/32][k*k][2][32] (raft_hip.h),
    rounded to the operand type of the conv precision (f16 / bf16 modes), cached per precision."""
    pc = pu.convf1
    prec = pc.precision
    cached = getattr(pu, "_convf1_vec", None)
    if cached is not None and cached[0] == prec:
        return cached[1]
    n, kk = pc.n, pc.kh * pc.kw
    w = pc.weight[:n, : kk * 2].reshape(n // 32, 32, kk, 2).permute(0, 2, 3, 1).contiguous()
    if prec == _lib.PREC_F16:
        w = w.half().float()
    elif prec == _lib.PREC_BF16:
        w = w.bfloat16().float()
    pu._convf1_vec = (prec, w)
    return w


def convc1_fused(pk: PackedRaft) -> bool:
    """Whether the all-pairs loop runs the lookup, convc1 and convf1 as ONE launch
    (raft_corr_lookup_conv: RAFT-full's radius 4 / 4 levels, split-precision convs;
    RAFT_FUSE_CONVC1=0 keeps lookup + convf1 and convc1 as two launches)."""
    pu = pk.update
    return (convf1_fused(pu) and pk.radius == 4 and pk.levels == 4 and pu.convc1.n == 256
            and pu.convc1.cin == 324 and pu.convf1.n == 128 and pu.convf1.weight.shape == (128, 128)
            and pu.convc1.precision in (_lib.PREC_F16X3, _lib.PREC_F16, _lib.PREC_BF16)
            and pu.convf1.precision == pu.convc1.precision
            and os.environ.get("RAFT_FUSE_CONVC1", "1") != "0")


def frag_weight(pc) -> torch.Tensor:
    """A conv's split weight in raft_corr_lookup_conv's fragment order (raft_hip.h), cached on the
    PackedConv per precision."""
    cached = getattr(pc, "_frag", None)
    if cached is not None and cached[0] == pc.precision:
        return cached[1]
    split = pc.launch_weight()
    n_pad, k_pad = split.shape
    out = torch.empty(int(_lib.load().raft_lookup_conv_weight_floats(pc.n, k_pad)), device=split.device,
                      dtype=torch.float32)
    _lib.call("raft_lookup_conv_pack_weight", split.data_ptr(), n_pad, k_pad, pc.n, out.data_ptr(), K.stream_handle())
    pc._frag = (pc.precision, out)
    return out


def plan_update(L, pu: PackedUpdate, ub: UpdateBuffers, B, h, w, with_mask: bool, convf1_done: bool = False,
                convc1_done: bool = False, last: bool = True):
    """One BasicUpdateBlock / SmallUpdateBlock step (core/update.py:297-325 / :250-263)
    followed by coords1 += delta_flow (core/raft.py:232).  Assumes ub.corr and the
    flow slot of HX were filled by the lookup and plan_gru_context ran for this pair
    (convf1_done: the lookup launch also wrote convf1's output, ub.flo1; convc1_done: and
    convc1's, ub.cor1)."""
    flow = Rows(ub.hx, ub.flow_off(pu), 2)
    cf = Rows(ub.cf)
    # RAFT-full: one stream; convc2 (corr branch) and convf2 (flow branch) are two 3x3 halo
    # convs with no data between them, run as ONE launch (raft_conv2d_pair: 168 + 56
    # work-groups fill the CUs that convc2 alone leaves idle).  RAFT_CONV_PAIR=0: the flow
    # branch on the side stream instead (a graph fork / join, as in round 1).
    # RAFT-small (different conv shapes per branch): side stream unless RAFT_FLOW_SIDE=0.
    pair = not pu.small and os.environ.get("RAFT_CONV_PAIR", "1") != "0"
    side = not pair and os.environ.get("RAFT_FLOW_SIDE", "1") != "0"

    def conv(pc, src, out, **kw):
        kw.setdefault("range_flag", _GUARD["flag"])
        L.append(conv_launch(conv_params(pc, src, B, h, w, out, **kw)))
    if side:
        L.append(K.FORK)
    if pu.small:
        _conv(L, pu.convf1, flow, B, h, w, Rows(ub.flo1), epilogue=_lib.EPI_RELU, side=side)
        _conv(L, pu.convf2, Rows(ub.flo1), B, h, w, cf.sub(96, 32), epilogue=_lib.EPI_RELU, side=side)
        _conv(L, pu.convc1, Rows(ub.corr), B, h, w, cf.sub(0, 96), epilogue=_lib.EPI_RELU)
    elif pair:
        if not convf1_done:
            _conv(L, pu.convf1, flow, B, h, w, Rows(ub.flo1), epilogue=_lib.EPI_RELU)
        if not convc1_done:
            _conv(L, pu.convc1, Rows(ub.corr), B, h, w, Rows(ub.cor1), epilogue=_lib.EPI_RELU)
        c2 = conv_params(pu.convc2, Rows(ub.cor1), B, h, w, cf.sub(0, 192), epilogue=_lib.EPI_RELU,
                         range_flag=_GUARD["flag"])
        f2 = conv_params(pu.convf2, Rows(ub.flo1), B, h, w, cf.sub(192, 64), epilogue=_lib.EPI_RELU,
                         range_flag=_GUARD["flag"])
        L.append(K.conv_pair_launch(c2, f2))
    else:
        _conv(L, pu.convf1, flow, B, h, w, Rows(ub.flo1), epilogue=_lib.EPI_RELU, side=side)
        _conv(L, pu.convf2, Rows(ub.flo1), B, h, w, cf.sub(192, 64), epilogue=_lib.EPI_RELU, side=side)
        _conv(L, pu.convc1, Rows(ub.corr), B, h, w, Rows(ub.cor1), epilogue=_lib.EPI_RELU)
        _conv(L, pu.convc2, Rows(ub.cor1), B, h, w, cf.sub(0, 192), epilogue=_lib.EPI_RELU)
    if side:
        L.append(K.JOIN)
    conv(pu.conv, cf, ub.motion(pu), epilogue=_lib.EPI_RELU)
    hd = pu.hdim
    hrows = ub.h(pu)
    for i, ((zr, q, _), ctx) in enumerate(zip(pu.gru, ub.ctx)):
        c = Rows(ctx)
        # (z, r*h and the new h are sigmoid / tanh blends of |h| <= 1: no range guard)
        conv(zr, ub.gru_in(pu), Rows(ub.z), epilogue=_lib.EPI_GRU_ZR, split=hd, aux0=hrows,
             out1=Rows(ub.rh), add0=c.sub(0, 2 * hd), range_flag=None)
        conv(q, Rows(ub.rh), hrows, src1=ub.x_dyn(pu), epilogue=_lib.EPI_GRU_Q, aux0=hrows,
             aux1=Rows(ub.z), add0=c.sub(2 * hd, hd), range_flag=None)
    coords = Rows(ub.coords)
    if pu.small:
        _conv(L, pu.fh1, hrows, B, h, w, Rows(ub.fh), epilogue=_lib.EPI_RELU, range_flag=None)  # feeds fp32 fh2
        _conv(L, pu.fh2, Rows(ub.fh), B, h, w, coords, epilogue=_lib.EPI_ADD_TO_OUT)
    else:
        fh = Rows(ub.fh)
        if with_mask:
            conv(pu.fh1_mask, hrows, fh, epilogue=_lib.EPI_RELU)
        else:  # (feeds only the fp32 flow-head conv2: no range guard)
            conv(pu.fh1, hrows, fh.sub(0, 256), epilogue=_lib.EPI_RELU, range_flag=None)
        _conv(L, pu.fh2, fh.sub(0, 256), B, h, w, coords, epilogue=_lib.EPI_ADD_TO_OUT)
        if with_mask:
            # the mask feeds only the fp32 softmax of the upsampling: no range guard
            _conv(L, pu.mask2, fh.sub(256, 256), B, h, w, Rows(ub.mask), epilogue=_lib.EPI_LINEAR, alpha=0.25,
                  range_flag=None)


def _order_context_branch(L, f0, c0):
    """Enqueue order of the two encoder branches: L[f0:c0] is the feature network + correlation build
    (main stream), L[c0:] the context network (side stream).  The streams fix the dependencies; the order
    only decides which launches the hipGraph executor dispatches first.  RAFT_CTX_ORDER: `late` (the
    context network enqueued after the whole feature branch), `early` (before it), `mix` (interleaved in
    proportion, so the context network's small 1/4- and 1/8-res layers run beside the feature network
    instead of after the correlation build)."""
    order = os.environ.get("RAFT_CTX_ORDER", "late")
    if order == "late":
        return
    feat, ctx = L[f0:c0], L[c0:]
    if order == "early":
        merged = ctx + feat
    elif order == "mix":
        merged, j = [], 0
        for i, l in enumerate(feat):
            merged.append(l)
            want = (i + 1) * len(ctx) // len(feat)
            merged.extend(ctx[j:want])
            j = max(j, want)
        merged.extend(ctx[j:])
    else:
        raise ValueError(f"RAFT_CTX_ORDER={order!r}: expected late, early or mix")
    L[f0:] = merged


# ----------------------------------------------------------------------------
# The whole forward
# ----------------------------------------------------------------------------


class RaftPlan:
    """RAFT.forward (core/raft.py:145-251, eval mode) as a fixed launch list."""

    def __init__(self, pk: PackedRaft, B, H, W, iters, test_mode=True, alternate=False, flow_init=False,
                 device=None, range_guard=True):
        if H % 8 or W % 8:
            raise ValueError(f"image size {H}x{W} must be a multiple of 8 (pad with InputPadder)")
        self.pk, self.B, self.H, self.W, self.iters = pk, B, H, W, iters
        self.test_mode, self.alternate = test_mode, alternate
        self.device = device
        # f16x3 range guard flag (raft_hip.h): raised by the convs and lookups whose outputs
        # feed split-precision convs; RAFT.forward checks it after the forward
        self.guarded = range_guard and pk.precision == _lib.PREC_F16X3
        self.range_flag = torch.zeros(1, dtype=torch.int32, device=device)
        _GUARD["flag"] = self.range_flag if self.guarded else None
        try:
            self._build(pk, B, H, W, iters, test_mode, alternate, flow_init, device)
        finally:
            _GUARD["flag"] = None
        self.graph = None
        self.side_stream = None
        self.runs = 0

    def _build(self, pk, B, H, W, iters, test_mode, alternate, flow_init, device):
        A = self.arena = Arena(device)
        L = self.launches = []
        h, w = H // 8, W // 8
        self.h, self.w = h, w
        P = B * h * w
        self.img1 = torch.empty(B, 3, H, W, device=device)
        self.img2 = torch.empty(B, 3, H, W, device=device)
        self.flow_init = torch.zeros(B, 2, h, w, device=device) if flow_init else None
        prep = Rows(A.rows(2 * B * H * W, 3))
        L.append(Launch("raft_prep_images", self.img1.data_ptr(), self.img2.data_ptr(), prep.ptr, B, H, W))
        # the context network (below) runs on the side stream beside the feature network and
        # the correlation build: independent work, and their 1/8-res stages alone leave CUs idle
        # (RAFT_CTX_SIDE=0: all on the main stream)
        ctx_side = os.environ.get("RAFT_CTX_SIDE", "1") != "0"
        if ctx_side:
            L.append(K.FORK)
        # feature network on [img1; img2] (core/raft.py:177-182)
        x, fh_, fw_ = plan_encoder_trunk(L, A, pk.fnet, prep, 2 * B, H, W)
        assert (fh_, fw_) == (h, w), ((fh_, fw_), (h, w))
        fm = Rows(A.rows(2 * B * h * w, pk.fdim))
        _conv(L, pk.fnet.head, x, 2 * B, h, w, fm)
        self.fmap = fm.t
        r, lv = pk.radius, pk.levels
        corr_ld = lv * (2 * r + 1) ** 2
        pu = pk.update
        ub = self.ub = UpdateBuffers(A, pu, P, corr_ld)
        fmap1 = fm.t[: B * h * w]
        fmap2 = fm.t[B * h * w:]
        C = pk.fdim
        div = K.sqrt_c(C)
        if not alternate:
            self.pyramid = A.flat(K.pyramid_floats(B, h, w, lv))
            # the correlation GEMM follows the conv arithmetic: exact f32 MFMA in "fp32"
            # mode, the fp32-accurate f16 split otherwise (raft_hip.h)
            cprec = _lib.PREC_FP32 if pk.precision == _lib.PREC_FP32 else _lib.PREC_F16X3
            # (f16x3: fmaps split once into the workspace, the volume on 256 x 256 tiles: raft_hip.h)
            # (the workspace only where the library takes that path: raft_corr_build_ws)
            # (the library's own rule: raft_corr_build_ws_bytes_prec is 0 where that kernel does not apply)
            wsb = int(_lib.load().raft_corr_build_ws_bytes_prec(B, h, w, C, cprec))
            fits4 = wsb > 0
            self.corr_ws = A.flat((wsb + 3) // 4) if fits4 else None
            L.append(Launch("raft_corr_build_ws", fmap1.data_ptr(), fmap2.data_ptr(), C, B, h, w, C, lv, div,
                            cprec, self.pyramid.data_ptr(), self.corr_ws.data_ptr() if fits4 else None, wsb))
        else:
            # AlternateCorrBlock pools num_levels times (core/corr.py:157-161); the
            # last level is never used, but its existence is the reference's size check.
            hh, ww = h, w
            for _ in range(lv):
                hh, ww = hh // 2, ww // 2
                if hh < 1 or ww < 1:
                    raise RuntimeError(f"AlternateCorrBlock: feature map {h}x{w} too small for {lv} pooling levels")
            self.f2levels = [(fmap2, h, w)]
            hh, ww = h, w
            for _ in range(lv - 1):
                nh, nw = hh // 2, ww // 2
                dst = A.rows(B * nh * nw, C)
                L.append(Launch("raft_avgpool2_nhwc", self.f2levels[-1][0].data_ptr(), dst.data_ptr(), B, hh, ww, C))
                self.f2levels.append((dst, nh, nw))
                hh, ww = nh, nw
        # context network (core/raft.py:193-200): tanh/relu split fused into its last conv
        n_ctx = len(L)
        xc, _, _ = plan_encoder_trunk(L, A, pk.cnet, Rows(prep.t[: B * H * W]), B, H, W)
        _conv(L, pk.cnet.head, xc, B, h, w, ub.h(pu), epilogue=_lib.EPI_TANH_RELU, split=pk.hdim, out1=ub.inp(pu))
        plan_gru_context(L, pu, ub, B, h, w)
        if ctx_side:
            for l in L[n_ctx:]:
                if isinstance(l, Launch):  # FORK / JOIN markers are plain strings
                    l.side = True
            _order_context_branch(L, L.index(K.FORK) + 1, n_ctx)
            L.append(K.JOIN)
        L.append(Launch("raft_init_coords", ub.coords.data_ptr(),
                        self.flow_init.data_ptr() if self.flow_init is not None else None, B, h, w))
        self.loop_start = len(L)
        self.flow_up = [torch.empty(B, 2, H, W, device=device) for _ in range(1 if test_mode else iters)]
        flow_slot = ub.flow_off(pu)
        gflag = self.range_flag.data_ptr() if self.guarded else None
        # all-pairs RAFT-full: the motion encoder's convf1 runs inside the lookup launch
        # (its own launch would be a K = 98 GEMM behind a launch's fixed cost)
        # (alternate corr: convf1 as its own VALU launch, raft_convf1_flow: the alternate lookup's
        # launch has no room for it)
        fuse_f1 = convf1_fused(pu) and os.environ.get("RAFT_CONV_PAIR", "1") != "0"
        if fuse_f1:
            f1w = convf1_vec_weight(pu)
            f1b = pu.convf1.bias.data_ptr() if pu.convf1.bias is not None else None
        fuse_c1 = fuse_f1 and not alternate and convc1_fused(pk)
        if fuse_c1:
            c1w, f1w_frag = frag_weight(pu.convc1), frag_weight(pu.convf1)
            c1b = pu.convc1.bias.data_ptr() if pu.convc1.bias is not None else None
        for it in range(iters):
            last = it == iters - 1
            if fuse_c1:
                L.append(Launch("raft_corr_lookup_conv", self.pyramid.data_ptr(), B, h, w, lv, r, ub.coords.data_ptr(),
                                ub.hx.data_ptr() + 4 * flow_slot, pu.ld, gflag, pu.convc1.precision, c1w.data_ptr(),
                                c1b, pu.convc1.n, ub.cor1.data_ptr(), ub.cor1.shape[1], gflag, f1w_frag.data_ptr(), f1b,
                                pu.convf1.n, pu.convf1.kh, ub.flo1.data_ptr(), ub.flo1.shape[1], gflag,
                                keep=(f1w_frag, c1w)))
            elif fuse_f1 and not alternate:
                L.append(Launch("raft_corr_lookup_convf1", self.pyramid.data_ptr(), B, h, w, lv, r,
                                ub.coords.data_ptr(), 0, ub.corr.data_ptr(), corr_ld, 0,
                                ub.hx.data_ptr() + 4 * flow_slot, pu.ld, gflag, f1w.data_ptr(), f1b, pu.convf1.n,
                                pu.convf1.kh, pu.convf1.precision, ub.flo1.data_ptr(), ub.flo1.shape[1], gflag,
                                keep=f1w))
            elif not alternate:
                L.append(Launch("raft_corr_lookup", self.pyramid.data_ptr(), B, h, w, lv, r, ub.coords.data_ptr(), 0,
                                ub.corr.data_ptr(), corr_ld, 0, ub.hx.data_ptr() + 4 * flow_slot, pu.ld, gflag))
            else:
                # every level in one call (one launch for RAFT's r = 4, C = 256: raft_hip.h)
                arrs = K.alt_levels_args(self.f2levels)
                # exact fp32 products in "fp32" mode (the range guard's re-run), the f16x3 box GEMM otherwise
                aprec = _lib.PREC_FP32 if pk.precision == _lib.PREC_FP32 else _lib.PREC_F16X3
                L.append(Launch("raft_alt_corr_lookup_levels_prec", fmap1.data_ptr(), *arrs, len(self.f2levels),
                                ub.coords.data_ptr(), 0, ub.corr.data_ptr(), corr_ld, B, h, w, C, r, div,
                                ub.hx.data_ptr() + 4 * flow_slot, pu.ld, gflag, aprec, keep=arrs))
                if fuse_f1:
                    L.append(Launch("raft_convf1_flow", ub.coords.data_ptr(), 0, B, h, w, f1w.data_ptr(), f1b,
                                    pu.convf1.n, pu.convf1.kh, pu.convf1.precision, ub.flo1.data_ptr(),
                                    ub.flo1.shape[1], gflag, keep=f1w))
            want_up = last or not test_mode
            plan_update(L, pu, ub, B, h, w, with_mask=want_up and not pu.small, convf1_done=fuse_f1,
                        convc1_done=fuse_c1, last=last)
            if want_up:
                dst = self.flow_up[-1 if test_mode else it]
                if pu.small:
                    L.append(Launch("raft_upflow8", ub.coords.data_ptr(), dst.data_ptr(), B, h, w))
                else:
                    L.append(Launch("raft_convex_upsample", ub.coords.data_ptr(), ub.mask.data_ptr(), 576,
                                    dst.data_ptr(), B, h, w))
        self.loop_end = len(L)
        self.flow_low = torch.empty(B, 2, h, w, device=device)
        L.append(Launch("raft_flow_from_coords", ub.coords.data_ptr(), self.flow_low.data_ptr(), B, h, w))

    # -- execution --------------------------------------------------------
    def run(self):
        if self.side_stream is None:
            self.side_stream = torch.cuda.Stream(device=self.device)
        K.run(self.launches, self.side_stream)
        self.runs += 1

    def release(self):
        """Drop the graph and every device buffer of the plan (it cannot run afterwards)."""
        if self.graph is not None:
            torch.cuda.synchronize(self.device)
            self.graph.reset()
            self.graph = None
        self.launches = []
        self.arena.bufs.clear()
        for name in ("pyramid", "fmap", "f2levels", "ub", "img1", "img2", "flow_init", "flow_low", "flow_up",
                     "range_flag"):
            if hasattr(self, name):
                setattr(self, name, None)

    def capture(self):
        """Record the whole launch list into a hipGraph (static buffers, no allocation)."""
        torch.cuda.synchronize()
        self.run()  # warm-up outside capture (first-launch code object loads)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.run()
        torch.cuda.synchronize()
        self.graph = g
        return g

    def replay(self):
        if self.graph is None:
            self.capture()
        self.graph.replay()

    def set_inputs(self, image1, image2, flow_init=None):
        self.img1.copy_(image1)
        self.img2.copy_(image2)
        if self.flow_init is not None:
            self.flow_init.copy_(flow_init)

    def outputs(self, clone=True):
        f = (lambda t: t.clone()) if clone else (lambda t: t)
        if self.test_mode:
            return f(self.flow_low), f(self.flow_up[0])
        return [f(t) for t in self.flow_up]

    def kernel_names(self):
        return [l.name for l in self.launches if isinstance(l, Launch)]
