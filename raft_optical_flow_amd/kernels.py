"""Torch-facing wrappers over the C-ABI (libraft_hip.so).

PyTorch is plumbing here: device memory, the current HIP stream and graph
capture.  Every function launches hand-written HIP kernels on
`torch.cuda.current_stream()`; nothing falls back to a CPU or torch op path.
"""
from __future__ import annotations

import ctypes
import math
from collections import OrderedDict
from dataclasses import dataclass

import torch

from . import _lib
from ._lib import ConvParams

BK = 32   # K-step of the conv GEMM (raft_conv2d)
BN = 64   # N tile of the conv GEMM


def stream_handle() -> int:
    return torch.cuda.current_stream().cuda_stream


def require_device(*tensors):
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError("raft_optical_flow_amd runs on a ROCm GPU only: got a tensor on "
                               f"{t.device} (no CPU fallback)")
        if t.dtype != torch.float32:
            raise TypeError(f"raft_optical_flow_amd kernels take float32 tensors, got {t.dtype}")


def ptr(t: torch.Tensor | None, offset_floats: int = 0) -> int | None:
    if t is None:
        return None
    return t.data_ptr() + 4 * offset_floats


class Rows:
    """NHWC rows view: (tensor [npix, ld] contiguous, channel offset, channels)."""

    __slots__ = ("t", "off", "c")

    def __init__(self, t: torch.Tensor, off: int = 0, c: int | None = None):
        assert t.dim() == 2 and t.is_contiguous(), t.shape
        self.t = t
        self.off = off
        self.c = t.shape[1] - off if c is None else c

    @property
    def ld(self) -> int:
        return self.t.shape[1]

    @property
    def ptr(self) -> int:
        return self.t.data_ptr() + 4 * self.off

    def sub(self, off: int, c: int) -> "Rows":
        return Rows(self.t, self.off + off, c)


# ----------------------------------------------------------------------------
# Convolution (implicit GEMM on MFMA)
# ----------------------------------------------------------------------------


@dataclass
class PackedConv:
    weight: torch.Tensor      # packed [n_pad, k_pad]
    bias: torch.Tensor | None
    n: int
    cin: int                  # declared input channels (sum of segments, incl. zero pad channels)
    kh: int
    kw: int
    stride: tuple
    pad: tuple
    mode: int
    cin_real: int = 0         # input channels of the original weight (FLOP accounting)
    precision: int = _lib.PREC_FP32
    split: torch.Tensor | None = None   # hi/lo f16 (F16X3 / F16) or bf16 (BF16) form of `weight`, made on first use
    split_prec: int = -1
    split_s: torch.Tensor | None = None  # column-scaled f16x3 split (raft_conv2d_split_weight_scaled), on first use

    def launch_precision(self) -> int:
        # N <= 4 convs run on the VALU kernel, which reads the fp32 weight
        return self.precision if self.n > 4 else _lib.PREC_FP32

    def launch_weight(self) -> torch.Tensor:
        if self.launch_precision() == _lib.PREC_FP32:
            return self.weight
        # F16X3 and F16 share one split form; BF16 has its own
        fmt = _lib.PREC_BF16 if self.precision == _lib.PREC_BF16 else _lib.PREC_F16X3
        if self.split is None or self.split_prec != fmt:
            w = self.weight
            self.split = torch.empty_like(w)
            _lib.call("raft_conv2d_split_weight_prec", w.data_ptr(), self.split.data_ptr(), w.shape[0], w.shape[1],
                      fmt, stream_handle())
            self.split_prec = fmt
        return self.split

    def launch_weight_s(self) -> torch.Tensor | None:
        """The column-scaled f16x3 split (raft_conv2d_params.weight_s) for the convs the halo kernel may
        run on its multi-round tiles (stride-1 3x3 / 1x5 / 5x1, VEC mode, f16x3); None otherwise."""
        if not (self.precision == _lib.PREC_F16X3 and self.n > 4 and (self.kh, self.kw) in ((3, 3), (1, 5), (5, 1))
                and self.stride == (1, 1) and self.mode == _lib.RAFT_CONV_VEC):
            return None
        if self.split_s is None:
            w = self.weight
            nbytes = int(_lib.load().raft_conv2d_split_scaled_bytes(w.shape[0], w.shape[1]))
            self.split_s = torch.empty(nbytes // 4, device=w.device, dtype=torch.float32)
            _lib.call("raft_conv2d_split_weight_scaled", w.data_ptr(), self.split_s.data_ptr(), w.shape[0], w.shape[1],
                      stream_handle())
        return self.split_s


def set_precision(obj, precision: int, _seen=None):
    """Set the conv arithmetic of every PackedConv reachable from obj (attributes, lists, dicts)."""
    _seen = set() if _seen is None else _seen
    if id(obj) in _seen:
        return
    _seen.add(id(obj))
    if isinstance(obj, PackedConv):
        if obj.precision != precision:
            obj.precision = precision
        return
    if isinstance(obj, (list, tuple)):
        items = obj
    elif isinstance(obj, dict):
        items = obj.values()
    elif hasattr(obj, "__dict__") and not isinstance(obj, torch.Tensor):
        items = vars(obj).values()
    else:
        return
    for v in items:
        set_precision(v, precision, _seen)


def pack_conv(weight: torch.Tensor, bias: torch.Tensor | None, stride=1, padding=0,
              seg_real=None, seg_decl=None, mode=None, device=None) -> PackedConv:
    """Pack an OIHW conv weight into the raft_conv2d layout (include/raft_hip.h).

    seg_real / seg_decl: channel counts of the input segments as the weight
    sees them and as the NHWC buffers declare them (extra declared channels are
    zero columns, e.g. a buffer padded to a multiple of 4)."""
    w = weight.detach().to(device=device, dtype=torch.float32)
    o, i, kh, kw = w.shape
    if seg_real is None:
        seg_real = [i]
    if seg_decl is None:
        seg_decl = list(seg_real)
    assert sum(seg_real) == i, (seg_real, i)
    if sum(seg_decl) != i:
        parts, c0 = [], 0
        for r, d in zip(seg_real, seg_decl):
            parts.append(w[:, c0:c0 + r])
            if d > r:
                parts.append(w.new_zeros(o, d - r, kh, kw))
            c0 += r
        w = torch.cat(parts, 1)
    cin = w.shape[1]
    if mode is None:
        mode = _lib.RAFT_CONV_VEC if (cin % 4 == 0 and all(d % 4 == 0 for d in seg_decl)
                                      and (len(seg_decl) == 1 or seg_decl[0] % BK == 0)) else _lib.RAFT_CONV_GATHER
    n_pad = -(-o // BN) * BN
    wt = w.permute(0, 2, 3, 1).contiguous()  # [o, kh, kw, cin]
    if mode == _lib.RAFT_CONV_VEC:
        c_pad = -(-cin // BK) * BK
        wt = torch.nn.functional.pad(wt, (0, c_pad - cin))
        wt = wt.reshape(o, kh * kw * c_pad)
    else:
        k = kh * kw * cin
        k_pad = -(-k // BK) * BK
        wt = torch.nn.functional.pad(wt.reshape(o, k), (0, k_pad - k))
    wt = torch.nn.functional.pad(wt, (0, 0, 0, n_pad - o)).contiguous()
    b = None if bias is None else bias.detach().to(device=device, dtype=torch.float32).contiguous()
    st = (stride, stride) if isinstance(stride, int) else tuple(stride)
    pd = (padding, padding) if isinstance(padding, int) else tuple(padding)
    return PackedConv(wt, b, o, cin, kh, kw, st, pd, mode, i)


def fold_bn(weight, bias, bn: torch.nn.BatchNorm2d):
    """Eval-mode BatchNorm folded into the preceding conv (w*s, (b-mean)*s+beta)."""
    s = bn.weight.detach() / torch.sqrt(bn.running_var.detach() + bn.eps)
    w = weight.detach() * s.reshape(-1, 1, 1, 1)
    b0 = bias.detach() if bias is not None else torch.zeros_like(s)
    b = (b0 - bn.running_mean.detach()) * s + bn.bias.detach()
    return w, b


def conv_params(pc: PackedConv, src0: Rows, batch: int, in_h: int, in_w: int, out: Rows,
                epilogue=_lib.EPI_LINEAR, src1: Rows | None = None, alpha=1.0, split=0,
                aux0: Rows | None = None, aux1: Rows | None = None, out1: Rows | None = None,
                add0: Rows | None = None, range_flag: torch.Tensor | None = None) -> ConvParams:
    """Build (and validate shapes of) a raft_conv2d_params for one launch."""
    sh, sw = pc.stride
    ph, pw = pc.pad
    out_h = (in_h + 2 * ph - pc.kh) // sh + 1
    out_w = (in_w + 2 * pw - pc.kw) // sw + 1
    c1 = src1.c if src1 is not None else 0
    if src0.c + c1 != pc.cin:
        raise ValueError(f"conv input channels {src0.c}+{c1} != packed {pc.cin}")
    npix_in = batch * in_h * in_w
    npix_out = batch * out_h * out_w
    for r, n in ((src0, npix_in), (src1, npix_in), (out, npix_out), (aux0, npix_out), (aux1, npix_out),
                 (out1, npix_out), (add0, npix_out)):
        if r is not None and r.t.shape[0] < n:
            raise ValueError(f"rows buffer has {r.t.shape[0]} pixels, need {n}")
    p = ConvParams()
    p.in0, p.in0_ld, p.in0_c = src0.ptr, src0.ld, src0.c
    if src1 is not None:
        p.in1, p.in1_ld, p.in1_c = src1.ptr, src1.ld, src1.c
    p.batch, p.in_h, p.in_w, p.out_h, p.out_w = batch, in_h, in_w, out_h, out_w
    p.kh, p.kw, p.stride_h, p.stride_w, p.pad_h, p.pad_w = pc.kh, pc.kw, sh, sw, ph, pw
    p.mode = pc.mode
    p.weight = pc.launch_weight().data_ptr()
    ws = pc.launch_weight_s()
    p.weight_s = ws.data_ptr() if ws is not None else None
    p.precision = pc.launch_precision()
    p.bias = pc.bias.data_ptr() if pc.bias is not None else None
    p.n = pc.n
    p.out, p.out_ld = out.ptr, out.ld
    p.epilogue, p.alpha, p.split = epilogue, float(alpha), split
    if aux0 is not None:
        p.aux0, p.aux0_ld = aux0.ptr, aux0.ld
    if aux1 is not None:
        p.aux1, p.aux1_ld = aux1.ptr, aux1.ld
    if out1 is not None:
        p.out1, p.out1_ld = out1.ptr, out1.ld
    if add0 is not None:
        p.add0, p.add0_ld = add0.ptr, add0.ld
    if range_flag is not None and p.precision == _lib.PREC_F16X3:
        p.range_flag = range_flag.data_ptr()
    return p


def conv_out_hw(pc: PackedConv, in_h: int, in_w: int):
    return ((in_h + 2 * pc.pad[0] - pc.kh) // pc.stride[0] + 1, (in_w + 2 * pc.pad[1] - pc.kw) // pc.stride[1] + 1)


class Launch:
    """A pre-built kernel launch: fn(*args, stream)."""

    __slots__ = ("fn", "args", "name", "keep", "side")

    def __init__(self, name: str, *args, keep=None, side=False):
        lib = _lib.load()
        self.name = name
        self.fn = getattr(lib, name)
        self.args = args
        self.keep = keep  # objects whose lifetime the launch depends on (ConvParams structs)
        self.side = side  # run on the plan's side stream (between a FORK and a JOIN)

    def __call__(self, stream: int):
        rc = self.fn(*self.args, stream)
        if rc != 0:
            _lib.check(rc, self.name)


def conv_launch(params: ConvParams, side=False) -> Launch:
    return Launch("raft_conv2d", ctypes.byref(params), keep=params, side=side)


def conv_pair_launch(p0: ConvParams, p1: ConvParams) -> Launch:
    """Two independent convs as one launch where the halo kernel can take both (raft_conv2d_pair)."""
    return Launch("raft_conv2d_pair", ctypes.byref(p0), ctypes.byref(p1), keep=(p0, p1))


def alt_levels_args(f2_levels):
    """ctypes arrays (fmap2 pointers, heights, widths) of raft_alt_corr_lookup_levels for
    [(fmap2 rows tensor, h, w), ...]; keep them alive with the launch."""
    n = len(f2_levels)
    ptrs = (ctypes.c_void_p * n)(*[t.data_ptr() for t, _, _ in f2_levels])
    hs = (ctypes.c_int * n)(*[hh for _, hh, _ in f2_levels])
    ws = (ctypes.c_int * n)(*[ww for _, _, ww in f2_levels])
    return ptrs, hs, ws


FORK = "fork"   # side stream waits for the main stream
JOIN = "join"   # main stream waits for the side stream


def run(launches, side_stream: torch.cuda.Stream | None = None):
    """Replay a launch list on the current stream; FORK/JOIN markers move the
    `side` launches onto `side_stream` (captured as parallel graph branches)."""
    main = torch.cuda.current_stream()
    s = main.cuda_stream
    ss = side_stream.cuda_stream if side_stream is not None else s
    for l in launches:
        if l is FORK:
            if side_stream is not None:
                side_stream.wait_stream(main)
        elif l is JOIN:
            if side_stream is not None:
                main.wait_stream(side_stream)
        else:
            l(ss if l.side else s)


# ----------------------------------------------------------------------------
# One-shot helpers (used by the module-level API)
# ----------------------------------------------------------------------------


def module_precision(mod) -> str:
    """Conv arithmetic of a block-level call: `mod.conv_precision` if set, else exact fp32."""
    prec = getattr(mod, "conv_precision", None) or "fp32"
    if prec not in _lib.PRECISIONS:
        raise ValueError(f"conv_precision must be one of {sorted(_lib.PRECISIONS)}, got {prec!r}")
    return prec


def cached_pack(mod, device, build):
    """The packed weights of `mod` for a block-level forward, rebuilt only when a parameter or
    buffer changes (data_ptr / version), the device or the conv precision changes; kept on the
    module outside its state_dict."""
    prec = module_precision(mod)
    key = (tuple((p.data_ptr(), p._version) for p in mod.parameters()) +
           tuple((b.data_ptr(), b._version) for b in mod.buffers()), str(device), prec)
    hit = mod.__dict__.get("_hip_pack")
    if hit is None or hit[0] != key:
        with torch.no_grad():
            obj = build()
        set_precision(obj, _lib.PRECISIONS[prec])
        hit = (key, obj)
        mod.__dict__["_hip_pack"] = hit
    return hit[1]


def cached_plan(mod, packed, key, build, max_streams=4):
    """A block-level forward's device buffers and pre-built launch list for one input shape, kept on
    the module (the last shape per stream) and rebuilt when the packed weights object (cached_pack's,
    compared by identity) or the key (shape, device) changes: repeated calls allocate nothing and
    only copy their inputs in.  The cache is per current stream: calls on one stream are ordered, so
    they may share buffers; a call on another stream (or inside another stream's graph capture) gets
    buffers of its own, so calls from two streams never race on one set of buffers."""
    sid = torch.cuda.current_stream().cuda_stream if torch.cuda.is_available() else 0
    plans = mod.__dict__.setdefault("_hip_plan", OrderedDict())
    hit = plans.get(sid)
    if hit is None or hit[0] is not packed or hit[1] != key:
        hit = (packed, key, build())
        plans[sid] = hit
        while len(plans) > max_streams:
            plans.popitem(last=False)
    plans.move_to_end(sid)
    return hit[2]


def conv2d_rows(pc: PackedConv, src0: Rows, batch, in_h, in_w, out: Rows, **kw):
    conv_launch(conv_params(pc, src0, batch, in_h, in_w, out, **kw))(stream_handle())


def nchw_to_rows(x: torch.Tensor, ld: int | None = None) -> torch.Tensor:
    require_device(x)
    x = x.contiguous()
    b, c, h, w = x.shape
    ld = c if ld is None else ld
    out = (torch.zeros if ld != c else torch.empty)(b * h * w, ld, device=x.device, dtype=torch.float32)
    _lib.call("raft_nchw_to_nhwc", x.data_ptr(), out.data_ptr(), ld, b, c, h, w, stream_handle())
    return out


def rows_to_nchw(r: Rows, b, h, w) -> torch.Tensor:
    out = torch.empty(b, r.c, h, w, device=r.t.device, dtype=torch.float32)
    _lib.call("raft_nhwc_to_nchw", r.ptr, r.ld, out.data_ptr(), b, r.c, h, w, stream_handle())
    return out


def pyramid_dims(h, w, levels):
    dims = [(h, w)]
    for _ in range(levels - 1):
        h, w = h // 2, w // 2
        dims.append((h, w))
    return dims


def pyramid_floats(b, h, w, levels) -> int:
    return int(_lib.load().raft_corr_pyramid_floats(b, h, w, levels))


def sqrt_c(c: int) -> float:
    """torch.sqrt(torch.tensor(dim).float()) in fp32 (core/corr.py:127, :198)."""
    return float(torch.sqrt(torch.tensor(float(c), dtype=torch.float32)).item())


def instnorm_workspace(b, hw, c, device):
    n = int(_lib.load().raft_instnorm_workspace_floats(b, hw, c))
    return torch.empty(max(n, 1), device=device, dtype=torch.float32)


__all__ = [n for n in dir() if not n.startswith("_")] + ["math"]
