"""RAFT — drop-in for core/raft.py (inference on MI355X).

`RAFT(args)` builds the same module tree as the reference (`core/raft.py:37-78`:
fnet / cnet / update_block with identical parameter names, so reference
checkpoints — including DataParallel `module.` ones via the caller's wrapper —
load unchanged) and `forward(image1, image2, iters=12, flow_init=None,
upsample=True, test_mode=False)` keeps the reference's contract
(`core/raft.py:145-251`): NCHW float images in [0, 255] with H, W multiples of
8 on the model's device; returns `(flow_low, flow_up)` in test_mode, else the
list of `iters` upsampled flows.

Execution is an engine.RaftPlan: every kernel is hand-written HIP (encoders,
correlation build + pyramid, window lookup, update block, upsampling), the
launch list is fixed per input shape.  The first forward of a shape runs the
launch list eagerly; from the second one on the whole forward (including the
32-iteration loop) is captured once and replays as one hipGraph, so unchanged
callers (demo.py, evaluate.py) get graph replay without setting anything
(`args.hip_graph = False`, `model.hip_graph = False` or RAFT_HIP_GRAPH=0 keep
eager launches).  Plans live in a small LRU (RAFT_MAX_PLANS, default 2): a
plan pins its correlation pyramid (275 MB at 440x1024) and buffers, so
evaluate.py's many KITTI sizes do not accumulate device memory.

f16x3 range guard: the default fp32-accurate split arithmetic holds only while every
conv input stays below 65504 in magnitude (include/raft_hip.h).  The convs and lookups
whose outputs feed split convs raise a device flag above 2^15.  `model.range_guard`
(env RAFT_RANGE_GUARD) chooses what happens then:
  "fallback" (default)  forward() waits for its flag (one host sync per forward) and, when it
                        is raised, warns and returns the result of a re-run on exact f32 MFMA:
                        what forward() returns is always the exact-range result ("sync" is
                        the same mode);
  "deferred"            opt-in, for callers that queue forwards back to back: the flag is
                        copied to pinned host memory behind the forward and read once that
                        copy has completed (at a later forward() call, at
                        model.check_range_guard(), which waits, or at interpreter exit).  A
                        raised flag warns and re-runs that forward on exact f32 MFMA INTO the
                        tensors it returned; values read from them before that point were
                        the inexact ones (the warning says so);
  "raise"               as "fallback", but raises FloatingPointError;
  "off"                 no device checks at all.
"""
from __future__ import annotations

import atexit
import os
import warnings
import weakref
from collections import OrderedDict, deque

import threading

import torch
import torch.nn as nn

from . import kernels as K
from .engine import PackedRaft, RaftPlan
from .extractor import BasicEncoder, SmallEncoder
from .update import BasicUpdateBlock, SmallUpdateBlock
from .utils.utils import coords_grid

# module attribute kept for API parity with core/raft.py:11-22 (callers monkeypatch it);
# the HIP path never autocasts: its arithmetic is RAFT.conv_precision
autocast = torch.amp.autocast

# default conv arithmetic of an fp32 model (include/raft_hip.h, RAFT_PREC_*):
# "f16x3" = fp32-accurate split-f16 MFMA, "fp32" = f32 MFMA
DEFAULT_PRECISION = "f16x3"

_CACHE_LOCK = threading.Lock()  # creation of per-device cache entries (DataParallel threads)


class RAFT(nn.Module):
    def __init__(self, args):
        super().__init__()
        self.args = args
        if args.small:
            self.hidden_dim = hdim = 96
            self.context_dim = cdim = 64
            args.corr_levels = 4
            args.corr_radius = 3
        else:
            self.hidden_dim = hdim = 128
            self.context_dim = cdim = 128
            args.corr_levels = 4
            args.corr_radius = 4
        if "dropout" not in self.args:
            self.args.dropout = 0
        if "alternate_corr" not in self.args:
            self.args.alternate_corr = False
        if "mixed_precision" not in self.args:
            self.args.mixed_precision = False
        if args.small:
            self.fnet = SmallEncoder(output_dim=128, norm_fn="instance", dropout=args.dropout)
            self.cnet = SmallEncoder(output_dim=hdim + cdim, norm_fn="none", dropout=args.dropout)
            self.update_block = SmallUpdateBlock(self.args, hidden_dim=hdim)
        else:
            self.fnet = BasicEncoder(output_dim=256, norm_fn="instance", dropout=args.dropout)
            self.cnet = BasicEncoder(output_dim=hdim + cdim, norm_fn="batch", dropout=args.dropout)
            self.update_block = BasicUpdateBlock(self.args, hidden_dim=hdim)
        # execution state (not part of state_dict)
        self.hip_graph = bool(getattr(args, "hip_graph", os.environ.get("RAFT_HIP_GRAPH", "1") != "0"))
        self.max_plans = int(os.environ.get("RAFT_MAX_PLANS", "2"))
        self.range_guard = os.environ.get("RAFT_RANGE_GUARD", "fallback")
        # conv arithmetic: "fp32" | "f16x3" | "f16"; args.mixed_precision (the
        # reference's fp16 autocast, core/raft.py:156) selects "f16"
        self.conv_precision = getattr(args, "conv_precision", None)
        # packed weights and plans per device: {str(device): {"packed": {precision: (weights key,
        # PackedRaft)}, "plans": OrderedDict}}; nn.DataParallel replicas share their source's
        # (_replicate_for_data_parallel), each replica touching only its own device's entry
        self._caches = {}
        self._pending = deque()     # deferred range-guard checks ("deferred"), oldest first

    def _replicate_for_data_parallel(self):
        """nn.DataParallel (the reference's multi-GPU API, train.py:172, evaluate.py:179) re-replicates
        the module on every forward by shallow-copying __dict__.  A replica keeps the per-device caches
        of its SOURCE module (so packing and graph capture happen once per device, not per forward;
        the weights key is the source's, whose values every replica copies) and a range-guard queue of
        its own; replicas on different devices never touch the same cache entry."""
        replica = super()._replicate_for_data_parallel()
        replica.__dict__["_dp_source"] = self.__dict__.get("_dp_source") or self
        replica.__dict__["_pending"] = deque()
        return replica

    def _source(self):
        return self.__dict__.get("_dp_source") or self

    def _dev_cache(self, device):
        caches = self._source().__dict__["_caches"]
        d = str(torch.device(device))
        c = caches.get(d)
        if c is None:
            with _CACHE_LOCK:
                c = caches.setdefault(d, {"packed": {}, "plans": OrderedDict()})
        return c

    @property
    def _plans(self):
        """The plans of the device this module's parameters are on (inspection / tests)."""
        return self._dev_cache(next(self.parameters()).device)["plans"]

    def freeze_bn(self):
        for m in self.modules():
            if isinstance(m, nn.BatchNorm2d):
                m.eval()

    def initialize_flow(self, img):
        n, c, h, w = img.shape
        coords0 = coords_grid(n, h // 8, w // 8, device=img.device)
        coords1 = coords_grid(n, h // 8, w // 8, device=img.device)
        return coords0, coords1

    def upsample_flow(self, flow, mask):
        """Convex upsampling (core/raft.py:112-142) on the HIP kernel; flow [N,2,H,W], mask [N,576,H,W]."""
        from . import _lib
        K.require_device(flow, mask)
        n, _, h, w = flow.shape
        coords = coords_grid(n, h, w, device=flow.device) + flow
        crow = K.nchw_to_rows(coords.contiguous())
        mrow = K.nchw_to_rows(mask.contiguous())
        out = torch.empty(n, 2, 8 * h, 8 * w, device=flow.device)
        _lib.call("raft_convex_upsample", crow.data_ptr(), mrow.data_ptr(), 576, out.data_ptr(), n, h, w,
                  K.stream_handle())
        return out

    # -- weights / plans ---------------------------------------------------
    def _weights_key(self):
        return tuple((p.data_ptr(), p._version) for p in self.parameters()) + tuple(
            (b.data_ptr(), b._version) for b in self.buffers())

    def resolved_precision(self) -> str:
        from . import _lib
        prec = self.conv_precision or ("f16" if self.args.mixed_precision else DEFAULT_PRECISION)
        if prec not in _lib.PRECISIONS:
            raise ValueError(f"conv_precision must be one of {sorted(_lib.PRECISIONS)}, got {prec!r}")
        return prec

    def packed(self, device, prec=None):
        from . import _lib
        prec = prec or self.resolved_precision()
        # (a DataParallel replica's parameters are this forward's copies of its source's: the
        # source's key names the values)
        key = (self._source()._weights_key(), str(device))
        cache = self._dev_cache(device)
        packs = cache["packed"]
        got = packs.get(prec)
        if got is None or got[0] != key:
            if got is not None or any(k != key for k, _ in packs.values()):
                # new weights: every packed form and plan of this device is stale
                packs.clear()
                self._release(cache["plans"])
            with torch.no_grad():
                got = (key, PackedRaft(self, device, _lib.PRECISIONS[prec]))
            packs[prec] = got
        return got[1]

    def _plan_key(self, batch, height, width, iters, test_mode, flow_init, prec):
        # the stream layout knobs are read when a plan is built, so they are part of its key
        knobs = (os.environ.get("RAFT_CTX_SIDE", "1"), os.environ.get("RAFT_FLOW_SIDE", "1"),
                 os.environ.get("RAFT_CONV_PAIR", "1"), os.environ.get("RAFT_FUSE_CONVF1", "1"),
                 os.environ.get("RAFT_FUSE_CONVC1", "1"), os.environ.get("RAFT_EPI_STATS", "1"),
                 os.environ.get("RAFT_IN_NORM", "1"))
        guard = self.range_guard != "off"  # "off": no device-side checks either
        return (batch, height, width, iters, bool(test_mode), bool(self.args.alternate_corr), bool(flow_init), prec,
                knobs, guard)

    def _cached_plan(self, batch, height, width, iters, test_mode, flow_init, device):
        """The cached plan of this call and the weights key its packed weights were made from, WITHOUT
        checking that key against the parameters (forward() checks it while the plan runs); None when
        the call has no plan yet."""
        prec = self.resolved_precision()
        cache = self._dev_cache(device)
        got = cache["packed"].get(prec)
        if got is None:
            return None
        pl = cache["plans"].get(self._plan_key(batch, height, width, iters, test_mode, flow_init, prec))
        if pl is None or pl.pk is not got[1]:
            return None
        return pl, got[0]

    def plan(self, batch, height, width, iters, test_mode=True, flow_init=False, device=None, prec=None):
        device = device or next(self.parameters()).device
        prec = prec or self.resolved_precision()
        pk = self.packed(device, prec)
        key = self._plan_key(batch, height, width, iters, test_mode, flow_init, prec)
        plans = self._dev_cache(device)["plans"]
        pl = plans.get(key)
        if pl is None:
            while len(plans) >= max(1, self.max_plans):
                plans.popitem(last=False)[1].release()
            pl = RaftPlan(pk, batch, height, width, iters, test_mode=test_mode,
                          alternate=bool(self.args.alternate_corr), flow_init=flow_init, device=device,
                          range_guard=key[-1])
            plans[key] = pl
        else:
            plans.move_to_end(key)
        return pl

    @staticmethod
    def _release(plans, keep=None):
        for k in list(plans):
            if plans[k] is not keep:
                plans.pop(k).release()

    def release_plans(self, keep=None):
        """Free the cached plans' device memory and graphs (all but `keep`), on every device."""
        for cache in list(self._source().__dict__["_caches"].values()):
            self._release(cache["plans"], keep)

    # -- deferred range guard ------------------------------------------------
    _MAX_PENDING = 2  # forwards whose flag may be unread: the third waits for the oldest

    def check_range_guard(self, block=True):
        """Resolve the deferred range-guard checks of earlier forwards ("fallback" mode): with
        block=True wait for all of them, else only read those whose flag copy has completed.
        A raised flag warns and re-runs that forward on exact f32 MFMA into its output tensors."""
        while self._pending:
            rec = self._pending[0]
            if not block and len(self._pending) <= self._MAX_PENDING and not rec["event"].query():
                break
            rec["event"].synchronize()
            self._pending.popleft()
            if int(rec["flag"].item()):
                self._guard_fallback(rec)

    def _guard_fallback(self, rec):
        msg = ("f16x3 range guard (deferred): an activation of an earlier forward exceeded 2^15 in "
               "magnitude, outside the exact range of the split-f16 conv arithmetic; values read from its "
               "outputs before this point were inexact")
        ins = [x for x in rec["inputs"] if x is not None]
        if any(x._version != v for x, v in zip(ins, rec["versions"])):
            warnings.warn(msg + "; the inputs of that forward were modified in place since, so its outputs "
                          "cannot be recomputed and stay inexact", RuntimeWarning)
            return
        warnings.warn(msg + "; that forward was re-run with exact f32 MFMA convs into its output tensors",
                      RuntimeWarning)
        i1, i2, fi = rec["inputs"]
        exact = self.forward(i1, i2, rec["iters"], fi, True, rec["test_mode"], _prec="fp32")
        outs, new = rec["outputs"], exact
        if isinstance(outs, tuple):
            for o, n in zip(outs, new):
                o.copy_(n)
        else:
            for o, n in zip(outs, new):
                o.copy_(n)

    def forward(self, image1, image2, iters=12, flow_init=None, upsample=True, test_mode=False, _prec=None):
        if image1.is_cuda and image1.device != torch.device("cuda", torch.cuda.current_device()):
            # launches go to the current device's stream: make the images' device current
            with torch.cuda.device(image1.device):
                return self.forward(image1, image2, iters, flow_init, upsample, test_mode, _prec)
        if self.training:
            raise NotImplementedError("raft_optical_flow_amd.RAFT is an inference path: call model.eval() "
                                      "(training / BatchNorm batch statistics are out of scope)")
        K.require_device(image1, image2, flow_init)
        if image1.shape != image2.shape or image1.dim() != 4 or image1.shape[1] != 3:
            raise ValueError(f"images must both be [N, 3, H, W], got {tuple(image1.shape)} / {tuple(image2.shape)}")
        if self._pending and _prec is None:
            self.check_range_guard(block=False)  # earlier forwards whose flags have landed
        b, _, H, W = image1.shape
        mode = self.range_guard
        if mode == "deferred" and self.__dict__.get("_is_replica", False):
            mode = "fallback"  # a DataParallel replica lives for one forward: nothing can be deferred
        # Steady state (same weights, shape and settings as a cached plan): the plan is enqueued first and
        # the weights key -- a walk over every parameter, ~0.2-0.7 ms of host time -- is checked while it
        # runs, instead of leaving the GPU idle between back-to-back forwards.  Changed weights (in-place
        # edits, load_state_dict, .to()) are caught by that check: the stale run is discarded and the
        # forward re-run on freshly packed weights, so the result is the one the reference would return.
        cached = None
        if _prec is None and self.hip_graph and not self.__dict__.get("_is_replica", False):
            cached = self._cached_plan(b, H, W, iters, test_mode, flow_init is not None, image1.device)
        while True:
            if cached is not None:
                pl, wkey = cached
            else:
                pl = self.plan(b, H, W, iters, test_mode, flow_init is not None, image1.device, prec=_prec)
            pl.set_inputs(image1, image2, flow_init)
            guard = pl.guarded and mode != "off"
            if guard:
                pl.range_flag.zero_()
            if self.hip_graph and (pl.graph is not None or pl.runs > 0):
                pl.replay()
            else:
                pl.run()
            if cached is None or (self._source()._weights_key(), str(image1.device)) == wkey:
                break
            # the weights changed since the plan was packed: let the stale run finish before its plan
            # can be released, then take the checked path
            torch.cuda.current_stream().synchronize()
            cached = None
        outs = pl.outputs(clone=True)
        if not guard:
            return outs
        if mode != "deferred":  # "fallback" (default), "sync", "raise"
            if int(pl.range_flag.item()):
                msg = ("f16x3 range guard: an activation exceeded 2^15 in magnitude, outside the exact range "
                       "of the split-f16 conv arithmetic")
                if mode == "raise":
                    raise FloatingPointError(msg)
                warnings.warn(msg + "; this forward was re-run with exact f32 MFMA convs", RuntimeWarning)
                return self.forward(image1, image2, iters, flow_init, upsample, test_mode, _prec="fp32")
            return outs
        # "deferred": the flag travels to pinned host memory behind the forward; read later
        if not self._pending:
            _register_exit_check(self)
        flag = torch.empty(1, dtype=torch.int32, pin_memory=True)
        flag.copy_(pl.range_flag, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        ins = (image1, image2, flow_init)
        self._pending.append({"event": ev, "flag": flag, "inputs": ins, "outputs": outs, "iters": iters,
                              "test_mode": test_mode,
                              "versions": [x._version for x in ins if x is not None]})
        if len(self._pending) > self._MAX_PENDING:
            self.check_range_guard(block=False)
        return outs


def _register_exit_check(model):
    """Resolve a model's deferred range-guard checks at interpreter exit (a weak reference: the
    hook keeps no model alive)."""
    if getattr(model, "_exit_hook", False):
        return
    ref = weakref.ref(model)

    def _flush():
        m = ref()
        if m is not None and m._pending:
            try:
                m.check_range_guard(block=True)
            except Exception as e:  # noqa: BLE001 (the GPU context may already be gone)
                warnings.warn(f"range guard: deferred checks could not be resolved at exit: {e}", RuntimeWarning)

    atexit.register(_flush)
    model.__dict__["_exit_hook"] = True
