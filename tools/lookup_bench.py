"""Corr-lookup kernel in isolation at the config-2 shape (B x 55 x 128, r=4, 4 levels),
plus a calibration copy of known byte count for the rocprofv3 FETCH_SIZE/WRITE_SIZE
passes.  Usage: python tools/lookup_bench.py [B] [spread_px]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raft_optical_flow_amd import _lib  # noqa: E402
from raft_optical_flow_amd import kernels as K  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
spread = float(sys.argv[2]) if len(sys.argv) > 2 else 0.7
reps = int(os.environ.get("REPS", "50"))
h, w, L, r, C = 55, 128, 4, 4, 256
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
f1 = torch.randn(B * h * w, C, device=dev, generator=g)
f2 = torch.randn(B * h * w, C, device=dev, generator=g)
pyr = torch.empty(K.pyramid_floats(B, h, w, L), device=dev)
s = K.stream_handle()
_lib.call("raft_corr_build", f1.data_ptr(), f2.data_ptr(), C, B, h, w, C, L, 16.0, pyr.data_ptr(), s)
ys, xs = torch.meshgrid(torch.arange(h, device=dev), torch.arange(w, device=dev), indexing="ij")
grid = torch.stack([xs, ys], -1).float().reshape(1, h * w, 2).repeat(B, 1, 1).reshape(-1, 2)
coords = (grid + spread * torch.randn(grid.shape, device=dev, generator=g)).contiguous()
out = torch.empty(B * h * w, L * 81, device=dev)
flow = torch.empty(B * h * w, 2, device=dev)


def lookup():
    _lib.call("raft_corr_lookup", pyr.data_ptr(), B, h, w, L, r, coords.data_ptr(), 0, out.data_ptr(), L * 81, 0,
              flow.data_ptr(), 2, None, s)


calib_src = torch.randn(64 * 1024 * 1024 // 4, device=dev)  # 64 MiB, read once per launch
calib_dst = torch.empty_like(calib_src)
nP = calib_src.numel()


def calib():
    # one-channel NHWC -> NCHW "transpose" = a fully coalesced 4-byte-per-lane copy:
    # every byte read once and written once (the FETCH/WRITE_SIZE calibrator)
    _lib.call("raft_nhwc_to_nchw", calib_src.data_ptr(), 1, calib_dst.data_ptr(), 1, 1, 1, nP, s)


for f in (lookup, calib):
    f()
torch.cuda.synchronize()
# the repetitions captured as one hipGraph: no host launch overhead in the timing
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph):
    s = K.stream_handle()
    for _ in range(reps):
        lookup()
graph.replay()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
graph.replay()
e1.record()
e1.synchronize()
t = e0.elapsed_time(e1) / reps * 1e-3
P = B * h * w
alg = P * (L * 100 * 4 + L * 81 * 4 + 8)
print(f"lookup B={B} spread={spread}: {t*1e6:.2f} us/launch, algorithmic {alg/1e6:.2f} MB -> {alg/t/1e9:.0f} GB/s")
for _ in range(reps):
    calib()
torch.cuda.synchronize()
print(f"calib copy: {calib_src.numel()*4/1e6:.1f} MB read + written per launch")

if os.environ.get("LKSTAMPS"):
    import ctypes
    import numpy as np
    lib = _lib.load()
    buf = np.zeros(8 * 65536, dtype=np.uint64)
    lib.raft_debug_lkstamps(ctypes.c_void_p(buf.ctypes.data), buf.size)
    st = buf.reshape(-1, 8).astype(np.float64)
    st = st[st[:, 0] > 0]
    st = st[st[:, 0] > st[:, 0].max() - 20000]
    m = st.mean(0)
    print(f"   lookup stamps, {len(st)} waves: span {(st[:, 1].max() - st[:, 0].min()) * 0.01:.2f} us, entry skew "
          f"{(st[:, 0].max() - st[:, 0].min()) * 0.01:.2f} us, life {((st[:, 1] - st[:, 0]) * 0.01).mean():.2f} us; "
          f"cycles: coords {m[2]:.0f} issue {m[3]:.0f} phase2+land {m[4]:.0f} taps {m[5]:.0f} stores {m[6]:.0f}")
