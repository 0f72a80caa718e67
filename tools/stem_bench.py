"""The encoders' 7x7 / stride-2 stem (conv_stem_kernel) alone at config 2's feature-network shape
(B = 2 frames of 440 x 1024 -> 220 x 512 x 64, linear epilogue + InstanceNorm partials, as the forward
runs it): microseconds per launch (hipGraph of 20 launches, best of 5).

    python tools/stem_bench.py [B H W]      (PREC=f16x3|bf16|f16, default f16x3)"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raft_optical_flow_amd import _lib  # noqa: E402
from raft_optical_flow_amd import kernels as K  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 2
H = int(sys.argv[2]) if len(sys.argv) > 2 else 440
W = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
PREC = os.environ.get("PREC", "f16x3")
dev = "cuda"
g = torch.Generator().manual_seed(0)
x = torch.randn(B * H * W, 3, generator=g).to(dev)
w = torch.randn(64, 3, 7, 7, generator=g) * 0.1
pc = K.pack_conv(w, torch.zeros(64), 2, 3, mode=_lib.RAFT_CONV_GATHER, device=dev)
pc.precision = _lib.PRECISIONS[PREC]
ho, wo = K.conv_out_hw(pc, H, W)
out = torch.empty(B * ho * wo, 64, device=dev)
p = K.conv_params(pc, K.Rows(x), B, H, W, K.Rows(out))
slots = _lib.load().raft_conv2d_stats_slots(ctypes.byref(p))
part = torch.empty(B * slots * 64 * 4, device=dev)
p.stats_part, p.stats_ld = part.data_ptr(), 64
fn = K.conv_launch(p)
fn(K.stream_handle())
torch.cuda.synchronize()
REPS = 20
gr = torch.cuda.CUDAGraph()
with torch.cuda.graph(gr):
    for _ in range(REPS):
        fn(K.stream_handle())
best = 1e30
for _ in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    gr.replay()
    e1.record()
    e1.synchronize()
    best = min(best, e0.elapsed_time(e1) / REPS * 1e3)
fl = 2.0 * B * ho * wo * 64 * 147
print(f"stem B={B} {H}x{W} -> {ho}x{wo} ({PREC}): {best:.1f} us, {fl / best / 1e6:.1f} TF/s, "
      f"{B * ho * wo * 64 * 4 / best / 1e3:.0f} GB/s of output")
