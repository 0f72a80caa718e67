"""The f16x3 correlation build two ways at one map size: raft_corr_build_prec (corr_build2, 128 x 128
tiles) vs raft_corr_build_ws (split maps + corr_build4, 256 x 256 tiles); microseconds per launch
(hipGraph of REPS launches, best of 5) and their max difference.

    python tools/corr4_bench.py [B H8 W8]     (55 128 = config 2's map, 135 240 = config 5's, 68 120 = config 4's)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raft_optical_flow_amd import _lib  # noqa: E402
from raft_optical_flow_amd import kernels as K  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
H = int(sys.argv[2]) if len(sys.argv) > 2 else 55
W = int(sys.argv[3]) if len(sys.argv) > 3 else 128
C, L, REPS = 256, 4, 10
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
fm = torch.randn(2 * B * H * W, C, device=dev, generator=g)
f1, f2 = fm[: B * H * W], fm[B * H * W:]
pyrs = [torch.empty(K.pyramid_floats(B, H, W, L), device=dev) for _ in range(2)]
wsb = int(_lib.load().raft_corr_build_ws_bytes(B, H, W, C))
ws = torch.empty((wsb + 3) // 4, device=dev)


def plain():
    _lib.call("raft_corr_build_prec", f1.data_ptr(), f2.data_ptr(), C, B, H, W, C, L, K.sqrt_c(C), _lib.PREC_F16X3,
              pyrs[0].data_ptr(), K.stream_handle())


def wsb_build():
    _lib.call("raft_corr_build_ws", f1.data_ptr(), f2.data_ptr(), C, B, H, W, C, L, K.sqrt_c(C), _lib.PREC_F16X3,
              pyrs[1].data_ptr(), ws.data_ptr(), wsb, K.stream_handle())


res = {}
for name, fn in (("corr_build2", plain), ("split+corr_build4", wsb_build)):
    fn()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(REPS):
            fn()
    best = 1e30
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        gr.replay()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / REPS * 1e3)
    res[name] = best
d = float((pyrs[0] - pyrs[1]).abs().max())
print(f"corr build B={B} {H}x{W}: " + ", ".join(f"{k} {v:.1f} us" for k, v in res.items()) +
      f"; max |diff| {d:.3g} (scale {float(pyrs[0].abs().max()):.3g})")
