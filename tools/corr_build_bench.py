"""Correlation-pyramid build alone (raft_corr_build_prec, f16x3, config-2 geometry: B x 55 x 128 x 256,
4 levels), 20 launches in a hipGraph; prints microseconds per launch.

    python tools/corr_build_bench.py [B]      (RAFT_HIP_LIB selects a variant library)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raft_optical_flow_amd import _lib  # noqa: E402
from raft_optical_flow_amd import kernels as K  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
H, W, C, L = 55, 128, 256, 4
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
f1 = torch.randn(B * H * W, C, device=dev, generator=g)
f2 = torch.randn(B * H * W, C, device=dev, generator=g)
pyr = torch.empty(K.pyramid_floats(B, H, W, L), device=dev)


def launch():
    _lib.call("raft_corr_build_prec", f1.data_ptr(), f2.data_ptr(), C, B, H, W, C, L, K.sqrt_c(C), _lib.PREC_F16X3,
              pyr.data_ptr(), K.stream_handle())


for _ in range(3):
    launch()
torch.cuda.synchronize()
reps = 20
gr = torch.cuda.CUDAGraph()
with torch.cuda.graph(gr):
    for _ in range(reps):
        launch()
gr.replay()
torch.cuda.synchronize()
best = 1e9
for _ in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    gr.replay()
    e1.record()
    e1.synchronize()
    best = min(best, e0.elapsed_time(e1) / reps * 1e3)
print(f"corr build (+ pooling) B={B}: {best:.1f} us per launch, {K.pyramid_floats(B, H, W, L) * 4 / 1e6:.0f} MB pyramid")
