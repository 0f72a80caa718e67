"""Alternate-corr lookup (raft_alt_corr_lookup_nhwc) in isolation at the config-3 shape:
B x 55 x 128 query pixels, C = 256, r = 4, one launch per level (fmap2 pooled 2^l).
Usage: python tools/alt_bench.py [B] [spread_px]   (RAFT_HIP_LIB selects a library variant)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raft_optical_flow_amd import _lib  # noqa: E402
from raft_optical_flow_amd import kernels as K  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
spread = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
reps = int(os.environ.get("REPS", "20"))
h, w, L, r, C = 55, 128, 4, 4, 256
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
f1 = torch.randn(B, h, w, C, device=dev, generator=g)
f2s = [torch.randn(B, h >> l, w >> l, C, device=dev, generator=g) for l in range(L)]
ys, xs = torch.meshgrid(torch.arange(h, device=dev), torch.arange(w, device=dev), indexing="ij")
grid = torch.stack([xs, ys], -1).float().reshape(1, h * w, 2).repeat(B, 1, 1).reshape(-1, 2)
# a smooth flow field (per-tile divergence ~ spread) plus the grid
flow = spread * torch.randn(B, 2, 7, 16, device=dev, generator=g)
flow = torch.nn.functional.interpolate(flow, size=(h, w), mode="bilinear", align_corners=True)
coords = (grid + flow.permute(0, 2, 3, 1).reshape(-1, 2) * 4).contiguous()
ntap = L * (2 * r + 1) ** 2
out = torch.empty(B * h * w, ntap, device=dev)


ARRS = K.alt_levels_args([(f2s[l], h >> l, w >> l) for l in range(L)])
PER_LEVEL = os.environ.get("ALT_PER_LEVEL") == "1"  # L raft_alt_corr_lookup_nhwc calls instead of one levels call


def run():
    s = K.stream_handle()
    if not PER_LEVEL:
        _lib.call("raft_alt_corr_lookup_levels", f1.data_ptr(), *ARRS, L, coords.data_ptr(), 0, out.data_ptr(), ntap,
                  B, h, w, C, r, 16.0, None, 0, None, s)
        return
    for l in range(L):
        _lib.call("raft_alt_corr_lookup_nhwc", f1.data_ptr(), f2s[l].data_ptr(), coords.data_ptr(), 0, float(2 ** l),
                  out.data_ptr() + 4 * l * 81, ntap, B, h, w, h >> l, w >> l, C, r, 16.0, None, 0, None, s)


run()
torch.cuda.synchronize()
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph):
    for _ in range(reps):
        run()
graph.replay()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
graph.replay()
e1.record()
e1.synchronize()
t = e0.elapsed_time(e1) / reps * 1e-3
fl = 2 * B * h * w * L * (2 * r + 2) ** 2 * C
print(f"alt lookup B={B} spread={spread}: {t*1e6:.1f} us per iteration (4 levels), {fl/t/1e12:.2f} TF/s")
