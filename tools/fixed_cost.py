"""Fixed vs per-K-step cost of the halo convs at B=1 (55x128): time one conv shape at several
input channel counts (hipGraph of 50 dependent launches each) and fit t = fixed + slope * K-steps.
Also times a trivial torch kernel the same way (the bare dependent-launch boundary).

    python tools/fixed_cost.py            (PREC=f16x3 default)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raft_optical_flow_amd import _lib
from raft_optical_flow_amd import kernels as K

PREC = os.environ.get("PREC", "f16x3")
dev = "cuda"
H, W = 55, 128


def graph_us(fn, reps=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps * 1e3)
    return best


t = torch.zeros(64, device=dev)
print(f"trivial torch kernel (dependent, in a graph): {graph_us(lambda: t.add_(1.0)):.2f} us")

for name, cout, kh, kw, pad in [("1x5 BN64", 256, 1, 5, (0, 2)), ("1x5 BN32", 128, 1, 5, (0, 2)),
                                 ("3x3 BN64", 256, 3, 3, (1, 1)), ("3x3 BN32", 128, 3, 3, (1, 1)),
                                 ("1x1 BN64", 256, 1, 1, (0, 0))]:
    pts = []
    for cin in (32, 64, 128, 256, 384):
        x = torch.randn(H * W, cin, device=dev)
        w = torch.randn(cout, cin, kh, kw) * 0.05
        pc = K.pack_conv(w, torch.zeros(cout), 1, pad, device=dev)
        pc.precision = _lib.PRECISIONS[PREC]
        out = torch.empty(H * W, cout, device=dev)
        prm = K.conv_params(pc, K.Rows(x), 1, H, W, K.Rows(out), epilogue=_lib.EPI_RELU)
        L = K.conv_launch(prm)
        us = graph_us(lambda: L(K.stream_handle()))
        ksteps = (cin // 32) * kh * kw
        pts.append((ksteps, us))
        print(f"  {name} cin {cin:4d}: {ksteps:4d} K-steps  {us:7.2f} us", flush=True)
    n = len(pts)
    mx = sum(p[0] for p in pts) / n
    my = sum(p[1] for p in pts) / n
    sl = sum((p[0] - mx) * (p[1] - my) for p in pts) / sum((p[0] - mx) ** 2 for p in pts)
    print(f"{name}: fixed {my - sl * mx:.2f} us + {sl * 1000:.1f} ns per K-step")
