"""Correlation-pyramid build alone (raft_corr_build_prec, f16x3, 4 levels, C = 256), 20 launches in a
hipGraph per tile order; prints microseconds per launch (best of 5 replays, orders interleaved).

    python tools/corr_build_bench.py [B [H8 W8]] [--orders "gm,nfast,xcd;..."]
    (H8 x W8 = the 1/8-resolution map: 55 128 = config 2, 135 240 = config 5; RAFT_HIP_LIB selects a
    variant library; an order "-" is the library default)"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raft_optical_flow_amd import _lib  # noqa: E402
from raft_optical_flow_amd import kernels as K  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("B", nargs="?", type=int, default=1)
ap.add_argument("H", nargs="?", type=int, default=55)
ap.add_argument("W", nargs="?", type=int, default=128)
ap.add_argument("--orders", default="-")
ap.add_argument("--reps", type=int, default=20)
args = ap.parse_args()
B, H, W, C, L = args.B, args.H, args.W, 256, 4
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
f1 = torch.randn(B * H * W, C, device=dev, generator=g)
f2 = torch.randn(B * H * W, C, device=dev, generator=g)
pyr = torch.empty(K.pyramid_floats(B, H, W, L), device=dev)


fm = torch.cat([f1, f2])
f1, f2 = fm[: B * H * W], fm[B * H * W:]


def launch():
    _lib.call("raft_corr_build_prec", f1.data_ptr(), f2.data_ptr(), C, B, H, W, C, L, K.sqrt_c(C),
              _lib.PREC_F16X3, pyr.data_ptr(), K.stream_handle())


orders = args.orders.split(";")
graphs = []
ref = None
for o in orders:
    if o == "-":
        os.environ.pop("RAFT_CB_ORDER", None)
    else:
        os.environ["RAFT_CB_ORDER"] = o
    for _ in range(2):
        launch()
    torch.cuda.synchronize()
    if ref is None:
        ref = pyr.clone()
    elif not torch.equal(ref, pyr):
        print(f"order {o}: pyramid differs from order {orders[0]}!")
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(args.reps):
            launch()
    graphs.append(gr)
os.environ.pop("RAFT_CB_ORDER", None)
best = [1e9] * len(orders)
for _ in range(5):
    for i, gr in enumerate(graphs):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        gr.replay()
        e1.record()
        e1.synchronize()
        best[i] = min(best[i], e0.elapsed_time(e1) / args.reps * 1e3)
mb = K.pyramid_floats(B, H, W, L) * 4 / 1e6
for o, t in zip(orders, best):
    print(f"corr build (+ pooling) B={B} {H}x{W} order {o}: {t:.1f} us per launch, {mb:.0f} MB pyramid "
          f"({mb / t:.2f} TB/s)")
