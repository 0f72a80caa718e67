"""Time InstanceNorm stats + apply (raft_instnorm_*) at the fnet shapes of config 2 (2 images).

    python tools/norm_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raft_optical_flow_amd import _lib
from raft_optical_flow_amd import kernels as K

dev = "cuda"
lib = _lib.load()


def graph_us(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for n, h, w, c in [(2, 220, 512, 64), (2, 110, 256, 96), (2, 55, 128, 128)]:
    hw = h * w
    x = torch.randn(n * hw, c, device=dev)
    r = torch.randn(n * hw, c, device=dev)
    out = torch.empty_like(x)
    st = torch.empty(2 * n * c, device=dev)
    ws = torch.empty(max(1, lib.raft_instnorm_workspace_floats(n, hw, c)), device=dev)

    def stats():
        _lib.call("raft_instnorm_stats", x.data_ptr(), c, n, hw, c, 1e-5, st.data_ptr(), ws.data_ptr(), K.stream_handle())

    def apply():
        _lib.call("raft_instnorm_apply", x.data_ptr(), c, st.data_ptr(), r.data_ptr(), c, None, 2, out.data_ptr(), c, n,
                  hw, c, K.stream_handle())

    ts, ta = graph_us(stats), graph_us(apply)
    mb = x.numel() * 4 / 1e6
    print(f"{n}x{h}x{w}x{c}: stats {ts:7.1f} us ({mb / ts * 1e3:6.0f} GB/s)  apply+resid {ta:7.1f} us "
          f"({3 * mb / ta * 1e3:6.0f} GB/s)")
    # numerics vs torch
    xx = x.view(n, hw, c).double()
    mean, var = xx.mean(1), xx.var(1, unbiased=False)
    ref = torch.relu(r.view(n, hw, c).double() + torch.relu((xx - mean[:, None]) / torch.sqrt(var[:, None] + 1e-5)))
    print("   max err vs fp64", float((out.view(n, hw, c).double() - ref).abs().max()))
