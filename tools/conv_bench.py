"""Time each update-block convolution shape of RAFT-full at B x 55 x 128 in isolation.

    python tools/conv_bench.py B [name,name...]      (PREC=fp32|f16x3|f16, default f16x3)"""
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from raft_optical_flow_amd import _lib
from raft_optical_flow_amd import kernels as K

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
ONLY = sys.argv[2].split(",") if len(sys.argv) > 2 else None
PREC = __import__("os").environ.get("PREC", "f16x3")
H, W = 55, 128
dev = "cuda"
SHAPES = [  # name, cin, cout, kh, kw, pad
    ("convc1", 324, 256, 1, 1, (0, 0)), ("convc2", 256, 192, 3, 3, (1, 1)), ("convf2", 128, 64, 3, 3, (1, 1)),
    ("conv", 256, 126, 3, 3, (1, 1)), ("zr", 384, 256, 1, 5, (0, 2)), ("q", 384, 128, 1, 5, (0, 2)),
    ("zr_split", 256, 256, 1, 5, (0, 2)), ("q_split", 256, 128, 1, 5, (0, 2)), ("fh1", 128, 256, 3, 3, (1, 1)), ("fh1mask", 128, 512, 3, 3, (1, 1)), ("mask2", 256, 576, 1, 1, (0, 0)),
    ("fh2", 256, 2, 3, 3, (1, 1)),
]
# encoder 3x3 convs at config 2 (fnet runs on both frames: B x 2), as (name, cin, cout, kh, kw, pad, b, h, w)
ENC = [("l1", 64, 64, 3, 3, (1, 1), 2, 220, 512), ("l2", 96, 96, 3, 3, (1, 1), 2, 110, 256),
       ("l3", 128, 128, 3, 3, (1, 1), 2, 55, 128)]
if __import__("os").environ.get("SHAPESET") == "enc":
    SHAPES = [(n, ci, co, kh, kw, pd) for n, ci, co, kh, kw, pd, _, _, _ in ENC]
    DIMS = {n: (bb * B, hh, ww) for n, _, _, _, _, _, bb, hh, ww in ENC}
else:
    DIMS = {}
tot_t = 0
for name, cin, cout, kh, kw, pad in SHAPES:
    if ONLY and name not in ONLY:
        continue
    Bq, H, W = DIMS.get(name, (B, int(__import__("os").environ.get("CB_H", 55)), int(__import__("os").environ.get("CB_W", 128))))
    x = torch.randn(Bq * H * W, cin, device=dev)
    w = torch.randn(cout, cin, kh, kw) * 0.05
    pc = K.pack_conv(w, torch.zeros(cout), 1, pad, device=dev)
    pc.precision = _lib.PRECISIONS[PREC]
    out = torch.empty(Bq * H * W, cout, device=dev)
    prm = K.conv_params(pc, K.Rows(x), Bq, H, W, K.Rows(out), epilogue=_lib.EPI_RELU)
    L = [K.conv_launch(prm)]
    if __import__("os").environ.get("HSTAMPS"):
        _lib.load().raft_debug_lstamps(None, 0, 1)
    for _ in range(3):
        L[0](K.stream_handle())
    torch.cuda.synchronize()
    # capture the repetitions in a hipGraph: the replay has no host launch overhead
    reps = 50
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s = K.stream_handle()
        for _ in range(reps):
            L[0](s)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    if __import__("os").environ.get("HSTAMPS"):
        import ctypes
        import numpy as np
        lib = _lib.load()
        buf = np.zeros(8 * 16384, dtype=np.uint64)
        lib.raft_debug_hstamps(ctypes.c_void_p(buf.ctypes.data), buf.size)
        st = buf.reshape(-1, 8).astype(np.float64)
        st = st[st[:, 0] > 0]
        st = st[st[:, 0] > st[:, 0].max() - 20000]  # the last launch (realtime ticks of 10 ns)
        mean = st.mean(0)
        span = (st[:, 1].max() - st[:, 0].min()) * 0.01
        clk = (st[:, 6] / np.maximum(st[:, 1] - st[:, 0], 1)).mean() * 100
        print(f"   halo stamps, {len(st)} compute waves: span {span:.1f} us, entry skew {(st[:, 0].max() - st[:, 0].min()) * 0.01:.1f} us, "
              f"clock {clk:.0f} MHz; cycles/wave: prologue {mean[2]:.0f} compute {mean[3]:.0f} "
              f"wait+barrier {mean[4]:.0f} epilogue {mean[5]:.0f} total {mean[6]:.0f}")
        lb = np.zeros(8 * 16384, dtype=np.uint64)
        lib.raft_debug_lstamps(ctypes.c_void_p(lb.ctypes.data), lb.size, 0)
        ls = lb.reshape(-1, 8).astype(np.float64)
        ls = ls[ls[:, 6] > 0]
        if len(ls):
            lm = ls.mean(0)
            print(f"   loader stamps, {len(ls)} waves (cycles in the last launch): "
                  f"patch store {lm[0]:.0f} patch load {lm[1]:.0f} weight DMA issue {lm[2]:.0f} vm wait {lm[3]:.0f} "
                  f"barrier {lm[4]:.0f} loop {lm[5]:.0f}")
    if __import__("os").environ.get("STAMPS"):
        import ctypes
        import numpy as np
        lib = _lib.load()
        buf = np.zeros(4 * 16384, dtype=np.uint64)
        lib.raft_debug_stamps(ctypes.c_void_p(buf.ctypes.data), buf.size)
        st = buf.reshape(-1, 4).astype(np.float64)
        st = st[st[:, 3] > 0]
        mean = st.mean(0)
        print(f"   stamps over {len(st)} waves (cycles per wave): work {mean[0]:.0f} barrier {mean[1]:.0f} "
              f"issue {mean[2]:.0f} loop {mean[3]:.0f}; max loop {st[:, 3].max():.0f}")
    fl = 2.0 * Bq * H * W * cout * cin * kh * kw
    tot_t += us
    print(f"{name:8s} M={Bq*H*W:6d} N={cout:4d} K={cin*kh*kw:5d}  {us:8.1f} us  {fl/us/1e6:7.1f} TF/s")
print(f"total {tot_t:.1f} us ({PREC})")
