"""One encoder-shaped 3x3 conv (64 -> 64, 2 x 220 x 512, f16x3) launched back to back: the weight-resident
kernel (default) or the halo kernel (RAFT_RESIDENT=0); prints the mean launch time (HIP events around a
graph of the launches).   python tools/res_bench.py [norm] [cin] [H] [W] [B]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from raft_optical_flow_amd import _lib  # noqa: E402
from raft_optical_flow_amd import kernels as K  # noqa: E402

norm = len(sys.argv) > 1 and sys.argv[1] == "norm"
cin = int(sys.argv[2]) if len(sys.argv) > 2 else 64
H = int(sys.argv[3]) if len(sys.argv) > 3 else 220
W = int(sys.argv[4]) if len(sys.argv) > 4 else 512
B = int(sys.argv[5]) if len(sys.argv) > 5 else 2
cout = cin
dev = "cuda"
g = torch.Generator().manual_seed(1)
x = torch.randn(B, cin, H, W, generator=g)
w = torch.randn(cout, cin, 3, 3, generator=g) / np.sqrt(cin * 9)
pc = K.pack_conv(w, torch.zeros(cout), 1, 1, device=dev)
pc.precision = _lib.PREC_F16X3
src = K.Rows(K.nchw_to_rows(x.to(dev)))
out = K.Rows(torch.empty(B * H * W, cout, device=dev))
p = K.conv_params(pc, src, B, H, W, out)
if norm:
    st = torch.stack([torch.zeros(B, cin), torch.ones(B, cin)], -1).contiguous().to(dev)
    p.in_norm, p.in_norm_relu = st.data_ptr(), 1
launch = K.conv_launch(p)
for _ in range(3):
    launch(K.stream_handle())
torch.cuda.synchronize()
gr = torch.cuda.CUDAGraph()
with torch.cuda.graph(gr):
    for _ in range(20):
        launch(K.stream_handle())
gr.replay()
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
gr.replay()
b.record()
b.synchronize()
us = a.elapsed_time(b) / 20 * 1e3
fl = 2.0 * B * H * W * cout * cin * 9
print(f"resident={os.environ.get('RAFT_RESIDENT', '1')} norm={norm} cin={cin} {B}x{H}x{W}: {us:.1f} us "
      f"({fl / us / 1e6:.1f} TF/s fp32-equiv)")
