"""Phase stamps of corr_build4_kernel (a -DCB4_STAMPS variant):

    make -C raft_optical_flow_amd/csrc variant NAME=cb4st DEFS=-DCB4_STAMPS
    RAFT_HIP_LIB=ab/cb4st/libraft_hip.so python tools/cb4_stamps.py [B H8 W8]

One raft_corr_build_ws launch; per-wave cycle means of each phase (waves 0 and 7) and units per
work-group."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raft_optical_flow_amd import _lib  # noqa: E402
from raft_optical_flow_amd import kernels as K  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
H = int(sys.argv[2]) if len(sys.argv) > 2 else 55
W = int(sys.argv[3]) if len(sys.argv) > 3 else 128
C, L = 256, 4
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
fm = torch.randn(2 * B * H * W, C, device=dev, generator=g)
f1, f2 = fm[: B * H * W], fm[B * H * W:]
pyr = torch.empty(K.pyramid_floats(B, H, W, L), device=dev)
lib = _lib.load()
wsb = int(lib.raft_corr_build_ws_bytes(B, H, W, C))
ws = torch.empty((wsb + 3) // 4, device=dev)
for _ in range(3):
    _lib.call("raft_corr_build_ws", f1.data_ptr(), f2.data_ptr(), C, B, H, W, C, L, K.sqrt_c(C), _lib.PREC_F16X3,
              pyr.data_ptr(), ws.data_ptr(), wsb, K.stream_handle())
torch.cuda.synchronize()
buf = np.zeros(8 * 8 * 1024, dtype=np.uint64)
lib.raft_debug_cb4stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
lib.raft_debug_cb4stamps(ctypes.c_void_p(buf.ctypes.data), buf.size)
st = buf.reshape(1024, 8, 8).astype(np.float64)
st = st[st[:, 0, 6] > 0]
names = ["DMA wait", "barrier", "DMA issue", "frag reads + MFMAs", "epilogue", "loop overhead"]
print(f"corr_build4 stamps B={B} {H}x{W}: {len(st)} work-groups, units per WG mean {st[:, 0, 7].mean():.2f}")
for wv in (0, 7):
    tot = st[:, wv, 6].mean()
    print(f"  wave {wv}: total {tot:.0f} cyc")
    for k, n in enumerate(names):
        v = st[:, wv, k].mean()
        print(f"    {n:28s} {v:9.0f} cyc {100 * v / tot:5.1f} %")
