"""Phase stamps of the alternate lookup's MFMA tile kernel (a -DALT_STAMPS variant):

    make -C raft_optical_flow_amd/csrc variant NAME=altst DEFS=-DALT_STAMPS
    RAFT_HIP_LIB=ab/altst/libraft_hip.so python tools/alt_stamps.py [B] [spread_px]

One raft_alt_corr_lookup_levels launch at the config-3 shape (tools/alt_bench.py's smooth
synthetic flow); prints per-wave cycle means of each phase for an MFMA wave (0) and a
non-MFMA wave (7), and bands per work-group."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raft_optical_flow_amd import _lib  # noqa: E402
from raft_optical_flow_amd import kernels as K  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
spread = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
h, w, L, r, C = 55, 128, 4, 4, 256
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
f1 = torch.randn(B, h, w, C, device=dev, generator=g)
f2s = [torch.randn(B, h >> l, w >> l, C, device=dev, generator=g) for l in range(L)]
ys, xs = torch.meshgrid(torch.arange(h, device=dev), torch.arange(w, device=dev), indexing="ij")
grid = torch.stack([xs, ys], -1).float().reshape(1, h * w, 2).repeat(B, 1, 1).reshape(-1, 2)
flow = spread * torch.randn(B, 2, 7, 16, device=dev, generator=g)
flow = torch.nn.functional.interpolate(flow, size=(h, w), mode="bilinear", align_corners=True)
coords = (grid + flow.permute(0, 2, 3, 1).reshape(-1, 2) * 4).contiguous()
ntap = L * (2 * r + 1) ** 2
out = torch.empty(B * h * w, ntap, device=dev)
ARRS = K.alt_levels_args([(f2s[l], h >> l, w >> l) for l in range(L)])


def run():
    _lib.call("raft_alt_corr_lookup_levels", f1.data_ptr(), *ARRS, L, coords.data_ptr(), 0, out.data_ptr(), ntap,
              B, h, w, C, r, 16.0, None, 0, None, K.stream_handle())


for _ in range(3):
    run()
torch.cuda.synchronize()
lib = _lib.load()
lib.raft_debug_altstamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
nwg = B * (-(-h // 8)) * (-(-w // 8))
buf = np.zeros(nwg * 8 * 24, dtype=np.uint64)
lib.raft_debug_altstamps(buf.ctypes.data, buf.size)
st = buf.reshape(nwg, 8, 24).astype(np.float64)
names = ["F1 tile", "level setup + band 0 issue", "band split + store (load wait)", "sync 1", "next band issue",
         "MFMAs", "sync 2", "S stores", "sync 3", "tap picks", "sync 4", "tap sums -> LDS + sync",
         "next level setup + issue", "binning + output stores", "flags, flow, final sync"]
print(f"alt mfma stamps B={B} spread={spread}: {nwg} work-groups, bands per WG mean {st[:, 0, 17].mean():.2f}")
for wv in (0, 7):
    tot = st[:, wv, 16].mean()
    print(f"  wave {wv}: total {tot:.0f} cyc")
    for k, n in enumerate(names):
        print(f"    {n:34s} {st[:, wv, k].mean():9.0f} cyc  {100 * st[:, wv, k].mean() / tot:5.1f} %")
