"""Phase stamps of the fused lookup + convc1 + convf1 kernel (a -DLC_STAMPS variant):

    make -C raft_optical_flow_amd/csrc variant NAME=lcst DEFS=-DLC_STAMPS
    RAFT_HIP_LIB=ab/lcst/libraft_hip.so python tools/lc_stamps.py

Runs config 2 forwards eagerly, then replays the last iteration's fused launch alone once and
prints per-wave cycle means of each phase and the launch's wall span (100 MHz realtime).
--h/--w/--precision select another workload (config 5: --h 1080 --w 1920 --precision bf16)."""
import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from raft_optical_flow_amd import RAFT, _lib  # noqa: E402
from raft_optical_flow_amd import kernels as K  # noqa: E402
from raft_optical_flow_amd.init import seeded_images, seeded_state_dict  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--h", type=int, default=440)
ap.add_argument("--w", type=int, default=1024)
ap.add_argument("--precision", default=None)
args = ap.parse_args()
dev = torch.device("cuda:0")
m = RAFT(argparse.Namespace(small=False, mixed_precision=False, alternate_corr=False))
m.load_state_dict(seeded_state_dict(m, 0))
m.to(dev).eval()
m.hip_graph = False
if args.precision:
    m.conv_precision = args.precision
i1, i2 = seeded_images(1, args.h, args.w, seed=1)
with torch.no_grad():
    for _ in range(2):
        m(i1.to(dev), i2.to(dev), iters=32, test_mode=True)
pl = next(iter(m._plans.values()))
lk = [l for l in pl.launches if getattr(l, "name", "") == "raft_corr_lookup_conv"]
lib = _lib.load()
lib.raft_debug_lcstamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
for rep in range(3):
    torch.cuda.synchronize()
    lk[-1](K.stream_handle())
    torch.cuda.synchronize()
nwg = 2048
buf = np.zeros(nwg * 8 * 16, dtype=np.uint64)
lib.raft_debug_lcstamps(buf.ctypes.data, buf.size)
s = buf.reshape(nwg * 8, 16).astype(np.int64)
s = s[s[:, 1] > 0]
print(f"  {s.shape[0]} waves stamped")
r0, r1, t = s[:, 0], s[:, 1], s[:, 2:9]
names = ["issue loads", "axis entries + flow patch", "taps x4 (tile wait incl.)", "sync + convf1 A + sync",
         "GEMMs", "epilogues"]
d = np.diff(t, axis=1)
for k, n in enumerate(names):
    print(f"  {n:26s} mean {d[:, k].mean():8.0f} cyc  max {d[:, k].max():8.0f}")
print(f"  total per wave mean {(t[:, 6] - t[:, 0]).mean():.0f} cycles")
c7 = s[:, 9]
if (c7 > 0).all():
    print(f"  (issue loads = coords round trip {(c7 - t[:, 0]).mean():.0f} + tile issue {(t[:, 1] - c7).mean():.0f} cyc)")
print(f"  launch span (realtime 100 MHz): {(r1.max() - r0.min()) / 100:.2f} us; wave mean {(r1 - r0).mean() / 100:.2f} us;"
      f" start spread {(r0.max() - r0.min()) / 100:.2f} us")
# resident rounds: the start times of the work-groups, in 1 us bins
st = np.sort((r0 - r0.min()) / 100)
print("  wave starts by us: " + " ".join(str(int(c)) for c in np.bincount(st.astype(np.int64))[:64]))
