"""Dev diagnostic: re-launch the forward's last raft_corr_lookup_conv on the forward's final state
and check its outputs for run-to-run differences; then per-iteration eager forwards."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from raft_optical_flow_amd import RAFT, _lib  # noqa: E402
from raft_optical_flow_amd import kernels as K  # noqa: E402
from raft_optical_flow_amd.init import seeded_state_dict, smooth_images  # noqa: E402

m = RAFT(argparse.Namespace(small=False, mixed_precision=False, alternate_corr=False))
m.load_state_dict(seeded_state_dict(m, 0))
m.to("cuda").eval()
m.hip_graph = False
i1, i2 = smooth_images(1, 128, 192, seed=3)
i1, i2 = i1.cuda(), i2.cuda()
with torch.no_grad():
    m(i1, i2, iters=12, test_mode=True)
torch.cuda.synchronize()
pl = next(iter(m._plans.values()))
lk = [l for l in pl.launches if getattr(l, "name", "") == "raft_corr_lookup_conv"]
ub = pl.ub
co = ub.coords.view(16, 24, 2)
print("final coords range x", float(co[..., 0].min()), float(co[..., 0].max()), "y", float(co[..., 1].min()),
      float(co[..., 1].max()))
ref = None
for rep in range(20):
    lk[-1](K.stream_handle())
    torch.cuda.synchronize()
    cur = (ub.cor1.clone(), ub.flo1.clone(), ub.hx[:, 254:256].clone())
    if ref is None:
        ref = cur
    else:
        d = [float((a - b).abs().max()) for a, b in zip(cur, ref)]
        if max(d) > 0:
            bad = (cur[0] - ref[0]).abs().amax(1).nonzero().flatten().tolist()
            print(f"rep {rep}: cor1 {d[0]:.3e} flo1 {d[1]:.3e} flow {d[2]:.3e}; cor1 rows differing {bad[:20]}")
print("done")
