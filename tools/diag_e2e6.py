"""Dev diagnostic: run a fused RAFT plan's launch list by hand; after every raft_corr_lookup_conv
re-launch it and compare (does the in-sequence launch differ from a re-run on the same state?)."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from raft_optical_flow_amd import RAFT  # noqa: E402
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
ub = pl.ub
side = torch.cuda.Stream()
main = torch.cuda.current_stream()
for trial in range(3):
    pl.set_inputs(i1, i2)
    it = 0
    for l in pl.launches:
        if l is K.FORK:
            side.wait_stream(main)
            continue
        if l is K.JOIN:
            main.wait_stream(side)
            continue
        name = getattr(l, "name", "")
        if name == "raft_corr_lookup_conv" and os.environ.get("SYNC_BEFORE") == "1":
            torch.cuda.synchronize()
        l(side.cuda_stream if l.side else main.cuda_stream)
        if name == "raft_corr_lookup_conv":
            torch.cuda.synchronize()
            a = (ub.cor1.clone(), ub.flo1.clone(), ub.hx[:, 254:256].clone(), ub.coords.clone())
            l(main.cuda_stream)
            torch.cuda.synchronize()
            d = [float((x - y).abs().max()) for x, y in zip(a, (ub.cor1, ub.flo1, ub.hx[:, 254:256], ub.coords))]
            if max(d) > 0:
                print(f"trial {trial} iter {it}: in-sequence vs re-run cor1 {d[0]:.3e} flo1 {d[1]:.3e} flow {d[2]:.3e}",
                      flush=True)
            it += 1
    torch.cuda.synchronize()
    print(f"trial {trial}: flow_up[0,0,0,0] {float(pl.flow_up[-1][0, 0, 0, 0]):.6f}", flush=True)
