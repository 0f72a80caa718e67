"""Dev diagnostic: determinism of the encoders (first call vs later calls, eager launches)."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from raft_optical_flow_amd import RAFT  # noqa: E402
from raft_optical_flow_amd.init import seeded_state_dict, smooth_images  # noqa: E402

m = RAFT(argparse.Namespace(small=False, mixed_precision=False, alternate_corr=False))
m.load_state_dict(seeded_state_dict(m, 0))
m.to("cuda").eval()
i1, i2 = smooth_images(1, 128, 192, seed=3)
img = torch.cat([i1, i2]).cuda()
with torch.no_grad():
    f = [m.fnet(img) for _ in range(4)]
    c = [m.cnet(img[:1]) for _ in range(4)]
print("fnet call diffs vs first", ["%.2e" % float((x - f[0]).abs().max()) for x in f[1:]],
      "cnet", ["%.2e" % float((x - c[0]).abs().max()) for x in c[1:]], flush=True)
