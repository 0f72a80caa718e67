"""Dev diagnostic: RAFT-full forward under each engine knob vs all knobs off (same weights and
frames), and the encoders alone, to localise an end-to-end difference.
    python tools/diag_e2e.py"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raft_optical_flow_amd import RAFT  # noqa: E402
from raft_optical_flow_amd.init import seeded_state_dict, smooth_images  # noqa: E402

DEV = "cuda"
KNOBS = ["RAFT_FUSE_CONVC1", "RAFT_CONV_STEM", "RAFT_EPI_STATS", "RAFT_IN_NORM"]


def setk(on):
    for k in KNOBS:
        os.environ[k] = "1" if k in on else "0"


m = RAFT(argparse.Namespace(small=False, mixed_precision=False, alternate_corr=False))
m.load_state_dict(seeded_state_dict(m, 0))
m.to(DEV).eval()
i1, i2 = smooth_images(1, 128, 192, seed=3)
i1, i2 = i1.to(DEV), i2.to(DEV)
img = torch.cat([i1, i2])
with torch.no_grad():
    setk([])
    f0 = m.fnet(img)
    c0 = m.cnet(i1)
    _, up0 = m(i1, i2, iters=12, test_mode=True)
    for on in [[k] for k in KNOBS] + [KNOBS[1:], KNOBS, []]:
        setk(on)
        f = m.fnet(img)
        c = m.cnet(i1)
        _, up = m(i1, i2, iters=12, test_mode=True)
        print(f"{'+'.join(on) or 'none':60s} fnet {float((f - f0).abs().max()):.3e} cnet "
              f"{float((c - c0).abs().max()):.3e} flow {float((up - up0).abs().max()):.3e}", flush=True)
