"""Run config-2 forwards (graph replay) for a rocprofv3 kernel trace; pair with tools/phase_summary.py.

    rocprofv3 --kernel-trace -d gpurun_out/fp -o run --output-format csv -- python tools/fwd_profile.py [B] [H] [W] [prec]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from raft_optical_flow_amd import RAFT  # noqa: E402
from raft_optical_flow_amd.init import seeded_state_dict  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
H = int(sys.argv[2]) if len(sys.argv) > 2 else 440
W = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
prec = sys.argv[4] if len(sys.argv) > 4 else "f16x3"
alt = os.environ.get("ALT", "0") == "1"
dev = torch.device("cuda:0")
m = RAFT(argparse.Namespace(small=False, mixed_precision=False, alternate_corr=alt))
m.load_state_dict(seeded_state_dict(m, 0))
m.to(dev).eval()
m.conv_precision = prec
g = torch.Generator().manual_seed(1)
i1 = (torch.rand(B, 3, H, W, generator=g) * 255).floor().to(dev)
i2 = (torch.rand(B, 3, H, W, generator=g) * 255).floor().to(dev)
with torch.no_grad():
    for _ in range(6):
        m(i1, i2, iters=32, test_mode=True)
torch.cuda.synchronize()
print("done")
